// api_ws.hip -- pooled per-call workspaces and one-time kernel attributes
// for the synchronous drop-in entry points (api_common.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <thread>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

#include "api_common.h"
#include "match_internal.h"

namespace orbx {

namespace {
std::mutex g_pool_mu;
std::map<int, std::vector<CallWs*>>* g_pool = nullptr;  // never freed: process lifetime
std::mutex g_attr_mu;
std::map<std::pair<const void*, int>, int>* g_attr = nullptr;
}  // namespace

int CallWs::reserve(size_t dbytes, size_t hbytes) {
  if (dbytes > dcap) {
    if (d) {
      if (hipStreamSynchronize(stream) != hipSuccess) return ORBX_ERR_HIP;
      hipFree(d);
      d = nullptr;
      dcap = 0;
    }
    const size_t n = dbytes + dbytes / 2 + 4096;
    if (hipMalloc((void**)&d, n) != hipSuccess) return ORBX_ERR_HIP;
    dcap = n;
  }
  if (hbytes > hcap) {
    if (h) {
      if (hipStreamSynchronize(stream) != hipSuccess) return ORBX_ERR_HIP;
      hipHostFree(h);
      h = nullptr;
      hcap = 0;
    }
    const size_t n = hbytes + hbytes / 2 + 4096;
    if (hipHostMalloc((void**)&h, n, hipHostMallocDefault) != hipSuccess) return ORBX_ERR_HIP;
    hcap = n;
  }
  return ORBX_OK;
}

CallWs* ws_acquire(int device) {
  {
    std::lock_guard<std::mutex> g(g_pool_mu);
    if (!g_pool) g_pool = new std::map<int, std::vector<CallWs*>>();
    std::vector<CallWs*>& v = (*g_pool)[device];
    if (!v.empty()) {
      CallWs* w = v.back();
      v.pop_back();
      return w;
    }
  }
  CallWs* w = new CallWs();
  w->device = device;
  if (hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking) != hipSuccess) {
    delete w;
    return nullptr;
  }
  return w;
}

void ws_release(CallWs* w) {
  // an early error return may leave copies into / out of the pinned staging
  // buffer or kernels queued on the workspace's stream: the next user must
  // not see them, so a busy stream is drained first, and a workspace whose
  // stream cannot be drained is destroyed instead of pooled
  if (hipStreamQuery(w->stream) != hipSuccess && hipStreamSynchronize(w->stream) != hipSuccess) {
    (void)hipGetLastError();
    hipSetDevice(w->device);
    if (w->d) hipFree(w->d);
    if (w->h) hipHostFree(w->h);
    hipStreamDestroy(w->stream);
    delete w;
    return;
  }
  std::lock_guard<std::mutex> g(g_pool_mu);
  (*g_pool)[w->device].push_back(w);
}

// Spin budget: about twice the p99 of the slowest synchronous call (the
// compat operator() with the pyramid, ~270 us at 1080p), so a call that
// completes on time never pays the blocking wake-up, and a caller on a
// shared or busy GPU holds a core for at most this long before sleeping in
// hipStreamSynchronize (it was 20 ms: the Tracking, LocalMapping and
// LoopClosing threads could each spin a core that long).  After the first
// 50 us the loop yields between polls.
#ifndef ORBX_SPIN_US
#define ORBX_SPIN_US 600
#endif
hipError_t stream_wait(hipStream_t s) {
  const auto t0 = std::chrono::steady_clock::now();
  const auto t_yield = t0 + std::chrono::microseconds(50);
  const auto t_end = t0 + std::chrono::microseconds(ORBX_SPIN_US);
  for (;;) {
    const hipError_t q = hipStreamQuery(s);
    if (q != hipErrorNotReady) return q;
    const auto now = std::chrono::steady_clock::now();
    if (now >= t_end) return hipStreamSynchronize(s);
    if (now >= t_yield) std::this_thread::yield();
    else __builtin_ia32_pause();
  }
}

__global__ void k_stage_in(uint4*, const uint4*, size_t);  // kernels_match.hip

int stage_in(void* d, const void* h, size_t bytes, hipStream_t s) {
#if ORBM_STAGE_KERNEL
  const size_t n16 = bytes / 16;
  if (n16 == 0) return ORBX_OK;
  hipLaunchKernelGGL(k_stage_in, dim3((unsigned)std::min<size_t>((n16 + 255) / 256, 1024)), dim3(256), 0, s,
                     reinterpret_cast<uint4*>(d), reinterpret_cast<const uint4*>(h), n16);
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_ERR_HIP;
#else
  return hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s) == hipSuccess ? ORBX_OK : ORBX_ERR_HIP;
#endif
}

int stage_out(void* h, const void* d, size_t bytes, hipStream_t s) {
#if ORBM_STAGE_KERNEL
  // the same copy kernel, the pinned buffer as the destination: the GPU
  // writes the results over PCIe, no DMA copy and its completion handover
  const size_t n16 = bytes / 16;
  if (n16 == 0) return ORBX_OK;
  hipLaunchKernelGGL(k_stage_in, dim3((unsigned)std::min<size_t>((n16 + 255) / 256, 1024)), dim3(256), 0, s,
                     reinterpret_cast<uint4*>(h), reinterpret_cast<const uint4*>(d), n16);
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_ERR_HIP;
#else
  return hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s) == hipSuccess ? ORBX_OK : ORBX_ERR_HIP;
#endif
}

int set_max_dynamic_lds(const void* kernel, int device) {
  std::lock_guard<std::mutex> g(g_attr_mu);
  if (!g_attr) g_attr = new std::map<std::pair<const void*, int>, int>();
  auto key = std::make_pair(kernel, device);
  auto it = g_attr->find(key);
  if (it != g_attr->end()) return it->second;
  int lds = 0, optin = 0;
  int rc = ORBX_OK;
  if (hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, device) != hipSuccess)
    rc = ORBX_ERR_HIP;
  if (hipDeviceGetAttribute(&optin, hipDeviceAttributeSharedMemPerBlockOptin, device) == hipSuccess &&
      optin > lds)
    lds = optin;
  // the dynamic maximum excludes the kernel's static __shared__ arrays
  hipFuncAttributes fa;
  if (rc == ORBX_OK && hipFuncGetAttributes(&fa, kernel) != hipSuccess) rc = ORBX_ERR_HIP;
  if (rc == ORBX_OK &&
      hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          lds - (int)fa.sharedSizeBytes) != hipSuccess)
    rc = ORBX_ERR_HIP;
  if (rc != ORBX_OK) (void)hipGetLastError(); /* do not leave a sticky error for the caller */
  (*g_attr)[key] = rc;
  return rc;
}

}  // namespace orbx
