// api_misc.hip -- C ABI of SURVEY.md §8f rank 4: distinctive descriptors and
// keypoint undistortion.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>

#include "../../include/orbx.h"
#include "api_common.h"

namespace orbx {
struct UndistortArgs {
  double fx, fy, cx, cy, ifx, ify;
  double k[14];
};
__global__ void k_distinctive(const uint8_t*, const int32_t*, int, int32_t*);
__global__ void k_undistort(const orbx_keypoint*, int, const UndistortArgs, orbx_keypoint*);
__global__ void k_boundary_copy(const uint8_t*, size_t, const uint8_t*, size_t, const uint8_t*, size_t,
                                uint8_t*, int, uint8_t*, uint8_t*, uint8_t*);
}  // namespace orbx

using namespace orbx;

static int check_device(int device) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return ORBX_ERR_NO_DEVICE;
  return hipSetDevice(device) == hipSuccess ? ORBX_OK : ORBX_ERR_HIP;
}

extern "C" int orbm_compute_distinctive_descriptors(const uint8_t* desc, const int32_t* off,
                                                    int nmp, int device, int32_t* best) {
  if (nmp < 0 || (nmp > 0 && (!off || !best))) return ORBX_ERR_ARG;
  if (nmp == 0) return ORBX_OK;
  const int total = off[nmp];
  if (off[0] != 0 || total < 0 || (total > 0 && !desc)) return ORBX_ERR_ARG;
  for (int m = 0; m < nmp; ++m)
    if (off[m + 1] < off[m] || off[m + 1] - off[m] > (1 << 20)) return ORBX_ERR_ARG;
  int rc = check_device(device);
  if (rc) return rc;
  WsLease L(device);
  CallWs* w = L.w;
  if (!w) return ORBX_ERR_HIP;
  Carve C;
  const size_t o_desc = C.take((size_t)total * 32), o_off = C.take((size_t)(nmp + 1) * 4);
  const size_t in_end = C.off, o_best = C.take((size_t)nmp * 4);
  rc = w->reserve(C.off, C.off);
  if (rc) return rc;
  if (total) memcpy(w->h + o_desc, desc, (size_t)total * 32);
  memcpy(w->h + o_off, off, (size_t)(nmp + 1) * 4);
  if (stage_in(w->d, w->h, in_end, w->stream)) return ORBX_ERR_HIP;
  hipLaunchKernelGGL(k_distinctive, dim3((nmp + 3) / 4), dim3(256), 0, w->stream, w->d + o_desc,
                     reinterpret_cast<const int32_t*>(w->d + o_off), nmp,
                     reinterpret_cast<int32_t*>(w->d + o_best));
  if (hipGetLastError() != hipSuccess) return ORBX_ERR_HIP;
  ORBX_TRY(hipMemcpyAsync(w->h + o_best, w->d + o_best, (size_t)nmp * 4, hipMemcpyDeviceToHost,
                          w->stream));
  ORBX_TRY(stream_wait(w->stream));
  memcpy(best, w->h + o_best, (size_t)nmp * 4);
  return ORBX_OK;
}

extern "C" int orbx_undistort_keypoints(const orbx_keypoint* kps, int n, const float* K,
                                        const float* dist, int ndist, int device,
                                        orbx_keypoint* out) {
  if (n < 0 || !K || (ndist > 0 && !dist) || ndist < 0 || ndist > 14 || (n > 0 && (!kps || !out)))
    return ORBX_ERR_ARG;
  if (n == 0) return ORBX_OK;
  if (ndist == 0 || dist[0] == 0.0f) { /* mvKeysUn = mvKeys (:386-390) */
    memmove(out, kps, n * sizeof(orbx_keypoint));
    return ORBX_OK;
  }
  int rc = check_device(device);
  if (rc) return rc;
  UndistortArgs A;
  memset(&A, 0, sizeof(A));
  A.fx = K[0];
  A.fy = K[4];
  A.cx = K[2];
  A.cy = K[5];
  A.ifx = 1. / A.fx;
  A.ify = 1. / A.fy;
  for (int j = 0; j < ndist; ++j) A.k[j] = dist[j];
  WsLease L(device);
  CallWs* w = L.w;
  if (!w) return ORBX_ERR_HIP;
  Carve C;
  const size_t o_in = C.take((size_t)n * sizeof(orbx_keypoint));
  const size_t o_out = C.take((size_t)n * sizeof(orbx_keypoint));
  rc = w->reserve(C.off, C.off);
  if (rc) return rc;
  memcpy(w->h + o_in, kps, (size_t)n * sizeof(orbx_keypoint));
  if (stage_in(w->d + o_in, w->h + o_in, ((size_t)n * sizeof(orbx_keypoint) + 15) & ~(size_t)15, w->stream))
    return ORBX_ERR_HIP;
  hipLaunchKernelGGL(k_undistort, dim3((n + 255) / 256), dim3(256), 0, w->stream,
                     reinterpret_cast<const orbx_keypoint*>(w->d + o_in), n, A,
                     reinterpret_cast<orbx_keypoint*>(w->d + o_out));
  if (hipGetLastError() != hipSuccess) return ORBX_ERR_HIP;
  ORBX_TRY(hipMemcpyAsync(w->h + o_out, w->d + o_out, (size_t)n * sizeof(orbx_keypoint),
                          hipMemcpyDeviceToHost, w->stream));
  ORBX_TRY(stream_wait(w->stream));
  memcpy(out, w->h + o_out, (size_t)n * sizeof(orbx_keypoint));
  return ORBX_OK;
}

extern "C" size_t orbx_boundary_record_bytes(int kcap) {
  return kcap > 0 ? (size_t)kcap * (sizeof(orbx_keypoint) + 32) + 16 : 0;
}

static int boundary_copy(int kcap, const void* a, const void* b, const void* c, void* rec, int unpack,
                         void* oa, void* ob, void* oc, void* stream) {
  if (kcap < 1) return ORBX_ERR_ARG;
  const size_t na = (size_t)kcap * sizeof(orbx_keypoint), nb = (size_t)kcap * 32, nc = 4;
  const size_t n = na + nb + nc;
  const unsigned blocks = (unsigned)std::min<size_t>((n + 4095) / 4096, 1024);
  hipLaunchKernelGGL(k_boundary_copy, dim3(blocks), dim3(256), 0, (hipStream_t)stream,
                     (const uint8_t*)a, na, (const uint8_t*)b, nb, (const uint8_t*)c, nc,
                     (uint8_t*)rec, unpack, (uint8_t*)oa, (uint8_t*)ob, (uint8_t*)oc);
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_ERR_HIP;
}

extern "C" int orbx_boundary_pack(const orbx_keypoint* d_kps, const uint8_t* d_desc,
                                  const int* d_count, int kcap, uint8_t* d_record, void* stream) {
  if (!d_kps || !d_desc || !d_count || !d_record) return ORBX_ERR_ARG;
  return boundary_copy(kcap, d_kps, d_desc, d_count, d_record, 0, nullptr, nullptr, nullptr, stream);
}

extern "C" int orbx_boundary_unpack(const uint8_t* d_record, int kcap, orbx_keypoint* d_kps,
                                    uint8_t* d_desc, int* d_count, void* stream) {
  if (!d_kps || !d_desc || !d_count || !d_record) return ORBX_ERR_ARG;
  return boundary_copy(kcap, d_record, nullptr, nullptr, nullptr, 1, d_kps, d_desc, d_count, stream);
}
