// api_common.h -- host helpers shared by the C-ABI translation units.
#ifndef ORBX_API_COMMON_H
#define ORBX_API_COMMON_H

#include <hip/hip_runtime.h>

#include <vector>

#include "../../include/orbx.h"

#define ORBX_TRY(expr)                              \
  do {                                              \
    if ((expr) != hipSuccess) return ORBX_ERR_HIP;  \
  } while (0)

enum {
  ORBX_STAGE_RESIZE = 0,
  ORBX_STAGE_FAST,
  ORBX_STAGE_QUADTREE,
  ORBX_STAGE_BLUR,
  ORBX_STAGE_BRIEF,
  ORBX_STAGE_MSELECT,
  ORBX_STAGE_MCAND,
  ORBX_STAGE_MRESOLVE,
  ORBX_STAGE_MFINAL,
  ORBX_STAGE_SROWS,
  ORBX_STAGE_SMATCH,
  ORBX_STAGE_SFILTER,
  ORBX_NSTAGES
};

namespace orbx {

// HIP events recorded around every launch group of a stage, on the stream
// the kernels run on.  collect() must be called after that stream is idle.
struct StageTimer {
  bool enabled = false;
  struct Rec {
    int stage;
    hipEvent_t a, b;
  };
  std::vector<Rec> recs;
  std::vector<hipEvent_t> pool;
  hipEvent_t pending[ORBX_NSTAGES] = {};

  hipEvent_t get() {
    if (!pool.empty()) {
      hipEvent_t e = pool.back();
      pool.pop_back();
      return e;
    }
    hipEvent_t e = nullptr;
    hipEventCreate(&e);
    return e;
  }
  void begin(int stage, hipStream_t s) {
    if (!enabled) return;
    pending[stage] = get();
    hipEventRecord(pending[stage], s);
  }
  void end(int stage, hipStream_t s) {
    if (!enabled || !pending[stage]) return;
    hipEvent_t b = get();
    hipEventRecord(b, s);
    recs.push_back({stage, pending[stage], b});
    pending[stage] = nullptr;
  }
  void reset(bool en) {
    for (auto& r : recs) {
      pool.push_back(r.a);
      pool.push_back(r.b);
    }
    recs.clear();
    enabled = en;
  }
  int collect(double* ms, int* launches, int n) {
    for (int i = 0; i < n; ++i) {
      if (ms) ms[i] = 0;
      if (launches) launches[i] = 0;
    }
    for (auto& r : recs) {
      float t = 0;
      if (hipEventElapsedTime(&t, r.a, r.b) != hipSuccess) return ORBX_ERR_HIP;
      if (r.stage < n) {
        if (ms) ms[r.stage] += t;
        if (launches) launches[r.stage] += 1;
      }
    }
    reset(enabled);
    return ORBX_OK;
  }
  void release() {
    reset(false);
    for (auto e : pool) hipEventDestroy(e);
    pool.clear();
  }
};

// ---------------------------------------------------------------------------
// Per-call workspaces of the synchronous drop-in entry points
// (orbm_search_by_bow, orbm_descriptor_distance_batch,
// orbm_search_by_projection, ...): a grow-only device arena, a grow-only
// pinned host staging buffer and a non-blocking stream.  Workspaces live in a
// per-device pool: a call takes one (a concurrent call takes another, so the
// entry points stay re-entrant from the Tracking / LocalMapping /
// LoopClosing threads) and returns it; steady-state calls do no hipMalloc,
// hipFree or stream creation, and never synchronise the device.
// ---------------------------------------------------------------------------
struct CallWs {
  int device = -1;
  hipStream_t stream = nullptr;
  uint8_t* d = nullptr;  // device arena
  size_t dcap = 0;
  uint8_t* h = nullptr;  // pinned host staging
  size_t hcap = 0;
  // grow-only; a grow waits for this workspace's stream only
  int reserve(size_t dbytes, size_t hbytes);
};

// arena carving: 256-B aligned offsets
struct Carve {
  size_t off = 0;
  size_t take(size_t bytes) {
    const size_t o = off;
    off += (bytes + 255) & ~(size_t)255;
    return o;
  }
};

CallWs* ws_acquire(int device);  // after hipSetDevice(device); nullptr on failure
void ws_release(CallWs* w);

// RAII lease of a pooled workspace
struct WsLease {
  CallWs* w;
  explicit WsLease(int device) : w(ws_acquire(device)) {}
  ~WsLease() {
    if (w) ws_release(w);
  }
  WsLease(const WsLease&) = delete;
  WsLease& operator=(const WsLease&) = delete;
};

// Completion wait of the synchronous drop-in calls: the caller (Tracking,
// LoopClosing) blocks on the result anyway, so the stream is polled for up
// to ORBX_SPIN_US microseconds before falling back to hipStreamSynchronize,
// whose blocking wake-up showed up as 2-4x p50 outliers in the per-call
// latency (bench latency leg).
hipError_t stream_wait(hipStream_t s);

// hipFuncAttributeMaxDynamicSharedMemorySize is process-wide per kernel:
// set it once per (kernel, device) to the CU's whole LDS, never per call (a
// concurrent call writing a smaller value could undercut a larger launch).
int set_max_dynamic_lds(const void* kernel, int device);

// a drop-in call's inputs [0, bytes) from its pinned staging buffer h into
// its device arena d, on stream s: a kernel (k_stage_in) when
// ORBM_STAGE_KERNEL, else a DMA copy.  bytes: a multiple of 16 (Carve's
// 256-byte blocks)
int stage_in(void* d, const void* h, size_t bytes, hipStream_t s);
// its results [.., + bytes) from the device arena d back into the pinned
// staging h (device-accessible host memory): the copy kernel writing host
// memory when ORBM_STAGE_KERNEL, else a DMA copy.  bytes: a multiple of 16
int stage_out(void* h, const void* d, size_t bytes, hipStream_t s);

}  // namespace orbx

#endif
