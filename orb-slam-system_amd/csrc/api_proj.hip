// api_proj.hip -- C ABI of the frame grid + ORBmatcher::SearchByProjection
// (query form, /root/reference/src/ORBmatcher.cc:19-61,732-818,820-894).
#include <hip/hip_runtime.h>

#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/orbx.h"
#include "api_common.h"

namespace orbx {
struct ProjFrame {
  int n;
  float minX, minY, wInv, hInv;
};
struct ProjProblem {  // kernels_proj.hip
  ProjFrame F;
  const orbx_keypoint* keys;
  const uint8_t* desc;
  const float* uright;
  const uint8_t* occupied;
  const orbx_query_proj* qs;
  const uint8_t* qdesc;
  int nq;
  int32_t* match;
  int* nmatches;
  int* cell_off;
  int* cell_feat;
  uint32_t* cand;
  int* ncand;
};
__global__ void k_grid_build(const ProjProblem*);
__global__ void k_proj_cand(const ProjProblem*, int);
__global__ void k_proj_resolve(const ProjProblem*, int, float, int, int);
}  // namespace orbx

using namespace orbx;

#define PJ_T 8
#define PJ_MAXN 8192
#define PG_CELLS (64 * 48)

static ProjFrame proj_frame(const orbx_proj_frame* F) {
  ProjFrame PF;
  PF.n = F->n;
  PF.minX = F->min_x;
  PF.minY = F->min_y;
  PF.wInv = F->grid_w_inv;
  PF.hInv = F->grid_h_inv;
  return PF;
}

// the three launches over nprob problems (device table d_probs): grid per
// problem, candidates per (query, problem), the greedy walk per problem
static void launch_proj(const ProjProblem* d_probs, int nprob, int max_n, int max_nq, int mode,
                        float nnratio, int th_dist, int check_ori, hipStream_t s) {
  int P = 1;
  while (P < max_n) P <<= 1;
  hipLaunchKernelGGL(k_grid_build, dim3((unsigned)nprob), dim3(1024), (size_t)P * 4, s, d_probs);
  if (max_nq > 0)
    hipLaunchKernelGGL(k_proj_cand, dim3((unsigned)((max_nq + 3) / 4), (unsigned)nprob), dim3(256), 0, s,
                       d_probs, mode);
  const size_t lds = (size_t)((max_n + 31) / 32) * 4 + (size_t)max_n;
  hipLaunchKernelGGL(k_proj_resolve, dim3((unsigned)nprob), dim3(64), lds, s, d_probs, mode, nnratio,
                     th_dist, check_ori);
}

extern "C" int orbm_search_by_projection(int mode, const orbx_proj_frame* F,
                                         const orbx_query_proj* q, const uint8_t* qdesc, int nq,
                                         float nnratio, int th_dist, int check_ori, int device,
                                         int32_t* match, int* nmatches) {
  if (!F || mode < 1 || mode > 3 || nq < 0 || F->n < 0 || !nmatches ||
      (nq > 0 && (!q || !qdesc)) || (F->n > 0 && (!F->keys || !F->desc || !match)))
    return ORBX_ERR_ARG;
  *nmatches = 0;
  const int n = F->n;
  if (n > PJ_MAXN) return ORBX_ERR_UNSUPPORTED;
  for (int i = 0; i < n; ++i) match[i] = -1;
  if (n == 0 || nq == 0) return ORBX_OK;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return ORBX_ERR_NO_DEVICE;
  ORBX_TRY(hipSetDevice(device));
  WsLease L(device);
  CallWs* w = L.w;
  if (!w) return ORBX_ERR_HIP;
  hipStream_t s = w->stream;
  set_max_dynamic_lds((const void*)k_grid_build, device);
  set_max_dynamic_lds((const void*)k_proj_resolve, device);
  Carve C;
  const size_t o_keys = C.take((size_t)n * sizeof(orbx_keypoint)), o_desc = C.take((size_t)n * 32);
  const size_t o_ur = F->uright ? C.take((size_t)n * 4) : 0, o_occ = F->occupied ? C.take(n) : 0;
  const size_t o_q = C.take((size_t)nq * sizeof(orbx_query_proj)), o_qd = C.take((size_t)nq * 32);
  const size_t o_prob = C.take(sizeof(ProjProblem));
  const size_t in_end = C.off;
  const size_t o_match = C.take((size_t)n * 4), o_nm = C.take(4), out_end = C.off;
  const size_t o_off = C.take((PG_CELLS + 1) * 4), o_feat = C.take((size_t)n * 4);
  const size_t o_cand = C.take((size_t)nq * PJ_T * 4), o_nc = C.take((size_t)nq * 4);
  int rc = w->reserve(C.off, out_end);
  if (rc) return rc;
  uint8_t* h = w->h;
  uint8_t* d = w->d;
  memcpy(h + o_keys, F->keys, (size_t)n * sizeof(orbx_keypoint));
  memcpy(h + o_desc, F->desc, (size_t)n * 32);
  if (F->uright) memcpy(h + o_ur, F->uright, (size_t)n * 4);
  if (F->occupied) memcpy(h + o_occ, F->occupied, n);
  memcpy(h + o_q, q, (size_t)nq * sizeof(orbx_query_proj));
  memcpy(h + o_qd, qdesc, (size_t)nq * 32);
  ProjProblem* hp = reinterpret_cast<ProjProblem*>(h + o_prob);
  ProjProblem* dp = reinterpret_cast<ProjProblem*>(d + o_prob);
  hp->F = proj_frame(F);
  hp->keys = reinterpret_cast<orbx_keypoint*>(d + o_keys);
  hp->desc = d + o_desc;
  hp->uright = F->uright ? reinterpret_cast<float*>(d + o_ur) : nullptr;
  hp->occupied = F->occupied ? d + o_occ : nullptr;
  hp->qs = reinterpret_cast<orbx_query_proj*>(d + o_q);
  hp->qdesc = d + o_qd;
  hp->nq = nq;
  hp->match = reinterpret_cast<int32_t*>(d + o_match);
  hp->nmatches = reinterpret_cast<int*>(d + o_nm);
  hp->cell_off = reinterpret_cast<int*>(d + o_off);
  hp->cell_feat = reinterpret_cast<int*>(d + o_feat);
  hp->cand = reinterpret_cast<uint32_t*>(d + o_cand);
  hp->ncand = reinterpret_cast<int*>(d + o_nc);
  if (stage_in(d, h, in_end, s)) return ORBX_ERR_HIP;
  launch_proj(dp, 1, n, nq, mode, nnratio, th_dist, check_ori, s);
  if (hipGetLastError() != hipSuccess) return ORBX_ERR_HIP;
  if (stage_out(h + in_end, d + in_end, out_end - in_end, s)) return ORBX_ERR_HIP;
  ORBX_TRY(stream_wait(s));
  memcpy(match, h + o_match, (size_t)n * 4);
  memcpy(nmatches, h + o_nm, sizeof(int));
  return ORBX_OK;
}

// ---------------------------------------------------------------------------
// Batched device form: many SearchByProjection problems (frames, each with
// its query set) in one set of launches on device-resident inputs.
// ---------------------------------------------------------------------------
struct orbm_proj_plan {
  int device = 0, max_prob = 0, max_n = 0, max_nq = 0;
  ProjProblem* d_probs = nullptr;
  ProjProblem* h_probs = nullptr;  // pinned staging of the problem table
  hipEvent_t ev = nullptr;         // the last table upload (h_probs reusable after it)
  hipEvent_t ev_done = nullptr;    // the last call's kernels (its grid / candidate scratch free after it)
  int* d_cell_off = nullptr;
  int* d_cell_feat = nullptr;
  uint32_t* d_cand = nullptr;
  int* d_ncand = nullptr;
};

static void proj_plan_free(orbm_proj_plan* p) {
  if (!p) return;
  hipSetDevice(p->device);
  if (p->ev) hipEventDestroy(p->ev);
  if (p->ev_done) hipEventDestroy(p->ev_done);
  if (p->h_probs) hipHostFree(p->h_probs);
  void* bufs[] = {p->d_probs, p->d_cell_off, p->d_cell_feat, p->d_cand, p->d_ncand};
  for (void* b : bufs)
    if (b) hipFree(b);
  delete p;
}

extern "C" int orbm_proj_plan_create(int max_problems, int max_n, int max_nq, int device, orbm_proj_plan** out) {
  if (!out || max_problems < 1 || max_n < 1 || max_nq < 0) return ORBX_ERR_ARG;
  *out = nullptr;
  if (max_n > PJ_MAXN || max_problems > 65535) return ORBX_ERR_UNSUPPORTED;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return ORBX_ERR_NO_DEVICE;
  ORBX_TRY(hipSetDevice(device));
  orbm_proj_plan* p = new orbm_proj_plan();
  p->device = device;
  p->max_prob = max_problems;
  p->max_n = max_n;
  p->max_nq = max_nq;
  const size_t B = (size_t)max_problems;
  if (hipMalloc((void**)&p->d_probs, B * sizeof(ProjProblem)) != hipSuccess ||
      hipHostMalloc((void**)&p->h_probs, B * sizeof(ProjProblem), hipHostMallocDefault) != hipSuccess ||
      hipEventCreateWithFlags(&p->ev, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&p->ev_done, hipEventDisableTiming) != hipSuccess ||
      hipMalloc((void**)&p->d_cell_off, B * (PG_CELLS + 1) * sizeof(int)) != hipSuccess ||
      hipMalloc((void**)&p->d_cell_feat, B * (size_t)max_n * sizeof(int)) != hipSuccess ||
      hipMalloc((void**)&p->d_cand, B * (size_t)std::max(max_nq, 1) * PJ_T * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc((void**)&p->d_ncand, B * (size_t)std::max(max_nq, 1) * sizeof(int)) != hipSuccess) {
    proj_plan_free(p);
    return ORBX_ERR_HIP;
  }
  if (set_max_dynamic_lds((const void*)k_grid_build, device) ||
      set_max_dynamic_lds((const void*)k_proj_resolve, device)) {
    proj_plan_free(p);
    return ORBX_ERR_HIP;
  }
  *out = p;
  return ORBX_OK;
}

extern "C" int orbm_proj_plan_destroy(orbm_proj_plan* p) {
  proj_plan_free(p);
  return ORBX_OK;
}

extern "C" int orbm_proj_plan_search(orbm_proj_plan* p, int mode, int nprob, const orbx_proj_problem* probs,
                                     float nnratio, int th_dist, int check_ori, void* stream) {
  if (!p || mode < 1 || mode > 3 || nprob < 0 || nprob > p->max_prob || (nprob > 0 && !probs))
    return ORBX_ERR_ARG;
  int max_n = 1, max_nq = 0;
  for (int i = 0; i < nprob; ++i) {
    const orbx_proj_problem& q = probs[i];
    const orbx_proj_frame& F = q.frame;
    if (F.n < 0 || F.n > p->max_n || q.nq < 0 || q.nq > p->max_nq || !q.match || !q.nmatches ||
        (F.n > 0 && (!F.keys || !F.desc)) || (q.nq > 0 && (!q.q || !q.qdesc)))
      return ORBX_ERR_ARG;
    max_n = std::max(max_n, F.n);
    max_nq = std::max(max_nq, q.nq);
  }
  if (nprob == 0) return ORBX_OK;
  ORBX_TRY(hipSetDevice(p->device));
  hipStream_t s = (hipStream_t)stream;
  ORBX_TRY(hipEventSynchronize(p->ev));  // the previous call's table has left the staging buffer
  // every call reuses the plan's device scratch (problem table, grids,
  // candidates): a call on another stream than the previous one's must not
  // overwrite them under the previous call's kernels -- the
  // stream waits for them on the device; no host block
  ORBX_TRY(hipStreamWaitEvent(s, p->ev_done, 0));
  for (int i = 0; i < nprob; ++i) {
    const orbx_proj_problem& q = probs[i];
    ProjProblem& P = p->h_probs[i];
    P.F = proj_frame(&q.frame);
    P.keys = q.frame.keys;
    P.desc = q.frame.desc;
    P.uright = q.frame.uright;
    P.occupied = q.frame.occupied;
    P.qs = q.q;
    P.qdesc = q.qdesc;
    P.nq = q.nq;
    P.match = q.match;
    P.nmatches = q.nmatches;
    P.cell_off = p->d_cell_off + (size_t)i * (PG_CELLS + 1);
    P.cell_feat = p->d_cell_feat + (size_t)i * p->max_n;
    P.cand = p->d_cand + (size_t)i * std::max(p->max_nq, 1) * PJ_T;
    P.ncand = p->d_ncand + (size_t)i * std::max(p->max_nq, 1);
  }
  ORBX_TRY(hipMemcpyAsync(p->d_probs, p->h_probs, (size_t)nprob * sizeof(ProjProblem), hipMemcpyHostToDevice, s));
  ORBX_TRY(hipEventRecord(p->ev, s));
  launch_proj(p->d_probs, nprob, max_n, max_nq, mode, nnratio, th_dist, check_ori, s);
  if (hipGetLastError() != hipSuccess) return ORBX_ERR_HIP;
  ORBX_TRY(hipEventRecord(p->ev_done, s));
  return ORBX_OK;
}
