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
__global__ void k_grid_build(const orbx_keypoint*, const ProjFrame, int, int*, int*);
__global__ void k_proj_cand(const ProjFrame, const orbx_keypoint*, const uint8_t*, const float*,
                            const uint8_t*, const int*, const int*, const orbx_query_proj*,
                            const uint8_t*, int, int, uint32_t*, int*);
__global__ void k_proj_resolve(const ProjFrame, const orbx_keypoint*, const uint8_t*, const float*,
                               const uint8_t*, const int*, const int*, const orbx_query_proj*,
                               const uint8_t*, int, int, float, int, int, const uint32_t*,
                               const int*, int32_t*, int*);
}  // namespace orbx

using namespace orbx;

#define PJ_T 8
#define PJ_MAXN 8192
#define PG_CELLS (64 * 48)

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
  ORBX_TRY(hipMemcpyAsync(d, h, in_end, hipMemcpyHostToDevice, s));
  orbx_keypoint* d_keys = reinterpret_cast<orbx_keypoint*>(d + o_keys);
  uint8_t* d_desc = d + o_desc;
  float* d_ur = F->uright ? reinterpret_cast<float*>(d + o_ur) : nullptr;
  uint8_t* d_occ = F->occupied ? d + o_occ : nullptr;
  int* d_off = reinterpret_cast<int*>(d + o_off);
  int* d_feat = reinterpret_cast<int*>(d + o_feat);
  orbx_query_proj* d_q = reinterpret_cast<orbx_query_proj*>(d + o_q);
  uint8_t* d_qd = d + o_qd;
  uint32_t* d_cand = reinterpret_cast<uint32_t*>(d + o_cand);
  int* d_nc = reinterpret_cast<int*>(d + o_nc);
  int32_t* d_match = reinterpret_cast<int32_t*>(d + o_match);
  int* d_nm = reinterpret_cast<int*>(d + o_nm);
  ProjFrame PF;
  PF.n = n;
  PF.minX = F->min_x;
  PF.minY = F->min_y;
  PF.wInv = F->grid_w_inv;
  PF.hInv = F->grid_h_inv;
  int P = 1;
  while (P < n) P <<= 1;
  hipLaunchKernelGGL(k_grid_build, dim3(1), dim3(1024), (size_t)P * 4, s, d_keys, PF, P, d_off,
                     d_feat);
  hipLaunchKernelGGL(k_proj_cand, dim3((nq + 3) / 4), dim3(256), 0, s, PF, d_keys, d_desc, d_ur,
                     d_occ, d_off, d_feat, d_q, d_qd, nq, mode, d_cand, d_nc);
  const size_t lds = (size_t)((n + 31) / 32) * 4 + (size_t)n;
  hipLaunchKernelGGL(k_proj_resolve, dim3(1), dim3(64), lds, s, PF, d_keys, d_desc, d_ur, d_occ,
                     d_off, d_feat, d_q, d_qd, nq, mode, nnratio, th_dist, check_ori, d_cand,
                     d_nc, d_match, d_nm);
  if (hipGetLastError() != hipSuccess) return ORBX_ERR_HIP;
  ORBX_TRY(hipMemcpyAsync(h + in_end, d + in_end, out_end - in_end, hipMemcpyDeviceToHost, s));
  ORBX_TRY(stream_wait(s));
  memcpy(match, h + o_match, (size_t)n * 4);
  memcpy(nmatches, h + o_nm, sizeof(int));
  return ORBX_OK;
}
