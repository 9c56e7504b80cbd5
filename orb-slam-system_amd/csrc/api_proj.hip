// api_proj.hip -- C ABI of the frame grid + ORBmatcher::SearchByProjection
// (query form, /root/reference/src/ORBmatcher.cc:19-61,732-818,820-894).
#include <hip/hip_runtime.h>

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

namespace {
struct Bufs {
  std::vector<void*> p;
  ~Bufs() {
    for (void* x : p) hipFree(x);
  }
  template <typename T>
  T* get(size_t n) {
    void* x = nullptr;
    if (hipMalloc(&x, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) return nullptr;
    p.push_back(x);
    return (T*)x;
  }
};
}  // namespace

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
  Bufs B;
  orbx_keypoint* d_keys = B.get<orbx_keypoint>(n);
  uint8_t* d_desc = B.get<uint8_t>((size_t)n * 32);
  float* d_ur = F->uright ? B.get<float>(n) : nullptr;
  uint8_t* d_occ = F->occupied ? B.get<uint8_t>(n) : nullptr;
  int* d_off = B.get<int>(PG_CELLS + 1);
  int* d_feat = B.get<int>(n);
  orbx_query_proj* d_q = B.get<orbx_query_proj>(nq);
  uint8_t* d_qd = B.get<uint8_t>((size_t)nq * 32);
  uint32_t* d_cand = B.get<uint32_t>((size_t)nq * PJ_T);
  int* d_nc = B.get<int>(nq);
  int32_t* d_match = B.get<int32_t>(n);
  int* d_nm = B.get<int>(1);
  if (!d_keys || !d_desc || (F->uright && !d_ur) || (F->occupied && !d_occ) || !d_off || !d_feat ||
      !d_q || !d_qd || !d_cand || !d_nc || !d_match || !d_nm)
    return ORBX_ERR_HIP;
  hipStream_t s = nullptr;
  ORBX_TRY(hipMemcpyAsync(d_keys, F->keys, n * sizeof(orbx_keypoint), hipMemcpyHostToDevice, s));
  ORBX_TRY(hipMemcpyAsync(d_desc, F->desc, (size_t)n * 32, hipMemcpyHostToDevice, s));
  if (d_ur) ORBX_TRY(hipMemcpyAsync(d_ur, F->uright, n * sizeof(float), hipMemcpyHostToDevice, s));
  if (d_occ) ORBX_TRY(hipMemcpyAsync(d_occ, F->occupied, n, hipMemcpyHostToDevice, s));
  ORBX_TRY(hipMemcpyAsync(d_q, q, nq * sizeof(orbx_query_proj), hipMemcpyHostToDevice, s));
  ORBX_TRY(hipMemcpyAsync(d_qd, qdesc, (size_t)nq * 32, hipMemcpyHostToDevice, s));
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
  ORBX_TRY(hipMemcpyAsync(match, d_match, n * sizeof(int32_t), hipMemcpyDeviceToHost, s));
  ORBX_TRY(hipMemcpyAsync(nmatches, d_nm, sizeof(int), hipMemcpyDeviceToHost, s));
  ORBX_TRY(hipStreamSynchronize(s));
  return ORBX_OK;
}
