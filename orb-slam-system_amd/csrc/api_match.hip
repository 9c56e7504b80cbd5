// api_match.hip -- C ABI of the matcher: ORBmatcher::SearchByBoW(KF, KF)
// and DescriptorDistance drop-ins, and the batched frame-pair matcher.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/orbx.h"
#include "api_common.h"
#include "match_internal.h"

namespace orbx {
__global__ void k_match_candidates(const MProblem*, const MNodePair*, int, int, uint2*, int4*,
                                   int2*);
template <int NJ>
__global__ void k_match_cand_lds(const MProblem*, const MNodePair*, uint2*, int4*, int2*);
__global__ void k_match_cand_rows(const MProblem*, const MNodePair*, const uint4*, const uint32_t*,
                                  uint2*, int4*, int2*);
__global__ void k_match_gather2(const MProblem*, const MNodePair*, uint4*, uint32_t*);
__global__ void k_match_resolve(const MProblem*, const MNodePair*, int, int, const uint2*,
                                const int4*, int2*);
__global__ void k_match_resolve_spec(const MProblem*, const MNodePair*, int, const uint2*,
                                     const int4*, int2*, int);
__global__ void k_match_finalize(const MProblem*, const MNodePair*, const int4*, int2*, int*,
                                 const int*);
__global__ void k_match_select(MProblem*, MNodePair*, const orbx_keypoint*, const int*,
                               const orbx_keypoint*, const int*, int, int, uint32_t*);
__global__ void k_hamming_pairs(const uint8_t*, const uint8_t*, const int32_t*, const int32_t*,
                                int, int32_t*);
}  // namespace orbx

using namespace orbx;

namespace {

// RAII device buffers for one synchronous call
struct DevBufs {
  std::vector<void*> ptrs;
  ~DevBufs() {
    for (void* p : ptrs) hipFree(p);
  }
  template <typename T>
  T* alloc(size_t n) {
    void* p = nullptr;
    if (hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)) != hipSuccess) return nullptr;
    ptrs.push_back(p);
    return (T*)p;
  }
  template <typename T>
  T* upload(const T* src, size_t n, hipStream_t s) {
    T* d = alloc<T>(n);
    if (!d) return nullptr;
    if (n && src && hipMemcpyAsync(d, src, n * sizeof(T), hipMemcpyHostToDevice, s) != hipSuccess)
      return nullptr;
    return d;
  }
};

int check_frame(const orbx_bow_frame* k) {
  if (!k || k->n < 0 || k->nnodes < 0) return ORBX_ERR_ARG;
  if (k->n > 0 && (!k->desc || !k->angle)) return ORBX_ERR_ARG;
  if (k->nnodes > 0 && (!k->node_id || !k->node_off || !k->feat)) return ORBX_ERR_ARG;
  for (int j = 0; j < k->nnodes; ++j) {
    if (j > 0 && k->node_id[j] <= k->node_id[j - 1]) return ORBX_ERR_ARG; /* std::map keys */
    if (k->node_off[j + 1] < k->node_off[j]) return ORBX_ERR_ARG;
  }
  const uint32_t nf = k->nnodes ? k->node_off[k->nnodes] : 0;
  for (uint32_t i = 0; i < nf; ++i)
    if (k->feat[i] >= (uint32_t)k->n) return ORBX_ERR_ARG;
  return ORBX_OK;
}

void launch_match(const MProblem* d_probs, int nprob, const MNodePair* d_nps, int nnp, int nrows,
                  int sequential, int max_n1, int max_n2, int max_bitmap_n2, uint4* d_gdesc2,
                  uint32_t* d_gval2, uint2* d_cand, int4* d_rowinfo, int2* d_ev, int* d_last,
                  const int* d_last_off, hipStream_t s, StageTimer* timer) {
  if (timer) timer->begin(ORBX_STAGE_MCAND, s);
  if (nrows > 0 && nnp > 0) {
    if (max_n2 <= ORBM_MAX_N2 && nnp <= 65535 && d_gdesc2) {
      // list2 descriptors gathered into node order, then two rows per lane,
      // the 4 waves splitting the positions; descriptors stream through LDS
      if (max_n2 > 0)
        hipLaunchKernelGGL(k_match_gather2, dim3((max_n2 + 127) / 128, nnp), dim3(256), 0, s, d_probs,
                           d_nps, d_gdesc2, d_gval2);
      hipLaunchKernelGGL(k_match_cand_rows, dim3((max_n1 + 127) / 128, nnp), dim3(256), 0, s,
                         d_probs, d_nps, d_gdesc2, d_gval2, d_cand, d_rowinfo, d_ev);
    } else if (max_n2 <= 64 * 32 && nnp <= 65535) {
      // list2 staged in LDS, distances in registers (32 per lane)
      const size_t lds = (size_t)std::max(max_n2, 1) * 32;
      hipFuncSetAttribute((const void*)k_match_cand_lds<32>,
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL(k_match_cand_lds<32>, dim3((max_n1 + 63) / 64, nnp), dim3(256), lds, s,
                         d_probs, d_nps, d_cand, d_rowinfo, d_ev);
    } else {
      hipLaunchKernelGGL(k_match_candidates, dim3((nrows + 3) / 4), dim3(256), 0, s, d_probs,
                         d_nps, nnp, nrows, d_cand, d_rowinfo, d_ev);
    }
  }
  if (timer) timer->end(ORBX_STAGE_MCAND, s);
  if (timer) timer->begin(ORBX_STAGE_MRESOLVE, s);
  const int units = sequential ? nprob : nnp;
  if (nrows > 0 && units > 0 && !sequential && max_bitmap_n2 <= 16384) {
    // speculative 64-row chunks; LDS = vbMatched2 bitmap + claim table
    const int n2cap = std::max(max_bitmap_n2, 32);
    const size_t lds = (size_t)((n2cap + 31) / 32) * 4 + (size_t)n2cap * 4;
    hipFuncSetAttribute((const void*)k_match_resolve_spec,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k_match_resolve_spec, dim3(units), dim3(64), lds, s, d_probs, d_nps, units,
                       d_cand, d_rowinfo, d_ev, n2cap);
  } else if (nrows > 0 && units > 0) {
    if (max_bitmap_n2 > 16384) {
      const size_t lds = (size_t)((max_bitmap_n2 + 31) / 32) * 4;
      hipFuncSetAttribute((const void*)k_match_resolve, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)lds);
      hipLaunchKernelGGL(k_match_resolve, dim3(units), dim3(64), lds, s, d_probs, d_nps, units,
                         sequential, d_cand, d_rowinfo, d_ev);
    } else {
      hipLaunchKernelGGL(k_match_resolve, dim3((units + 3) / 4), dim3(256), 0, s, d_probs, d_nps,
                         units, sequential, d_cand, d_rowinfo, d_ev);
    }
  }
  if (timer) timer->end(ORBX_STAGE_MRESOLVE, s);
  if (timer) timer->begin(ORBX_STAGE_MFINAL, s);
  hipLaunchKernelGGL(k_match_finalize, dim3(nprob), dim3(256), 0, s, d_probs, d_nps, d_rowinfo,
                     d_ev, d_last, d_last_off);
  if (timer) timer->end(ORBX_STAGE_MFINAL, s);
}

}  // namespace

extern "C" int orbm_search_by_bow(const orbx_bow_frame* kf1, const orbx_bow_frame* kf2,
                                  float nnratio, int check_ori, int device, int32_t* match12,
                                  int* nmatches) {
  if (!nmatches || (kf1 && kf1->n > 0 && !match12)) return ORBX_ERR_ARG;
  int rc = check_frame(kf1);
  if (rc) return rc;
  rc = check_frame(kf2);
  if (rc) return rc;
  if (kf2->n > ORBM_MAX_N2) return ORBX_ERR_UNSUPPORTED;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
    return ORBX_ERR_NO_DEVICE;
  // merge-join of the two FeatureVectors (ORBmatcher.cc:305-350): common
  // NodeIds in ascending order
  std::vector<MNodePair> nps;
  int rows = 0, max_n1 = 0, max_n2 = 0, g2 = 0;
  {
    int f1 = 0, f2 = 0;
    while (f1 < kf1->nnodes && f2 < kf2->nnodes) {
      const uint32_t a = kf1->node_id[f1], b = kf2->node_id[f2];
      if (a == b) {
        MNodePair np;
        np.prob = 0;
        np.off1 = (int)kf1->node_off[f1];
        np.n1 = (int)(kf1->node_off[f1 + 1] - kf1->node_off[f1]);
        np.off2 = (int)kf2->node_off[f2];
        np.n2 = (int)(kf2->node_off[f2 + 1] - kf2->node_off[f2]);
        if (np.n2 > 0xFFFF) return ORBX_ERR_UNSUPPORTED; /* 16-bit list positions */
        np.row_base = rows;
        np.g2 = g2;
        rows += np.n1;
        g2 += np.n2;
        max_n1 = std::max(max_n1, np.n1);
        max_n2 = std::max(max_n2, np.n2);
        nps.push_back(np);
        ++f1;
        ++f2;
      } else if (a < b) {
        ++f1;
      } else {
        ++f2;
      }
    }
  }
  // node pairs may run in parallel iff no KF2 feature appears in two of them
  int sequential = 0;
  {
    std::vector<uint8_t> seen(kf2->n > 0 ? kf2->n : 1, 0);
    for (const MNodePair& np : nps)
      for (int i = 0; i < np.n2 && !sequential; ++i) {
        const uint32_t f = kf2->feat[np.off2 + i];
        if (seen[f]) sequential = 1;
        seen[f] = 1;
      }
  }
  if (kf1->n == 0) {
    *nmatches = 0;
    return ORBX_OK;
  }
  ORBX_TRY(hipSetDevice(device));
  hipStream_t s;
  ORBX_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int result = ORBX_OK;
  {
    DevBufs B;
    const uint32_t nf1 = kf1->nnodes ? kf1->node_off[kf1->nnodes] : 0;
    const uint32_t nf2 = kf2->nnodes ? kf2->node_off[kf2->nnodes] : 0;
    MProblem P;
    memset(&P, 0, sizeof(P));
    P.desc1 = B.upload(kf1->desc, (size_t)kf1->n * 32, s);
    P.desc2 = B.upload(kf2->desc, (size_t)kf2->n * 32, s);
    P.ang1 = B.upload(kf1->angle, (size_t)kf1->n, s);
    P.ang2 = B.upload(kf2->angle, (size_t)kf2->n, s);
    P.valid1 = kf1->valid ? B.upload(kf1->valid, (size_t)kf1->n, s) : nullptr;
    P.valid2 = kf2->valid ? B.upload(kf2->valid, (size_t)kf2->n, s) : nullptr;
    P.feat1 = B.upload(kf1->feat, nf1, s);
    P.feat2 = B.upload(kf2->feat, nf2, s);
    P.match12 = B.alloc<int32_t>(kf1->n);
    P.nmatches = B.alloc<int>(1);
    P.ang_stride = 1;
    P.n1 = kf1->n;
    P.n2 = kf2->n;
    P.np_begin = 0;
    P.np_end = (int)nps.size();
    P.row_begin = 0;
    P.row_end = rows;
    P.check_ori = check_ori ? 1 : 0;
    P.nnratio = nnratio;
    P.sequential = sequential;
    P.dcap = orbm_dcap(nnratio);
    P.pad = 0;
    MProblem* d_prob = B.upload(&P, 1, s);
    MNodePair* d_nps = B.upload(nps.data(), nps.size(), s);
    uint2* d_cand = B.alloc<uint2>((size_t)rows * ORBM_T);
    int4* d_rowinfo = B.alloc<int4>(rows);
    int2* d_ev = B.alloc<int2>(rows);
    int* d_last = B.alloc<int>(kf1->n);
    uint4* d_gdesc2 = B.alloc<uint4>((size_t)g2 * 2);
    uint32_t* d_gval2 = kf2->valid ? B.alloc<uint32_t>((size_t)g2) : nullptr;
    const int zero = 0;
    int* d_last_off = B.upload(&zero, 1, s);
    if (!P.desc1 || !P.desc2 || !P.ang1 || !P.ang2 || !P.feat1 || !P.feat2 || !P.match12 ||
        !P.nmatches || !d_prob || !d_nps || !d_cand || !d_rowinfo || !d_ev || !d_last ||
        !d_last_off || !d_gdesc2 || (kf1->valid && !P.valid1) ||
        (kf2->valid && (!P.valid2 || !d_gval2))) {
      result = ORBX_ERR_HIP;
    } else {
      launch_match(d_prob, 1, d_nps, (int)nps.size(), rows, sequential, max_n1, max_n2, kf2->n,
                   d_gdesc2, d_gval2, d_cand, d_rowinfo, d_ev, d_last, d_last_off, s, nullptr);
      if (hipGetLastError() != hipSuccess ||
          hipMemcpyAsync(match12, P.match12, sizeof(int32_t) * (size_t)kf1->n,
                         hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipMemcpyAsync(nmatches, P.nmatches, sizeof(int), hipMemcpyDeviceToHost, s) !=
              hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess)
        result = ORBX_ERR_HIP;
    }
  }
  hipStreamDestroy(s);
  return result;
}

extern "C" int orbm_descriptor_distance_batch(const uint8_t* a, int na, const uint8_t* b, int nb,
                                              const int32_t* ia, const int32_t* ib, int npairs,
                                              int device, int32_t* dist) {
  if (npairs < 0 || (npairs > 0 && (!a || !b || !ia || !ib || !dist))) return ORBX_ERR_ARG;
  for (int i = 0; i < npairs; ++i)
    if (ia[i] < 0 || ia[i] >= na || ib[i] < 0 || ib[i] >= nb) return ORBX_ERR_ARG;
  if (npairs == 0) return ORBX_OK;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
    return ORBX_ERR_NO_DEVICE;
  ORBX_TRY(hipSetDevice(device));
  hipStream_t s;
  ORBX_TRY(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int result = ORBX_OK;
  {
    DevBufs B;
    const uint8_t* da = B.upload(a, (size_t)na * 32, s);
    const uint8_t* db = B.upload(b, (size_t)nb * 32, s);
    const int32_t* dia = B.upload(ia, (size_t)npairs, s);
    const int32_t* dib = B.upload(ib, (size_t)npairs, s);
    int32_t* dd = B.alloc<int32_t>(npairs);
    if (!da || !db || !dia || !dib || !dd) {
      result = ORBX_ERR_HIP;
    } else {
      hipLaunchKernelGGL(k_hamming_pairs, dim3((npairs + 255) / 256), dim3(256), 0, s, da, db,
                         dia, dib, npairs, dd);
      if (hipGetLastError() != hipSuccess ||
          hipMemcpyAsync(dist, dd, sizeof(int32_t) * (size_t)npairs, hipMemcpyDeviceToHost, s) !=
              hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess)
        result = ORBX_ERR_HIP;
    }
  }
  hipStreamDestroy(s);
  return result;
}

// ---------------------------------------------------------------------------
// batched frame-pair matcher
// ---------------------------------------------------------------------------
namespace orbx {
__global__ void k_match_setup(MProblem* probs, MNodePair* nps, int npairs,
                              const orbx_keypoint* kps_a, const uint8_t* desc_a,
                              const orbx_keypoint* kps_b, const uint8_t* desc_b, int kcap,
                              int topn, const uint32_t* sel, int32_t* match12, int* nmatches,
                              float nnratio, int check_ori, int* last_off) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= npairs) return;
  MProblem P;
  P.desc1 = desc_a + (size_t)p * kcap * 32;
  P.desc2 = desc_b + (size_t)p * kcap * 32;
  P.ang1 = &kps_a[(size_t)p * kcap].angle;
  P.ang2 = &kps_b[(size_t)p * kcap].angle;
  P.valid1 = nullptr;
  P.valid2 = nullptr;
  P.feat1 = sel + ((size_t)p * 2 + 0) * topn;
  P.feat2 = sel + ((size_t)p * 2 + 1) * topn;
  P.match12 = match12 + (size_t)p * kcap;
  P.nmatches = nmatches + p;
  P.ang_stride = (int)(sizeof(orbx_keypoint) / sizeof(float));
  P.n1 = 0;
  P.n2 = 0;
  P.np_begin = p;
  P.np_end = p + 1;
  P.row_begin = p * topn;
  P.row_end = (p + 1) * topn;
  P.check_ori = check_ori;
  P.nnratio = nnratio;
  P.sequential = 0;
  P.dcap = orbm_dcap(nnratio);
  P.pad = 0;
  probs[p] = P;
  MNodePair NP;
  NP.prob = p;
  NP.off1 = 0;
  NP.n1 = 0;
  NP.off2 = 0;
  NP.n2 = 0;
  NP.row_base = p * topn;
  NP.g2 = p * topn;
  nps[p] = NP;
  last_off[p] = p * kcap;
}
}  // namespace orbx

struct orbm_plan {
  int device = 0, max_pairs = 0, kcap = 0, topn = 0;
  MProblem* d_probs = nullptr;
  MNodePair* d_nps = nullptr;
  uint32_t* d_sel = nullptr;
  uint2* d_cand = nullptr;
  uint4* d_gdesc2 = nullptr;
  int4* d_rowinfo = nullptr;
  int2* d_ev = nullptr;
  int *d_last = nullptr, *d_last_off = nullptr;
  StageTimer timer;
};

static void mplan_free(orbm_plan* m) {
  if (!m) return;
  hipSetDevice(m->device);
  void* b[] = {m->d_probs, m->d_nps, m->d_sel, m->d_cand, m->d_gdesc2, m->d_rowinfo, m->d_ev,
               m->d_last, m->d_last_off};
  for (void* p : b)
    if (p) hipFree(p);
  m->timer.release();
  delete m;
}

extern "C" int orbm_plan_create(int max_pairs, int kcap, int topn, int device, orbm_plan** out) {
  if (!out || max_pairs < 1 || kcap < 1 || topn < 1 || topn > 0xFFFF || kcap > ORBM_MAX_N2)
    return ORBX_ERR_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
    return ORBX_ERR_NO_DEVICE;
  ORBX_TRY(hipSetDevice(device));
  orbm_plan* m = new orbm_plan();
  m->device = device;
  m->max_pairs = max_pairs;
  m->kcap = kcap;
  m->topn = topn;
  const size_t P = (size_t)max_pairs, rows = P * topn;
  if (hipMalloc((void**)&m->d_probs, P * sizeof(MProblem)) != hipSuccess ||
      hipMalloc((void**)&m->d_nps, P * sizeof(MNodePair)) != hipSuccess ||
      hipMalloc((void**)&m->d_sel, P * 2 * topn * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc((void**)&m->d_cand, rows * ORBM_T * sizeof(uint2)) != hipSuccess ||
      hipMalloc((void**)&m->d_gdesc2, rows * 2 * sizeof(uint4)) != hipSuccess ||
      hipMalloc((void**)&m->d_rowinfo, rows * sizeof(int4)) != hipSuccess ||
      hipMalloc((void**)&m->d_ev, rows * sizeof(int2)) != hipSuccess ||
      hipMalloc((void**)&m->d_last, P * kcap * sizeof(int)) != hipSuccess ||
      hipMalloc((void**)&m->d_last_off, P * sizeof(int)) != hipSuccess) {
    mplan_free(m);
    return ORBX_ERR_HIP;
  }
  *out = m;
  return ORBX_OK;
}

extern "C" int orbm_plan_destroy(orbm_plan* m) {
  mplan_free(m);
  return ORBX_OK;
}

extern "C" int orbm_plan_set_timing(orbm_plan* m, int enable) {
  if (!m) return ORBX_ERR_ARG;
  hipSetDevice(m->device);
  m->timer.reset(enable != 0);
  return ORBX_OK;
}

extern "C" int orbm_plan_stage_times(orbm_plan* m, double* ms, int* launches, int n) {
  if (!m) return ORBX_ERR_ARG;
  hipSetDevice(m->device);
  return m->timer.collect(ms, launches, n);
}

extern "C" int orbm_plan_match_frames(orbm_plan* m, int npairs, const orbx_keypoint* kps_a,
                                      const uint8_t* desc_a, const int* count_a,
                                      const orbx_keypoint* kps_b, const uint8_t* desc_b,
                                      const int* count_b, float nnratio, int check_ori,
                                      int32_t* match12, int* nmatches, void* stream) {
  if (!m || npairs < 1 || npairs > m->max_pairs || !kps_a || !desc_a || !count_a || !kps_b ||
      !desc_b || !count_b || !match12 || !nmatches)
    return ORBX_ERR_ARG;
  ORBX_TRY(hipSetDevice(m->device));
  hipStream_t s = (hipStream_t)stream;
  m->timer.begin(ORBX_STAGE_MSELECT, s);
  hipLaunchKernelGGL(k_match_setup, dim3((npairs + 63) / 64), dim3(64), 0, s, m->d_probs,
                     m->d_nps, npairs, kps_a, desc_a, kps_b, desc_b, m->kcap, m->topn, m->d_sel,
                     match12, nmatches, nnratio, check_ori ? 1 : 0, m->d_last_off);
  hipLaunchKernelGGL(k_match_select, dim3(npairs, 2), dim3(256), 0, s, m->d_probs, m->d_nps,
                     kps_a, count_a, kps_b, count_b, m->kcap, m->topn, m->d_sel);
  m->timer.end(ORBX_STAGE_MSELECT, s);
  launch_match(m->d_probs, npairs, m->d_nps, npairs, npairs * m->topn, 0, m->topn, m->topn,
               m->kcap, m->d_gdesc2, nullptr, m->d_cand, m->d_rowinfo, m->d_ev, m->d_last,
               m->d_last_off, s, &m->timer);
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_ERR_HIP;
}
