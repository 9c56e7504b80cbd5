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
template <int NW>
__global__ void k_match_cand_rows(const MProblem*, const MNodePair*, const uint4*, const uint32_t*,
                                  uint2*, int4*, int2*);
__global__ void k_match_gather2(const MProblem*, const MNodePair*, uint4*, uint32_t*);
typedef int v4i_ __attribute__((ext_vector_type(4)));
template <int NK>
__global__ void k_match_expand2(const MProblem*, const MNodePair*, v4i_*);
template <int NK, int RT, bool PK, int CS>
__global__ void k_match_cand_mfma(const MProblem*, const MNodePair*, const v4i_*, uint2*, int4*,
                                  int2*);

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

#ifndef ORBM_MFMA
#define ORBM_MFMA 1 /* 0: VALU distances everywhere (profiling variant) */
#endif


namespace {

// bytes 24..31 of every descriptor zero (orbx descriptors with the
// reference's pattern): the candidate kernel may skip dwords 6-7 exactly
bool upper_bytes_zero(const uint8_t* d, int n) {
  uint64_t acc = 0;
  for (int i = 0; i < n; ++i) {
    uint64_t w;
    memcpy(&w, d + (size_t)i * 32 + 24, 8);
    acc |= w;
  }
  return acc == 0;
}

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
                  uint32_t* d_gval2, void* d_gx2, uint2* d_cand, int4* d_rowinfo, int2* d_ev,
                  int* d_last, const int* d_last_off, hipStream_t s, StageTimer* timer,
                  bool six_words) {
  {
    int dev = 0;
    hipGetDevice(&dev);
    set_max_dynamic_lds((const void*)k_match_cand_lds<32>, dev);
    set_max_dynamic_lds((const void*)k_match_resolve_spec, dev);
    set_max_dynamic_lds((const void*)k_match_resolve, dev);
  }
  if (timer) timer->begin(ORBX_STAGE_MCAND, s);
  if (nrows > 0 && nnp > 0) {
    if (max_n2 <= ORBM_MAX_N2 && nnp <= 65535 && d_gdesc2) {
      const bool mfma = ORBM_MFMA && d_gx2 && !d_gval2 && max_n2 > 0;
      if (mfma) {
        // distances on the matrix cores (no validity masks on this path):
        // list2 gathered straight into +-1 bytes
        v4i_* gx2 = reinterpret_cast<v4i_*>(d_gx2);
        // a launch of fewer workgroups than CUs (one long node pair, e.g. a
        // drop-in call) splits each row tile's list 4 ways over a
        // workgroup's waves (MC_CSPLIT_WGS: below this many 128-row
        // workgroups; lists of 8+ tiles)
        const bool csplit = (size_t)nnp * (size_t)((max_n1 + 128 * MC_RT - 1) / (128 * MC_RT)) < (size_t)MC_CSPLIT_WGS &&
                            max_n2 >= 256;
        const dim3 g1((max_n1 + 128 * MC_RT - 1) / (128 * MC_RT), nnp), g4((max_n1 + 31) / 32, nnp);
#define MC_LAUNCH(NK, PK)                                                                               \
  do {                                                                                                  \
    if (csplit)                                                                                         \
      hipLaunchKernelGGL((k_match_cand_mfma<NK, 1, PK, 4>), g4, dim3(256), 0, s, d_probs, d_nps, gx2,   \
                         d_cand, d_rowinfo, d_ev);                                                      \
    else                                                                                                \
      hipLaunchKernelGGL((k_match_cand_mfma<NK, MC_RT, PK, 1>), g1, dim3(256), 0, s, d_probs, d_nps,    \
                         gx2, d_cand, d_rowinfo, d_ev);                                                 \
  } while (0)
        if (six_words) {
          hipLaunchKernelGGL(k_match_expand2<6>, dim3((max_n2 * ORBM_EXPAND_PER_POS(6) + 255) / 256, nnp), dim3(256), 0, s,
                             d_probs, d_nps, gx2);
          // positions in the accumulator while they fit its 2^MC_PB(6) slots
          if (ORBM_FP4 && MC_PK && max_n2 <= (1 << 14))
            MC_LAUNCH(6, ORBM_FP4 != 0);
          else
            MC_LAUNCH(6, false);
        } else {
          hipLaunchKernelGGL(k_match_expand2<8>, dim3((max_n2 * ORBM_EXPAND_PER_POS(8) + 255) / 256, nnp), dim3(256), 0, s,
                             d_probs, d_nps, gx2);
          if (ORBM_FP4 && MC_PK && max_n2 <= (1 << 13))
            MC_LAUNCH(8, ORBM_FP4 != 0);
          else
            MC_LAUNCH(8, false);
        }
#undef MC_LAUNCH
      } else {
        // list2 descriptors gathered into node order, then two rows per lane,
        // the 4 waves splitting the positions; descriptors stream through LDS
        if (max_n2 > 0)
          hipLaunchKernelGGL(k_match_gather2, dim3((max_n2 + 127) / 128, nnp), dim3(256), 0, s, d_probs,
                             d_nps, d_gdesc2, d_gval2);
        if (six_words)
          hipLaunchKernelGGL(k_match_cand_rows<6>, dim3((max_n1 + 127) / 128, nnp), dim3(256), 0, s,
                             d_probs, d_nps, d_gdesc2, d_gval2, d_cand, d_rowinfo, d_ev);
        else
          hipLaunchKernelGGL(k_match_cand_rows<8>, dim3((max_n1 + 127) / 128, nnp), dim3(256), 0, s,
                             d_probs, d_nps, d_gdesc2, d_gval2, d_cand, d_rowinfo, d_ev);
      }
    } else if (max_n2 <= 64 * 32 && nnp <= 65535) {
      // list2 staged in LDS, distances in registers (32 per lane)
      const size_t lds = (size_t)std::max(max_n2, 1) * 32;
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
    // (+ alignment to 8 B) + the chunk's candidate slots (64 lanes x ORBM_T)
    const int n2cap = std::max(max_bitmap_n2, 32);
    const size_t lds = (size_t)((((n2cap + 31) / 32 + n2cap) + 1) & ~1) * 4 + (size_t)64 * ORBM_T * sizeof(uint2);
    hipLaunchKernelGGL(k_match_resolve_spec, dim3(units), dim3(64), lds, s, d_probs, d_nps, units,
                       d_cand, d_rowinfo, d_ev, n2cap);
  } else if (nrows > 0 && units > 0) {
    if (max_bitmap_n2 > 16384) {
      const size_t lds = (size_t)((max_bitmap_n2 + 31) / 32) * 4;
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

// the KF-KF search (th_low = ORBM_TH_LOW) or upstream's KF-Frame search
// (th_low = ORBM_TH_LOW + 1, i.e. bestDist1 <= TH_LOW) of kf1's rows over
// kf2's candidates: match12 indexed by kf1 feature
static int bow_search(const orbx_bow_frame* kf1, const orbx_bow_frame* kf2, float nnratio,
                      int check_ori, int device, int th_low, int32_t* match12, int* nmatches) {
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
  WsLease L(device);
  CallWs* w = L.w;
  if (!w) return ORBX_ERR_HIP;
  hipStream_t s = w->stream;
  // one arena: inputs [0, in_end) go up in one copy from pinned staging,
  // outputs [in_end, out_end) come back in one copy, scratch after them
  const uint32_t nf1 = kf1->nnodes ? kf1->node_off[kf1->nnodes] : 0;
  const uint32_t nf2 = kf2->nnodes ? kf2->node_off[kf2->nnodes] : 0;
  const size_t n1 = (size_t)kf1->n, n2 = (size_t)kf2->n, nnp = nps.size();
  Carve C;
  const size_t o_desc1 = C.take(n1 * 32), o_desc2 = C.take(n2 * 32);
  const size_t o_ang1 = C.take(n1 * 4), o_ang2 = C.take(n2 * 4);
  const size_t o_val1 = kf1->valid ? C.take(n1) : 0, o_val2 = kf2->valid ? C.take(n2) : 0;
  const size_t o_feat1 = C.take((size_t)nf1 * 4), o_feat2 = C.take((size_t)nf2 * 4);
  const size_t o_prob = C.take(sizeof(MProblem)), o_nps = C.take(nnp * sizeof(MNodePair));
  const size_t o_loff = C.take(sizeof(int));
  const size_t in_end = C.off;
  const size_t o_m12 = C.take(n1 * 4), o_nm = C.take(sizeof(int));
  const size_t out_end = C.off;
  const size_t o_cand = C.take((size_t)rows * ORBM_T * sizeof(uint2));
  const size_t o_rowinfo = C.take((size_t)rows * sizeof(int4)), o_ev = C.take((size_t)rows * sizeof(int2));
  const size_t o_last = C.take(n1 * 4), o_g2 = C.take((size_t)g2 * 2 * sizeof(uint4));
  const size_t o_gv2 = kf2->valid ? C.take((size_t)g2 * 4) : 0;
  const size_t o_gx2 = kf2->valid ? 0 : C.take((size_t)g2 * 256);  /* +-1 bytes for the MFMA path */
  int rc2 = w->reserve(C.off, out_end);
  if (rc2) return rc2;
  uint8_t* d = w->d;
  uint8_t* h = w->h;
  memcpy(h + o_desc1, kf1->desc, n1 * 32);
  memcpy(h + o_desc2, kf2->desc, n2 * 32);
  memcpy(h + o_ang1, kf1->angle, n1 * 4);
  memcpy(h + o_ang2, kf2->angle, n2 * 4);
  if (kf1->valid) memcpy(h + o_val1, kf1->valid, n1);
  if (kf2->valid) memcpy(h + o_val2, kf2->valid, n2);
  if (nf1) memcpy(h + o_feat1, kf1->feat, (size_t)nf1 * 4);
  if (nf2) memcpy(h + o_feat2, kf2->feat, (size_t)nf2 * 4);
  MProblem P;
  memset(&P, 0, sizeof(P));
  P.desc1 = d + o_desc1;
  P.desc2 = d + o_desc2;
  P.ang1 = reinterpret_cast<const float*>(d + o_ang1);
  P.ang2 = reinterpret_cast<const float*>(d + o_ang2);
  P.valid1 = kf1->valid ? d + o_val1 : nullptr;
  P.valid2 = kf2->valid ? d + o_val2 : nullptr;
  P.feat1 = reinterpret_cast<const uint32_t*>(d + o_feat1);
  P.feat2 = reinterpret_cast<const uint32_t*>(d + o_feat2);
  P.match12 = reinterpret_cast<int32_t*>(d + o_m12);
  P.nmatches = reinterpret_cast<int*>(d + o_nm);
  P.ang_stride = 1;
  P.n1 = kf1->n;
  P.n2 = kf2->n;
  P.np_begin = 0;
  P.np_end = (int)nnp;
  P.row_begin = 0;
  P.row_end = rows;
  P.check_ori = check_ori ? 1 : 0;
  P.nnratio = nnratio;
  P.sequential = sequential;
  P.dcap = orbm_dcap(nnratio, th_low);
  P.th_low = th_low;
  memcpy(h + o_prob, &P, sizeof(P));
  if (nnp) memcpy(h + o_nps, nps.data(), nnp * sizeof(MNodePair));
  memset(h + o_loff, 0, sizeof(int));
  rc2 = stage_in(d, h, in_end, s);
  if (rc2) return rc2;
  launch_match(reinterpret_cast<MProblem*>(d + o_prob), 1, reinterpret_cast<MNodePair*>(d + o_nps),
               (int)nnp, rows, sequential, max_n1, max_n2, kf2->n,
               reinterpret_cast<uint4*>(d + o_g2),
               kf2->valid ? reinterpret_cast<uint32_t*>(d + o_gv2) : nullptr,
               kf2->valid ? nullptr : d + o_gx2, reinterpret_cast<uint2*>(d + o_cand), reinterpret_cast<int4*>(d + o_rowinfo),
               reinterpret_cast<int2*>(d + o_ev), reinterpret_cast<int*>(d + o_last),
               reinterpret_cast<const int*>(d + o_loff), s, nullptr,
               upper_bytes_zero(kf1->desc, kf1->n) && upper_bytes_zero(kf2->desc, kf2->n));
  if (hipGetLastError() != hipSuccess) return ORBX_ERR_HIP;
  rc2 = stage_out(h + in_end, d + in_end, out_end - in_end, s);
  if (rc2) return rc2;
  ORBX_TRY(stream_wait(s));
  memcpy(match12, h + o_m12, n1 * 4);
  memcpy(nmatches, h + o_nm, sizeof(int));
  return ORBX_OK;
}

extern "C" int orbm_search_by_bow(const orbx_bow_frame* kf1, const orbx_bow_frame* kf2,
                                  float nnratio, int check_ori, int device, int32_t* match12,
                                  int* nmatches) {
  return bow_search(kf1, kf2, nnratio, check_ori, device, ORBM_TH_LOW, match12, nmatches);
}

// upstream ORB-SLAM2's SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&)
// (this reference keeps only its stub, ORBmatcher.cc:88-119): the KF's
// features are the rows (valid = a non-null, non-bad MapPoint), the Frame's
// every feature a candidate, a claimed Frame feature is skipped, bestDist1 <=
// TH_LOW; output indexed by Frame feature.  The same device search with
// th_low = TH_LOW + 1, its row -> candidate result inverted here.
extern "C" int orbm_search_by_bow_kf_frame(const orbx_bow_frame* kf, const orbx_bow_frame* frame,
                                           float nnratio, int check_ori, int device, int32_t* match_f,
                                           int* nmatches) {
  if (!nmatches || !frame || (frame->n > 0 && !match_f)) return ORBX_ERR_ARG;
  /* the sentinel scheme assumes a second-best of 256 (upstream's initial
   * bestDist2) passes the ratio test for every acceptable best */
  if (orbm_dcap(nnratio, ORBM_TH_LOW + 1) > 256) return ORBX_ERR_UNSUPPORTED;
  /* a KF feature listed under two nodes (never in a DBoW2 FeatureVector) would
   * leave one row per KF index in the row -> candidate result while nmatches
   * counts both: rejected */
  if (kf && kf->n > 0 && kf->nnodes > 0 && kf->node_off && kf->feat) {
    std::vector<unsigned char> seen((size_t)kf->n, 0);
    for (uint32_t j = 0; j < kf->node_off[kf->nnodes]; ++j) {
      const uint32_t i = kf->feat[j];
      if (i >= (uint32_t)kf->n || seen[i]) return ORBX_ERR_ARG;
      seen[i] = 1;
    }
  }
  orbx_bow_frame fr = *frame;
  fr.valid = nullptr;  /* every Frame feature is a candidate */
  std::vector<int32_t> m(kf && kf->n > 0 ? (size_t)kf->n : 1, -1);
  const int rc = bow_search(kf, &fr, nnratio, check_ori, device, ORBM_TH_LOW + 1, m.data(), nmatches);
  if (rc) return rc;
  for (int i = 0; i < frame->n; ++i) match_f[i] = -1;
  for (int i = 0; kf && i < kf->n; ++i)
    if (m[i] >= 0) match_f[m[i]] = i;
  return ORBX_OK;
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
  WsLease L(device);
  CallWs* w = L.w;
  if (!w) return ORBX_ERR_HIP;
  hipStream_t s = w->stream;
  Carve C;
  const size_t o_a = C.take((size_t)na * 32), o_b = C.take((size_t)nb * 32);
  const size_t o_ia = C.take((size_t)npairs * 4), o_ib = C.take((size_t)npairs * 4);
  const size_t in_end = C.off, o_d = C.take((size_t)npairs * 4), out_end = C.off;
  int rc = w->reserve(out_end, out_end);
  if (rc) return rc;
  uint8_t* h = w->h;
  uint8_t* d = w->d;
  memcpy(h + o_a, a, (size_t)na * 32);
  memcpy(h + o_b, b, (size_t)nb * 32);
  memcpy(h + o_ia, ia, (size_t)npairs * 4);
  memcpy(h + o_ib, ib, (size_t)npairs * 4);
  rc = stage_in(d, h, in_end, s);
  if (rc) return rc;
  hipLaunchKernelGGL(k_hamming_pairs, dim3((npairs + 255) / 256), dim3(256), 0, s, d + o_a, d + o_b,
                     reinterpret_cast<const int32_t*>(d + o_ia),
                     reinterpret_cast<const int32_t*>(d + o_ib), npairs,
                     reinterpret_cast<int32_t*>(d + o_d));
  if (hipGetLastError() != hipSuccess) return ORBX_ERR_HIP;
  rc = stage_out(h + o_d, d + o_d, out_end - o_d, s);
  if (rc) return rc;
  ORBX_TRY(stream_wait(s));
  memcpy(dist, h + o_d, (size_t)npairs * 4);
  return ORBX_OK;
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
  P.th_low = ORBM_TH_LOW;
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
  /* ORBM_PLAN_ZERO_TAIL (opt-in, orbm_plan_set_options): the caller
   * guarantees bytes 24..31 of every descriptor are zero, as they are for
   * orbx_plan_extract outputs (static_assert on the pattern in
   * kernels_extract.hip), and the candidate kernels skip dwords 6-7.  Off by
   * default: any other descriptor source gets all 8 dwords. */
  bool six_words = false;
  bool force_valu = false; /* ORBM_PLAN_VALU: popcount kernel instead of the MFMA path */
  MProblem* d_probs = nullptr;
  MNodePair* d_nps = nullptr;
  uint32_t* d_sel = nullptr;
  uint2* d_cand = nullptr;
  uint4* d_gdesc2 = nullptr;
  void* d_gx2 = nullptr; /* list2 as +-1 bytes, 256 B per position */
  int4* d_rowinfo = nullptr;
  int2* d_ev = nullptr;
  int *d_last = nullptr, *d_last_off = nullptr;
  StageTimer timer;
};

static void mplan_free(orbm_plan* m) {
  if (!m) return;
  hipSetDevice(m->device);
  void* b[] = {m->d_probs, m->d_nps, m->d_sel, m->d_cand, m->d_gdesc2, m->d_gx2, m->d_rowinfo,
               m->d_ev, m->d_last, m->d_last_off};
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
      hipMalloc(&m->d_gx2, rows * 256) != hipSuccess ||
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

extern "C" int orbm_plan_set_options(orbm_plan* m, int flags) {
  if (!m || (flags & ~(ORBM_PLAN_ZERO_TAIL | ORBM_PLAN_VALU))) return ORBX_ERR_ARG;
  m->six_words = (flags & ORBM_PLAN_ZERO_TAIL) != 0;
  m->force_valu = (flags & ORBM_PLAN_VALU) != 0;
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
               m->kcap, m->d_gdesc2, nullptr, m->force_valu ? nullptr : m->d_gx2, m->d_cand, m->d_rowinfo, m->d_ev, m->d_last,
               m->d_last_off, s, &m->timer, m->six_words);
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_ERR_HIP;
}
