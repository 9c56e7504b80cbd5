// match_internal.h -- device tables of the SearchByBoW pipeline.
//
// One "problem" = one ORBmatcher::SearchByBoW(KF1, KF2) call
// (src/ORBmatcher.cc:278-366).  Its common vocabulary nodes become "node
// pairs" (list1 = node's features in KF1, list2 = in KF2) in ascending NodeId
// order.  Every list1 entry owns one "row" (row_base + position) of the
// candidate / event arrays.
#ifndef ORBX_MATCH_INTERNAL_H
#define ORBX_MATCH_INTERNAL_H

#include <stdint.h>

#ifndef ORBM_T
#define ORBM_T 8           /* candidates kept per row                     */
#endif
#define ORBM_TH_LOW 50     /* ORBmatcher::TH_LOW (ORBmatcher.cc:14)       */
#define ORBM_HISTO 30      /* ORBmatcher::HISTO_LENGTH (ORBmatcher.cc:15) */
#define ORBM_MAX_N2 65536  /* list positions / idx2 bitmap bound          */
/* k_match_cand_mfma operands: 1 = e2m1 +-1 nibbles on the MX-scaled
 * v_mfma_scale_f32_32x32x64_f8f6f4 (64 bits of K per instruction, 16 B per
 * 32 bits of a position), 0 = +-1 bytes on v_mfma_i32_32x32x32_i8 (32 bits
 * per instruction, 32 B); kernels_match.hip */
#ifndef ORBM_FP4
#define ORBM_FP4 1
#endif
/* row tiles of 32 per wave in k_match_cand_mfma (round 4, fp4 operands:
 * RT 1 at 95 VGPRs / 5 waves per SIMD beat RT 2 / 4 waves by 3 %, RT 4 lost
 * 15 %) and the waves per SIMD its register budget is cut for */
#ifndef MC_RT
#define MC_RT 1
#endif
/* k_match_cand_mfma column split (CS = 4 waves per row tile) below this many
   128-row workgroups in a launch (api_match.hip launch_match; 0 = never) */
/* drop-in calls stage their inputs with a kernel reading the pinned buffer
   (k_stage_in) instead of a DMA copy (A/B: 0) */
#ifndef ORBM_STAGE_KERNEL
#define ORBM_STAGE_KERNEL 1
#endif
#ifndef MC_CSPLIT_WGS
#define MC_CSPLIT_WGS 256
#endif
#ifndef MC_WPE
#define MC_WPE 5
#endif
/* k_match_cand_mfma: list positions carried in the MFMA accumulator (fp4
 * form, lists up to 2^14 / 2^13 positions for 6 / 8 live dwords; round 5),
 * 0 = keys built per element (A/B) */
#ifndef MC_PK
#define MC_PK 1
#endif
/* k_match_expand2 threads per list position: one per MFMA K step */
#define ORBM_EXPAND_PER_POS(NK) (ORBM_FP4 ? (NK) / 2 : (NK))

struct MProblem {
  const uint8_t* desc1;
  const uint8_t* desc2;
  const float* ang1;
  const float* ang2;
  const uint8_t* valid1;
  const uint8_t* valid2;
  const uint32_t* feat1;
  const uint32_t* feat2;
  int32_t* match12;
  int* nmatches;
  int ang_stride;  /* floats between consecutive angles (1, or 7 for orbx_keypoint) */
  int n1, n2;      /* features of KF1 / KF2 */
  int np_begin, np_end;
  int row_begin, row_end;
  int check_ori;
  float nnratio;
  int sequential;  /* 1: one wave walks all node pairs in order (malformed FeatureVectors) */
  int dcap;        /* candidate distance cap (orbm_dcap) */
  int th_low;      /* a best match needs d < th_low: ORBM_TH_LOW (KF-KF, :339), ORBM_TH_LOW + 1 for
                      upstream's KF-Frame form (bestDist1 <= TH_LOW) */
};

/* Smallest distance D >= th with (float)(th-1) < nnratio * (float)D, capped
 * at 257 (th = the problem's th_low).  Only candidates below D can change a
 * SearchByBoW decision: a best match needs d < th <= D, and a second-best
 * >= D always passes the ratio test (ORBmatcher.cc:339-342), exactly like the
 * true value. */
#if defined(__HIPCC__)
__host__ __device__
#endif
static inline int orbm_dcap(float nnratio, int th = ORBM_TH_LOW) {
  for (int D = th; D <= 256; ++D)
    if ((float)(th - 1) < nnratio * (float)D) return D;
  return 257;
}

struct MNodePair {
  int prob;
  int off1, n1;  /* list1 = feat1[off1 .. off1+n1) */
  int off2, n2;  /* list2 = feat2[off2 .. off2+n2) */
  int row_base;
  int g2;        /* list2 position j's descriptor is gdesc2[g2 + j] (k_match_gather2) */
};

#endif
