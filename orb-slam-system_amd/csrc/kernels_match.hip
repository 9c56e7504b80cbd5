// kernels_match.hip -- gfx950 kernels of ORBmatcher::SearchByBoW /
// DescriptorDistance (src/ORBmatcher.cc:278-366, 469-502, 896-908).
//
// SearchByBoW is greedy and order dependent (vbMatched2 excludes KF2
// features already taken by earlier KF1 features), so it is split into
//   k_match_candidates  fully parallel: per KF1 feature ("row") the ORBM_T
//                       best KF2 candidates by (distance, list position),
//                       one wavefront per row, XOR + v_bcnt Hamming.
//   k_match_resolve     the order-dependent part: one wavefront walks the
//                       rows of a node pair in list order; each row is one
//                       ballot over its candidates against an LDS bitmap of
//                       taken KF2 features (exact fallback: full rescan).
//                       Node pairs of a well-formed FeatureVector touch
//                       disjoint KF2 features, so they run in parallel.
//   k_match_finalize    rotation histogram + ComputeThreeMaxima + output.
#include <hip/hip_runtime.h>
#include <limits.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/orbx.h"
#include "match_internal.h"
#include "wave_ops.h"

namespace orbx {

__device__ __forceinline__ int hamming32(const uint32_t* a, const uint32_t* b) {
  const uint4 a0 = reinterpret_cast<const uint4*>(a)[0], a1 = reinterpret_cast<const uint4*>(a)[1];
  const uint4 b0 = reinterpret_cast<const uint4*>(b)[0], b1 = reinterpret_cast<const uint4*>(b)[1];
  return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
         __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

__device__ __forceinline__ int hamming_u(const uint32_t d1[8], const uint32_t* b) {
  const uint4 b0 = reinterpret_cast<const uint4*>(b)[0], b1 = reinterpret_cast<const uint4*>(b)[1];
  return __popc(d1[0] ^ b0.x) + __popc(d1[1] ^ b0.y) + __popc(d1[2] ^ b0.z) +
         __popc(d1[3] ^ b0.w) + __popc(d1[4] ^ b1.x) + __popc(d1[5] ^ b1.y) +
         __popc(d1[6] ^ b1.z) + __popc(d1[7] ^ b1.w);
}

// a generic pointer known to point into global memory: loads through it are
// global_load, which the wait counters order with the other vector memory
// ops (a flat_load may return out of order, so a flat load pending on any
// path makes the compiler wait for everything: vmcnt(0))
typedef const uint32_t __attribute__((address_space(1)))* gu32_t;
typedef const uint8_t __attribute__((address_space(1)))* gu8_t;
__device__ __forceinline__ int hamming_g(const uint32_t d1[8], gu32_t b) {
  int d = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) d += __popc(d1[k] ^ b[k]);  // two dwordx4 loads (32-B aligned rows)
  return d;
}

// 256-bit Hamming distance as one accumulate chain: v_bcnt_u32_b32 adds its
// second operand, so 8 xor + 8 bcnt (the compiler's add3 trees cost 3 more)
__device__ __forceinline__ uint32_t bcnt_acc(uint32_t x, uint32_t acc) {
  uint32_t r;
  asm("v_bcnt_u32_b32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(acc));
  return r;
}
__device__ __forceinline__ uint32_t ham256(uint4 a0, uint4 a1, uint4 b0, uint4 b1) {
  uint32_t d = bcnt_acc(a0.x ^ b0.x, 0u);
  d = bcnt_acc(a0.y ^ b0.y, d);
  d = bcnt_acc(a0.z ^ b0.z, d);
  d = bcnt_acc(a0.w ^ b0.w, d);
  d = bcnt_acc(a1.x ^ b1.x, d);
  d = bcnt_acc(a1.y ^ b1.y, d);
  d = bcnt_acc(a1.z ^ b1.z, d);
  return bcnt_acc(a1.w ^ b1.w, d);
}

typedef uint32_t v4u_ __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t ham256v(uint4 a0, uint4 a1, v4u_ b0, v4u_ b1) {
  uint32_t d = bcnt_acc(a0.x ^ b0.x, 0u);
  d = bcnt_acc(a0.y ^ b0.y, d);
  d = bcnt_acc(a0.z ^ b0.z, d);
  d = bcnt_acc(a0.w ^ b0.w, d);
  d = bcnt_acc(a1.x ^ b1.x, d);
  d = bcnt_acc(a1.y ^ b1.y, d);
  d = bcnt_acc(a1.z ^ b1.z, d);
  return bcnt_acc(a1.w ^ b1.w, d);
}

__device__ __forceinline__ int find_node_pair(const MNodePair* nps, int nnp, int r) {
  int lo = 0, hi = nnp;  // last np with row_base <= r
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (nps[mid].row_base <= r) lo = mid + 1; else hi = mid;
  }
  return lo - 1;
}

// ---------------------------------------------------------------------------
// k_match_candidates: one wave per row.  rowinfo[r] = {valid, nvalid2, minD}.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_match_candidates(
    const MProblem* __restrict__ probs, const MNodePair* __restrict__ nps, int nnp, int nrows,
    uint2* __restrict__ cand, int4* __restrict__ rowinfo, int2* __restrict__ ev) {
  __shared__ int hist[4][320];
  __shared__ uint32_t lessl[4][ORBM_T], eql[4][ORBM_T];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + wave;
  if (r >= nrows) return;
  if (lane == 0) ev[r] = make_int2(-1, 0);
  const int j = find_node_pair(nps, nnp, r);
  if (j < 0) { if (lane == 0) rowinfo[r] = make_int4(0, 0, 0, 0); return; }
  const MNodePair NP = nps[j];
  const int a = r - NP.row_base;
  if (a >= NP.n1) { if (lane == 0) rowinfo[r] = make_int4(0, 0, 0, 0); return; }
  const MProblem P = probs[NP.prob];
  const int idx1 = (int)P.feat1[NP.off1 + a];
  if (P.valid1 && !P.valid1[idx1]) { if (lane == 0) rowinfo[r] = make_int4(0, 0, 0, 0); return; }
  uint32_t d1[8];
  const uint32_t* q1 = reinterpret_cast<const uint32_t*>(P.desc1 + (size_t)idx1 * 32);
#pragma unroll
  for (int k = 0; k < 8; ++k) d1[k] = q1[k];
  for (int b = lane; b < 320; b += 64) hist[wave][b] = 0;
  __builtin_amdgcn_wave_barrier();
  int nvalid = 0;
  const uint32_t* f2 = P.feat2 + NP.off2;
  for (int jj = lane; jj < NP.n2; jj += 64) {
    const int idx2 = (int)f2[jj];
    if (P.valid2 && !P.valid2[idx2]) continue;
    const int d = hamming_u(d1, reinterpret_cast<const uint32_t*>(P.desc2 + (size_t)idx2 * 32));
    atomicAdd(&hist[wave][d], 1);
    ++nvalid;
  }
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) nvalid += __shfl_xor(nvalid, s, 64);
  __builtin_amdgcn_wave_barrier();
  // cutoff D: smallest d with #(dist <= d) >= T (5 bins per lane, wave scan)
  int h[5], hs = 0;
#pragma unroll
  for (int k = 0; k < 5; ++k) { h[k] = hist[wave][5 * lane + k]; hs += h[k]; }
  const int incl = wave_incl_scan(hs);
  const int excl = incl - hs;
  const uint64_t reach = __ballot(incl >= ORBM_T);
  int D = 1 << 20, cntLess = nvalid;  // nvalid < T: take everything
  if (reach) {
    const int L0 = __ffsll((unsigned long long)reach) - 1;
    int dd = 0, cl = 0;
    if (lane == L0) {
      int cum = excl;
      for (int k = 0; k < 5; ++k) {
        if (cum + h[k] >= ORBM_T) { dd = 5 * lane + k; cl = cum; break; }
        cum += h[k];
      }
    }
    D = lane_value(dd, L0);
    cntLess = lane_value(cl, L0);
  }
  const uint64_t nz = __ballot(hs > 0);
  int minD = 1 << 20;
  if (nz) {
    const int L1 = __ffsll((unsigned long long)nz) - 1;
    int md = 0;
    if (lane == L1) {
      for (int k = 4; k >= 0; --k) if (h[k] > 0) md = 5 * lane + k;
    }
    minD = lane_value(md, L1);
  }
  // ordered compaction: all entries with d < D, then the first (T - cntLess) with d == D
  const int needEq = ORBM_T - cntLess;
  int nl = 0, ne = 0;
  for (int base = 0; base < NP.n2; base += 64) {
    const int jj = base + lane;
    int d = 1 << 20;
    if (jj < NP.n2) {
      const int idx2 = (int)f2[jj];
      if (!(P.valid2 && !P.valid2[idx2]))
        d = hamming_u(d1, reinterpret_cast<const uint32_t*>(P.desc2 + (size_t)idx2 * 32));
    }
    const uint64_t ml = __ballot(d < D), me = __ballot(d == D);
    const uint64_t below = (1ull << lane) - 1ull;
    if (d < D) lessl[wave][nl + __popcll(ml & below)] = ((uint32_t)d << 16) | (uint32_t)jj;
    if (d == D) {
      const int rk = ne + __popcll(me & below);
      if (rk < needEq) eql[wave][rk] = ((uint32_t)d << 16) | (uint32_t)jj;
    }
    nl += __popcll(ml);
    ne += __popcll(me);
    if (nl >= cntLess && ne >= needEq) break;
  }
  __builtin_amdgcn_wave_barrier();
  const int nlt = min(nl, ORBM_T), neq = max(0, min(ne, needEq));
  uint2* out = cand + (size_t)r * ORBM_T;
  if (lane < nlt) {  // rank sort of the (< T) entries below the cutoff
    const uint32_t k = lessl[wave][lane];
    int rank = 0;
    for (int t = 0; t < nlt; ++t) rank += lessl[wave][t] < k;
    out[rank] = make_uint2(k, f2[k & 0xFFFFu]);
  }
  if (lane < ORBM_T && lane >= nlt) {
    const int e = lane - nlt;
    const uint32_t k = (e < neq) ? eql[wave][e] : 0xFFFFFFFFu;
    out[lane] = make_uint2(k, k != 0xFFFFFFFFu ? f2[k & 0xFFFFu] : 0u);
  }
  if (lane == 0) rowinfo[r] = make_int4(1, nvalid, minD, idx1);
}


// ---------------------------------------------------------------------------
// k_match_cand_lds: node pairs with n2 <= 64*NJ.  Workgroup = 64 rows of one
// node pair; list2 descriptors staged once in LDS; every row's distances stay
// in registers (NJ per lane).  rowinfo for every row; the sorted top-T
// (dist<<16|pos, idx2) list only for rows whose best distance is < TH_LOW
// (other rows can never be accepted and never change vbMatched2).
// ---------------------------------------------------------------------------
template <int NJ>
__global__ __launch_bounds__(256) void k_match_cand_lds(
    const MProblem* __restrict__ probs, const MNodePair* __restrict__ nps,
    uint2* __restrict__ cand, int4* __restrict__ rowinfo, int2* __restrict__ ev) {
  extern __shared__ uint4 sdesc[];  // 2 per list2 position
  __shared__ uint32_t svalid[NJ * 2];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const MNodePair NP = nps[blockIdx.y];
  const int a0 = blockIdx.x * 64;
  if (a0 >= NP.n1) return;
  const MProblem P = probs[NP.prob];
  const uint32_t* f2 = P.feat2 + NP.off2;
  const int n2 = NP.n2;
  for (int i = tid; i < NJ * 2; i += 256) svalid[i] = 0u;
  __syncthreads();
  for (int i = tid; i < 2 * n2; i += 256) {
    const uint32_t idx2 = f2[i >> 1];
    sdesc[i] = reinterpret_cast<const uint4*>(P.desc2 + (size_t)idx2 * 32)[i & 1];
    if ((i & 1) == 0 && !(P.valid2 && !P.valid2[idx2])) atomicOr(&svalid[(i >> 1) >> 5], 1u << ((i >> 1) & 31));
  }
  __syncthreads();
  const int INF = 0x7FFF;
  for (int rr = wave; rr < 64; rr += 4) {
    const int a = a0 + rr;
    if (a >= NP.n1) break;
    const int r = NP.row_base + a;
    if (lane == 0) ev[r] = make_int2(-1, 0);
    const int idx1 = (int)P.feat1[NP.off1 + a];
    if (P.valid1 && !P.valid1[idx1]) {
      if (lane == 0) rowinfo[r] = make_int4(0, 0, 0, idx1);
      continue;
    }
    const uint4 q0 = reinterpret_cast<const uint4*>(P.desc1 + (size_t)idx1 * 32)[0];
    const uint4 q1 = reinterpret_cast<const uint4*>(P.desc1 + (size_t)idx1 * 32)[1];
    int d[NJ];
    int mn = INF, nv = 0;
#pragma unroll
    for (int i = 0; i < NJ; ++i) {
      const int pos = lane + 64 * i;
      int dd = INF;
      if (pos < n2 && ((svalid[pos >> 5] >> (pos & 31)) & 1u)) {
        const uint4 b0 = sdesc[2 * pos], b1 = sdesc[2 * pos + 1];
        dd = __popc(q0.x ^ b0.x) + __popc(q0.y ^ b0.y) + __popc(q0.z ^ b0.z) + __popc(q0.w ^ b0.w) +
             __popc(q1.x ^ b1.x) + __popc(q1.y ^ b1.y) + __popc(q1.z ^ b1.z) + __popc(q1.w ^ b1.w);
        ++nv;
      }
      d[i] = dd;
      mn = min(mn, dd);
    }
#pragma unroll
    for (int s = 32; s >= 1; s >>= 1) {
      mn = min(mn, __shfl_xor(mn, s, 64));
      nv += __shfl_xor(nv, s, 64);
    }
    if (lane == 0) rowinfo[r] = make_int4(1, nv, mn >= INF ? (1 << 20) : mn, idx1);
    if (mn >= P.th_low) continue;
    uint2* out = cand + (size_t)r * ORBM_T;
    uint32_t key[NJ];
#pragma unroll
    for (int i = 0; i < NJ; ++i)
      key[i] = d[i] < INF ? (((uint32_t)d[i] << 16) | (uint32_t)(lane + 64 * i)) : 0xFFFFFFFFu;
    for (int t = 0; t < ORBM_T; ++t) {
      uint32_t best = key[0];
#pragma unroll
      for (int i = 1; i < NJ; ++i) best = min(best, key[i]);
#pragma unroll
      for (int s = 32; s >= 1; s >>= 1) best = min(best, (uint32_t)__shfl_xor((int)best, s, 64));
      if (lane == 0) out[t] = make_uint2(best, best != 0xFFFFFFFFu ? f2[best & 0xFFFFu] : 0u);
      if (best == 0xFFFFFFFFu) {
        if (lane > t && lane < ORBM_T) out[lane] = make_uint2(0xFFFFFFFFu, 0u);
        break;
      }
#pragma unroll
      for (int i = 0; i < NJ; ++i)
        if (key[i] == best) key[i] = 0xFFFFFFFFu;
    }
  }
}
template __global__ void k_match_cand_lds<32>(const MProblem*, const MNodePair*, uint2*, int4*, int2*);


// ---------------------------------------------------------------------------
// k_match_gather2: list2 descriptors of every node pair into node order,
// gdesc2[NP.g2 + j] = desc2[feat2[off2 + j]] (and, with a validity array,
// gval2[NP.g2 + j] = 0 if valid else ~0), so k_match_cand_rows reads each
// group of positions as contiguous scalar loads with no index indirection.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_match_gather2(const MProblem* __restrict__ probs,
                                                       const MNodePair* __restrict__ nps,
                                                       uint4* __restrict__ gdesc2,
                                                       uint32_t* __restrict__ gval2) {
  const MNodePair NP = nps[blockIdx.y];
  const int i = blockIdx.x * 256 + threadIdx.x;  // (position, half)
  const int j = i >> 1;
  if (j >= NP.n2) return;
  const MProblem& P = probs[NP.prob];
  const uint32_t idx2 = P.feat2[NP.off2 + j];
  gdesc2[(size_t)(NP.g2 + j) * 2 + (i & 1)] = reinterpret_cast<const uint4*>(P.desc2 + (size_t)idx2 * 32)[i & 1];
  if (gval2 && (i & 1) == 0) gval2[NP.g2 + j] = (P.valid2 && !P.valid2[idx2]) ? 0xFFFFFFFFu : 0u;
}

// ---------------------------------------------------------------------------
// k_match_cand_rows: 128 rows (KF1 features) per workgroup, two per lane
// (rows a0+lane and a0+64+lane); the 4 waves split the list2 positions
// (wave w takes quarter w of every chunk), so a 2000-row node pair runs 64
// waves and every descriptor read from LDS feeds 128 distances.  The
// gathered list2 descriptors (k_match_gather2) stream through two 16-KB LDS
// chunks: chunk c+1 is loaded into registers while chunk c is matched, then
// stored to the other buffer (one barrier per chunk).  Reads are
// wave-uniform (broadcast).  Each lane keeps, per row, its 8 smallest
// (distance<<16 | list position) keys sorted in registers; keys carry the
// position, so the 4 waves' lists merge (LDS) into exactly the first 8 of
// the reference's scan order.  A wave skips the insertion network when no
// lane improves.
// ---------------------------------------------------------------------------
#define MC_CHUNK 512  /* positions per LDS chunk (16 KB of descriptors) */

// sorted insertion of k into L (ascending): new L[t] = median(L[t-1], k, L[t])
// -- one v_min + 7 independent v_med3_u32 instead of a 16-deep min/max chain
__device__ __forceinline__ uint32_t med3u(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ void topk_insert(uint32_t (&L)[ORBM_T], uint32_t k) {
  // in place, last slot first: each result takes the register of the value
  // it replaces (ascending order made the allocator rotate 7 v_mov per insert)
#pragma unroll
  for (int t = ORBM_T - 1; t >= 1; --t) L[t] = med3u(L[t - 1], k, L[t]);
  L[0] = min(L[0], k);
}

// NW: descriptor dwords that can differ.  8 in general; 6 when both sides'
// bytes 24..31 are zero -- always so for orbx descriptors with the
// reference's 728-entry pattern (pairs 182..255 degenerate),
// checked by the host before choosing it: the same distances, 25 % fewer ops.
template <int NW>
__global__ __launch_bounds__(256) void k_match_cand_rows(
    const MProblem* __restrict__ probs, const MNodePair* __restrict__ nps,
    const uint4* __restrict__ gdesc2, const uint32_t* __restrict__ gval2,
    uint2* __restrict__ cand, int4* __restrict__ rowinfo, int2* __restrict__ ev) {
  static_assert(NW == 6 || NW == 8, "6 or 8 live descriptor dwords");
  __shared__ uint4 sdesc[2][2 * MC_CHUNK];        // 2 x 16 KB; the merge area aliases it
  __shared__ uint32_t sval[2][MC_CHUNK];          // per-position invalid masks (validity arrays only)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int bx, np;
  frame_unit(bx, np);  // a node pair's row chunks share one L2 (its list2)
  const MNodePair NP = nps[np];
  const int a0 = bx * 128;
  if (a0 >= NP.n1) return;  // workgroup-uniform
  const MProblem P = probs[NP.prob];
  const uint32_t* f2 = P.feat2 + NP.off2;
  const uint4* g2 = gdesc2 + (size_t)NP.g2 * 2;
  const uint32_t* gv = gval2 ? gval2 + NP.g2 : nullptr;
  const bool hasv = P.valid2 != nullptr;
  const int n2 = NP.n2;
  // the lane's two rows
  int idx1[2] = {0, 0};
  bool act[2], v1[2] = {false, false};
  uint4 q[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int a = a0 + 64 * h + lane;
    act[h] = a < NP.n1;
    q[h][0] = q[h][1] = make_uint4(0, 0, 0, 0);
    if (act[h]) {
      idx1[h] = (int)P.feat1[NP.off1 + a];
      v1[h] = !(P.valid1 && !P.valid1[idx1[h]]);
      q[h][0] = reinterpret_cast<const uint4*>(P.desc1 + (size_t)idx1[h] * 32)[0];
      q[h][1] = reinterpret_cast<const uint4*>(P.desc1 + (size_t)idx1[h] * 32)[1];
    }
  }
  // lists start full of sentinels at the distance cap: only d < dcap enters
  const uint32_t sent = (uint32_t)P.dcap << 16;
  uint32_t LA[ORBM_T], LB[ORBM_T];
#pragma unroll
  for (int t = 0; t < ORBM_T; ++t) LA[t] = LB[t] = sent;
  // chunk staging: thread loads uint4 entries tid + 256*u of a chunk
  uint4 pre[4];
  uint32_t prev[2];
  auto load_chunk = [&](int c0) {
    const int cn = min(MC_CHUNK, n2 - c0);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = tid + 256 * u;
      pre[u] = i < 2 * cn ? g2[(size_t)c0 * 2 + i] : make_uint4(0, 0, 0, 0);
    }
    if (hasv) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int i = tid + 256 * u;
        prev[u] = i < cn ? gv[c0 + i] : 0xFFFFFFFFu;
      }
    }
  };
  auto store_chunk = [&](int b) {
#pragma unroll
    for (int u = 0; u < 4; ++u) sdesc[b][tid + 256 * u] = pre[u];
    if (hasv) {
#pragma unroll
      for (int u = 0; u < 2; ++u) sval[b][tid + 256 * u] = prev[u];
    }
  };
  load_chunk(0);
  store_chunk(0);
  __syncthreads();
  int buf = 0;
  for (int c0 = 0; c0 < n2; c0 += MC_CHUNK, buf ^= 1) {  // workgroup-uniform
    const int cn = min(MC_CHUNK, n2 - c0);
    const bool more = c0 + MC_CHUNK < n2;
    if (more) load_chunk(c0 + MC_CHUNK);  // in flight while this chunk is matched
    const int qn = (((cn + 3) >> 2) + 7) & ~7;  // this wave's quarter (multiple of 8)
    const int jb = min(wave * qn, cn), je = min(jb + qn, cn);
    const int je8 = jb + ((je - jb) & ~3);
    const uint4* sd = sdesc[buf];
    for (int j0 = jb; j0 < je8; j0 += 4) {  // wave-uniform
      // 8 independent Hamming chains (4 positions x 2 rows), advanced one
      // descriptor word at a time: xors of all chains, then their v_bcnt
      // accumulates -- no back-to-back dependent VALU instructions
      uint4 lo[4], hi[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) lo[u] = sd[2 * (j0 + u)];
#pragma unroll
      for (int u = 0; u < 4; ++u) hi[u] = sd[2 * (j0 + u) + 1];
      uint32_t acc[2][4];
#pragma unroll
      for (int k = 0; k < NW; ++k) {
        uint32_t t[2][4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint4& b = k < 4 ? lo[u] : hi[u];
          const uint32_t bw = (k & 3) == 0 ? b.x : (k & 3) == 1 ? b.y : (k & 3) == 2 ? b.z : b.w;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const uint4& a = k < 4 ? q[h][0] : q[h][1];
            const uint32_t aw = (k & 3) == 0 ? a.x : (k & 3) == 1 ? a.y : (k & 3) == 2 ? a.z : a.w;
            t[h][u] = aw ^ bw;
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int h = 0; h < 2; ++h) acc[h][u] = bcnt_acc(t[h][u], k ? acc[h][u] : 0u);
      }
      uint32_t kA[4], kB[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t inval = hasv ? __builtin_amdgcn_readfirstlane(sval[buf][j0 + u]) : 0u;
        const uint32_t pos = (uint32_t)(c0 + j0 + u);
        kA[u] = ((acc[0][u] << 16) | pos) | inval;
        kB[u] = ((acc[1][u] << 16) | pos) | inval;
      }
      const uint32_t mA = min(min(kA[0], kA[1]), min(kA[2], kA[3]));
      const uint32_t mB = min(min(kB[0], kB[1]), min(kB[2], kB[3]));
      if (__ballot(mA < LA[ORBM_T - 1])) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (__ballot(kA[u] < LA[ORBM_T - 1])) topk_insert(LA, kA[u]);
      }
      if (__ballot(mB < LB[ORBM_T - 1])) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (__ballot(kB[u] < LB[ORBM_T - 1])) topk_insert(LB, kB[u]);
      }
    }
    for (int j = je8; j < je; ++j) {
      const uint4 b0 = sd[2 * j], b1 = sd[2 * j + 1];
      const uint32_t inval = hasv ? __builtin_amdgcn_readfirstlane(sval[buf][j]) : 0u;
      const uint32_t pos = (uint32_t)(c0 + j);
      const uint32_t ka = ((ham256(q[0][0], q[0][1], b0, b1) << 16) | pos) | inval;
      const uint32_t kb = ((ham256(q[1][0], q[1][1], b0, b1) << 16) | pos) | inval;
      if (__ballot(ka < LA[ORBM_T - 1])) topk_insert(LA, ka);
      if (__ballot(kb < LB[ORBM_T - 1])) topk_insert(LB, kb);
    }
    if (more) store_chunk(buf ^ 1);  // that buffer was last read before the previous barrier
    __syncthreads();
  }
  // merge the 4 waves' lists of each row (keys are unique: position inside)
  uint32_t* ml = reinterpret_cast<uint32_t*>(&sdesc[0][0]);  // [3][2][ORBM_T][64]
  if (wave > 0) {
#pragma unroll
    for (int t = 0; t < ORBM_T; ++t) {
      ml[(((wave - 1) * 2 + 0) * ORBM_T + t) * 64 + lane] = LA[t];
      ml[(((wave - 1) * 2 + 1) * ORBM_T + t) * 64 + lane] = LB[t];
    }
  }
  __syncthreads();
  if (wave > 0) return;
#pragma unroll
  for (int w = 0; w < 3; ++w)
#pragma unroll
    for (int t = 0; t < ORBM_T; ++t) {
      const uint32_t ka = ml[((w * 2 + 0) * ORBM_T + t) * 64 + lane];
      const uint32_t kb = ml[((w * 2 + 1) * ORBM_T + t) * 64 + lane];
      if (__ballot(ka < LA[ORBM_T - 1])) topk_insert(LA, ka);
      if (__ballot(kb < LB[ORBM_T - 1])) topk_insert(LB, kb);
    }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    uint32_t (&L)[ORBM_T] = h ? LB : LA;
    // a full list (no sentinel left) may have more candidates below the cap
    const bool full = L[ORBM_T - 1] < sent;
#pragma unroll
    for (int t = 0; t < ORBM_T; ++t)
      if (L[t] >= sent) L[t] = 0xFFFFFFFFu;
    if (!act[h]) continue;
    const int r = NP.row_base + a0 + 64 * h + lane;
    ev[r] = make_int2(-1, 0);
    if (!v1[h]) {
      rowinfo[r] = make_int4(0, 0, 0, idx1[h]);
      continue;
    }
    const int minD = L[0] != 0xFFFFFFFFu ? (int)(L[0] >> 16) : (1 << 20);
    // .y > ORBM_T: the list may be incomplete (resolve rescans when exhausted)
    rowinfo[r] = make_int4(1, full ? ORBM_T + 1 : 0, minD, idx1[h]);
    if (minD >= P.th_low) continue;
    uint4* out = reinterpret_cast<uint4*>(cand + (size_t)r * ORBM_T);
#pragma unroll
    for (int t = 0; t < ORBM_T / 2; ++t) {
      const uint32_t ka = L[2 * t], kb = L[2 * t + 1];
      out[t] = make_uint4(ka, ka != 0xFFFFFFFFu ? f2[ka & 0xFFFFu] : 0u, kb,
                          kb != 0xFFFFFFFFu ? f2[kb & 0xFFFFu] : 0u);
    }
  }
}

template __global__ void k_match_cand_rows<8>(const MProblem*, const MNodePair*, const uint4*,
                                              const uint32_t*, uint2*, int4*, int2*);
template __global__ void k_match_cand_rows<6>(const MProblem*, const MNodePair*, const uint4*,
                                              const uint32_t*, uint2*, int4*, int2*);

// ---------------------------------------------------------------------------
// Distances on the matrix cores.  With bits as +-1 bytes the i8 MFMA's dot
// product of a position's a' = 2a - 1 and a row's b' = 1 - 2b is
// sum_k -(+1 if a_k == b_k else -1) = 2 h - K (h = Hamming distance), so an
// accumulator started at K ends at 2 h and the candidate key
// (h << 16 | position) is (C << 15) + position.  k_match_expand2 writes the
// gathered list2 as such values; k_match_cand_mfma computes 32 positions x
// 32 rows per wave step and keeps the VALU for the top-T insertion only.
// Default (ORBM_FP4): the values are e2m1 nibbles (+-1.0 are exact) on the
// MX-scaled v_mfma_scale_f32_32x32x64_f8f6f4 with x1.0 block scales, K = 64
// bits per instruction in the cycles the i8 form spends on 32, and half the
// operand bytes; every partial sum is an integer below 2^24, so the f32
// accumulator is exact.  ORBM_FP4 0: +-1 bytes on v_mfma_i32_32x32x32_i8.
// ---------------------------------------------------------------------------
typedef int v4i_ __attribute__((ext_vector_type(4)));
typedef int v3i_ __attribute__((ext_vector_type(3)));
typedef int v16i_ __attribute__((ext_vector_type(16)));

// 4 bits -> 4 bytes of 0 / 1 (bit t -> byte t; the shifted copies never overlap)
__device__ __forceinline__ uint32_t nib_bytes(uint32_t n) { return (n * 0x00204081u) & 0x01010101u; }

// 16 bits -> 16 bytes: +1 / -1 for bit set / clear (pos = true), or the reverse
__device__ __forceinline__ v4i_ pm1_bytes(uint32_t bits, bool pos) {
  const uint32_t base = pos ? 0xFFFFFFFFu : 0x01010101u;  // x * 0xFE flips 0xFF <-> 0x01 per set bit
  v4i_ r;
#pragma unroll
  for (int q = 0; q < 4; ++q) r[q] = (int)(base ^ (nib_bytes((bits >> (4 * q)) & 15u) * 0xFEu));
  return r;
}

// 8 bits -> 8 nibbles (bit t -> bit 4t)
__device__ __forceinline__ uint32_t spread8_nib(uint32_t x) {
  x &= 0xFFu;
  x = (x | (x << 12)) & 0x000F000Fu;
  x = (x | (x << 6)) & 0x03030303u;
  return (x | (x << 3)) & 0x11111111u;
}

// 32 bits of K (16 from one dword, then 16 from the next) -> 32 e2m1
// nibbles: +1.0 (0x2) / -1.0 (0xA) for bit set / clear (pos = true), or the
// reverse; nibble t of the fragment is K element t
__device__ __forceinline__ v4i_ pm1_nibs(uint32_t lo16, uint32_t hi16, bool pos) {
  const uint32_t base = pos ? 0xAAAAAAAAu : 0x22222222u;  // ^ 8 flips 0xA <-> 0x2 per set bit
  v4i_ r;
  r[0] = (int)(base ^ (spread8_nib(lo16) << 3));
  r[1] = (int)(base ^ (spread8_nib(lo16 >> 8) << 3));
  r[2] = (int)(base ^ (spread8_nib(hi16) << 3));
  r[3] = (int)(base ^ (spread8_nib(hi16 >> 8) << 3));
  return r;
}

// i8 form (ORBM_FP4 0): gx2[(g2 + j) * 2 * NK + 2 * s + h] = bits 16h ..
// 16h+15 of dword s of the descriptor at list position j of the node pair
// (desc2[feat2[off2 + j]]), as +-1 bytes (a' = 2a - 1).  fp4 form:
// gx2[(g2 + j) * NK + 2 * m + h] = bits 16h .. 16h+15 of dwords 2m and
// 2m + 1 as +-1 nibbles (16 B per lane half and K step).  The list2 gather
// and the expansion in one pass (the MFMA path needs no packed copy).
template <int NK>
__global__ __launch_bounds__(256) void k_match_expand2(const MProblem* __restrict__ probs,
                                                       const MNodePair* __restrict__ nps,
                                                       v4i_* __restrict__ gx2) {
  const MNodePair NP = nps[blockIdx.y];
  constexpr int PER = ORBM_EXPAND_PER_POS(NK);
  const int i = blockIdx.x * 256 + threadIdx.x;  // (position, K step)
  const int j = i / PER, s = i - j * PER;
  if (j >= NP.n2) return;
  const MProblem& P = probs[NP.prob];
  const uint32_t idx2 = P.feat2[NP.off2 + j];
  v4i_* o = gx2 + ((size_t)(NP.g2 + j) * PER + s) * 2;
#if ORBM_FP4
  const uint2 w = reinterpret_cast<const uint2*>(P.desc2 + (size_t)idx2 * 32)[s];
  o[0] = pm1_nibs(w.x & 0xFFFFu, w.y & 0xFFFFu, true);
  o[1] = pm1_nibs(w.x >> 16, w.y >> 16, true);
#else
  const uint32_t w = reinterpret_cast<const uint32_t*>(P.desc2 + (size_t)idx2 * 32)[s];
  o[0] = pm1_bytes(w & 0xFFFFu, true);
  o[1] = pm1_bytes(w >> 16, true);
#endif
}
template __global__ void k_match_expand2<6>(const MProblem*, const MNodePair*, v4i_*);
template __global__ void k_match_expand2<8>(const MProblem*, const MNodePair*, v4i_*);

// one 32-position x 32-row tile: distances on the MFMA, keys and top-T
// insertions of the lane's 16 (row, position) values on the VALU
// hoff = 4h + (K << 15): the lane half's position offset and the K bias;
// value i of the tile is position t0 + (i & 3) + 8 (i >> 2) + 4h
typedef int v8i_ __attribute__((ext_vector_type(8)));
typedef float v16f_ __attribute__((ext_vector_type(16)));

// e2m1 operand in the f8f6f4 builtin's 8-dword slot (the backend keeps only
// the 4 dwords the FP4 format reads)
__device__ __forceinline__ v8i_ fp4_slot(const v4i_& x) { return v8i_{x[0], x[1], x[2], x[3], 0, 0, 0, 0}; }

// NS K steps (NK dwords: NK i8 steps of 32 bits, or NK / 2 fp4 steps of 64)
// fp4 form: the accumulator's start value 2^23 + K in every element (see
// mfma_tile), held in registers for the whole tile loop
template <int NS>
__device__ __forceinline__ v16f_ fp4_acc_init() {
  const float c0 = 8388608.0f + (float)(64 * NS);
  v16f_ ci = {c0, c0, c0, c0, c0, c0, c0, c0, c0, c0, c0, c0, c0, c0, c0, c0};
  asm volatile("" : "+v"(ci));  // a live tuple, not a per-tile re-splat
  return ci;
}

template <int NS>
__device__ __forceinline__ void mfma_tile(const v4i_ (&af)[NS], const v4i_ (&bf)[NS], uint32_t t0,
                                          int n2, uint32_t hoff, uint32_t (&L)[ORBM_T],
                                          const v16f_& ci) {
  uint32_t k[16];
#if ORBM_FP4
  // x1.0 block scales (E8M0 127); the f32 accumulator starts at 2^23 + K
  // (ci; hoff's K term is 0 here), so it ends at 2^23 + 2h: an exact integer
  // in [2^23, 2^24), whose bit pattern is 0x4B000000 + 2h, and 0x4B000000 <<
  // 15 vanishes mod 2^32, so key = bits << 15 + position as in the i8 form
  v16f_ C = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fp4_slot(af[0]), fp4_slot(bf[0]), ci, 4, 4,
                                                            0, 0x7F, 0, 0x7F);
#pragma unroll
  for (int s = 1; s < NS; ++s)
    C = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fp4_slot(af[s]), fp4_slot(bf[s]), C, 4, 4, 0,
                                                        0x7F, 0, 0x7F);
#pragma unroll
  for (int i = 0; i < 16; ++i)
    k[i] = (__float_as_uint(C[i]) << 15) + hoff + (t0 + (uint32_t)((i & 3) + 8 * (i >> 2)));
#else
  (void)ci;
  // accumulate from 0 (an inline-constant C operand, no per-tile init):
  // C = 2h - K, and K << 15 is folded into the position offsets
  v16i_ C = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[0], bf[0], v16i_{}, 0, 0, 0);
#pragma unroll
  for (int s = 1; s < NS; ++s) C = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[s], bf[s], C, 0, 0, 0);
#pragma unroll
  for (int i = 0; i < 16; ++i) k[i] = ((uint32_t)C[i] << 15) + hoff + (t0 + (uint32_t)((i & 3) + 8 * (i >> 2)));
#endif
  if (t0 + 32 > (uint32_t)n2) {  // last tile: positions past the list
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if ((hoff & 0x7FFFu) + t0 + (uint32_t)((i & 3) + 8 * (i >> 2)) >= (uint32_t)n2) k[i] = 0xFFFFFFFFu;
  }
  uint32_t m = min(min(min(k[0], k[1]), min(k[2], k[3])), min(min(k[4], k[5]), min(k[6], k[7])));
  m = min(m, min(min(min(k[8], k[9]), min(k[10], k[11])), min(min(k[12], k[13]), min(k[14], k[15]))));
  if (__ballot(m < L[ORBM_T - 1])) {
    // the 16 tests against the tile-start threshold, all issued before the
    // first insertion (an insertion of a key >= the current last entry is
    // a no-op, so a stale threshold only adds no-op insertions)
    const uint32_t l7 = L[ORBM_T - 1];
    unsigned long long bm[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) bm[i] = __ballot(k[i] < l7);
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (bm[i]) topk_insert(L, k[i]);
  }
}

#if ORBM_FP4
// Positions in the accumulator (fp4 form, round 5).  With A's MX block scale
// 2^PB every product is +-2^PB, so an accumulator started at
// 2^23 + K 2^PB + p (p = the element's list position, < 2^PB) ends at
// 2^23 + 2h 2^PB + p: an integer below 2^24 (2h <= 2K <= 384 for NK 6 with
// PB 14, <= 512 for NK 8 with PB 13), exact in f32, whose bit pattern
// 0x4B000000 + h 2^(PB+1) + p orders like (h, p) -- the key itself, with
// no per-key VALU (the plain form spends a shift and an add per key).  The
// per-tile start values are the lane's 16 constants plus t0 (8 v_pk_add_f32).
// Keys become (h << 16 | p) when the row's list is written out.
#define MC_PB(NK) ((NK) == 6 ? 14 : 13)
#define MC_KBASE 0x4B000000u
#ifndef MC_TOP3
#define MC_TOP3 1 /* 1: per-lane top-3 of the tile's 16 keys, two insertions (A/B: 0 = one per key) */
#endif
typedef float v2f_ __attribute__((ext_vector_type(2)));

template <int NS, int PB>
__device__ __forceinline__ void mfma_tile_pk(const v4i_ (&af)[NS], const v4i_ (&bf)[NS], float t0f,
                                             int n2, bool last, uint32_t (&L)[ORBM_T], const v16f_& cb) {
  v16f_ ci;
#pragma unroll
  for (int i = 0; i < 16; i += 2) {
    const v2f_ v = v2f_{cb[i], cb[i + 1]} + v2f_{t0f, t0f};
    ci[i] = v[0];
    ci[i + 1] = v[1];
  }
  v16f_ C = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fp4_slot(af[0]), fp4_slot(bf[0]), ci, 4, 4,
                                                            0, 0x7F + PB, 0, 0x7F);
#pragma unroll
  for (int s = 1; s < NS; ++s)
    C = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fp4_slot(af[s]), fp4_slot(bf[s]), C, 4, 4, 0,
                                                        0x7F + PB, 0, 0x7F);
  uint32_t k[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) k[i] = __float_as_uint(C[i]);
  if (last) {  // wave-uniform: positions past the list
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if ((k[i] & ((1u << PB) - 1u)) >= (uint32_t)n2) k[i] = 0xFFFFFFFFu;
  }
#if MC_TOP3
  // the lane's three smallest keys (two running chains of med3 insertions,
  // then the lower half of the bitonic 6-sequence a1 a2 a3 b3 b2 b1); on
  // these frames most tiles hold a lane with one key under its list's last
  // entry, few a lane with three: two wave-level insertions replace up to 16
  uint32_t a1 = min(k[0], k[1]), a2 = max(k[0], k[1]), a3 = 0xFFFFFFFFu;
  uint32_t b1 = min(k[8], k[9]), b2 = max(k[8], k[9]), b3 = 0xFFFFFFFFu;
#pragma unroll
  for (int i = 2; i < 8; ++i) {
    a3 = med3u(a2, k[i], a3);
    a2 = med3u(a1, k[i], a2);
    a1 = min(a1, k[i]);
    b3 = med3u(b2, k[8 + i], b3);
    b2 = med3u(b1, k[8 + i], b2);
    b1 = min(b1, k[8 + i]);
  }
  const uint32_t l1 = min(a1, b3), l2 = min(a2, b2), l3 = min(a3, b1);
  const uint32_t m1 = min(min(l1, l2), l3), m3 = max(max(l1, l2), l3);
  const uint32_t m2 = med3u(l1, l2, l3);
  if (__ballot(m1 < L[ORBM_T - 1])) {
    topk_insert(L, m1);
    if (__ballot(m2 < L[ORBM_T - 1])) {
      topk_insert(L, m2);
      if (__ballot(m3 < L[ORBM_T - 1])) {
        // some lane has a third key under its last entry: the remaining keys
        // (> m2; keys are unique in a lane) against the current threshold.
        // An insertion runs in every lane once any lane needs it, so keys a
        // lane already inserted (<= m2) become no-op keys first
        const uint32_t l7 = L[ORBM_T - 1];
        unsigned long long bm[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          k[i] = k[i] > m2 ? k[i] : 0xFFFFFFFFu;
          bm[i] = __ballot(k[i] < l7);
        }
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (bm[i]) topk_insert(L, k[i]);
      }
    }
  }
#else
  uint32_t m = min(min(min(k[0], k[1]), min(k[2], k[3])), min(min(k[4], k[5]), min(k[6], k[7])));
  m = min(m, min(min(min(k[8], k[9]), min(k[10], k[11])), min(min(k[12], k[13]), min(k[14], k[15]))));
  if (__ballot(m < L[ORBM_T - 1])) {
    const uint32_t l7 = L[ORBM_T - 1];
    unsigned long long bm[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) bm[i] = __ballot(k[i] < l7);
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (bm[i]) topk_insert(L, k[i]);
  }
#endif
}
#endif

// 128 * RT rows per workgroup, 32 * RT per wave: lane l holds rows
// a0 + 32 (RT w + t) + (l & 31), t < RT, as B operands (K bits of its half
// h = l >> 5 per step), and gets back C[position][row] for the 16 positions
// (i&3) + 8(i>>2) + 4h of each 32-position tile (gfx950 32x32 C layout).
// Each lane half keeps its own sorted top-T list per row; the halves merge
// through LDS at the end.  Positions are read as A fragments straight from
// gx2 (L1/L2: the waves of a workgroup and the node pair's other workgroups
// read the same tiles), one tile ahead; each fragment feeds RT MFMA chains.
// Validity arrays are not supported (k_match_cand_rows).
// PK (fp4 form, max n2 <= 2^MC_PB(NK)): positions in the accumulator
// (mfma_tile_pk); otherwise keys built per element (mfma_tile)
// CS > 1 (launches with fewer workgroups than CUs, e.g. one node pair of a
// drop-in call): the workgroup's CS waves take the same 32 rows and split
// the list's tiles CS ways; their top-T lists merge through LDS at the end
// (the exact top-T of the union: each part's top-T holds the union's members
// from that part).
template <int NK, int RT, bool PK, int CS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MC_WPE))) void k_match_cand_mfma(
    const MProblem* __restrict__ probs, const MNodePair* __restrict__ nps,
    const v4i_* __restrict__ gx2, uint2* __restrict__ cand, int4* __restrict__ rowinfo,
    int2* __restrict__ ev) {
  static_assert(NK == 6 || NK == 8, "6 or 8 live descriptor dwords");
  static_assert(CS == 1 || (CS == 4 && RT == 1), "column split: 4 waves on one row tile");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, c = lane & 31;
  int bx, np;
  frame_unit(bx, np);  // a node pair's row chunks share one L2 (its list2)
  const MNodePair NP = nps[np];
  const int a0 = bx * (CS == 1 ? 128 * RT : 32);
  if (a0 >= NP.n1) return;  // workgroup-uniform
  const MProblem P = probs[NP.prob];
  const uint32_t* f2 = P.feat2 + NP.off2;
  const int n2 = NP.n2;
  constexpr int NS = ORBM_EXPAND_PER_POS(NK);  // MFMA K steps per tile
  int a[RT], idx1[RT];
  bool act[RT], v1[RT];
  v4i_ bf[RT][NS];
  uint32_t L[RT][ORBM_T];
#if ORBM_FP4
  constexpr int PB = MC_PB(NK);
  const uint32_t sent = PK ? MC_KBASE + ((uint32_t)P.dcap << (PB + 1)) : (uint32_t)P.dcap << 16;
#else
  static_assert(!PK, "positions in the accumulator need the fp4 form");
  const uint32_t sent = (uint32_t)P.dcap << 16;
#endif
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    a[t] = a0 + 32 * (RT * (CS == 1 ? wave : 0) + t) + c;
    act[t] = a[t] < NP.n1;
    idx1[t] = 0;
    v1[t] = false;
    uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0;
    if (act[t]) {
      idx1[t] = (int)P.feat1[NP.off1 + a[t]];
      v1[t] = !(P.valid1 && !P.valid1[idx1[t]]);
      q0 = reinterpret_cast<const uint4*>(P.desc1 + (size_t)idx1[t] * 32)[0];
      q1 = reinterpret_cast<const uint4*>(P.desc1 + (size_t)idx1[t] * 32)[1];
    }
    const uint32_t dw[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
#pragma unroll
    for (int s = 0; s < NS; ++s)
#if ORBM_FP4
      bf[t][s] = pm1_nibs((dw[2 * s] >> (16 * h)) & 0xFFFFu, (dw[2 * s + 1] >> (16 * h)) & 0xFFFFu, false);
#else
      bf[t][s] = pm1_bytes((dw[s] >> (16 * h)) & 0xFFFFu, false);
#endif
#pragma unroll
    for (int u = 0; u < ORBM_T; ++u) L[t][u] = sent;
  }
  // the lane half's position offset (+ the i8 form's K bias, see mfma_tile)
  const uint32_t hoff = (uint32_t)(4 * h) + (ORBM_FP4 ? 0u : ((uint32_t)(32 * NK) << 15));
  const v4i_* gx = gx2 + (size_t)NP.g2 * NS * 2 + h;
  v4i_ af[NS], an[NS];
#if ORBM_FP4
  const v16f_ ci = fp4_acc_init<NS>();
  // PK: element i's start value without t0: 2^23 + K 2^PB + 4h + (i & 3) + 8 (i >> 2)
  v16f_ cb;
#pragma unroll
  for (int i = 0; i < 16; ++i)
    cb[i] = (float)(8388608 + (64 * NS << PB) + 4 * h + (i & 3) + 8 * (i >> 2));
#define MC_TILE(F, T0) \
  (PK ? mfma_tile_pk<NS, PB>(F, bf[t], (float)(T0), n2, (T0) + 32 > n2, L[t], cb) \
      : mfma_tile<NS>(F, bf[t], (uint32_t)(T0), n2, hoff, L[t], ci))
#else
  const v16f_ ci = {};
#define MC_TILE(F, T0) mfma_tile<NS>(F, bf[t], (uint32_t)(T0), n2, hoff, L[t], ci)
#endif
  // this wave's positions [tb, te): the whole list, or its tiles split CS ways
  int tb = 0, te = n2;
  if constexpr (CS > 1) {
    const int ntile = (n2 + 31) >> 5, tpw = (ntile + CS - 1) / CS;
    tb = 32 * min(ntile, wave * tpw);
    te = 32 * min(ntile, (wave + 1) * tpw);
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) af[s] = n2 > 0 ? gx[(size_t)min(tb + c, n2 - 1) * NS * 2 + 2 * s] : v4i_{0, 0, 0, 0};
#ifdef MC_NO_PINGPONG  // profiling variant: one fragment set copied forward per tile
  static_assert(CS == 1, "profiling variant: whole lists only");
  for (int t0 = 0; t0 < n2; t0 += 32) {  // wave-uniform
    const int pn = min(t0 + 32 + c, n2 - 1);
#pragma unroll
    for (int s = 0; s < NS; ++s) an[s] = gx[(size_t)pn * NS * 2 + 2 * s];  // next tile (clamped)
#pragma unroll
    for (int t = 0; t < RT; ++t) MC_TILE(af, t0);
#pragma unroll
    for (int s = 0; s < NS; ++s) af[s] = an[s];
  }
#else
  // two fragment sets in turn (tile t0 from af while an loads t0 + 32, then
  // the reverse): no register copies per tile
  for (int t0 = tb; t0 < te; t0 += 64) {  // wave-uniform
    const int pn = min(t0 + 32 + c, n2 - 1);
#pragma unroll
    for (int s = 0; s < NS; ++s) an[s] = gx[(size_t)pn * NS * 2 + 2 * s];
#pragma unroll
    for (int t = 0; t < RT; ++t) MC_TILE(af, t0);
    if (t0 + 32 >= te) break;  // wave-uniform
    const int pf = min(t0 + 64 + c, n2 - 1);
#pragma unroll
    for (int s = 0; s < NS; ++s) af[s] = gx[(size_t)pf * NS * 2 + 2 * s];
#pragma unroll
    for (int t = 0; t < RT; ++t) MC_TILE(an, t0 + 32);
  }
#endif
#undef MC_TILE
  // merge the two halves' lists of each row (keys unique: position inside):
  // lane c takes lane c + 32's list by cross-lane reads, so the kernel holds
  // no LDS and can share a CU with the extraction kernels of the next step
  // (k_pyramid leaves VGPRs but no LDS)
  uint32_t up[RT][ORBM_T];
#pragma unroll
  for (int t = 0; t < RT; ++t)
#pragma unroll
    for (int u = 0; u < ORBM_T; ++u) up[t][u] = (uint32_t)__shfl_down((int)L[t][u], 32, 64);
  if constexpr (CS > 1) {
    // halves first (lanes 32-63 insert no-op keys), then waves 1.. hand
    // their lists to wave 0 through LDS
    __shared__ uint32_t xl[CS - 1][32][ORBM_T + 1];
#pragma unroll
    for (int u = 0; u < ORBM_T; ++u) {
      const uint32_t kk = h ? 0xFFFFFFFFu : up[0][u];
      if (__ballot(kk < L[0][ORBM_T - 1])) topk_insert(L[0], kk);
    }
    if (wave > 0 && !h) {
#pragma unroll
      for (int u = 0; u < ORBM_T; ++u) xl[wave - 1][c][u] = L[0][u];
    }
    __syncthreads();
    if (wave > 0 || h) return;
    for (int w = 0; w < CS - 1; ++w) {
#pragma unroll
      for (int u = 0; u < ORBM_T; ++u) {
        const uint32_t kk = xl[w][c][u];
        if (__ballot(kk < L[0][ORBM_T - 1])) topk_insert(L[0], kk);
      }
    }
  } else {
    if (h) return;
  }
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    uint32_t (&Lt)[ORBM_T] = L[t];
    if constexpr (CS == 1) {
#pragma unroll
      for (int u = 0; u < ORBM_T; ++u) {
        const uint32_t kk = up[t][u];
        if (__ballot(kk < Lt[ORBM_T - 1])) topk_insert(Lt, kk);
      }
    }
    const bool full = Lt[ORBM_T - 1] < sent;
#pragma unroll
    for (int u = 0; u < ORBM_T; ++u) {
#if ORBM_FP4
      // PK: 0x4B000000 + h 2^(PB+1) + p -> h << 16 | p
      if (PK) Lt[u] = ((Lt[u] - MC_KBASE) >> (PB + 1) << 16) | (Lt[u] & ((1u << PB) - 1u));
#endif
      if (Lt[u] >= (PK ? (uint32_t)P.dcap << 16 : sent)) Lt[u] = 0xFFFFFFFFu;
    }
    if (!act[t]) continue;
    const int r = NP.row_base + a[t];
    ev[r] = make_int2(-1, 0);
    if (!v1[t]) {
      rowinfo[r] = make_int4(0, 0, 0, idx1[t]);
      continue;
    }
    const int minD = Lt[0] != 0xFFFFFFFFu ? (int)(Lt[0] >> 16) : (1 << 20);
    rowinfo[r] = make_int4(1, full ? ORBM_T + 1 : 0, minD, idx1[t]);
    if (minD >= P.th_low) continue;
    uint4* out = reinterpret_cast<uint4*>(cand + (size_t)r * ORBM_T);
#pragma unroll
    for (int u = 0; u < ORBM_T / 2; ++u) {
      const uint32_t ka = Lt[2 * u], kb = Lt[2 * u + 1];
      out[u] = make_uint4(ka, ka != 0xFFFFFFFFu ? f2[ka & 0xFFFFu] : 0u, kb,
                          kb != 0xFFFFFFFFu ? f2[kb & 0xFFFFu] : 0u);
    }
  }
}
#define MC_INST(NK, RT, PK, CS) \
  template __global__ void k_match_cand_mfma<NK, RT, PK, CS>(const MProblem*, const MNodePair*, const v4i_*, uint2*, int4*, int2*);
MC_INST(6, MC_RT, false, 1)
MC_INST(8, MC_RT, false, 1)
MC_INST(6, 1, false, 4)
MC_INST(8, 1, false, 4)
#if ORBM_FP4
MC_INST(6, MC_RT, true, 1)
MC_INST(8, MC_RT, true, 1)
MC_INST(6, 1, true, 4)
MC_INST(8, 1, true, 4)
#endif
#undef MC_INST

// ---------------------------------------------------------------------------
// k_match_resolve: greedy, in list order.  unit = node pair (parallel mode)
// or problem (sequential mode: all its node pairs, one bitmap).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void best_merge(uint32_t& k1, int& d2, uint32_t ok1, int od2) {
  // (k1, d2): smallest key (dist<<16|pos) and second-smallest distance of a multiset
  const uint32_t lo = min(k1, ok1), hi = max(k1, ok1);
  d2 = min(min(d2, od2), (int)(hi >> 16));
  k1 = lo;
}

__global__ __launch_bounds__(256) void k_match_resolve(
    const MProblem* __restrict__ probs, const MNodePair* __restrict__ nps, int nunits,
    int sequential, const uint2* __restrict__ cand, const int4* __restrict__ rowinfo,
    int2* __restrict__ ev) {
  __shared__ uint32_t bitmap[4][ORBM_MAX_N2 / 32 / 4];  // 512 words (16384 idx2) per wave
  __shared__ uint2 scand[4][64 * ORBM_T];                // one 64-row chunk of candidates per wave
  extern __shared__ uint32_t bigmap[];                   // used when n2 > 16384 (1 wave/block)
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int unit = blockIdx.x * (blockDim.x >> 6) + wave;
  if (unit >= nunits) return;
  int np0, np1;
  const MProblem* Pp;
  if (sequential) {
    Pp = &probs[unit];
    np0 = Pp->np_begin;
    np1 = Pp->np_end;
  } else {
    np0 = unit;
    np1 = unit + 1;
    Pp = &probs[nps[unit].prob];
  }
  const MProblem P = *Pp;
  uint32_t* bm = (P.n2 > 16384) ? bigmap : bitmap[wave];
  const int words = (P.n2 + 31) >> 5;
  for (int w = lane; w < words; w += 64) bm[w] = 0u;
  __builtin_amdgcn_wave_barrier();
  for (int j = np0; j < np1; ++j) {
    const MNodePair NP = nps[j];
    const uint32_t* f2 = P.feat2 + NP.off2;
    for (int base = 0; base < NP.n1; base += 64) {
      // rows in list order, 64 at a time; only rows that can pass TH_LOW matter
      int4 inf = make_int4(0, 0, 0, 0);
      if (base + lane < NP.n1) inf = rowinfo[NP.row_base + base + lane];
      uint64_t feas = __ballot(inf.x != 0 && inf.z < P.th_low);
      if (feas) {  // stage the chunk's candidate lists (contiguous rows) in LDS
        const int nr = min(64, NP.n1 - base);
        const uint4* src = reinterpret_cast<const uint4*>(cand + (size_t)(NP.row_base + base) * ORBM_T);
        uint4* dst = reinterpret_cast<uint4*>(scand[wave]);
        for (int q = lane; q < nr * ORBM_T / 2; q += 64) dst[q] = src[q];
        __builtin_amdgcn_wave_barrier();
      }
      while (feas) {
        const int l = __ffsll((unsigned long long)feas) - 1;
        feas &= feas - 1;
        const int r = NP.row_base + base + l;
        const int idx1 = lane_value(inf.w, l);
        const int nvalid2 = lane_value(inf.y, l);
        const uint2 c = lane < ORBM_T ? scand[wave][l * ORBM_T + lane] : make_uint2(0xFFFFFFFFu, 0u);
        const uint32_t key = c.x;
        const int idx2 = (int)c.y;
        const bool un = key != 0xFFFFFFFFu && !((bm[idx2 >> 5] >> (idx2 & 31)) & 1u);
        const uint64_t m = __ballot(un);
        int best1 = INT_MAX, best2 = INT_MAX, bidx2 = -1;
        if (__popcll(m) >= 2 || nvalid2 <= ORBM_T) {
          if (m) {
            const int l1 = __ffsll((unsigned long long)m) - 1;
            best1 = (int)(lane_value(key, l1) >> 16);
            bidx2 = lane_value(idx2, l1);
            const uint64_t m2 = m & (m - 1);
            if (m2) best2 = (int)(lane_value(key, __ffsll((unsigned long long)m2) - 1) >> 16);
          }
        } else {  // candidates exhausted: exact rescan of the node's list
          const uint32_t* q1 = reinterpret_cast<const uint32_t*>(P.desc1 + (size_t)idx1 * 32);
          uint32_t d1[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) d1[k] = q1[k];
          uint32_t k1 = 0xFFFFFFFFu;
          int d2 = INT_MAX;
          for (int jj = lane; jj < NP.n2; jj += 64) {
            const int i2 = (int)f2[jj];
            if (P.valid2 && !P.valid2[i2]) continue;
            if ((bm[i2 >> 5] >> (i2 & 31)) & 1u) continue;
            const int d = hamming_u(d1, reinterpret_cast<const uint32_t*>(P.desc2 + (size_t)i2 * 32));
            best_merge(k1, d2, ((uint32_t)d << 16) | (uint32_t)jj, INT_MAX);
          }
#pragma unroll
          for (int s = 32; s >= 1; s >>= 1) {
            const uint32_t ok = __shfl_xor(k1, s, 64);
            const int od = __shfl_xor(d2, s, 64);
            best_merge(k1, d2, ok, od);
          }
          if (k1 != 0xFFFFFFFFu) {
            best1 = (int)(k1 >> 16);
            bidx2 = (int)f2[k1 & 0xFFFFu];
            best2 = d2;
          }
        }
        if (best1 < P.th_low && (float)best1 < P.nnratio * (float)best2) {
          if (lane == 0) {  // rotation bin: k_match_finalize
            bm[bidx2 >> 5] |= 1u << (bidx2 & 31);
            ev[r] = make_int2(bidx2, 0);
          }
          __builtin_amdgcn_wave_barrier();
        }
      }
    }
  }
}


// ---------------------------------------------------------------------------
// k_match_resolve_spec: the greedy walk, 64 rows at a time, speculatively.
// One wavefront per node pair (well-formed FeatureVectors, n2 <= n2cap).
// Each round every pending row of the chunk decides against the committed
// vbMatched2 bitmap; accepted rows claim their KF2 feature (LDS atomicMin of
// the lane); a row whose examined candidates include a feature claimed by an
// earlier row of the chunk -- or whose candidate list ran out -- is a
// boundary: every pending row before it is exactly what the serial walk
// would decide, so those commit together and the rest re-decide.
// ---------------------------------------------------------------------------
#ifndef RS_NB
#define RS_NB 2
#endif
// RS_EVB: a chunk's accepted rows are stored once per lane after its rounds
// (each lane owns its row), so no store sits between the look-ahead loads
#ifndef RS_EVB
#define RS_EVB 1
#endif
#ifndef RS_RU  // rescan batch (list positions per lane)
#define RS_RU 8
#endif
#if RS_EVB
#define RS_EV_COMMIT(id) (evl = (id))
#else
#define RS_EV_COMMIT(id) (ev[r] = make_int2((id), 0))
#endif
__global__ __launch_bounds__(64) void k_match_resolve_spec(
    const MProblem* __restrict__ probs, const MNodePair* __restrict__ nps, int nunits,
    const uint2* __restrict__ cand, const int4* __restrict__ rowinfo, int2* __restrict__ ev,
    int n2cap) {
  extern __shared__ uint32_t sm[];
  uint32_t* bm = sm;                                   // (n2cap + 31) / 32 words
  int* claim = reinterpret_cast<int*>(sm + ((n2cap + 31) >> 5));  // n2cap
  uint2* cs = reinterpret_cast<uint2*>(sm + ((((n2cap + 31) >> 5) + n2cap + 1) & ~1));  // 64 * ORBM_T
  const int lane = threadIdx.x;
  const int unit = blockIdx.x;
  if (unit >= nunits) return;
  const MNodePair NP = nps[unit];
  const MProblem P = probs[NP.prob];
  const gu32_t gf2 = (gu32_t)(P.feat2 + NP.off2);
  for (int w = lane; w < ((P.n2 + 31) >> 5); w += 64) bm[w] = 0u;
  for (int w = lane; w < P.n2; w += 64) claim[w] = 64;
  __builtin_amdgcn_wave_barrier();
  // row info + candidate lists of the RS_NB chunks ahead are in flight while
  // a chunk resolves (RS_NB register buffers, used in turn; one wave per
  // node pair, so registers are not what limits this kernel -- the walk is
  // bound by the latency of these loads)
  // (unconditional loads at a clamped row: a load under a divergent branch
  // would be waited for at the branch join; rows past n1 are masked in chunk)
  // (the row info as a 3-vector: with an int4 the unused w register was
  // taken for a temporary, whose write then waited for the load in flight)
  auto fetch = [&](v3i_& inf_n, uint4 (&cv_n)[ORBM_T / 2], int base) {
    const int r = NP.row_base + min(base + lane, NP.n1 - 1);
    inf_n = *reinterpret_cast<const v3i_*>(rowinfo + r);
    const uint4* src = reinterpret_cast<const uint4*>(cand + (size_t)r * ORBM_T);
#pragma unroll
    for (int t = 0; t < ORBM_T / 2; ++t) cv_n[t] = src[t];
  };
#ifdef RS_STATS
  int st_feas = 0, st_chunks = 0, st_rounds = 0, st_hard = 0;
#endif
  auto chunk = [&](v3i_& inf_n, uint4 (&cv_n)[ORBM_T / 2], int base) {
    const int r = NP.row_base + base + lane;
    // nothing of the row info stays live across the refill below, so the
    // refill reuses the buffer's registers (with a buffer live across the
    // fetch, the refill took other registers and the loop latch copied them
    // back, waiting on every load in flight): the rounds need only the
    // wave-uniform "list longer than the candidates" mask, and the rare
    // rescan re-reads its row's idx1
    const v3i_ inf = inf_n;
    const bool feas = base + lane < NP.n1 && inf[0] != 0 && inf[2] < P.th_low;
    const uint64_t longl = __ballot(inf[1] > ORBM_T);
    uint2 c[ORBM_T];
#pragma unroll
    for (int t = 0; t < ORBM_T / 2; ++t) {
      c[2 * t] = feas ? make_uint2(cv_n[t].x, cv_n[t].y) : make_uint2(0xFFFFFFFFu, 0u);
      c[2 * t + 1] = feas ? make_uint2(cv_n[t].z, cv_n[t].w) : make_uint2(0xFFFFFFFFu, 0u);
    }
    // the selects happen here, not sunk past the refill (which would keep
    // cv_n live across it)
#pragma unroll
    for (int t = 0; t < ORBM_T; ++t) asm volatile("" : "+v"(c[t].x), "+v"(c[t].y));
    // the buffer is consumed before it is refilled, so the refill can take the
    // same registers (otherwise the loop latch copies it, waiting on vmcnt)
    __builtin_amdgcn_sched_barrier(0);
    fetch(inf_n, cv_n, base + 64 * RS_NB);  // unconditional (clamped rows)
    uint64_t pend = __ballot(feas);
    if (!pend) return;
#if RS_EVB
    int evl = -1;  // the lane's accepted KF2 feature, stored once after the rounds
#endif
#ifdef RS_STATS
    st_feas += __popcll(pend); st_chunks++;
#endif
    // per chunk: the lane's valid-slot mask, and its candidate list in LDS
    // (slot t of lane l at cs[64 t + l]) for the rounds' indexed reads
    uint32_t V = 0;
#pragma unroll
    for (int t = 0; t < ORBM_T; ++t) {
      V |= (c[t].x != 0xFFFFFFFFu ? 1u : 0u) << t;
      cs[64 * t + lane] = c[t];
    }
    while (pend) {
#ifdef RS_STATS
      st_rounds++;
#endif
      const bool mine = (pend >> lane) & 1ull;
      // all bitmap words first (independent LDS reads, one wait); empty
      // slots read word 0 harmlessly.  The in-order scan for the first two
      // unmatched candidates is a bit mask: U = valid & ~matched, first =
      // lowest set bit, second = next one; their keys come from the lane's
      // LDS slots (one read each) -- branch-free, where a per-slot scan
      // chained 8 conditional steps through exec masks
      uint32_t bw[ORBM_T];
#pragma unroll
      for (int t = 0; t < ORBM_T; ++t) bw[t] = bm[c[t].y >> 5];
      uint32_t B = 0;
#pragma unroll
      for (int t = 0; t < ORBM_T; ++t) B |= ((bw[t] >> (c[t].y & 31u)) & 1u) << t;
      const uint32_t U = V & ~B, U2 = U & (U - 1u);
      const int fi = __ffs(U) - 1, si = __ffs(U2) - 1;  // -1: none
      const uint2 e1 = cs[64 * max(fi, 0) + lane];
      const uint32_t e2 = cs[64 * max(si, 0) + lane].x;
      const int k1 = U ? (int)(e1.x >> 16) : INT_MAX;
      const int id1 = (int)e1.y;  // used only when accepted (U != 0)
      const int k2 = U2 ? (int)(e2 >> 16) : INT_MAX;
      const int plen = U2 ? si + 1 : ORBM_T;  // slots the serial walk examined
      const bool hard = mine && U2 == 0u && ((longl >> lane) & 1ull);  // list exhausted: needs a rescan
      const bool acc = mine && !hard && k1 < P.th_low && (float)k1 < P.nnratio * (float)k2;
      if (acc) atomicMin(&claim[id1], lane);
      __builtin_amdgcn_wave_barrier();
      int cl[ORBM_T];
#pragma unroll
      for (int t = 0; t < ORBM_T; ++t) cl[t] = claim[c[t].y];
      // slots claimed by an earlier lane (cl - lane < 0 for cl, lane in [0, 64])
      uint32_t CL = 0;
#pragma unroll
      for (int t = 0; t < ORBM_T; ++t) CL |= ((uint32_t)(cl[t] - lane) >> 31) << t;
      const bool conf = mine && (CL & V & ((1u << plen) - 1u)) != 0u;
      const uint64_t cm = __ballot(conf || hard);
      const int bnd = cm ? (__ffsll((unsigned long long)cm) - 1) : 64;
      __builtin_amdgcn_wave_barrier();
      if (acc) claim[id1] = 64;
      if (mine && lane < bnd && acc) {  // rotation bin: k_match_finalize
        atomicOr(&bm[id1 >> 5], 1u << (id1 & 31));
        RS_EV_COMMIT(id1);
      }
      __builtin_amdgcn_wave_barrier();
      pend &= (bnd >= 64) ? 0ull : ~((1ull << bnd) - 1ull);
      if (pend && bnd < 64 && ((__ballot(hard) >> bnd) & 1ull)) {
        // lowest pending row ran out of candidates: exact rescan of list2 (whole wave)
#ifdef RS_STATS
        st_hard++;
#endif
        const int idx1 = rowinfo[NP.row_base + base + bnd].w;
        const gu32_t q1 = (gu32_t)(P.desc1 + (size_t)idx1 * 32);
        uint32_t d1[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) d1[k] = q1[k];
        uint32_t kb = 0xFFFFFFFFu;
        int d2 = INT_MAX;
        // RS_RU list positions per lane at a time: every index, then every
        // descriptor (and validity byte) load of the batch issued before the
        // first use, unconditionally at clamped positions -- one loop step
        // per position, with its two dependent loads and a divergent
        // continue, made a rescan ~60 us (n2 = 2000), longer than the walk
        const gu8_t gv2 = (gu8_t)P.valid2;
        // validity bytes only when the problem has them (one uniform branch
        // per rescan, not a branch and a wait per position)
        auto scan = [&](auto hv) {
          constexpr bool HV = decltype(hv)::value;
          for (int j0 = 0; j0 < NP.n2; j0 += 64 * RS_RU) {
            int i2[RS_RU];
#pragma unroll
            for (int u = 0; u < RS_RU; ++u) i2[u] = (int)gf2[min(j0 + 64 * u + lane, NP.n2 - 1)];
            v4u_ da[RS_RU], db[RS_RU];
            uint8_t vv[RS_RU];
#pragma unroll
            for (int u = 0; u < RS_RU; ++u) {
              typedef const v4u_ __attribute__((address_space(1)))* gv4u_t;
              const gv4u_t q = (gv4u_t)(P.desc2 + (size_t)i2[u] * 32);
              da[u] = q[0];
              db[u] = q[1];
              vv[u] = HV ? gv2[i2[u]] : (uint8_t)1;
            }
#pragma unroll
            for (int u = 0; u < RS_RU; ++u) {
              const int jj = j0 + 64 * u + lane;
              const int d = (int)ham256v(make_uint4(d1[0], d1[1], d1[2], d1[3]),
                                         make_uint4(d1[4], d1[5], d1[6], d1[7]), da[u], db[u]);
              const bool ok = jj < NP.n2 && vv[u] && !((bm[i2[u] >> 5] >> (i2[u] & 31)) & 1u);
              if (ok) best_merge(kb, d2, ((uint32_t)d << 16) | (uint32_t)jj, INT_MAX);
            }
          }
        };
        if (gv2) scan(std::true_type{});
        else scan(std::false_type{});
#pragma unroll
        for (int s = 32; s >= 1; s >>= 1) {
          const uint32_t ok = __shfl_xor(kb, s, 64);
          const int od = __shfl_xor(d2, s, 64);
          best_merge(kb, d2, ok, od);
        }
        if (kb != 0xFFFFFFFFu) {
          const int b1 = (int)(kb >> 16), bi = (int)gf2[kb & 0xFFFFu];
          if (b1 < P.th_low && (float)b1 < P.nnratio * (float)d2 && lane == bnd) {
            atomicOr(&bm[bi >> 5], 1u << (bi & 31));
            RS_EV_COMMIT(bi);
          }
        }
        __builtin_amdgcn_wave_barrier();
        // nothing of the rescan left in flight: its last loads would otherwise
        // make the waitcnt pass wait for every load at the next round's first
        // register reuse -- the look-ahead loads included
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), rare path
        pend &= ~(1ull << bnd);
      }
    }
#if RS_EVB
    if (evl >= 0) ev[r] = make_int2(evl, 0);
#endif
  };
  v3i_ inf[RS_NB];
  uint4 cv[RS_NB][ORBM_T / 2];
  if (NP.n1 <= 0) return;
#pragma unroll
  for (int b = 0; b < RS_NB; ++b) {
    fetch(inf[b], cv[b], 64 * b);
    __builtin_amdgcn_sched_barrier(0);  // issue order = use order (the loop's waits count on it)
  }
  // every buffer is refilled exactly once per iteration and the loop has one
  // exit, at the latch: a chunk past n1 only refills its buffer (clamped
  // rows) and finds no pending row.  With an exit after each chunk the CFG
  // structurizer merged the exits into one flow block that also reaches the
  // header, on a path where the other buffer was never refilled, and the
  // waitcnt pass then waited for every load in flight at the header (the
  // look-ahead was one chunk, not RS_NB)
  for (int base = 0; base < NP.n1; base += 64 * RS_NB) {
#pragma unroll
    for (int b = 0; b < RS_NB; ++b) chunk(inf[b], cv[b], base + 64 * b);
  }
#ifdef RS_STATS
  if (lane == 0)
    printf("RS unit %d n1 %d n2 %d feas %d chunks %d rounds %d hard %d\n", unit, NP.n1, NP.n2,
           st_feas, st_chunks, st_rounds, st_hard);
#endif
}

// ---------------------------------------------------------------------------
// k_match_finalize: one workgroup per problem.
// ---------------------------------------------------------------------------
// ComputeThreeMaxima (ORBmatcher.cc:469-502), one thread
__device__ __forceinline__ void three_maxima(const int* hist, int* ind) {
  int ti[3] = {-1, -1, -1}, tv[3] = {0, 0, 0};
  int hv[ORBM_HISTO];  // every bin read up front (independent LDS reads)
#pragma unroll
  for (int i = 0; i < ORBM_HISTO; ++i) hv[i] = hist[i];
#pragma unroll
  for (int i = 0; i < ORBM_HISTO; ++i) {
    const int v = hv[i];
    for (int jj = 0; jj < 3; ++jj) {
      if (v > tv[jj]) {
        for (int k = 2; k > jj; --k) { tv[k] = tv[k - 1]; ti[k] = ti[k - 1]; }
        tv[jj] = v;
        ti[jj] = i;
        break;
      }
    }
  }
  if (tv[1] < 0.1f * tv[0]) { ti[1] = -1; ti[2] = -1; }
  else if (tv[2] < 0.1f * tv[0]) { ti[2] = -1; }
  ind[0] = ti[0]; ind[1] = ti[1]; ind[2] = ti[2];
}

__global__ __launch_bounds__(256) void k_match_finalize(const MProblem* __restrict__ probs,
                                                        const MNodePair* __restrict__ nps,
                                                        const int4* __restrict__ rowinfo,
                                                        int2* __restrict__ ev,
                                                        int* __restrict__ last_scratch,
                                                        const int* __restrict__ scratch_off) {
  __shared__ int hist[ORBM_HISTO];
  __shared__ int ind[3];
  __shared__ int s_nev, s_nfilt;
  const int p = blockIdx.x, tid = threadIdx.x;
  const MProblem P = probs[p];
  const float factor = 1.0f / ORBM_HISTO;
  int* last = last_scratch + scratch_off[p];
  // global views of the problem's arrays (generic pointers read from
  // MProblem would compile to flat_load / flat_store)
  typedef int __attribute__((address_space(1)))* gi32_t;
  typedef const float __attribute__((address_space(1)))* gf32_t;
  const gi32_t m12 = (gi32_t)P.match12;
  // the problem's rows are one contiguous range: node pairs are laid out in
  // order from np_begin (api_match.hip: the merge-join assigns row_base
  // sequentially; a batched plan has one node pair per problem)
  const int rb = P.np_end > P.np_begin ? nps[P.np_begin].row_base : 0;
  const int re = P.np_end > P.np_begin ? nps[P.np_end - 1].row_base + nps[P.np_end - 1].n1 : 0;
  constexpr int FZ_U = 8;
  // every row in one batch per thread (a problem of <= 2048 rows: the
  // bench's, a drop-in call's): the rows' matches, KF1 indices and bins
  // stay in registers for the three passes instead of being re-read, and
  // their loads are issued ahead of the initialisation below
  const bool one = re > rb && re - rb <= 256 * FZ_U;
  int2 e1[FZ_U];
  int i1r[FZ_U];
  if (one) {
#pragma unroll
    for (int u = 0; u < FZ_U; ++u) {
      const int r = min(rb + tid + 256 * u, re - 1);
      e1[u] = ev[r];
      i1r[u] = rowinfo[r].w;
    }
  }
  for (int i = tid; i < P.n1; i += 256) {
    m12[i] = -1;
    last[i] = -1;
  }
  if (tid < ORBM_HISTO) hist[tid] = 0;
  if (tid == 0) { s_nev = 0; s_nfilt = 0; }
  __syncthreads();
  // Otherwise each thread walks its rows FZ_U at a time: every load of a
  // batch is issued before the first use (clamped rows, masked below),
  // instead of three dependent round trips per row
  int nev = 0;
  if (one) {
    int2 e[FZ_U];
    int i1[FZ_U], bin[FZ_U];
#pragma unroll
    for (int u = 0; u < FZ_U; ++u) {
      e[u] = e1[u];
      i1[u] = i1r[u];
      bin[u] = 0;
    }
    if (P.check_ori) {
      float rot[FZ_U];
#pragma unroll
      for (int u = 0; u < FZ_U; ++u)
        rot[u] = e[u].x >= 0 ? ((gf32_t)P.ang1)[(size_t)i1[u] * P.ang_stride] -
                                   ((gf32_t)P.ang2)[(size_t)e[u].x * P.ang_stride]
                             : 0.0f;
#pragma unroll
      for (int u = 0; u < FZ_U; ++u) {
        float ro = rot[u];
        if (ro < 0.0f) ro += 360.0f;
        bin[u] = (int)roundf(ro * factor);  // rotation histogram bin (ORBmatcher.cc:332-340)
        if (bin[u] == ORBM_HISTO) bin[u] = 0;
      }
    }
#pragma unroll
    for (int u = 0; u < FZ_U; ++u) {
      const int r = rb + tid + 256 * u;
      if (r >= re || e[u].x < 0) continue;
      atomicMax(&last[i1[u]], r);
      atomicAdd(&hist[bin[u]], 1);
      ++nev;
    }
    atomicAdd(&s_nev, nev);
    __syncthreads();
    if (tid == 0) three_maxima(hist, ind);
    __syncthreads();
    int l[FZ_U];
#pragma unroll
    for (int u = 0; u < FZ_U; ++u) l[u] = last[i1[u]];
#pragma unroll
    for (int u = 0; u < FZ_U; ++u) {
      const int r = rb + tid + 256 * u;
      if (r < re && e[u].x >= 0 && l[u] == r) m12[i1[u]] = e[u].x;
    }
    __syncthreads();
    int nf = 0;
    if (P.check_ori) {
      const int b0 = ind[0], b1 = ind[1], b2 = ind[2];
#pragma unroll
      for (int u = 0; u < FZ_U; ++u) {
        const int r = rb + tid + 256 * u;
        if (r >= re || e[u].x < 0) continue;
        if (bin[u] == b0 || bin[u] == b1 || bin[u] == b2) continue;
        m12[i1[u]] = -2;  // set to nullptr by the rotation check (:359)
        ++nf;
      }
    }
    atomicAdd(&s_nfilt, nf);
    __syncthreads();
    if (tid == 0) *P.nmatches = s_nev - s_nfilt;
    return;
  }
  for (int r0 = rb + tid; r0 < re; r0 += 256 * FZ_U) {
    int2 e[FZ_U];
    int i1[FZ_U];
#pragma unroll
    for (int u = 0; u < FZ_U; ++u) {
      const int r = min(r0 + 256 * u, re - 1);
      e[u] = ev[r];
      i1[u] = rowinfo[r].w;
    }
    float rot[FZ_U];
    if (P.check_ori) {
#pragma unroll
      for (int u = 0; u < FZ_U; ++u)
        rot[u] = e[u].x >= 0 ? ((gf32_t)P.ang1)[(size_t)i1[u] * P.ang_stride] -
                                   ((gf32_t)P.ang2)[(size_t)e[u].x * P.ang_stride]
                             : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < FZ_U; ++u) {
      const int r = r0 + 256 * u;
      if (r >= re || e[u].x < 0) continue;
      int bin = 0;  // rotation histogram bin (ORBmatcher.cc:332-340)
      if (P.check_ori) {
        float ro = rot[u];
        if (ro < 0.0f) ro += 360.0f;
        bin = (int)roundf(ro * factor);
        if (bin == ORBM_HISTO) bin = 0;
        ev[r].y = bin;  // read back by this thread below
      }
      atomicMax(&last[i1[u]], r);
      atomicAdd(&hist[bin], 1);
      ++nev;
    }
  }
  atomicAdd(&s_nev, nev);
  __syncthreads();
  if (tid == 0) three_maxima(hist, ind);
  __syncthreads();
  for (int r0 = rb + tid; r0 < re; r0 += 256 * FZ_U) {
    int2 e[FZ_U];
    int i1[FZ_U], l[FZ_U];
#pragma unroll
    for (int u = 0; u < FZ_U; ++u) {
      const int r = min(r0 + 256 * u, re - 1);
      e[u] = ev[r];
      i1[u] = rowinfo[r].w;
    }
#pragma unroll
    for (int u = 0; u < FZ_U; ++u) l[u] = last[i1[u]];
#pragma unroll
    for (int u = 0; u < FZ_U; ++u) {
      const int r = r0 + 256 * u;
      if (r < re && e[u].x >= 0 && l[u] == r) m12[i1[u]] = e[u].x;
    }
  }
  __syncthreads();
  int nf = 0;
  if (P.check_ori) {
    const int b0 = ind[0], b1 = ind[1], b2 = ind[2];
    for (int r0 = rb + tid; r0 < re; r0 += 256 * FZ_U) {
      int2 e[FZ_U];
      int i1[FZ_U];
#pragma unroll
      for (int u = 0; u < FZ_U; ++u) {
        const int r = min(r0 + 256 * u, re - 1);
        e[u] = ev[r];
        i1[u] = rowinfo[r].w;
      }
#pragma unroll
      for (int u = 0; u < FZ_U; ++u) {
        const int r = r0 + 256 * u;
        if (r >= re || e[u].x < 0) continue;
        if (e[u].y == b0 || e[u].y == b1 || e[u].y == b2) continue;
        m12[i1[u]] = -2;  // set to nullptr by the rotation check (:359)
        ++nf;
      }
    }
  }
  atomicAdd(&s_nfilt, nf);
  __syncthreads();
  if (tid == 0) *P.nmatches = s_nev - s_nfilt;
}

// ---------------------------------------------------------------------------
// k_match_select: top-`topn` keypoints of one frame by (response desc,
// index asc), written in ascending index order (one vocabulary node).
// grid (npairs, 2): y = side (0: frame A -> list1, 1: frame B -> list2).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_match_select(
    MProblem* __restrict__ probs, MNodePair* __restrict__ nps, const orbx_keypoint* __restrict__ kps_a,
    const int* __restrict__ count_a, const orbx_keypoint* __restrict__ kps_b,
    const int* __restrict__ count_b, int kcap, int topn, uint32_t* __restrict__ sel) {
  __shared__ int hist[256];
  __shared__ int s_R, s_above, wtot[4];
  const int p = blockIdx.x, side = blockIdx.y, tid = threadIdx.x;
  const orbx_keypoint* kp = (side ? kps_b : kps_a) + (size_t)p * kcap;
  const int K = side ? count_b[p] : count_a[p];
  uint32_t* out = sel + ((size_t)p * 2 + side) * topn;
  hist[tid] = 0;
  // the first SEL_U blocks of 256 responses stay in registers for the
  // selection pass below (all loads issued at once; no reload per block)
  constexpr int SEL_U = 8;
  int rr[SEL_U];
#pragma unroll
  for (int u = 0; u < SEL_U; ++u) {
    const int i = tid + 256 * u;
    rr[u] = i < K ? (int)kp[i].response : -2;
  }
  __syncthreads();
#pragma unroll
  for (int u = 0; u < SEL_U; ++u)
    if (tid + 256 * u < K) atomicAdd(&hist[rr[u] & 255], 1);
  for (int i = tid + 256 * SEL_U; i < K; i += 256) atomicAdd(&hist[(int)kp[i].response & 255], 1);
  __syncthreads();
  if (tid < 64) {
    // the response cutoff R: the first bin, from 255 down, where the count
    // of keypoints at or above it reaches topn (above = count strictly
    // above).  Wave 0, 4 bins per lane in descending order, a lane scan,
    // then the crossing lane walks its 4 bins (a single-thread walk over
    // 256 bins was a chain of up to 256 LDS reads)
    const int lane = tid;
    int R = -1, above = 0;
    if (K > topn) {
      int h[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) h[j] = hist[255 - 4 * lane - j];
      const int sum = h[0] + h[1] + h[2] + h[3];
      const int incl = wave_incl_scan(sum);
      // exists: the bins hold all K > topn keypoints
      const int L = __ffsll((unsigned long long)__ballot(incl >= topn)) - 1;
      int cum = incl - sum;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (R < 0 && cum + h[j] >= topn) { R = 255 - 4 * lane - j; above = cum; }
        cum += h[j];
      }
      R = lane_value(R, L);
      above = lane_value(above, L);
    }
    if (lane == 0) {
      s_R = R;
      s_above = above;
    }
  }
  __syncthreads();
  const int R = s_R, needEq = topn - s_above;
  const int wave = tid >> 6, lane = tid & 63;
  int nsel = 0, neq = 0;
  auto block = [&](int base, int resp) {
    const int i = base + tid;
    const bool eq = (i < K) && resp == R;
    // rank among equal-response entries (ordered)
    const uint64_t meq = __ballot(eq);
    if (lane == 0) wtot[wave] = __popcll(meq);
    __syncthreads();
    int eqoff = neq;
    for (int w = 0; w < wave; ++w) eqoff += wtot[w];
    const int eqrank = eqoff + __popcll(meq & ((1ull << lane) - 1ull));
    const int eqtot = wtot[0] + wtot[1] + wtot[2] + wtot[3];
    __syncthreads();
    const bool take = (i < K) && (resp > R || (eq && eqrank < needEq));
    const uint64_t mt = __ballot(take);
    if (lane == 0) wtot[wave] = __popcll(mt);
    __syncthreads();
    int off = nsel;
    for (int w = 0; w < wave; ++w) off += wtot[w];
    if (take) out[off + __popcll(mt & ((1ull << lane) - 1ull))] = (uint32_t)i;
    nsel += wtot[0] + wtot[1] + wtot[2] + wtot[3];
    neq += eqtot;
    __syncthreads();
  };
#pragma unroll
  for (int u = 0; u < SEL_U; ++u)
    if (256 * u < K) block(256 * u, rr[u]);
  for (int base = 256 * SEL_U; base < K; base += 256) block(base, base + tid < K ? (int)kp[base + tid].response : -2);
  if (tid == 0) {
    if (side == 0) { nps[p].n1 = nsel; probs[p].n1 = K; }
    else { nps[p].n2 = nsel; probs[p].n2 = K; }
  }
}

// DescriptorDistance over index pairs
// ---------------------------------------------------------------------------
// k_stage_in: a call's inputs from the pinned staging buffer (host memory the
// GPU reads over PCIe) into its device arena, as a kernel on the call's
// stream: the kernels after it start without the copy engine -> compute
// queue handover a DMA copy needs (~8 us between the copy's end and the first
// kernel in the drop-in SearchByBoW trace).  bytes: a multiple of 16.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_stage_in(uint4* __restrict__ d, const uint4* __restrict__ h,
                                                  size_t n16) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += (size_t)gridDim.x * 256) d[i] = h[i];
}

__global__ void k_hamming_pairs(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b,
                                const int32_t* __restrict__ ia, const int32_t* __restrict__ ib,
                                int npairs, int32_t* __restrict__ dist) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= npairs) return;
  dist[i] = hamming32(reinterpret_cast<const uint32_t*>(a + (size_t)ia[i] * 32),
                      reinterpret_cast<const uint32_t*>(b + (size_t)ib[i] * 32));
}

}  // namespace orbx
