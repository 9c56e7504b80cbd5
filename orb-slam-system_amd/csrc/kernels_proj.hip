// kernels_proj.hip -- gfx950 kernels of the frame grid and the projection
// matchers:
//   Frame::AssignFeaturesToGrid / PosInGrid (src/Frame.cc:210-225,361-371)  -> k_grid_build
//   Frame::GetFeaturesInArea (src/Frame.cc:307-358) + DescriptorDistance    -> k_proj_cand
//   ORBmatcher::SearchByProjection greedy walk + rotation check              -> k_proj_resolve
//     mode 1 (Frame&, vector<MapPoint*>, th)        src/ORBmatcher.cc:19-61
//     mode 2 (Frame& Current, const Frame& Last)    src/ORBmatcher.cc:732-818
//     mode 3 (Frame& Current, KeyFrame*, set, ...)  src/ORBmatcher.cc:820-894
// The candidate visiting order of GetFeaturesInArea is (ix, iy, index) =
// the position ("rank") of a feature in the ix-major cell list, so "first
// strict minimum" = smallest (distance, rank) key.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/orbx.h"
#include "wave_ops.h"

namespace orbx {

#define PG_COLS 64 /* FRAME_GRID_COLS (include/Frame.h:18) */
#define PG_ROWS 48 /* FRAME_GRID_ROWS (include/Frame.h:17) */
#define PG_CELLS (PG_COLS * PG_ROWS)
#define PJ_T 8     /* candidates kept per query */
#define PJ_MAXN 8192
#define PJ_DEVERR 16

struct ProjFrame {
  int n;
  float minX, minY, wInv, hInv;
};

// one SearchByProjection call: the frame, its queries, outputs and grid /
// candidate scratch (device pointers).  The drop-in call launches one; the
// batched plan (orbm_proj_plan_search) launches many at once, problem =
// blockIdx.y (candidates) or blockIdx.x (grid, walk).
struct ProjProblem {
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
  int* cell_off;   // PG_CELLS + 1
  int* cell_feat;  // n
  uint32_t* cand;  // nq x PJ_T
  int* ncand;      // nq
};

// one workgroup: cells of every feature, ix-major stable order by an LDS
// bitonic sort of (cell << 16 | index) keys (index order inside a cell, as
// push_back in index order)
__global__ __launch_bounds__(1024) void k_grid_build(const ProjProblem* __restrict__ probs) {
  extern __shared__ uint32_t sk[];  // P keys (LDS sized for the largest problem)
  __shared__ int cnt[PG_CELLS];
  const ProjProblem& PP = probs[blockIdx.x];
  const ProjFrame F = PP.F;
  const orbx_keypoint* __restrict__ keys = PP.keys;
  int* __restrict__ cell_off = PP.cell_off;
  int* __restrict__ cell_feat = PP.cell_feat;
  int P = 1;
  while (P < F.n) P <<= 1;
  const int tid = threadIdx.x;
  for (int c = tid; c < PG_CELLS; c += 1024) cnt[c] = 0;
  __syncthreads();
  for (int i = tid; i < P; i += 1024) {
    uint32_t key = 0xFFFFFFFFu;
    if (i < F.n) {
      const orbx_keypoint k = keys[i];
      const int px = (int)roundf((k.x - F.minX) * F.wInv);  // PosInGrid (:363-364)
      const int py = (int)roundf((k.y - F.minY) * F.hInv);
      if (!(px < 0 || px >= PG_COLS || py < 0 || py >= PG_ROWS)) {
        const int c = px * PG_ROWS + py;
        key = ((uint32_t)c << 16) | (uint32_t)i;
        atomicAdd(&cnt[c], 1);
      }
    }
    sk[i] = key;
  }
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = tid; t < (P >> 1); t += 1024) {
        const int lo = 2 * t - (t & (stride - 1)), hi = lo + stride;
        const bool up = (lo & size) == 0;
        const uint32_t x = sk[lo], y = sk[hi];
        if ((x > y) == up) {
          sk[lo] = y;
          sk[hi] = x;
        }
      }
      __syncthreads();
    }
  if (tid == 0) {  // 3072 counters: one thread, once per frame
    int run = 0;
    for (int c = 0; c < PG_CELLS; ++c) {
      cell_off[c] = run;
      run += cnt[c];
    }
    cell_off[PG_CELLS] = run;
  }
  for (int i = tid; i < P; i += 1024)
    if (sk[i] != 0xFFFFFFFFu) cell_feat[i] = (int)(sk[i] & 0xFFFFu);
}

// GetFeaturesInArea cell bounds (:312-326); false = empty
__device__ __forceinline__ bool area_cells(const ProjFrame& F, float x, float y, float r,
                                           int* x0, int* x1, int* y0, int* y1) {
  const int mincx = (int)floorf((x - F.minX - r) * F.wInv);
  *x0 = mincx > 0 ? mincx : 0;
  if (*x0 >= PG_COLS) return false;
  const int maxcx = (int)ceilf((x - F.minX + r) * F.wInv);
  *x1 = maxcx < PG_COLS - 1 ? maxcx : PG_COLS - 1;
  if (*x1 < 0) return false;
  const int mincy = (int)floorf((y - F.minY - r) * F.hInv);
  *y0 = mincy > 0 ? mincy : 0;
  if (*y0 >= PG_ROWS) return false;
  const int maxcy = (int)ceilf((y - F.minY + r) * F.hInv);
  *y1 = maxcy < PG_ROWS - 1 ? maxcy : PG_ROWS - 1;
  if (*y1 < 0) return false;
  return true;
}

// candidate filter of one feature (level, box, stereo gate) and its key
__device__ __forceinline__ uint32_t proj_key(const orbx_query_proj& Q, const orbx_keypoint& k,
                                             const uint8_t* __restrict__ desc,
                                             const float* __restrict__ uright, int mode, int idx,
                                             int rank, uint4 q0, uint4 q1, bool* is_cand) {
  *is_cand = false;
  const bool bCheckLevels = (Q.min_level > 0) || (Q.max_level >= 0);
  if (bCheckLevels) {
    if (k.octave < Q.min_level) return 0xFFFFFFFFu;
    if (Q.max_level >= 0 && k.octave > Q.max_level) return 0xFFFFFFFFu;
  }
  const float distx = k.x - Q.x, disty = k.y - Q.y;
  if (!(fabsf(distx) < Q.radius && fabsf(disty) < Q.radius)) return 0xFFFFFFFFu;
  *is_cand = true;
  if (mode == 1 && uright && uright[idx] > 0) {  // :39-43 (claim-independent gate)
    const float er = fabsf(Q.xr - uright[idx]);
    if (er > Q.radius) return 0xFFFFFFFFu;
  }
  const uint4* dp = reinterpret_cast<const uint4*>(desc + (size_t)idx * 32);
  const uint4 b0 = dp[0], b1 = dp[1];
  const uint32_t d = __popc(q0.x ^ b0.x) + __popc(q0.y ^ b0.y) + __popc(q0.z ^ b0.z) +
                     __popc(q0.w ^ b0.w) + __popc(q1.x ^ b1.x) + __popc(q1.y ^ b1.y) +
                     __popc(q1.z ^ b1.z) + __popc(q1.w ^ b1.w);
  return (d << 16) | (uint32_t)rank;
}

// One wavefront per query: the PJ_T smallest (distance << 16 | rank) keys
// over the candidates not occupied before the call (claims made during the
// walk are resolved by k_proj_resolve), and whether that list is complete.
__global__ __launch_bounds__(256) void k_proj_cand(const ProjProblem* __restrict__ probs, int mode) {
  const ProjProblem& PP = probs[blockIdx.y];
  const int lane = threadIdx.x & 63;
  const int qi = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (qi >= PP.nq) return;
  const ProjFrame F = PP.F;
  const orbx_keypoint* __restrict__ keys = PP.keys;
  const uint8_t* __restrict__ desc = PP.desc;
  const float* __restrict__ uright = PP.uright;
  const uint8_t* __restrict__ occupied = PP.occupied;
  const int* __restrict__ cell_off = PP.cell_off;
  const int* __restrict__ cell_feat = PP.cell_feat;
  const orbx_query_proj* __restrict__ qs = PP.qs;
  const uint8_t* __restrict__ qdesc = PP.qdesc;
  uint32_t* __restrict__ cand = PP.cand;
  int* __restrict__ ncand = PP.ncand;
  const orbx_query_proj Q = qs[qi];
  const uint4* qd = reinterpret_cast<const uint4*>(qdesc + (size_t)qi * 32);
  const uint4 q0 = qd[0], q1 = qd[1];
  uint32_t L[PJ_T];
#pragma unroll
  for (int t = 0; t < PJ_T; ++t) L[t] = 0xFFFFFFFFu;
  int nkeys = 0;  // keyed candidates seen by this lane
  int x0, x1, y0, y1;
  if (area_cells(F, Q.x, Q.y, Q.radius, &x0, &x1, &y0, &y1)) {
    for (int ix = x0; ix <= x1; ++ix) {
      // cells (ix, y0..y1) are contiguous in the ix-major list
      const int b = cell_off[ix * PG_ROWS + y0], e = cell_off[ix * PG_ROWS + y1 + 1];
      for (int j = b + lane; j < e; j += 64) {
        const int idx = cell_feat[j];
        if (occupied && occupied[idx]) continue;
        bool isc;
        uint32_t k = proj_key(Q, keys[idx], desc, uright, mode, idx, j, q0, q1, &isc);
        if (k == 0xFFFFFFFFu) continue;
        ++nkeys;
#pragma unroll
        for (int t = 0; t < PJ_T; ++t) {
          const uint32_t lo = min(L[t], k);
          k = max(L[t], k);
          L[t] = lo;
        }
      }
    }
  }
  // merge the 64 lane lists: PJ_T rounds of a wave minimum
  int total = nkeys;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) total += __shfl_xor(total, d, 64);
  int head = 0;
  uint32_t out = 0xFFFFFFFFu;
  for (int t = 0; t < PJ_T; ++t) {
    const uint32_t mine = head < PJ_T ? L[0] : 0xFFFFFFFFu;
    uint32_t m = mine;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) m = min(m, (uint32_t)__shfl_xor((int)m, d, 64));
    if (lane == t) out = m;
    if (mine == m && m != 0xFFFFFFFFu) {  // keys are unique (rank): one winner
#pragma unroll
      for (int s = 0; s < PJ_T - 1; ++s) L[s] = L[s + 1];
      L[PJ_T - 1] = 0xFFFFFFFFu;
      ++head;
    }
  }
  if (lane < PJ_T) cand[(size_t)qi * PJ_T + lane] = out;
  if (lane == 0) ncand[qi] = total;
}

// exact rescan of one query under the current claims (list exhausted):
// smallest key and second-smallest distance among unclaimed candidates
__device__ void proj_rescan(const ProjFrame& F, const orbx_query_proj& Q,
                            const orbx_keypoint* __restrict__ keys,
                            const uint8_t* __restrict__ desc, const float* __restrict__ uright,
                            const int* __restrict__ cell_off, const int* __restrict__ cell_feat,
                            const uint8_t* __restrict__ qdesc, int qi, int mode,
                            const uint32_t* taken, uint32_t* k1, uint32_t* d2) {
  const int lane = threadIdx.x & 63;
  const uint4* qd = reinterpret_cast<const uint4*>(qdesc + (size_t)qi * 32);
  const uint4 q0 = qd[0], q1 = qd[1];
  uint32_t a = 0xFFFFFFFFu, b = 0xFFFFFFFFu;  // smallest key, second-smallest distance
  int x0, x1, y0, y1;
  if (area_cells(F, Q.x, Q.y, Q.radius, &x0, &x1, &y0, &y1)) {
    for (int ix = x0; ix <= x1; ++ix) {
      const int bb = cell_off[ix * PG_ROWS + y0], e = cell_off[ix * PG_ROWS + y1 + 1];
      for (int j = bb + lane; j < e; j += 64) {
        const int idx = cell_feat[j];
        if ((taken[idx >> 5] >> (idx & 31)) & 1u) continue;
        bool isc;
        const uint32_t k = proj_key(Q, keys[idx], desc, uright, mode, idx, j, q0, q1, &isc);
        if (k == 0xFFFFFFFFu) continue;
        if (k < a) {
          b = min(b, a >> 16);
          a = k;
        } else {
          b = min(b, k >> 16);
        }
      }
    }
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint32_t oa = (uint32_t)__shfl_xor((int)a, d, 64);
    const uint32_t ob = (uint32_t)__shfl_xor((int)b, d, 64);
    const uint32_t lo = min(a, oa), hi = max(a, oa);
    b = min(min(b, ob), hi >> 16);
    a = lo;
  }
  *k1 = a;
  *d2 = b;
}

// One wavefront walks the queries in order (the reference's greedy loop):
// best = first unclaimed entry of the query's list, second = the next
// unclaimed entry's distance; an exhausted incomplete list is rescanned.
__global__ __launch_bounds__(64) void k_proj_resolve(const ProjProblem* __restrict__ probs, int mode,
                                                    float nnratio, int th_dist, int check_ori) {
  extern __shared__ uint32_t taken[];  // (n + 31) / 32 bits, then n bins (int8 in int32)
  const ProjProblem& PP = probs[blockIdx.x];
  const ProjFrame F = PP.F;
  const orbx_keypoint* __restrict__ keys = PP.keys;
  const uint8_t* __restrict__ desc = PP.desc;
  const float* __restrict__ uright = PP.uright;
  const uint8_t* __restrict__ occupied = PP.occupied;
  const int* __restrict__ cell_off = PP.cell_off;
  const int* __restrict__ cell_feat = PP.cell_feat;
  const orbx_query_proj* __restrict__ qs = PP.qs;
  const uint8_t* __restrict__ qdesc = PP.qdesc;
  const int nq = PP.nq;
  const uint32_t* __restrict__ cand = PP.cand;
  const int* __restrict__ ncand = PP.ncand;
  int32_t* __restrict__ match = PP.match;
  int* __restrict__ nmatches = PP.nmatches;
  int8_t* bin_of = reinterpret_cast<int8_t*>(taken + ((F.n + 31) >> 5));
  __shared__ int hist[32];
  const int lane = threadIdx.x;
  const int nw = (F.n + 31) >> 5;
  for (int i = lane; i < nw; i += 64) {
    uint32_t w = 0;
    if (occupied)
      for (int b = 0; b < 32; ++b) {
        const int idx = i * 32 + b;
        if (idx < F.n && occupied[idx]) w |= 1u << b;
      }
    taken[i] = w;
  }
  for (int i = lane; i < F.n; i += 64) {
    match[i] = -1;
    bin_of[i] = -1;
  }
  if (lane < 32) hist[lane] = 0;
  __syncthreads();
  const float factor = 1.0f / 30;
  int nm = 0;
  for (int qi = 0; qi < nq; ++qi) {
    const uint32_t e = lane < PJ_T ? cand[(size_t)qi * PJ_T + lane] : 0xFFFFFFFFu;
    const int nc = ncand[qi];
    bool ok = false;
    int idx = 0;
    if (__ballot(e != 0xFFFFFFFFu) == 0 && nc == 0) continue;
    const int fidx = e != 0xFFFFFFFFu ? cell_feat[e & 0xFFFFu] : 0;
    const bool free_ = e != 0xFFFFFFFFu && !((taken[fidx >> 5] >> (fidx & 31)) & 1u);
    const unsigned long long fb = __ballot(free_);
    const bool complete = nc <= PJ_T;
    uint32_t k1 = 0xFFFFFFFFu, d2 = 0xFFFFFFFFu;
    const int nfree = __popcll(fb);
    if (nfree >= 2 || complete) {
      if (nfree >= 1) {
        const int l1 = __ffsll(fb) - 1;
        k1 = lane_value(e, l1);
        if (nfree >= 2) {
          const int l2 = __ffsll(fb & (fb - 1)) - 1;
          d2 = lane_value(e, l2) >> 16;
        }
      }
    } else {
      const orbx_query_proj Q = qs[qi];
      proj_rescan(F, Q, keys, desc, uright, cell_off, cell_feat, qdesc, qi, mode, taken, &k1, &d2);
    }
    if (k1 == 0xFFFFFFFFu) continue;
    const int bestDist = (int)(k1 >> 16);
    const int secondBestDist = d2 == 0xFFFFFFFFu ? 0x7FFFFFFF : (int)d2;
    if (mode == 1)
      ok = bestDist <= 100 && ((float)bestDist <= nnratio * (float)secondBestDist);  // :55
    else
      ok = bestDist <= th_dist;  // :790 TH_HIGH, :869 ORBdist
    if (!ok) continue;
    idx = cell_feat[k1 & 0xFFFFu];
    if (lane == 0) {
      taken[idx >> 5] |= 1u << (idx & 31);
      match[idx] = qi;
      if (mode != 1 && check_ori) {
        float rot = qs[qi].angle - keys[idx].angle;
        if (rot < 0) rot += 360.0f;  // :874 (mode 2: upstream wrap)
        const int bin = (int)roundf(rot * factor) % 30;
        bin_of[idx] = (int8_t)bin;
        hist[bin]++;
      }
    }
    ++nm;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
  }
  if (mode != 1 && check_ori) {  // ComputeThreeMaxima (:469-502) + removal
    __syncthreads();
    int ind1 = -1, ind2 = -1, ind3 = -1;
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < 30; ++i) {
      const int s = hist[i];
      if (s > max1) {
        max3 = max2; max2 = max1; max1 = s;
        ind3 = ind2; ind2 = ind1; ind1 = i;
      } else if (s > max2) {
        max3 = max2; max2 = s;
        ind3 = ind2; ind2 = i;
      } else if (s > max3) {
        max3 = s;
        ind3 = i;
      }
    }
    if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
    else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
    int removed = 0;
    for (int i = lane; i < F.n; i += 64) {
      const int b = bin_of[i];
      if (b >= 0 && b != ind1 && b != ind2 && b != ind3) {
        match[i] = -1;
        ++removed;
      }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) removed += __shfl_xor(removed, d, 64);
    nm -= removed;
  }
  if (lane == 0) *nmatches = nm;
}

}  // namespace orbx
