// kernels_extract.hip -- gfx950 kernels of the ORB extractor hot path.
//
// Stage map (reference file:line -> kernel):
//   ComputePyramid / cv::resize      ORBextractor.cc:497-515  -> k_resize
//   cell FAST + NMS + retry          ORBextractor.cc:316-340  -> k_fast_cells
//   DistributeOctTree                ORBextractor.cc:228-286  -> k_quadtree
//   GaussianBlur 7x7 (descriptors)   ORBextractor.cc:478-479  -> k_blur
//   IC_Angle + computeOrbDescriptor  ORBextractor.cc:21-73    -> k_orient_brief
//   + output assembly (:455-494)
// All integer work is exact; the float work (fastAtan2, BRIEF rotation) is
// written operation-for-operation with -ffp-contract=off and explicit fmaf.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/orbx.h"
#include "orbx_internal.h"
#include "orbx_sincos.h"

#define ORBX_BRIEF_STORAGE static __constant__ const
#include "brief_pattern.inc"
#define ORBX_SINCOS_STORAGE static __constant__ const
#include "sincos_exceptions.inc"

namespace orbx {

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ const uint8_t* level_base(const uint8_t* frames, size_t fstride,
                                                     size_t rstride, const uint8_t* pyr,
                                                     size_t pstride, const LevelInfo& U, int u,
                                                     int f, int* pitch) {
  if (u == 0) {
    *pitch = (int)rstride;
    return frames + (size_t)f * fstride;
  }
  *pitch = U.pitch;
  return pyr + (size_t)f * pstride + U.pyr_off;
}

// ---------------------------------------------------------------------------
// k_resize: level l (unique, >= 1) from level l-1 with OpenCV's INTER_LINEAR
// fixed-point arithmetic: D = S[sx]*a0 + S[sx1]*a1 (int32),
// dst = (((b0*(D0>>4))>>16) + ((b1*(D1>>4))>>16) + 2) >> 2.
// Block 64x4 threads, 4 output pixels per thread (one 32-bit store).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_resize(const uint8_t* __restrict__ frames, size_t fstride,
                                                size_t rstride, uint8_t* __restrict__ pyr,
                                                size_t pstride, const LevelInfo* __restrict__ lv,
                                                int l, const int32_t* __restrict__ xofs,
                                                const int32_t* __restrict__ xofs1,
                                                const int16_t* __restrict__ alpha,
                                                const int32_t* __restrict__ yofs,
                                                const int16_t* __restrict__ beta) {
  const LevelInfo D = lv[l];
  const int u = D.src_level;
  const LevelInfo S = lv[u];
  const int f = blockIdx.z;
  int spitch;
  const uint8_t* src = level_base(frames, fstride, rstride, pyr, pstride, S, u, f, &spitch);
  uint8_t* dst = pyr + (size_t)f * pstride + D.pyr_off;
  const int y = blockIdx.y * 4 + threadIdx.y;
  const int x0 = (blockIdx.x * 64 + threadIdx.x) * 4;
  if (y >= D.h || x0 >= D.w) return;
  const int sy = yofs[D.lut_y + y];
  const int r0 = min(max(sy, 0), S.h - 1), r1 = min(max(sy + 1, 0), S.h - 1);
  const int b0 = beta[2 * (D.lut_y + y)], b1 = beta[2 * (D.lut_y + y) + 1];
  const uint8_t* S0 = src + (size_t)r0 * spitch;
  const uint8_t* S1 = src + (size_t)r1 * spitch;
  uint32_t packed = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int x = x0 + k;
    if (x < D.w) {
      const int j = D.lut_x + x;
      const int sx = xofs[j], sx1 = xofs1[j];
      const int a0 = alpha[2 * j], a1 = alpha[2 * j + 1];
      const int d0 = S0[sx] * a0 + S0[sx1] * a1;
      const int d1 = S1[sx] * a0 + S1[sx1] * a1;
      const int v = (((b0 * (d0 >> 4)) >> 16) + ((b1 * (d1 >> 4)) >> 16) + 2) >> 2;
      packed |= (uint32_t)(v & 0xFF) << (8 * k);
    }
  }
  uint8_t* out = dst + (size_t)y * D.pitch + x0;
  if (x0 + 3 < D.w) {
    *reinterpret_cast<uint32_t*>(out) = packed;  // pitch is a multiple of 16
  } else {
    for (int k = 0; x0 + k < D.w; ++k) out[k] = (uint8_t)(packed >> (8 * k));
  }
}

// ---------------------------------------------------------------------------
// k_fast_cells: one workgroup per (FAST cell, frame).
// FAST-9/16 "strength" A(p) = max(0, max_arc min_k I_k - p, p - min_arc max_k I_k)
// over the 16 arcs of 9 contiguous circle pixels.  cv::FAST at threshold t
// reports p iff A(p) > t, with cornerScore<16> == A(p) - 1 (proof: DESIGN §5).
// NMS is cv::FAST's strict 3x3 test on the uchar score buffer, which holds
// A-1 for corners inside the cell's scan band and 0 elsewhere.  A cell whose
// ini-threshold result is empty is re-run at the min threshold
// (ORBextractor.cc:293-296,330-331).  Survivors are compacted in raster order
// into the cell's slot list, packed (x-16)<<20 | (y-16)<<8 | score.
// ---------------------------------------------------------------------------
__constant__ int8_t c_circle_dx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
__constant__ int8_t c_circle_dy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};

__device__ __forceinline__ int min3i(int a, int b, int c) { return min(min(a, b), c); }
__device__ __forceinline__ int max3i(int a, int b, int c) { return max(max(a, b), c); }

__device__ __forceinline__ int fast_strength(const uint8_t* t, int tw) {
  int I[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) I[k] = t[c_circle_dy[k] * tw + c_circle_dx[k]];
  const int v = t[0];
  int mn3[16], mx3[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    mn3[k] = min3i(I[k], I[(k + 1) & 15], I[(k + 2) & 15]);
    mx3[k] = max3i(I[k], I[(k + 1) & 15], I[(k + 2) & 15]);
  }
  int Mb = 0, Md = 255;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    Mb = max(Mb, min3i(mn3[k], mn3[(k + 3) & 15], mn3[(k + 6) & 15]));
    Md = min(Md, max3i(mx3[k], mx3[(k + 3) & 15], mx3[(k + 6) & 15]));
  }
  return max3i(0, Mb - v, v - Md);
}

__device__ __forceinline__ int nms_keep(const uint8_t* amap, int bw, int bh, int bx, int by,
                                        int th) {
  const int a = amap[by * bw + bx];
  if (a <= th) return 0;
  const int s = a - 1;
#pragma unroll
  for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx) {
      if (dx == 0 && dy == 0) continue;
      const int qx = bx + dx, qy = by + dy;
      int nb = 0;
      if (qx >= 0 && qx < bw && qy >= 0 && qy < bh) {
        const int aq = amap[qy * bw + qx];
        nb = aq > th ? aq - 1 : 0;
      }
      if (!(s > nb)) return 0;
    }
  return 1;
}

__global__ __launch_bounds__(256) void k_fast_cells(
    const uint8_t* __restrict__ frames, size_t fstride, size_t rstride,
    const uint8_t* __restrict__ pyr, size_t pstride, const LevelInfo* __restrict__ lv,
    const CellInfo* __restrict__ cells, uint32_t* __restrict__ slots, size_t slot_stride,
    uint32_t* __restrict__ ccount, int ncells, int ini_th, int min_th) {
  __shared__ uint8_t tile[ORBX_CELL_MAX * ORBX_CELL_MAX];
  __shared__ uint8_t amap[(ORBX_CELL_MAX - 6) * (ORBX_CELL_MAX - 6)];
  __shared__ uint8_t keep[(ORBX_CELL_MAX - 6) * (ORBX_CELL_MAX - 6)];
  __shared__ int s_wtot[4];
  const int c = blockIdx.x, f = blockIdx.y, tid = threadIdx.x;
  const CellInfo ci = cells[c];
  int pitch;
  const uint8_t* base =
      level_base(frames, fstride, rstride, pyr, pstride, lv[ci.level], ci.level, f, &pitch);
  const int tw = ci.w, th = ci.h, bw = tw - 6, bh = th - 6, nb = bw * bh;
  for (int i = tid; i < tw * th; i += 256) {
    const int ty = i / tw, tx = i - ty * tw;
    tile[i] = base[(size_t)(ci.y + ty) * pitch + ci.x + tx];
  }
  __syncthreads();
  for (int i = tid; i < nb; i += 256) {
    const int by = i / bw, bx = i - by * bw;
    amap[i] = (uint8_t)fast_strength(&tile[(by + 3) * tw + bx + 3], tw);
  }
  __syncthreads();
  int cnt = 0;
  for (int i0 = 0; i0 < nb; i0 += 256) {
    const int i = i0 + tid;
    int k = 0;
    if (i < nb) {
      const int by = i / bw, bx = i - by * bw;
      k = nms_keep(amap, bw, bh, bx, by, ini_th);
      keep[i] = (uint8_t)k;
    }
    cnt += __syncthreads_count(k);
  }
  if (cnt == 0) {  // handleKeyPoints: FAST again at minThFAST when the cell is empty
    for (int i0 = 0; i0 < nb; i0 += 256) {
      const int i = i0 + tid;
      int k = 0;
      if (i < nb) {
        const int by = i / bw, bx = i - by * bw;
        k = nms_keep(amap, bw, bh, bx, by, min_th);
        keep[i] = (uint8_t)k;
      }
      cnt += __syncthreads_count(k);
    }
  }
  // raster-order compaction
  const int wave = tid >> 6, lane = tid & 63;
  uint32_t* out = slots + (size_t)f * slot_stride + ci.slot_off;
  int basepos = 0;
  if (cnt > 0) {
    for (int i0 = 0; i0 < nb; i0 += 256) {
      const int i = i0 + tid;
      const int k = (i < nb) ? keep[i] : 0;
      const uint64_t m = __ballot(k);
      const int rank = __popcll(m & ((1ull << lane) - 1ull));
      if (lane == 0) s_wtot[wave] = __popcll(m);
      __syncthreads();
      int off = basepos;
      for (int w = 0; w < wave; ++w) off += s_wtot[w];
      if (k) {
        const int by = i / bw, bx = i - by * bw;
        const int gx = ci.x + 3 + bx - ORBX_MINB, gy = ci.y + 3 + by - ORBX_MINB;
        const uint32_t score = (uint32_t)amap[i] - 1u;
        out[off + rank] = orbx_pack_key((uint32_t)gx, (uint32_t)gy, score);
      }
      basepos += s_wtot[0] + s_wtot[1] + s_wtot[2] + s_wtot[3];
      __syncthreads();
    }
  }
  if (tid == 0) ccount[(size_t)f * ncells + c] = (uint32_t)cnt;
}

// ---------------------------------------------------------------------------
// Block-wide exclusive scan of an LDS int array (256 threads), returns total.
// ---------------------------------------------------------------------------
__device__ int block_scan_excl(int* a, int n, int* wtmp) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int chunk = (n + 255) / 256;
  const int b = tid * chunk, e = min(n, b + chunk);
  int s = 0;
  for (int i = b; i < e; ++i) s += a[i];
  int incl = s;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    int t = __shfl_up(incl, d, 64);
    if (lane >= d) incl += t;
  }
  if (lane == 63) wtmp[wave] = incl;
  __syncthreads();
  int woff = 0;
  for (int w = 0; w < wave; ++w) woff += wtmp[w];
  const int total = wtmp[0] + wtmp[1] + wtmp[2] + wtmp[3];
  int run = woff + incl - s;
  for (int i = b; i < e; ++i) {
    const int v = a[i];
    a[i] = run;
    run += v;
  }
  __syncthreads();
  return total;
}

// ---------------------------------------------------------------------------
// k_quadtree: DistributeOctTree for one (level, frame) per workgroup.
// The reference's std::list is replaced by per-pass arrays; the list order
// of one pass is reproduced with two scans (children of split parents in
// reverse parent order, each as n4,n3,n2,n1; then kept single-key nodes in
// their previous order).  Node membership is recomputed from coordinates,
// so keys never move; each node keeps the first maximal response of its
// keys (ties -> lowest key index = earliest in vToDistributeKeys).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int quadrant(uint32_t key, int rx, int ry) {
  const int x = (int)(key >> 20), y = (int)((key >> 8) & 0xFFF);
  const int x0 = rx & 0xFFFF, x1 = rx >> 16, y0 = ry & 0xFFFF, y1 = ry >> 16;
  const int hx = (x1 - x0) / 2, hy = (y1 - y0) / 2;
  const int right = x >= x0 + hx, bottom = y >= y0 + hy;
  return right + 2 * bottom;  // 0 n1, 1 n2, 2 n3, 3 n4
}

__device__ __forceinline__ void child_rect(int rx, int ry, int q, int* crx, int* cry) {
  const int x0 = rx & 0xFFFF, x1 = rx >> 16, y0 = ry & 0xFFFF, y1 = ry >> 16;
  const int hx = (x1 - x0) / 2, hy = (y1 - y0) / 2;
  const int nx0 = (q & 1) ? x0 + hx : x0, nx1 = (q & 1) ? x1 : x0 + hx;
  const int ny0 = (q & 2) ? y0 + hy : y0, ny1 = (q & 2) ? y1 : y0 + hy;
  *crx = nx0 | (nx1 << 16);
  *cry = ny0 | (ny1 << 16);
}

__device__ __forceinline__ int upper_bound_i(const int* a, int n, int v) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (a[mid] <= v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(256) void k_quadtree(
    const LevelInfo* __restrict__ lv, const CellInfo* __restrict__ cells,
    const uint32_t* __restrict__ slots, size_t slot_stride, const uint32_t* __restrict__ ccount,
    int ncells_total, uint32_t* __restrict__ qkeys, int32_t* __restrict__ qnode, size_t qk_stride,
    uint32_t* __restrict__ qout, size_t qout_stride, int* __restrict__ lcount, int nlevels,
    int smax, int maxcells, int* __restrict__ err) {
  extern __shared__ __align__(16) int smem[];
  const int l = blockIdx.x, f = blockIdx.y, tid = threadIdx.x;
  const LevelInfo L = lv[l];
  const LevelInfo U = lv[L.unique];
  int* cell_off = smem;                       // maxcells + 1
  int* rx = cell_off + maxcells + 1;          // smax
  int* ry = rx + smax;                        // smax
  int* cnt = ry + smax;                       // smax
  int* child = cnt + smax;                    // 4*smax (counts, then positions; then best)
  int* nrx = child + 4 * smax;                // smax
  int* nry = nrx + smax;                      // smax
  int* ncnt = nry + smax;                     // smax
  int* tmp1 = ncnt + smax;                    // smax
  int* tmp2 = tmp1 + smax;                    // smax
  __shared__ int wtmp[4];
  __shared__ int s_flag;

  uint32_t* keys = qkeys + (size_t)f * qk_stride + L.qk_off;
  int32_t* node = qnode + (size_t)f * qk_stride + L.qk_off;

  // gather vToDistributeKeys (cell-major, raster within cell)
  const int nc = U.ncells;
  for (int i = tid; i < nc; i += 256) cell_off[i] = (int)ccount[(size_t)f * ncells_total + U.cell_begin + i];
  __syncthreads();
  const int C = block_scan_excl(cell_off, nc, wtmp);
  if (tid == 0) cell_off[nc] = C;
  __syncthreads();
  const uint32_t* fslots = slots + (size_t)f * slot_stride;
  for (int k = tid; k < C; k += 256) {
    const int c = upper_bound_i(cell_off, nc, k) - 1;
    keys[k] = fslots[cells[U.cell_begin + c].slot_off + (k - cell_off[c])];
  }
  // initial nodes (:230-252)
  const int nIni = L.nini;
  int S = nIni;
  for (int i = tid; i < nIni; i += 256) {
    rx[i] = (int)(L.hX * (float)i) | ((int)(L.hX * (float)(i + 1)) << 16);
    ry[i] = 0 | (L.Hr << 16);
    cnt[i] = 0;
  }
  __syncthreads();
  for (int k = tid; k < C; k += 256) {
    int n = -1;
    if (nIni > 0) {
      const float x = (float)(keys[k] >> 20);
      const int idx = (int)(x / L.hX);
      if (idx >= 0 && idx < nIni) n = idx;
    }
    node[k] = n;
    if (n >= 0) atomicAdd(&cnt[n], 1);
  }
  __syncthreads();

  int newS = 0;
  for (int pass = 0;; ++pass) {
    if (pass >= ORBX_QT_MAX_PASSES) {
      if (tid == 0) atomicOr(err, ORBX_DEVERR_QUADTREE);
      newS = 0;
      break;
    }
    for (int i = tid; i < 4 * S; i += 256) child[i] = 0;
    if (tid == 0) s_flag = 0;
    __syncthreads();
    for (int k = tid; k < C; k += 256) {
      const int n = node[k];
      if (n >= 0 && cnt[n] >= 2) atomicAdd(&child[4 * n + quadrant(keys[k], rx[n], ry[n])], 1);
    }
    __syncthreads();
    for (int i = tid; i < S; i += 256) {
      const int cn = cnt[i];
      int nch = 0;
      if (cn >= 2) nch = (child[4 * i] > 0) + (child[4 * i + 1] > 0) + (child[4 * i + 2] > 0) + (child[4 * i + 3] > 0);
      tmp1[S - 1 - i] = nch;
      tmp2[i] = cn == 1;
    }
    __syncthreads();
    const int totC = block_scan_excl(tmp1, S, wtmp);
    const int totK = block_scan_excl(tmp2, S, wtmp);
    newS = totC + totK;
    for (int i = tid; i < S; i += 256) {
      const int cn = cnt[i];
      if (cn >= 2) {
        int pos = tmp1[S - 1 - i];
        for (int q = 3; q >= 0; --q) {
          const int cc = child[4 * i + q];
          if (cc > 0) {
            if (pos < smax) {
              int crx, cry;
              child_rect(rx[i], ry[i], q, &crx, &cry);
              nrx[pos] = crx;
              nry[pos] = cry;
              ncnt[pos] = cc;
            }
            if (cc >= 2) s_flag = 1;
            child[4 * i + q] = pos++;
          } else {
            child[4 * i + q] = -1;
          }
        }
      } else if (cn == 1) {
        const int pos = totC + tmp2[i];
        if (pos < smax) {
          nrx[pos] = rx[i];
          nry[pos] = ry[i];
          ncnt[pos] = 1;
        }
        child[4 * i] = pos;
      }
    }
    __syncthreads();
    for (int k = tid; k < C; k += 256) {
      const int n = node[k];
      if (n < 0) continue;
      node[k] = (cnt[n] >= 2) ? child[4 * n + quadrant(keys[k], rx[n], ry[n])] : child[4 * n];
    }
    const bool finish = (newS >= L.N) || (s_flag == 0);
    __syncthreads();
    if (finish) break;
    for (int i = tid; i < newS; i += 256) {
      rx[i] = nrx[i];
      ry[i] = nry[i];
      cnt[i] = ncnt[i];
    }
    S = newS;
    __syncthreads();
  }
  // per final node: first key with maximal response (:277-284)
  uint32_t* best = (uint32_t*)child;  // 4*smax >= newS
  if (newS > L.kcap) {
    if (tid == 0) atomicOr(err, ORBX_DEVERR_QTCAP);
    newS = 0;
  }
  for (int i = tid; i < newS; i += 256) best[i] = 0u;
  __syncthreads();
  for (int k = tid; k < C; k += 256) {
    const int n = node[k];
    if (n >= 0 && n < newS)
      atomicMax(&best[n], ((keys[k] & 0xFFu) << 24) | (0xFFFFFFu - (uint32_t)k));
  }
  __syncthreads();
  uint32_t* out = qout + (size_t)f * qout_stride + L.kout_off;
  for (int i = tid; i < newS; i += 256) {
    const uint32_t k = 0xFFFFFFu - (best[i] & 0xFFFFFFu);
    out[i] = keys[k];
  }
  if (tid == 0) lcount[(size_t)f * nlevels + l] = newS;
}

// ---------------------------------------------------------------------------
// k_blur: cv::GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101) on 8U with the
// bit-exact fixed-point kernel [18,34,48,56,48,34,18]/256:
// H = sum k_i p (u16), out = (sum k_j H_j + 32768) >> 16.
// Tile 64x16 outputs per workgroup.
// ---------------------------------------------------------------------------
__constant__ int c_gk[7] = {18, 34, 48, 56, 48, 34, 18};

__device__ __forceinline__ int reflect101(int p, int len) {
  p = p < 0 ? -p : p;
  return p >= len ? 2 * len - 2 - p : p;
}

__global__ __launch_bounds__(256) void k_blur(const uint8_t* __restrict__ frames, size_t fstride,
                                              size_t rstride, const uint8_t* __restrict__ pyr,
                                              size_t pstride, uint8_t* __restrict__ blur,
                                              size_t bstride, const LevelInfo* __restrict__ lv,
                                              int u) {
  __shared__ uint8_t in[22][72];
  __shared__ uint16_t hs[22][64];
  const LevelInfo U = lv[u];
  const int f = blockIdx.z, tid = threadIdx.x;
  int pitch;
  const uint8_t* src = level_base(frames, fstride, rstride, pyr, pstride, U, u, f, &pitch);
  const int bx0 = blockIdx.x * 64, by0 = blockIdx.y * 16;
  for (int i = tid; i < 22 * 70; i += 256) {
    const int ty = i / 70, tx = i - ty * 70;
    const int gx = reflect101(min(bx0 + tx - 3, U.w + 2), U.w);
    const int gy = reflect101(min(by0 + ty - 3, U.h + 2), U.h);
    in[ty][tx] = src[(size_t)gy * pitch + gx];
  }
  __syncthreads();
  for (int i = tid; i < 22 * 64; i += 256) {
    const int ty = i >> 6, tx = i & 63;
    int s = 0;
#pragma unroll
    for (int k = 0; k < 7; ++k) s += c_gk[k] * in[ty][tx + k];
    hs[ty][tx] = (uint16_t)s;
  }
  __syncthreads();
  const int ox = tid & 63, oy0 = (tid >> 6) * 4;
  const int gx = bx0 + ox;
  const int bp = (int)((U.w + 15) & ~15);
  uint8_t* dst = blur + (size_t)f * bstride + U.blur_off;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int oy = oy0 + r, gy = by0 + oy;
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < 7; ++k) s += (uint32_t)c_gk[k] * hs[oy + k][ox];
    if (gx < U.w && gy < U.h) dst[(size_t)gy * bp + gx] = (uint8_t)min((s + 32768u) >> 16, 255u);
  }
}

// ---------------------------------------------------------------------------
// k_orient_brief: one wavefront per output keypoint.
//   IC_Angle (:21-48): m10 = sum u*I, m01 = sum v*I over the 749-pixel disk
//   (umax), on the unblurred level, reduced across the wave; angle =
//   cv::fastAtan2(m01, m10).
//   computeOrbDescriptor (:57-73): 256 tests, 4 per lane, on the blurred
//   level, row = rint(fma(x, sin, RN(y*cos))), col = rint(fma(x, cos,
//   -RN(y*sin))), bits gathered with __ballot.
//   Assembly (:471-494): level-major order, pt *= mvScaleFactor[level].
// ---------------------------------------------------------------------------
__device__ __forceinline__ float fast_atan2(float y, float x) {
  const float r2d = (float)(180 / 3.141592653589793238462643383279502884);
  const float p1 = 0.9997878412794807f * r2d, p3 = -0.3258083974640975f * r2d,
              p5 = 0.1555786518463281f * r2d, p7 = -0.04432655554792128f * r2d;
  const float eps = (float)2.220446049250313080847e-16;
  const float ax = fabsf(x), ay = fabsf(y);
  float a, c, c2;
  if (ax >= ay) {
    c = ay / (ax + eps);
    c2 = c * c;
    a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  } else {
    c = ax / (ay + eps);
    c2 = c * c;
    a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
  }
  if (x < 0) a = 180.f - a;
  if (y < 0) a = 360.f - a;
  return a;
}

__device__ __forceinline__ void brief_sincos(float x, float* s, float* c) {
  orbx_sincos_core(x, s, c);
  const uint32_t b = orbx_f2u(x);
  int lo = 0, hi = ORBX_SINCOS_NEXC;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (ORBX_SINCOS_EXC[mid][0] < b) lo = mid + 1; else hi = mid;
  }
  if (lo < ORBX_SINCOS_NEXC && ORBX_SINCOS_EXC[lo][0] == b) {
    *s = orbx_u2f(ORBX_SINCOS_EXC[lo][1]);
    *c = orbx_u2f(ORBX_SINCOS_EXC[lo][2]);
  }
}

__global__ __launch_bounds__(256) void k_orient_brief(
    const uint8_t* __restrict__ frames, size_t fstride, size_t rstride,
    const uint8_t* __restrict__ pyr, size_t pstride, const uint8_t* __restrict__ blur,
    size_t bstride, const LevelInfo* __restrict__ lv, int nlevels,
    const uint32_t* __restrict__ qout, size_t qout_stride, const int* __restrict__ lcount,
    const int16_t* __restrict__ disk, int ndisk, orbx_keypoint* __restrict__ kps,
    uint8_t* __restrict__ desc, int* __restrict__ counts, int kcap) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int f = blockIdx.y;
  const int g = blockIdx.x * 4 + wave;
  const int* lc = lcount + (size_t)f * nlevels;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    int t = 0;
    for (int l = 0; l < nlevels; ++l) t += lc[l];
    counts[f] = t;
  }
  if (g >= kcap) return;
  int l = 0;
  while (l < nlevels && !(g >= lv[l].kout_off && g < lv[l].kout_off + lv[l].kcap)) ++l;
  if (l >= nlevels) return;
  const LevelInfo L = lv[l];
  const int i = g - L.kout_off;
  if (i >= lc[l]) return;
  int o = i;
  for (int t = 0; t < l; ++t) o += lc[t];
  const uint32_t key = qout[(size_t)f * qout_stride + L.kout_off + i];
  const int x = (int)(key >> 20) + ORBX_MINB, y = (int)((key >> 8) & 0xFFF) + ORBX_MINB;
  const int score = (int)(key & 0xFF);
  const int u = L.unique;
  const LevelInfo U = lv[u];
  int pitch;
  const uint8_t* img = level_base(frames, fstride, rstride, pyr, pstride, U, u, f, &pitch);
  const uint8_t* center = img + (size_t)y * pitch + x;
  int m10 = 0, m01 = 0;
  for (int j = lane; j < ndisk; j += 64) {
    const int du = disk[2 * j], dv = disk[2 * j + 1];
    const int I = center[dv * pitch + du];
    m10 += du * I;
    m01 += dv * I;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    m10 += __shfl_xor(m10, d, 64);
    m01 += __shfl_xor(m01, d, 64);
  }
  const float angle = fast_atan2((float)m01, (float)m10);
  const float factorPI = (float)(3.1415926535897932384626433832795 / 180.f);
  float sn, cs;
  brief_sincos(angle * factorPI, &sn, &cs);
  const int bp = (U.w + 15) & ~15;
  const uint8_t* bc = blur + (size_t)f * bstride + U.blur_off + (size_t)y * bp + x;
  uint64_t words[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int p = lane + 64 * r;
    int t[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const float px = (float)ORBX_BRIEF_PATTERN[p][2 * e];
      const float py = (float)ORBX_BRIEF_PATTERN[p][2 * e + 1];
      const float ya = py * cs, yb = py * sn;
      const int row = (int)__builtin_rintf(__builtin_fmaf(px, sn, ya));
      const int col = (int)__builtin_rintf(__builtin_fmaf(px, cs, -yb));
      t[e] = bc[row * bp + col];
    }
    words[r] = __ballot(t[0] < t[1]);
  }
  if (lane < 4) {
    const uint64_t w = lane == 0 ? words[0] : lane == 1 ? words[1] : lane == 2 ? words[2] : words[3];
    reinterpret_cast<uint64_t*>(desc + ((size_t)f * kcap + o) * 32)[lane] = w;
  }
  if (lane == 0) {
    orbx_keypoint kp;
    kp.x = (float)x;
    kp.y = (float)y;
    if (l != 0) {
      kp.x *= L.scale;
      kp.y *= L.scale;
    }
    kp.size = (float)L.patch_size;
    kp.angle = angle;
    kp.response = (float)score;
    kp.octave = l;
    kp.class_id = -1;
    kps[(size_t)f * kcap + o] = kp;
  }
}

// ---------------------------------------------------------------------------
// k_synth: deterministic synthetic frames (orbx/synth.py is the spec).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t sm_mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t sm_at(uint64_t seed, uint64_t i) {
  return sm_mix(seed + (i + 1) * 0x9E3779B97F4A7C15ull);
}

__global__ __launch_bounds__(256) void k_synth(uint8_t* __restrict__ frames, int W, int H,
                                               size_t fstride, int first_idx, int kind) {
  __shared__ int rect[96][5];
  const int f = blockIdx.y, tid = threadIdx.x;
  const uint64_t seed = 0x5EED0000ull + (uint64_t)(first_idx + f);
  if (kind == 0) {
    for (int i = tid; i < 96 * 5; i += 256) {
      const uint64_t v = sm_at(seed, (uint64_t)i);
      const int r = i / 5, c = i - r * 5;
      const uint64_t m = (c == 0 || c == 1) ? (uint64_t)W : (c == 4) ? 256ull : (uint64_t)H;
      rect[r][c] = (int)(v % m);
    }
    __syncthreads();
  }
  const long long npx = (long long)W * H;
  uint8_t* out = frames + (size_t)f * fstride;
  for (long long p = (long long)blockIdx.x * 4096 + tid; p < npx && p < (long long)(blockIdx.x + 1) * 4096;
       p += 256) {
    const int y = (int)(p / W), x = (int)(p - (long long)y * W);
    int v;
    if (kind == 2) {
      v = 128;
    } else if (kind == 1) {
      v = (int)(sm_at(seed, (uint64_t)p) % 256ull);
    } else {
      v = 64 + (128 * x) / (W > 1 ? W - 1 : 1);
      for (int r = 0; r < 96; ++r) {
        const int xa = min(rect[r][0], rect[r][1]), xb = max(rect[r][0], rect[r][1]);
        const int ya = min(rect[r][2], rect[r][3]), yb = max(rect[r][2], rect[r][3]);
        if (x >= xa && x <= xb && y >= ya && y <= yb) v = rect[r][4];
      }
      v += (int)(sm_at(seed, 480ull + (uint64_t)p) % 13ull) - 6;
      v = min(max(v, 0), 255);
    }
    out[(size_t)y * W + x] = (uint8_t)v;
  }
}

}  // namespace orbx
