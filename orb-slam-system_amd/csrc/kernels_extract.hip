// kernels_extract.hip -- gfx950 kernels of the ORB extractor hot path.
//
// Stage map (reference file:line -> kernel):
//   ComputePyramid / cv::resize      ORBextractor.cc:497-515  -> k_pyramid
//   cell FAST + NMS + retry          ORBextractor.cc:316-340  -> k_fast_strips
//   DistributeOctTree                ORBextractor.cc:228-286  -> k_quadtree
//   IC_Angle + GaussianBlur 7x7 +   ORBextractor.cc:21-73,   -> k_orient_brief
//   computeOrbDescriptor             478-479
//   + output assembly (:455-494)
// All integer work is exact; the float work (fastAtan2, BRIEF rotation) is
// written operation-for-operation with -ffp-contract=off and explicit fmaf.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/orbx.h"
#include "orbx_internal.h"
#include "orbx_sincos.h"
#include "wave_ops.h"
#include "fast_ops.h"

#define ORBX_BRIEF_STORAGE static __constant__ const
#include "brief_pattern.inc"
#define ORBX_SINCOS_STORAGE static __constant__ const
#include "sincos_exceptions.inc"
#ifndef OB_HPASS
#define OB_HPASS 1 /* BRIEF horizontal blur pass: 1 = i8 MFMA over the signed patch, 0 = v_dot4 tasks (A/B) */
#endif
#if OB_HPASS == 0
// the horizontal-blur task table, packed per lane for k_orient_brief: entry
// (cc - 21, lane) holds the lane's three rounds as bytes 10 rp + q (0xFF =
// none), one dword load per keypoint instead of an LDS copy of the table
namespace orbx_htask_src {
#define ORBX_HTASK_STORAGE constexpr
#include "brief_htasks.inc"
#undef ORBX_HTASK_STORAGE
}
struct BriefHtaskPacked {
  uint32_t v[4][64];
};
constexpr BriefHtaskPacked brief_htask_pack() {
  BriefHtaskPacked t{};
  for (int c = 0; c < 4; ++c)
    for (int l = 0; l < 64; ++l) {
      uint32_t w = 0;
      for (int k = 0; k < 3; ++k) {
        const uint32_t e = orbx_htask_src::ORBX_HTASK[c][l + 64 * k];
        const uint32_t b = e == 0xFFFFu ? 0xFFu : (e >> 8) * 10u + (e & 0xFFu);
        w |= b << (8 * k);
      }
      t.v[c][l] = w;
    }
  return t;
}
static __constant__ const BriefHtaskPacked c_htask = brief_htask_pack();
#endif

namespace orbx {

__device__ __forceinline__ int lane_id() { return __lane_id(); }

// LDS byte address of a __shared__ pointer (an operand of hand-written ds_*)
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}


// 16-B chunk as a native LLVM vector: HIP's uint4 class defeats SROA when it
// is held in a local array (stage_region's loads would bounce through scratch).
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

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

// Block-cooperative copy of a 2-D byte region into LDS with U loads in flight
// per thread: all loads of a round are issued before the first LDS store,
// so a workgroup pays one memory latency per round instead of one per load.
// T = uint4 / uint32_t / uint8_t (src, pitches and offsets aligned to T).
template <typename T, int U, int NT>
__device__ __forceinline__ void stage_region(uint8_t* __restrict__ lds, int lpitch,
                                             const uint8_t* __restrict__ src, size_t sp, int nrows,
                                             int nper, int tid) {
  // (row, column) of element tid + NT*k advance by (dr, dc) per step: no
  // per-load division; offsets are 24-bit products (rows * pitch < 2^32,
  // both factors < 2^24) added to the wave-uniform base
  const int total = nrows * nper;
  if (total <= 0) return;
  const int dr = NT / nper, dc = NT - dr * nper;
  int r = tid / nper, c = tid - r * nper;
  const uint32_t spu = (uint32_t)sp;
  for (int i0 = tid; i0 < total; i0 += NT * U) {
    T v[U];
    int rr[U], cc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      rr[u] = r;
      cc[u] = c;
      // unconditional (a guarded load is waited for at its branch join):
      // elements past the end read the last row, and are not stored
      v[u] = *reinterpret_cast<const T*>(
          src + (__umul24((uint32_t)min(r, nrows - 1), spu) + (uint32_t)c * (uint32_t)sizeof(T)));
      r += dr;
      c += dc;
      if (c >= nper) { c -= nper; ++r; }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + NT * u < total)
        reinterpret_cast<T*>(lds + __mul24(rr[u], lpitch))[cc[u]] = v[u];
  }
}

// dword load at any byte address (gfx950 global memory accepts unaligned
// dword accesses; the memcpy form lets the compiler emit one global_load_dword)
__device__ __forceinline__ uint32_t ld32u(const uint8_t* p) {
  uint32_t w;
  __builtin_memcpy(&w, p, 4);
  return w;
}

// Rows of nbytes at any byte alignment into dword-aligned LDS rows: one
// unaligned dword load per 4 bytes.  A row's last dword is loaded ending at
// the row's last byte and shifted into place, so nothing past the row is read
// (the caller's frame may end there).  Same indexing as stage_region.
template <int U, int NT>
__device__ __forceinline__ void stage_rows_u32(uint8_t* __restrict__ lds, int lpitch,
                                               const uint8_t* __restrict__ src, size_t sp,
                                               int nrows, int nbytes, int tid) {
  const int nper = (nbytes + 3) >> 2;
  const int total = nrows * nper;
  if (total <= 0) return;
  const int dr = NT / nper, dc = NT - dr * nper;
  int r = tid / nper, c = tid - r * nper;
  const uint32_t spu = (uint32_t)sp;
  const int lastc = max(nbytes - 4, 0);
  for (int i0 = tid; i0 < total; i0 += NT * U) {
    uint32_t v[U];
    int rr[U], cc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      rr[u] = r;
      cc[u] = c;
      const int cb = 4 * c, cl = min(cb, lastc);
      v[u] = ld32u(src + (__umul24((uint32_t)min(r, nrows - 1), spu) + (uint32_t)cl)) >> (8 * (cb - cl));
      r += dr;
      c += dc;
      if (c >= nper) { c -= nper; ++r; }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + NT * u < total)
        reinterpret_cast<uint32_t*>(lds + __mul24(rr[u], lpitch))[cc[u]] = v[u];
  }
}


// ---------------------------------------------------------------------------
// k_pyramid: a chain of unique levels (PyrSeg) with OpenCV's INTER_LINEAR
// fixed-point arithmetic (resize.cpp HResizeLinear / VResizeLinear<uchar>):
// D = S[sx]*a0 + S[sx1]*a1 (int32),
// dst = (((b0*(D0>>4))>>16) + ((b1*(D1>>4))>>16) + 2) >> 2.
// Workgroup = one tile of the segment's last level.  The source region is
// staged in LDS once; every finer level is computed into the other LDS
// buffer (ping-pong); the tile's computed rows of every 4-pixel group that
// holds an owned column go to HBM as dwords (bytes it does not own are exact
// recomputations, equal to their owner's), and the intermediate levels are
// never re-read from HBM.
// Thread = 4 consecutive columns (dword in LDS and HBM) of a row.
// ---------------------------------------------------------------------------
#ifndef PYR_U
#define PYR_U 1
#endif
#ifdef PYR_PROBE_NOSTORE  // profiling only: no HBM stores of the levels
#define PYR_STORE_ON 0
#else
#define PYR_STORE_ON 1
#endif
// PYR_U: rows in flight per thread (more measured slower)

__global__ __launch_bounds__(256) void k_pyramid(const uint8_t* __restrict__ frames, size_t fstride,
                                                 size_t rstride, uint8_t* __restrict__ pyr,
                                                 size_t pstride, const PyrSeg S,
                                                 const int4* __restrict__ xs,
                                                 const int4* __restrict__ ys,
                                                 const uint4* __restrict__ blob,
                                                 const int* __restrict__ bo, int dbg) {
  extern __shared__ __align__(16) uint8_t plds[];
#if ORBX_EX_PRIO
  if (S.prio) __builtin_amdgcn_s_setprio(ORBX_EX_PRIO);  // ahead of a co-resident matcher's waves
#endif
  const int tid = threadIdx.x;
  int bx, f;
  frame_unit(bx, f);
  const int tx = bx % S.ntx, ty = bx / S.ntx;
  // the column LUT is read once per level and thread: straight from global
  // memory (L2); the row LUT, read every row iteration, is staged in LDS
  // (keeping the column LUT out of LDS raises occupancy from 5 to 7
  // workgroups per CU at 1080p).  Row entries hold the LDS byte offsets of
  // their two source rows: every tile lays a level out at the same pitch
  // (PyrSeg::lpitch), so the planner writes final offsets.
  const uint2* xl = reinterpret_cast<const uint2*>(blob) + bo[S.xbo_off + tx];
  {
    uint2* yl = reinterpret_cast<uint2*>(plds + S.lds_a + S.lds_b);
    const int y0 = bo[S.ybo_off + ty], ny = (bo[S.ybo_off + ty + 1] - y0) >> 1;
    const uint4* yb = blob + (y0 >> 1);
    for (int i = tid; i < ny; i += 256) reinterpret_cast<uint4*>(yl)[i] = yb[i];
  }
  // ---- stage the source region (level lev[0]) ----
  int4 X = xs[S.xs_off + tx], Y = ys[S.ys_off + ty];
  {
    const int cay = Y.x, cax = X.x & ~15, cpitch = S.lpitch[0];
    const uint8_t* src;
    size_t sp;
#ifdef PYR_PROBE_SAMESRC  // profiling only: every frame stages frame 0's source region
    const int fsrc = 0;
#else
    const int fsrc = f;
#endif
    if (S.off[0] < 0) {
      src = frames + (size_t)fsrc * fstride;
      sp = rstride;
    } else {
      src = pyr + (size_t)fsrc * pstride + S.off[0];
      sp = (size_t)S.pitch[0];
    }
    const int nr = Y.y - Y.x;
    const uintptr_t al = reinterpret_cast<uintptr_t>(src) | (uintptr_t)sp;
    const uint8_t* s0 = src + (size_t)cay * sp;
    if ((al & 15) == 0) {  // this tile's own 16-B columns (the pitch may be wider)
      stage_region<v4u, 4, 256>(plds, cpitch, s0 + cax, sp, nr, (((X.y + 15) & ~15) - cax) >> 4, tid);
    } else if ((al & 3) == 0) {
      const int d0 = (X.x & ~3) - cax, nd = (((X.y + 3) & ~3) - (X.x & ~3)) >> 2;
      stage_region<uint32_t, 8, 256>(plds + d0, cpitch, s0 + cax + d0, sp, nr, nd, tid);
    } else {
      stage_rows_u32<8, 256>(plds, cpitch, s0 + cax, sp, nr, X.y - cax, tid);
    }
  }
  __syncthreads();
  if (dbg == 11) return;
  // ---- levels 1..nl ----
  int xo = 0, yo = 0;  // this level's entries in the LUT blobs
  for (int s = 1; s <= S.nl; ++s) {
    X = xs[S.xs_off + s * S.ntx + tx];
    Y = ys[S.ys_off + s * S.nty + ty];
    const int dax = X.x & ~3;
    const int ncg = X.y > X.x ? (X.y - dax + 3) >> 2 : 0;
    const int nrows = max(Y.y - Y.x, 0);
    const uint32_t dpitch = (uint32_t)S.lpitch[s];
    if (ncg > 0 && nrows > 0) {
      // tid / ncg and 256 / ncg through the float reciprocal: exact for
      // integers <= 256.5 (relative error ~1e-7 against a margin >= 0.5 / ncg)
      const float rcp = __builtin_amdgcn_rcpf((float)ncg);
      const int R = __builtin_amdgcn_readfirstlane((int)(256.5f * rcp));
      if (tid < R * ncg) {
        const int r0 = (int)(((float)tid + 0.5f) * rcp), cg = tid - r0 * ncg;
        // the 4 columns' source bytes lie in an 8-byte window from sx[0]
        // (scale < 2: sx1[3] - sx[0] <= 7, checked by the planner): two
        // v_alignbyte of three LDS dwords per source row (one unaligned
        // ds_read_b64 instead: 0.685 -> 1.20 ms, c4), then one v_perm (bytes
        // sx, sx1 -> u16 pair) and one v_dot2_u32_u16 with the (a0, a1) pair
        // per column: D = S[sx]*a0 + S[sx1]*a1
        // blob (geometry.cpp build_blobs): column 0 of the group holds
        // s0 | (sx1 - s0) << 16, columns 1..3 their v_perm selectors
        // relative to s0; .y = a0 | a1 << 16, both in [0, 2048]
        uint32_t hsel[4], hcoef[4];
        uint32_t hbase, hsh;
        {
          const uint2 e0 = xl[xo + 4 * cg];
          hbase = (e0.x & 0xFFFCu) + lds_addr(plds);  // LDS byte address of the window's first dword
          hsh = e0.x & 3u;
          hsel[0] = (e0.x & 0xFFFF0000u) | 0x0C000C00u;
          hcoef[0] = e0.y;
#pragma unroll
          for (int k = 1; k < 4; ++k) {
            const uint2 e = xl[xo + 4 * cg + k];
            hsel[k] = e.x;
            hcoef[k] = e.y;
          }
        }
        const int gx0 = dax + 4 * cg;
        // HBM stores through a buffer resource over the level: a group
        // holding no owned column gets an offset past num_records, so its
        // stores are dropped by the range check (no per-row branch)
        const bool own = PYR_STORE_ON && gx0 + 4 > X.z && gx0 < X.w;
        const int gp = S.pitch[s];
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            pyr + (size_t)f * pstride + S.off[s], 0, gp * S.h[s], 0x00020000);
        const uint32_t gbase = own ? (uint32_t)(Y.x * gp + gx0) : 0xC0000000u;
        const uint32_t lbase = (uint32_t)((s & 1) ? S.lds_a : 0) + 4u * (uint32_t)cg;  // from plds
        const uint32_t ylb = __builtin_amdgcn_readfirstlane((uint32_t)(S.lds_a + S.lds_b) + 8u * (uint32_t)yo);
        // wave-uniform trip count (the wave's first active lane has its
        // smallest row): lanes past the level's last row recompute and
        // re-store that row (same bytes), so the loop needs no exec masking
        const int nm1 = nrows - 1;
        int rv = r0, rw = __builtin_amdgcn_readfirstlane(r0);
        while (rw < nrows) {
          const uint32_t r = (uint32_t)min(rv, nm1);
          rv += R;
          rw = __builtin_amdgcn_readfirstlane(rw + R);  // a separate scalar trip counter (opaque: not folded into rv)
          const uint2 e = *reinterpret_cast<const uint2*>(plds + (ylb + 8u * r));
          // SDWA halves of the entry: hbase + off0 / off1, b0 << 12 / b1 << 12
          // (the u24 multiply reads the low 24 bits: b0's shift needs no mask)
          uint32_t a0, a1, bs0, bs1;
          asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0"
              : "=v"(a0) : "v"(hbase), "v"(e.x));
          asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1"
              : "=v"(a1) : "v"(hbase), "v"(e.x));
          bs0 = e.y << 12;
          asm("v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1"
              : "=v"(bs1) : "v"(12u), "v"(e.y));
          typedef const __attribute__((address_space(3))) uint32_t* lds_u32p;
          const lds_u32p R0 = (lds_u32p)(size_t)a0, R1 = (lds_u32p)(size_t)a1;
          const uint32_t lo0 = __builtin_amdgcn_alignbyte(R0[1], R0[0], hsh);
          const uint32_t hi0 = __builtin_amdgcn_alignbyte(R0[2], R0[1], hsh);
          const uint32_t lo1 = __builtin_amdgcn_alignbyte(R1[1], R1[0], hsh);
          const uint32_t hi1 = __builtin_amdgcn_alignbyte(R1[2], R1[1], hsh);
          uint32_t v[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            // vertical: ((b*(D>>4))>>16) == mulhi_u24(b << 12, D & ~15)
            // (b <= 2048, D <= 255*2048: both operands < 2^24, exact)
            const uint32_t d0 = __builtin_amdgcn_udot2(as_us2(__builtin_amdgcn_perm(hi0, lo0, hsel[k])),
                                                       as_us2(hcoef[k]), 0u, false);
            const uint32_t d1 = __builtin_amdgcn_udot2(as_us2(__builtin_amdgcn_perm(hi1, lo1, hsel[k])),
                                                       as_us2(hcoef[k]), 0u, false);
            // (operands from LDS: the 24-bit form is spelled out, the
            // compiler would emit the quarter-rate v_mul_hi_u32)
            uint32_t t0, t1;
            asm("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(t0) : "v"(bs0), "v"(d0 & 0xFFFFF0u));
            asm("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(t1) : "v"(bs1), "v"(d1 & 0xFFFFF0u));
            v[k] = t0 + t1 + 2u;  // < 1024
          }
          // (v >> 2) of the four columns as bytes: two u16 pairs shifted as
          // whole dwords (v < 1024: the pair's high value lands whole in
          // bits 16..23), then one v_perm
          uint32_t p01, p23;
          asm("v_lshl_or_b32 %0, %1, 16, %2" : "=v"(p01) : "v"(v[1]), "v"(v[0]));
          asm("v_lshl_or_b32 %0, %1, 16, %2" : "=v"(p23) : "v"(v[3]), "v"(v[2]));
          p01 >>= 2;
          p23 >>= 2;
          const uint32_t packed = __builtin_amdgcn_perm(p23, p01, 0x06040200u);
          *reinterpret_cast<uint32_t*>(plds + (lbase + __umul24(r, dpitch))) = packed;
          // every computed row, also the ones another tile owns: computed
          // rows are exact, so their bytes equal the owner's (benign); the
          // whole group, also at the owned interval's edges: the planner
          // computes every group holding an owned pixel whole, so the bytes
          // this tile does not own carry the values their owner writes (or
          // lie past the level's last column, in the row padding)
          __builtin_amdgcn_raw_buffer_store_b32(packed, rs, gbase + __umul24(r, (uint32_t)gp), 0, 0);
        }
      }
    }
#ifndef PYR_PROBE_NOSYNC  // profiling only: level passes without the block barrier (wrong pixels)
    __syncthreads();
#endif
    xo += 4 * ncg;
    yo += nrows;
  }
}

// ---------------------------------------------------------------------------
// k_pyr_area2: one exact-2x level (cv::resize's INTER_AREA fast path, which
// resize(INTER_LINEAR) takes when both ratios are exactly 2: OpenCV 3.4
// resizeAreaFast_ with ResizeAreaFastVec, SIMD part and scalar remainder
// both (S[2x] + S[2x+1] + S'[2x] + S'[2x+1] + 2) >> 2).  Thread = 4
// destination pixels of a row (a dword: level pitches are 16-B multiples);
// grid (row groups, rows, frames).  Only for scale factors of exactly 2,
// outside every benchmark configuration.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_pyr_area2(const uint8_t* __restrict__ frames, size_t fstride,
                                                   size_t rstride, uint8_t* __restrict__ pyr,
                                                   size_t pstride, const PyrSeg S) {
  const int f = blockIdx.z, y = blockIdx.y;
  const int x4 = (blockIdx.x * 256 + threadIdx.x) * 4;
  const int dw = S.w[1];
  if (x4 >= dw) return;
  const uint8_t* src;
  size_t sp;
  if (S.off[0] < 0) {
    src = frames + (size_t)f * fstride;
    sp = rstride;
  } else {
    src = pyr + (size_t)f * pstride + S.off[0];
    sp = (size_t)S.pitch[0];
  }
  const uint8_t* a = src + (size_t)(2 * y) * sp + 2 * x4;
  const uint8_t* b = a + sp;
  const int n = min(4, dw - x4);
  uint32_t w = 0;
  for (int k = 0; k < n; ++k)
    w |= (uint32_t)((a[2 * k] + a[2 * k + 1] + b[2 * k] + b[2 * k + 1] + 2) >> 2) << (8 * k);
  uint8_t* o = pyr + (size_t)f * pstride + S.off[1] + (size_t)y * S.pitch[1] + x4;
  if (n == 4) {
    *reinterpret_cast<uint32_t*>(o) = w;
  } else {
    for (int k = 0; k < n; ++k) o[k] = (uint8_t)(w >> (8 * k));
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

// ---------------------------------------------------------------------------
// k_fast_strips: one workgroup per (strip of cells, frame).
//  1. the strip tile (cells + 3-px rings) is staged in LDS with dword loads;
//  2. every thread tests 4 adjacent band pixels with the 4 cardinal circle
//     points (necessary for a 9-arc at t_lo = min(ini, min) thresholds) and
//     pushes survivors into an LDS queue;
//  3. the full FAST strength A is computed only for queued pixels;
//  4. cv::FAST's NMS per cell at iniThFAST, then minThFAST for cells left
//     empty, into one 64-bit mask per (cell, band row);
//  5. each (cell, row) writes its kept pixels at the cell's raster offset.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int tbyte(const uint32_t* dw, int i) { return (dw[i >> 2] >> ((i & 3) * 8)) & 0xFF; }

__device__ __forceinline__ bool nms_keep_tile(const uint8_t* amap, int tpitch, int r, int c, int a,
                                              int th, int bh, int cb0, int cb1) {
  bool keep = true;
#pragma unroll
  for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
    for (int dx = -1; dx <= 1; ++dx) {
      if (!dx && !dy) continue;
      const int rr = r + dy, cc = c + dx;
      int nb = 0;
      if (rr >= 3 && rr < 3 + bh && cc >= cb0 && cc < cb1) {
        const int aq = amap[rr * tpitch + cc];
        nb = aq > th ? aq - 1 : 0;
      }
      keep = keep && (a - 1 > nb);
    }
  return keep;
}


__device__ __forceinline__ bool fast_even_test(const uint8_t* t, int tw, int th) {
  const int v = t[0];
  const int hi = v + th, lo = v - th;
  int mb = 0, md = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int I = t[c_circle_dy[2 * k] * tw + c_circle_dx[2 * k]];
    mb |= (I > hi) << k;
    md |= (I < lo) << k;
  }
  mb |= mb << 8;
  md |= md << 8;
  const int rb = mb & (mb >> 1) & (mb >> 2) & (mb >> 3);
  const int rd = md & (md >> 1) & (md >> 2) & (md >> 3);
  return ((rb | rd) & 0xFF) != 0;
}

__device__ __forceinline__ int wave_excl_scan(int n, int lane, int* total) {
  const int incl = wave_incl_scan(n);  // all 64 lanes active
  *total = lane_value(incl, 63);
  return incl - n;
}


#define FS_NW (FS_NT / 64)
#ifndef FS_L1FLUSH
#define FS_L1FLUSH 64 /* stage B runs once a wave's L1 holds this many entries */
#endif
#define FS_L1CAP (FS_L1FLUSH + 256) /* per-wave cardinal survivors: < FS_L1FLUSH carried + <= 256 new */
#define FS_L2CAP 128 /* per-wave even-test survivors: < 64 carried + <= 64 new */
#ifndef FS_CW_RMAX
/* FS_CW_RMAX: orbx_internal.h (the planner's column-walk test uses it too) */
#endif


// ---------------------------------------------------------------------------
// Everything after a strip's tile is in LDS: per-cell counters, pass 1,
// NMS, raster-order output.
// ---------------------------------------------------------------------------
// TP: the tile pitch as a compile-time constant (every LDS offset of stage A
// an immediate of one address register), 0 = runtime pitch
template <int TP>
__device__ __forceinline__ void fs_strip_body(
    uint8_t* __restrict__ tile, uint8_t* __restrict__ amap_mem, int* __restrict__ cnt,
    unsigned long long* __restrict__ mask, unsigned long long* __restrict__ mask2,
    uint16_t (*wlist1)[FS_L1CAP], uint16_t (*wlist2)[FS_L2CAP], uint16_t* __restrict__ clist,
    int* __restrict__ cslot, int& ncorner, const StripInfo& st, int f, int lead, int xal,
    int slot_pref, uint32_t* __restrict__ slots, size_t slot_stride,
    uint32_t* __restrict__ ccount, int ncells, int ini_th, int min_th, int tpitch_rt, int ccap,
    int* __restrict__ ovf, int dbg, const uint8_t* __restrict__ gsrc, int gpitch, bool cw, int kxs) {
  const int tpitch = TP ? TP : tpitch_rt;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: list bases in SGPRs
  const int bh = st.h - 6;
  uint8_t* amap = amap_mem - 3 * tpitch;  // indexed by tile row 3 .. 3+bh
  if (tid < st.ncells) {
    cnt[tid] = 0;
    cslot[tid] = slot_pref;
  }
  if (tid == 0) ncorner = 0;
  __syncthreads();
  if (dbg == 1) return;
  // band columns [c0, c1) in tile coordinates, rows [3, 3+bh); the strip's
  // cells tile [st.x, st.x + st.w)
  const int c0 = lead + 3, c1 = lead + st.w - 3;
  const int t_lo = min(ini_th, min_th);
  // pass 1 (per wave, no block barrier).  Stage A: cardinal pre-test on a
  // group of 4 pixels (tile cols 4g..4g+3) in packed 16-bit lanes + zero-fill
  // of the strength map; survivors are appended to list L1.  Stage B: the
  // even-point test, 64 L1 entries at a time, appends to L2.  Stage C: the
  // full 16-point strength, 64 L2 entries at a time.  Lists are per wave, so
  // only wave-level LDS ordering is needed.
  // nothing of the staging is in flight any more: an explicit vmcnt(0) here
  // lets the waitcnt pass drop the (run-time no-op) vmcnt waits it otherwise
  // re-inserts every stage-A iteration for registers the staging loads used
  __builtin_amdgcn_s_waitcnt(0x0F70);
  const int g0 = c0 >> 2, g1 = (c1 + 3) >> 2, ng = g1 - g0;
  const int ntask = ng * bh;
  uint16_t* L1 = wlist1[wave];
  uint16_t* L2 = wlist2[wave];
  int n2 = 0;  // wave-uniform list length of L2
  int n1 = 0;  // wave-uniform L1 length
#ifndef FS_APPEND_CC
  // L1's end as an LDS byte address (SGPR): stage A's appends advance it in
  // scalar code, n1 is derived from it only where the list is consumed
  const uint32_t l1base = lds_addr(L1);
  uint32_t l1a = l1base;
  const unsigned long long exec_all = __builtin_amdgcn_read_exec();
#endif
#ifdef FS_PROBE_NOAPP
  uint32_t probe_sink = 0;
#endif
  auto strength_batch = [&](int e, bool act) {
    bool corner = false;
    if (act) {
      const int rr = e >> 9, cc = e & 511;
      const int a = fast_strength(tile + __mul24(rr, tpitch) + cc, tpitch);
      corner = a > t_lo;
      amap[__mul24(rr, tpitch) + cc] = (uint8_t)(corner ? a : 0);
    }
    const unsigned long long bal = __ballot(corner);
    int b = 0;
    if (lane == 0 && bal) b = atomicAdd(&ncorner, __popcll(bal));
    b = __builtin_amdgcn_readfirstlane(b);
    const int q = b + lanes_below(bal);
    if (corner && q < ccap) clist[q] = (uint16_t)e;
  };
  auto even_batch = [&](int e, bool act) {
    const int ec = e & 511;
#ifdef FS_EVEN_SCALAR  // profiling only: the scalar bit-mask form
    const bool keep = act && ec >= c0 && ec < c1 && fast_even_test(tile + __mul24(e >> 9, tpitch) + ec, tpitch, t_lo);
#else
    const bool keep = act && ec >= c0 && ec < c1 && fast_even_test_pk(tile + __mul24(e >> 9, tpitch) + ec, tpitch, t_lo);
#endif
    const unsigned long long bal = __ballot(keep);
    if (keep) L2[n2 + lanes_below(bal)] = (uint16_t)e;
    n2 += __popcll(bal);
    if (n2 >= 64) {
      wave_sync_lds();
      n2 -= 64;
#ifndef FAST_SKIP_C  // profiling only: drop the even-test survivors
      strength_batch(L2[n2 + lane], true);
#endif
      wave_sync_lds();
    }
  };
  {
    const uint32_t tt = (uint32_t)t_lo * 0x00010001u;
    // stage A's v_perm selectors in SGPRs, set once (as literals the compiler
    // re-materialised some into VGPRs every group: gfx9 VOP3 takes no literal)
    uint32_t sel_v0, sel_v1, sel_a4lo, sel_a4hi, sel_a12hi;
    asm volatile("s_mov_b32 %0, 0x0c020c00" : "=s"(sel_v0));
    asm volatile("s_mov_b32 %0, 0x0c030c01" : "=s"(sel_v1));  // also a12 of the low half
    asm volatile("s_mov_b32 %0, 0x0c050c03" : "=s"(sel_a4lo));
    asm volatile("s_mov_b32 %0, 0x0c060c04" : "=s"(sel_a4hi));
    asm volatile("s_mov_b32 %0, 0x0c040c02" : "=s"(sel_a12hi));
    // one 4-pixel group: tile byte offset off = r * tpitch + 4 g, list entry
    // ebase = r << 9 | 4 g; a lane with threshold 0xFF00 per 16-bit lane
    // (padding) finds no survivors; zf: zero the group's strength-map dword
    // (a padding lane may only repeat a group some lane of the same call
    // zeroes: a later zero would erase strengths already written)
    // gb = tile + off - 3 tpitch - 4 (every read of the group at a
    // non-negative constant offset from it: one address register when the
    // pitch is a compile-time constant), zp = amap + off
    // (g = 0: w0 is the previous row's last dword -- only pixels left of
    // the band, rejected in stage B, read it; r >= 3 keeps it in the tile)
    auto gload = [&](const uint8_t* gb) {
      const uint32_t* row0 = reinterpret_cast<const uint32_t*>(gb + 3 * tpitch);
      GroupWords q;
      q.w0 = row0[0];
      q.w1 = row0[1];
      q.w2 = row0[2];
      q.up = *reinterpret_cast<const uint32_t*>(gb + 4);
      q.dn = *reinterpret_cast<const uint32_t*>(gb + 6 * tpitch + 4);
      return q;
    };
    // the cardinal test of one group: clo / chi hold pixels 0, 2 / 1, 3 in
    // 16-bit lanes, nonzero = survivor
    auto gcore = [&](const GroupWords& q, uint8_t* zp, uint32_t ttl, bool zf, uint32_t& clo,
                     uint32_t& chi) {
      const uint32_t w0 = q.w0, w1 = q.w1, w2 = q.w2, up = q.up, dn = q.dn;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t sel = h ? sel_v1 : sel_v0;
        const us2 v = as_us2(__builtin_amdgcn_perm(0u, w1, sel));
        const us2 a0 = as_us2(__builtin_amdgcn_perm(0u, dn, sel));
        const us2 a8 = as_us2(__builtin_amdgcn_perm(0u, up, sel));
        // (x+3, y) and (x-3, y) straight from the byte pairs {w2:w1} / {w1:w0}
        // (one v_perm each, no v_alignbyte): pixel i's point 4 is byte i+3 of
        // {w2:w1}, its point 12 byte i+1 of {w1:w0}
        const us2 a4 = as_us2(__builtin_amdgcn_perm(w2, w1, h ? sel_a4hi : sel_a4lo));
        const us2 a12 = as_us2(__builtin_amdgcn_perm(w1, w0, h ? sel_a12hi : sel_v1));
        const us2 t2 = as_us2(ttl);
        const us2 mb = __builtin_elementwise_min(__builtin_elementwise_max(a0, a8),
                                                 __builtin_elementwise_max(a4, a12));
        const us2 md = __builtin_elementwise_max(__builtin_elementwise_min(a0, a8),
                                                 __builtin_elementwise_min(a4, a12));
        const us2 db = __builtin_elementwise_sub_sat(mb, v + t2);       // > 0 iff brighter arc
        const us2 dd = __builtin_elementwise_sub_sat(__builtin_elementwise_sub_sat(v, md), t2);
        uint32_t x = as_u32(db) | as_u32(dd);
        asm("" : "+v"(x));  // one OR per half, shared by both pixels' tests
        if (h) chi = x; else clo = x;
      }
      if (zf) *reinterpret_cast<uint32_t*>(zp) = 0u;
    };
    auto l1_flush = [&]() {
#ifndef FS_APPEND_CC
      if (l1a >= l1base + 2u * FS_L1FLUSH) {  // wave-uniform
        n1 = (int)((l1a - l1base) >> 1);
#else
      if (n1 >= FS_L1FLUSH) {  // wave-uniform
#endif
        wave_sync_lds();
        while (n1 >= 64) {
          n1 -= 64;
#ifndef FS_PROBE_NOB  // profiling only: appends without stages B / C
          even_batch(L1[n1 + lane], true);
#endif
        }
        wave_sync_lds();
#ifndef FS_APPEND_CC
        l1a = l1base + 2u * (uint32_t)n1;
#endif
      }
    };
    auto gtest = [&](const GroupWords& q, uint8_t* zp, uint32_t ebase, uint32_t ttl, bool zf) {
      uint32_t clo, chi;
      gcore(q, zp, ttl, zf, clo, chi);
      // append: the ballot is the compare's SGPR result, the lane's slot is
      // mbcnt of it from 0 at the uniform L1 + n1, only survivors store
      // (stores of every lane to a dummy slot measured 13 % slower).
      // Columns outside [c0, c1) are appended too and rejected in stage B.
#ifdef FS_PROBE_NOAPP  // profiling only: stage A tests without appends
      probe_sink |= clo | chi;
      return;
#endif
#ifndef FS_APPEND_CC
      // Branch-free appends (round 6).  The CU's one scalar unit issues about
      // one instruction per cycle (tools/probe/issue_rates.hip: 0.93-0.96
      // SALU per CU-cycle at 4-8 waves per SIMD), and the compiler's form of
      // `if (k) L1[n1 + mbcnt] = e; n1 += popcount` spent 7 scalar
      // instructions per append (s_and_saveexec, s_cbranch_execz, s_lshl,
      // s_add, s_or exec, s_bcnt1, s_add).  Here exec is set straight from
      // each compare's ballot around its store and the list end advances by
      // one s_lshl1_add per append: 13 scalar instructions per group of 4
      // pixels instead of 28 (a store with no active lane writes nothing).
      // The whole group's appends are skipped when no lane has a survivor
      // (one compare and a branch; c4 FAST 1.08 -> 1.05 ms, c1 / c5 -2 %,
      // c2 +2 %: its 640x480 frames leave few survivor-free wave groups).
      if (__ballot((clo | chi) != 0u)) {
        const unsigned long long b0 = __ballot((uint16_t)clo != 0), b1 = __ballot((uint16_t)chi != 0),
                                 b2 = __ballot(clo > 0xFFFFu), b3 = __ballot(chi > 0xFFFFu);
        const uint32_t p0 = (uint32_t)lanes_below(b0), p1 = (uint32_t)lanes_below(b1),
                       p2 = (uint32_t)lanes_below(b2), p3 = (uint32_t)lanes_below(b3);
        const uint32_t e0 = ebase, e1 = ebase + 1u, e2 = ebase + 2u, e3 = ebase + 3u;
        uint32_t a0, a1, a2, a3, t;
        asm volatile(
            "s_bcnt1_i32_b64 %[t], %[b0]\n\t"
            "v_lshl_add_u32 %[a0], %[p0], 1, %[la]\n\t"
            "s_lshl1_add_u32 %[la], %[t], %[la]\n\t"
            "s_bcnt1_i32_b64 %[t], %[b1]\n\t"
            "v_lshl_add_u32 %[a1], %[p1], 1, %[la]\n\t"
            "s_lshl1_add_u32 %[la], %[t], %[la]\n\t"
            "s_bcnt1_i32_b64 %[t], %[b2]\n\t"
            "v_lshl_add_u32 %[a2], %[p2], 1, %[la]\n\t"
            "s_lshl1_add_u32 %[la], %[t], %[la]\n\t"
            "s_bcnt1_i32_b64 %[t], %[b3]\n\t"
            "v_lshl_add_u32 %[a3], %[p3], 1, %[la]\n\t"
            "s_lshl1_add_u32 %[la], %[t], %[la]\n\t"
            "s_mov_b64 exec, %[b0]\n\t"
            "ds_write_b16 %[a0], %[e0]\n\t"
            "s_mov_b64 exec, %[b1]\n\t"
            "ds_write_b16 %[a1], %[e1]\n\t"
            "s_mov_b64 exec, %[b2]\n\t"
            "ds_write_b16 %[a2], %[e2]\n\t"
            "s_mov_b64 exec, %[b3]\n\t"
            "ds_write_b16 %[a3], %[e3]\n\t"
            "s_mov_b64 exec, %[ex]"
            : [la] "+s"(l1a), [t] "=&s"(t), [a0] "=&v"(a0), [a1] "=&v"(a1), [a2] "=&v"(a2), [a3] "=&v"(a3)
            : [b0] "s"(b0), [b1] "s"(b1), [b2] "s"(b2), [b3] "s"(b3), [p0] "v"(p0), [p1] "v"(p1),
              [p2] "v"(p2), [p3] "v"(p3), [e0] "v"(e0), [e1] "v"(e1), [e2] "v"(e2), [e3] "v"(e3),
              [ex] "s"(exec_all)
            : "memory", "scc");
      }
#else
      // profiling variant: the compiler's branchy appends (rounds 1-5)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t x = (j & 1) ? chi : clo;
        const bool k = (j & 2) ? x > 0xFFFFu : (uint16_t)x != 0;
        const unsigned long long bal = __ballot(k);
        const int pos = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                       __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
        uint16_t* const L1n = L1 + __builtin_amdgcn_readfirstlane(n1);
        if (k) L1n[pos] = (uint16_t)(ebase + (uint32_t)j);
        n1 += __popcll(bal);
      }
#endif
#ifdef FS_PROBE_SALU  // profiling only: FS_PROBE_SALU extra scalar instructions per group
      {
        int sv = __builtin_amdgcn_readfirstlane(n1);
#pragma unroll
        for (int q = 0; q < FS_PROBE_SALU; ++q) asm volatile("s_add_u32 %0, %0, 1" : "+s"(sv));
        if (sv == -12345) asm volatile("s_nop 0");
      }
#endif
#ifdef FS_PROBE_VALU  // profiling only: FS_PROBE_VALU extra independent VALU per group
      {
        uint32_t vv = ebase;
#pragma unroll
        for (int q = 0; q < FS_PROBE_VALU; ++q) asm volatile("v_xor_b32 %0, 1, %0" : "+v"(vv));
        if (__builtin_amdgcn_readfirstlane((int)(vv == 0xFFFFFFFEu))) asm volatile("s_nop 0");
      }
#endif
      l1_flush();
    };
    auto group = [&](const uint8_t* gb, uint8_t* zp, uint32_t ebase, uint32_t ttl, bool zf) {
      gtest(gload(gb), zp, ebase, ttl, zf);
    };
    if (cw) {
      // column walk (no block-wide staging): lane l <-> tile dword column
      // gb + l (gb = g0, or g0 - 1 when the band's first pixel needs the
      // dword left of it); wave w owns band rows [rb, re) and loads tile rows
      // [rb, re + 6) straight into registers, writes them to the tile for
      // stages B / C (rows shared with the neighbouring waves are written
      // twice with the same bytes) and runs stage A from the registers: the
      // row's own dword, rows -3 / +3 of the column, and the neighbouring
      // columns' dwords by DPP wave shifts (no LDS reads, no barrier)
      const int gb = g0 - ((c0 & 3) != 3 ? 1 : 0);
      const int rpwv = (bh + FS_NW - 1) / FS_NW;
      const int rb = wave * rpwv, re = min(bh, rb + rpwv);
      const int gl = min(gb + lane, g1);  // lanes past the right halo repeat it
      const bool lact = gb + lane >= g0 && gb + lane < g1;
      const uint32_t tl = lact ? tt : 0xFF00FF00u;
      if (rb < re) {  // wave-uniform
        uint32_t V[FS_CW_RMAX + 6];
        // the wave's rows through a buffer resource over [row rb, the tile's
        // last row]: one scalar offset add per row, no 64-bit address math,
        // and rows past the tile read 0 from the range check instead of a
        // clamped address (those rows are never stored or tested; round 6)
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t*>(gsrc) + __umul24((uint32_t)rb, (uint32_t)gpitch), 0, (st.h - rb) * gpitch, 0x00020000);
        const int voff = 4 * gl;
#pragma unroll
        for (int k = 0; k < FS_CW_RMAX + 6; ++k) V[k] = __builtin_amdgcn_raw_buffer_load_b32(rs, voff, k * gpitch, 0);
        uint8_t* trow = tile + __mul24(rb, tpitch) + 4 * gl;
        const int nr = re - rb;
#ifdef FS_CW_STORE_FIRST  // profiling variant: every row to the tile before the first test (rounds 3-5)
        if (true) {
#else
        if (dbg == 5) {  // profiling only: loads and tile stores
#endif
#pragma unroll
          for (int k = 0; k < FS_CW_RMAX + 6; ++k)
            if (k < nr + 6) *reinterpret_cast<uint32_t*>(trow + k * tpitch) = V[k];
          if (dbg == 5) return;
        }
        // rows 0..5 to the tile now, row k + 6 just before band row k's test
        // (round 6): the rows arrive in load order and each store waits only
        // for its own row, so the first tests run while later rows are still
        // in flight (stages B / C read rows up to r + 3 of an entry at row
        // r <= k, already stored)
#ifndef FS_CW_STORE_FIRST
#pragma unroll
        for (int k = 0; k < 6; ++k) *reinterpret_cast<uint32_t*>(trow + k * tpitch) = V[k];
#endif
        uint8_t* zrow = amap + __mul24(3 + rb, tpitch) + 4 * gl;
        uint32_t er = ((uint32_t)(3 + rb) << 9) | (uint32_t)(4 * gl);
#pragma unroll
        for (int k = 0; k < FS_CW_RMAX; ++k) {
          if (k < nr) {  // wave-uniform
#ifndef FS_CW_STORE_FIRST
            *reinterpret_cast<uint32_t*>(trow + (k + 6) * tpitch) = V[k + 6];
#endif
            GroupWords q;
            q.up = V[k];
            q.w1 = V[k + 3];
            q.dn = V[k + 6];
            // bound_ctrl: the lane past the wave's edge reads 0 (a halo lane,
            // its results are dropped) and no "old" operand is materialised
            q.w0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)V[k + 3], 0x138, 0xf, 0xf, true);  // wave_shr:1
            q.w2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)V[k + 3], 0x130, 0xf, 0xf, true);  // wave_shl:1
            // zero-fill in every lane: halo lanes (and lanes repeating the
            // right halo) zero dwords wholly outside [c0, c1), where no
            // strength is ever written (gb >= 0 since c0 >= 3)
            gtest(q, zrow + k * tpitch, er + ((uint32_t)k << 9), tl, true);
          }
        }
      }
    } else if (ng <= 64) {
      // row-mapped: lane = (row lr of the step, group lg); a step covers
      // rpw = 64 / ngp rows (ngp = 16 / 32 / 64 >= ng); offsets and entries
      // are lane constants plus a uniform row term, the loop is scalar
      const int sh = ng <= 16 ? 4 : ng <= 32 ? 5 : 6;
      const int rpw = 64 >> sh, lr = lane >> sh, lg = lane & ((1 << sh) - 1);
      const bool lact = lg < ng;
      const int g = g0 + min(lg, ng - 1);  // padding lanes repeat the last group
      const uint32_t tl = lact ? tt : 0xFF00FF00u;
      const int offl = __mul24(3 + lr, tpitch) + 4 * g;
      const uint32_t el = ((uint32_t)(3 + lr) << 9) | (uint32_t)(4 * g);
      // per-lane pointers advanced by a uniform step (one VALU add each)
      const int step = FS_NW * rpw * tpitch;
      const uint8_t* gbl = tile + (offl - 3 * tpitch - 4 + __mul24(wave * rpw, tpitch));
      uint8_t* zpl = amap + (offl + __mul24(wave * rpw, tpitch));
      // full row blocks first (no per-iteration bounds test), then the
      // wave's partial last block if it has one
      int rb = wave * rpw;
      uint32_t eb = el + ((uint32_t)rb << 9);
      for (; rb + rpw <= bh; rb += FS_NW * rpw, gbl += step, zpl += step, eb += (uint32_t)(FS_NW * rpw) << 9)
        group(gbl, zpl, eb, tl, true);  // wave-uniform trip count
      if (rb < bh) {  // last rows: lanes past the band repeat its last row, no survivors
        const int r = min(rb + lr, bh - 1);
        const int off = __mul24(3 + r, tpitch) + 4 * g;
        group(tile + (off - 3 * tpitch - 4), amap + off, ((uint32_t)(3 + r) << 9) | (uint32_t)(4 * g),
              rb + lr < bh ? tl : 0xFF00FF00u, true);
      }
    } else {
      // flattened (row, group) tasks for bands wider than 64 groups
      const int it_first = wave * 64 + lane;
      int r = 3 + it_first / ng, g = g0 + it_first % ng;
      const int dr = FS_NT / ng, dg = FS_NT - dr * ng;
      for (int it0 = wave * 64; it0 < ntask; it0 += FS_NT) {  // wave-uniform trip count
        const bool act = it0 + lane < ntask;
        const int rc = act ? r : 3, gc = act ? g : g0;
        const int off = __mul24(rc, tpitch) + 4 * gc;
        group(tile + (off - 3 * tpitch - 4), amap + off, ((uint32_t)rc << 9) | (uint32_t)(4 * gc),
              act ? tt : 0xFF00FF00u, act);
        r += dr;
        g += dg;
        if (g >= g1) { g -= ng; ++r; }
      }
    }
    wave_sync_lds();
#ifndef FS_APPEND_CC
    n1 = (int)((l1a - l1base) >> 1);
#endif
    while (n1 >= 64) {  // leftovers above one batch (FS_L1FLUSH > 64)
      n1 -= 64;
      even_batch(L1[n1 + lane], true);
    }
    if (n1 > 0) even_batch(lane < n1 ? (int)L1[lane] : 0, lane < n1);
    wave_sync_lds();
    if (n2 > 0) strength_batch(lane < n2 ? (int)L2[lane] : 0, lane < n2);
  }
#ifdef FS_PROBE_NOAPP
  if (probe_sink == 0x9E3779B9u) ovf[1] = 1;
#endif
  __syncthreads();
  if (dbg == 2) return;
  for (int i = tid; i < st.ncells * bh; i += FS_NT) mask[i] = mask2[i] = 0ull;  // over the dead tile
  __syncthreads();
  // pass 2: cv::FAST NMS over the (sparse) nonzero strength map at both
  // thresholds in one scan: iniThFAST into mask (+ per-cell counts) and
  // minThFAST into mask2, used for cells left empty at iniThFAST (:293-296)
  const int wcell = st.wcell;
  // (c - c0) / wcell through the float reciprocal (exact: c - c0 < 512)
  const float rwcell = __builtin_amdgcn_rcpf((float)wcell);
  auto nms_pixel = [&](int r, int c, int a) {
    const int k = min((int)(((float)(c - c0) + 0.5f) * rwcell), st.ncells - 1);
    const int cb0 = c0 + k * wcell, cb1 = (k == st.ncells - 1) ? c1 : cb0 + wcell;
    // the neighbours' largest strength first: the per-threshold score
    // a > th ? a - 1 : 0 is non-decreasing in a, so its maximum over the
    // neighbours is the score of their maximum (one max per neighbour
    // instead of two compares, two selects and two max; c1 / c2 FAST -1 %)
    // branch-free: the 8 reads issued together at offsets clamped into the
    // band / cell (an outside neighbour reads the centre row or column), the
    // outside ones zeroed by selects.  The bounds-tested loop compiled to 8
    // exec-masked reads, each waited for alone: FAST c4 1.064 -> 1.024 ms,
    // c1 / c2 / c5 -2 to -3 %
    const bool vu = r > 3, vd = r + 1 < 3 + bh, vl = c > cb0, vr = c + 1 < cb1;
    const int ou = vu ? tpitch : 0, od = vd ? tpitch : 0, ol = vl ? 1 : 0, orr = vr ? 1 : 0;
    const uint8_t* pc = amap + __mul24(r, tpitch) + c;
    const int nu = pc[-ou], nd = pc[od], nl = pc[-ol], nr = pc[orr];
    const int nul = pc[-ou - ol], nur = pc[orr - ou], ndl = pc[od - ol], ndr = pc[od + orr];
    int mx = max(max(vu ? nu : 0, vd ? nd : 0), max(vl ? nl : 0, vr ? nr : 0));
    mx = max(mx, max(max(vu && vl ? nul : 0, vu && vr ? nur : 0), max(vd && vl ? ndl : 0, vd && vr ? ndr : 0)));
    const int nbm = max(0, mx > min_th ? mx - 1 : 0), nbi = max(0, mx > ini_th ? mx - 1 : 0);
    const unsigned long long bit = 1ull << (c - cb0);
    if (a > ini_th && a - 1 > nbi) {
      atomicOr(&mask[k * bh + (r - 3)], bit);
      atomicAdd(&cnt[k], 1);
    }
    if (a > min_th && a - 1 > nbm) atomicOr(&mask2[k * bh + (r - 3)], bit);
  };
  const int nc = ncorner;
  if (nc <= ccap) {
    for (int q = tid; q < nc; q += FS_NT) {
      const int e = clist[q];
      const int r = e >> 9, c = e & 511;
      nms_pixel(r, c, amap[r * tpitch + c]);
    }
  } else {  // list overflow: scan the strength map
    if (tid == 0) atomicAdd(ovf, 1);  // strips that took this path (orbx_plan_debug_counters)
    const int dr = FS_NT / ng, dg = FS_NT - dr * ng;
    int r = 3 + tid / ng, g = g0 + tid % ng;
    for (; r < 3 + bh;) {
      const uint32_t w4 = reinterpret_cast<const uint32_t*>(amap + r * tpitch)[g];
      if (w4) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int a = (w4 >> (8 * j)) & 0xFF, c = 4 * g + j;
          if (a == 0 || c < c0 || c >= c1) continue;
          nms_pixel(r, c, a);
        }
      }
      r += dr;
      g += dg;
      if (g >= g1) { g -= ng; ++r; }
    }
  }
  __syncthreads();
  if (dbg == 3 || dbg == 4) return;
  // pass 4: raster-order output per cell: one wave per cell, lane = band row,
  // row offsets by a wave prefix sum of the row popcounts
  uint32_t* fslots = slots + (size_t)f * slot_stride;
#ifndef FS_OUT_ONE_CELL
  if (bh <= 32) {
    // two cells per wave (lane halves), so a wave walks its cells' corners
    // once instead of once per cell
    for (int kk = 2 * wave; kk < st.ncells; kk += 2 * FS_NW) {  // wave-uniform
      const int k = kk + (lane >> 5), br = lane & 31;
      const bool act = k < st.ncells && br < bh;
      const int kc = act ? k : kk;
      const unsigned long long* mk = (cnt[kc] != 0 ? mask : mask2) + __mul24(kc, bh);
      unsigned long long m = act ? mk[br] : 0ull;
      const int n = __popcll(m);
      const int incl = wave_incl_scan(n);
      int tlo = lane_value(incl, 31), tall = lane_value(incl, 63);
      int off = incl - n - (lane >= 32 ? tlo : 0);
      const int cb0 = c0 + k * wcell, so = cslot[kc];
      const int gy = st.y + 3 + br - ORBX_MINB;
      const uint8_t* arow = amap + __mul24(3 + br, tpitch);
#ifdef FS_PROBE_NOOUT  // profiling only: no key stores (a dependent sink instead)
      uint32_t sink = 0;
      while (m) {
        const int b = __ffsll(m) - 1;
        m &= m - 1;
        sink += (uint32_t)arow[cb0 + b] + (uint32_t)off++;
      }
      if (sink == 0x9E3779B9u) fslots[so] = sink;
      tall = tlo = 0;  // no keypoints downstream
#else
      while (m) {
        const int b = __ffsll(m) - 1;
        m &= m - 1;
        const int c = cb0 + b;
        const int gx = xal + c - ORBX_MINB;
        fslots[so + off++] = orbx_pack_key((uint32_t)gx, (uint32_t)gy, (uint32_t)arow[c] - 1u, kxs);
      }
#endif
      if (lane == 0) ccount[(size_t)f * ncells + st.cell_begin + kk] = (uint32_t)tlo;
      if (lane == 32 && kk + 1 < st.ncells)
        ccount[(size_t)f * ncells + st.cell_begin + kk + 1] = (uint32_t)(tall - tlo);
    }
    return;
  }
#endif
  for (int k = wave; k < st.ncells; k += FS_NW) {
    const unsigned long long* mk = (cnt[k] != 0 ? mask : mask2) + k * bh;
    const int cb0 = c0 + k * wcell, so = cslot[k];
    int carry = 0;
    for (int rb = 0; rb < bh; rb += 64) {
      const int br = rb + lane;
      unsigned long long m = br < bh ? mk[br] : 0ull;
      int tot;
      int off = carry + wave_excl_scan(__popcll(m), lane, &tot);
      const int gy = st.y + 3 + br - ORBX_MINB;
      while (m) {
        const int b = __ffsll(m) - 1;
        m &= m - 1;
        const int c = cb0 + b;
        const int gx = xal + c - ORBX_MINB;
        fslots[so + off++] =
            orbx_pack_key((uint32_t)gx, (uint32_t)gy, (uint32_t)amap[(3 + br) * tpitch + c] - 1u, kxs);
      }
      carry += tot;
    }
    if (lane == 0) ccount[(size_t)f * ncells + st.cell_begin + k] = (uint32_t)carry;
  }
}

template <int TP>
__device__ __forceinline__ void fs_kernel(
    const uint8_t* __restrict__ frames, size_t fstride, size_t rstride,
    const uint8_t* __restrict__ pyr, size_t pstride, const LevelArgs& LA,
    const CellInfo* __restrict__ cells, const StripInfo* __restrict__ strips,
    uint32_t* __restrict__ slots, size_t slot_stride, uint32_t* __restrict__ ccount, int ncells,
    int ini_th, int min_th, int tpitch_rt, int tmax_h, int mcells, int ccap, int* __restrict__ ovf,
    int strip0, int dbg) {
  const int tpitch = TP ? TP : tpitch_rt;
  // LDS (occupancy is LDS-bound and the kernel is latency-bound: +12 KB per
  // workgroup measured +38 % time): tile | strength map of the band rows only
  // | per-cell counts; the NMS row masks reuse the tile, which is dead after
  // pass 1 (fs_lds in api_extract.hip mirrors this layout)
  extern __shared__ __align__(16) uint32_t sm[];
#if ORBX_EX_PRIO
  if (LA.prio) __builtin_amdgcn_s_setprio(ORBX_EX_PRIO);  // ahead of a co-resident matcher's waves
#endif
  uint8_t* tile = reinterpret_cast<uint8_t*>(sm);                    // tpitch * tmax_h
  uint8_t* amap_mem = tile + tpitch * tmax_h;                         // tpitch * (tmax_h - 6)
  int* cnt = reinterpret_cast<int*>(amap_mem + tpitch * (tmax_h - 6));  // mcells
  int* cslot = cnt + ((mcells + 3) & ~3);                               // mcells
  // corners at t_lo (A > t_lo), any order: ccap entries (the plan sizes it,
  // orbx_internal.h FS_CCAP)
  uint16_t* clist = reinterpret_cast<uint16_t*>(cslot + ((mcells + 3) & ~3));
  const bool masks_in_tile = 16 * mcells * (tmax_h - 6) <= tpitch * tmax_h;
  unsigned long long* mask = masks_in_tile ? reinterpret_cast<unsigned long long*>(tile)
                                           : reinterpret_cast<unsigned long long*>(clist + ((ccap + 3) & ~3));
  unsigned long long* mask2 = mask + mcells * (tmax_h - 6);
  __shared__ uint16_t wlist1[FS_NW][FS_L1CAP];
  __shared__ uint16_t wlist2[FS_NW][FS_L2CAP];
  __shared__ int ncorner;
  const int tid = threadIdx.x;
  // plain grid: with 8 strip columns at 1080p level 0, XCD (f*S + s) % 8 is
  // a strip column, whose ring rows then meet in one L2.  Frame-grouped
  // (frame_unit) and 4..256-strip chunked mappings cut the traffic 1.66x ->
  // 1.0x of the level bytes but measured 1.5-3 % slower.
#ifdef FS_FRAME_UNIT  // profiling variant: every strip of frame f on XCD f % 8
  int sx, f;
  frame_unit(sx, f);
  sx += strip0;
#else
  const int sx = blockIdx.x + strip0, f = blockIdx.y;
#endif
  const StripInfo st = strips[sx];
  const int pitch = st.pitch ? st.pitch : (int)rstride;
#ifdef FS_PROBE_SAMESRC  // profiling only: every frame's strips read frame 0 (cache-resident source)
  const int fsrc = 0;
#else
  const int fsrc = f;
#endif
  const int slot_pref = tid < st.ncells ? cells[st.cell_begin + tid].slot_off : 0;  // in flight
  bool aligned, aligned16, cw;
  int xal, lead;
  const uint8_t* s0;
  if (st.level != 0 || LA.l0al16) {
    // 16-B-aligned level base (the common case): the planner's lead, column
    // walk decision and pyramid offset (StripInfo::lead16 / cw16 / soff16)
    aligned = aligned16 = true;
    lead = st.lead16;
    xal = st.x - lead;
    s0 = st.level == 0 ? frames + ((size_t)fsrc * fstride + (size_t)st.y * rstride + (size_t)xal)
                       : pyr + ((size_t)fsrc * pstride + (size_t)st.soff16);
    cw = FS_NW == 4 && st.cw16;
  } else {
    const uint8_t* base = frames + (size_t)fsrc * fstride;
    const uintptr_t alb = reinterpret_cast<uintptr_t>(base) | (uintptr_t)pitch;
    aligned = (alb & 3) == 0;
    aligned16 = (alb & 15) == 0;
    xal = aligned16 ? (st.x & ~15) : aligned ? (st.x & ~3) : st.x;
    lead = st.x - xal;  // tile col of global st.x
    s0 = base + (size_t)st.y * pitch + xal;
    // column walk (fs_strip_body): dword-aligned rows, band rows <= 4 waves x
    // FS_CW_RMAX, and the band's dword columns plus both halo dwords within
    // the 64 lanes (every strip of the bench workloads but wCell-32 levels),
    // on levels the planner marks (st.colwalk: wide levels, where it measured
    // faster; block staging on the narrow ones); api_extract.hip makes the
    // same test for StripInfo::cw16
    const int cg0 = (lead + 3) >> 2, cg1 = (lead + st.w) >> 2;
    const int cgb = cg0 - (((lead + 3) & 3) != 3 ? 1 : 0);
    cw = FS_NW == 4 && st.colwalk && aligned && st.h - 6 <= FS_NW * FS_CW_RMAX && cg1 - cgb <= 63;
  }
#ifdef FS_NO_COLWALK  // profiling variant: block-wide staging for every strip
  cw = false;
#endif
  const int tw = lead + st.w;  // columns in use
  if (!cw) {
    if (aligned16) stage_region<v4u, 4, FS_NT>(tile, tpitch, s0, pitch, st.h, (tw + 15) >> 4, tid);
    else if (aligned) stage_region<uint32_t, 12, FS_NT>(tile, tpitch, s0, pitch, st.h, (tw + 3) >> 2, tid);
    else stage_rows_u32<12, FS_NT>(tile, tpitch, s0, pitch, st.h, tw, tid);
  }
  fs_strip_body<TP>(tile, amap_mem, cnt, mask, mask2, wlist1, wlist2, clist, cslot, ncorner, st, f, lead,
                             xal, slot_pref, slots, slot_stride, ccount, ncells, ini_th, min_th, tpitch, ccap, ovf,
                             dbg, s0, pitch, cw, LA.key_xs);
}

#define FS_KERNEL_ARGS                                                                              \
  const uint8_t *__restrict__ frames, size_t fstride, size_t rstride, const uint8_t *__restrict__ pyr, \
      size_t pstride, const LevelArgs LA, const CellInfo *__restrict__ cells,                       \
      const StripInfo *__restrict__ strips, uint32_t *__restrict__ slots, size_t slot_stride,      \
      uint32_t *__restrict__ ccount, int ncells, int ini_th, int min_th, int tpitch, int tmax_h,   \
      int mcells, int ccap, int *__restrict__ ovf, int strip0, int dbg
#define FS_KERNEL_PASS \
  frames, fstride, rstride, pyr, pstride, LA, cells, strips, slots, slot_stride, ccount, ncells, ini_th, min_th, tpitch, tmax_h, mcells, ccap, ovf, strip0, dbg

#ifdef FS_WPE  // profiling variant: occupancy target (7 measured +20 % at c4: 72 VGPRs)
#define FS_ATTR __attribute__((amdgpu_waves_per_eu(FS_WPE)))
#else
#define FS_ATTR
#endif
__global__ __launch_bounds__(FS_NT) FS_ATTR void k_fast_strips(FS_KERNEL_ARGS) { fs_kernel<0>(FS_KERNEL_PASS); }
// the plan's tile pitch is 288 for every strip width in 224..264 (all the
// bench workloads): immediates instead of per-iteration address adds
__global__ __launch_bounds__(FS_NT) FS_ATTR void k_fast_strips_p288(FS_KERNEL_ARGS) { fs_kernel<288>(FS_KERNEL_PASS); }

// ---------------------------------------------------------------------------
// Block-wide exclusive scan of an LDS int array (NT threads), returns total.
// ---------------------------------------------------------------------------
template <int NT>
__device__ int block_scan_excl(int* a, int n, int* wtmp) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int chunk = (n + NT - 1) / NT;
  const int b = tid * chunk, e = min(n, b + chunk);
  int s = 0;
  for (int i = b; i < e; ++i) s += a[i];
  const int incl = wave_incl_scan(s);
  if (lane == 63) wtmp[wave] = incl;
  __syncthreads();
  int woff = 0;
  for (int w = 0; w < wave; ++w) woff += wtmp[w];
  int total = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) total += wtmp[w];
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
__device__ __forceinline__ int quadrant(uint32_t key, int rx, int ry, int kxs) {
  const int x = orbx_key_x(key, kxs), y = orbx_key_y(key, kxs);
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

#define QT_KERNEL_ARGS                                                                      \
  const LevelInfo *__restrict__ lv, const CellInfo *__restrict__ cells,                    \
      const uint32_t *__restrict__ slots, size_t slot_stride,                              \
      const uint32_t *__restrict__ ccount, int ncells_total, uint32_t *__restrict__ qkeys, \
      int32_t *__restrict__ qnode, size_t qk_stride, uint32_t *__restrict__ qout,          \
      size_t qout_stride, int *__restrict__ lcount, int nlevels, int smax, int maxcells,   \
      int *__restrict__ err, uint32_t *__restrict__ qperm
#define QT_KERNEL_PASS \
  lv, cells, slots, slot_stride, ccount, ncells_total, qkeys, qnode, qk_stride, qout, qout_stride, lcount, nlevels, smax, maxcells, err, qperm

// QJ: keys per thread held in registers (NT QJ per level; more spill to the
// global keys/node arrays).  Both instantiations are built for 8 waves per
// SIMD (<= 64 VGPRs, 8 workgroups per CU): the kernel is latency-bound, so
// occupancy beats a larger register file of keys.  Measured (same-run A/B,
// ms per step): 12 keys at 95 VGPRs (5 waves) 0.089 / 0.173 / 0.117 (c4 /
// c1 / c5); 8 keys at 8 waves 0.089 / 0.123 / 0.078; 6 keys at 8 waves
// 0.092 / 0.115 / 0.075 -- 8 for 1080p-class levels, 6 below.
template <int QJ, int NT>
__device__ __forceinline__ void qt_body(QT_KERNEL_ARGS) {
  extern __shared__ __align__(16) int smem[];
  // grid (frames, levels): dispatch is round-robin over the 8 XCDs in
  // linear-id order, so consecutive frames of a level land on different XCDs,
  // and every frame's big levels 0 and 1 are dispatched first -- when the
  // workgroups need more than one round, the small levels fill the second
  // (the earlier (levels, frames) frame-grouped order put big levels of the
  // later frames into the second round: 0.139 -> 0.089 ms, c4)
  const int f = blockIdx.x, l = blockIdx.y;
  const int tid = threadIdx.x;
  const LevelInfo L = lv[l];
  const LevelInfo U = lv[L.unique];
  // cell offsets live only through the key gather: the node arrays reuse
  // their LDS (max(2 maxcells + 1, 11 smax) ints: one round of workgroups)
  int* cell_off = smem;                       // maxcells + 1
  int* cell_slot = smem + maxcells + 1;        // maxcells (slot_off of each cell)
  int* rx = smem;                             // smax  (rx / ry / cnt and nrx / nry / ncnt
  int* ry = rx + smax;                        // smax   swap roles every pass)
  int* cnt = ry + smax;                       // smax
  int* child = cnt + smax;                    // 4*smax (counts, then positions; then best)
  int* nrx = child + 4 * smax;                // smax
  int* nry = nrx + smax;                      // smax
  int* ncnt = nry + smax;                     // smax
  int* tmp1 = ncnt + smax;                    // smax
  // wide form: a second child array (4*smax, qt_lds_wide) so the next pass's
  // counts are zeroed inside this pass (one barrier less per pass)
  constexpr bool DB = NT >= 1024;
  int* const child2 = DB ? tmp1 + smax : child;
  __shared__ int wtmp[NT / 64];
  __shared__ int s_flag[2];

  uint32_t* keys = qkeys + (size_t)f * qk_stride + L.qk_off;
  int32_t* node = qnode + (size_t)f * qk_stride + L.qk_off;

  // gather vToDistributeKeys (cell-major, raster within cell)
  const int nc = U.ncells;
  const uint32_t* fcc = ccount + (size_t)f * ncells_total + U.cell_begin;
  // the cells' slot offsets are loaded beside their counts (independent
  // loads), so a key's gather below is one dependent global load, not two
  for (int i = tid; i < nc; i += NT) {
    cell_off[i] = (int)fcc[i];
    cell_slot[i] = cells[U.cell_begin + i].slot_off;
  }
  __syncthreads();
  const int C = block_scan_excl<NT>(cell_off, nc, wtmp);
  if (tid == 0) cell_off[nc] = C;
  __syncthreads();
  const uint32_t* fslots = slots + (size_t)f * slot_stride;
  // keys k = tid + NT j (j < QJ) and their node ids live in registers for
  // the whole distribution (every pass walks all keys twice: from global
  // memory that was a load-latency chain per pass); more keys than that
  // spill to the global scratch.  keys[] in global memory also serves the
  // final gather of the winners.
  uint32_t kr[QJ];
  int nr[QJ];
#pragma unroll
  for (int j = 0; j < QJ; ++j) {
    const int k = tid + NT * j;
    kr[j] = 0u;
    nr[j] = -1;
    if (k < C) {
      const int c = upper_bound_i(cell_off, nc, k) - 1;
      kr[j] = fslots[cell_slot[c] + (k - cell_off[c])];
      keys[k] = kr[j];
    }
  }
  for (int k = tid + NT * QJ; k < C; k += NT) {
    const int c = upper_bound_i(cell_off, nc, k) - 1;
    keys[k] = fslots[cell_slot[c] + (k - cell_off[c])];
  }
  __syncthreads();  // cell_off is dead: its LDS becomes the node arrays
#if defined(QT_PROBE_STOP) && QT_PROBE_STOP == 1  // profiling only: the gather alone
  if (tid == 0) lcount[(size_t)f * nlevels + l] = 0;
  return;
#endif
  auto for_keys = [&](auto&& body) {  // body(k, key, node&)
#pragma unroll
    for (int j = 0; j < QJ; ++j) {
      const int k = tid + NT * j;
      if (k < C) body(k, kr[j], nr[j]);
    }
    for (int k = tid + NT * QJ; k < C; k += NT) {
      int n = node[k];
      body(k, keys[k], n);
      node[k] = n;
    }
  };
  // initial nodes (:230-252)
  const int nIni = L.nini;
  int S = nIni;
  for (int i = tid; i < nIni; i += NT) {
    rx[i] = (int)(L.hX * (float)i) | ((int)(L.hX * (float)(i + 1)) << 16);
    ry[i] = 0 | (L.Hr << 16);
    cnt[i] = 0;
  }
  __syncthreads();
  if (DB) {  // the first pass's child counts and flag (the fast pass zeroes the next ones)
    for (int i = tid; i < 4 * min(nIni, smax); i += NT) child[i] = 0;
    if (tid == 0) s_flag[0] = 0;
  }
  for_keys([&](int, uint32_t key, int& n) {
    n = -1;
    if (nIni > 0) {
      const float x = (float)orbx_key_x(key, L.key_xs);
      const int idx = (int)(x / L.hX);
      if (idx >= 0 && idx < nIni) n = idx;
    }
    if (n >= 0) atomicAdd(&cnt[n], 1);
  });
  __syncthreads();

  int newS = 0;
  int* chc = child;  // this pass's child array (DB: alternates with child2)
  int* chn = child2;
  // fast passes: each key's child slot (4 n + quadrant, or 4 n for a
  // single-key node; -1 none) and whether it counts, from one batch of node
  // reads (one LDS round trip, not one per key); kept for the reassignment
  int tq[QJ];
  uint32_t split = 0;
  bool pre = false;
  auto qt_targets = [&]() {
    split = 0;
#pragma unroll
    for (int j = 0; j < QJ; ++j) {
      tq[j] = -1;
      if (NT * j >= C) continue;  // wave-uniform: key slots past the level's keys cost nothing
      const int n = nr[j], ns = max(n, 0);
      const int c = cnt[ns], x = rx[ns], y = ry[ns];
      tq[j] = n < 0 ? -1 : c >= 2 ? 4 * n + quadrant(kr[j], x, y, L.key_xs) : 4 * n;
      split |= (n >= 0 && c >= 2 ? 1u : 0u) << j;
    }
#pragma unroll
    for (int j = 0; j < QJ; ++j)
      if ((split >> j) & 1u) atomicAdd(&chc[tq[j]], 1);
  };
  for (int pass = 0;; ++pass) {
#ifdef QT_PROBE_MAXPASS  // profiling only: stop after this many passes (wrong keypoints)
    if (pass >= QT_PROBE_MAXPASS) break;
#endif
    if (pass >= ORBX_QT_MAX_PASSES) {
      if (tid == 0) atomicOr(err, ORBX_DEVERR_QUADTREE);
      newS = 0;
      break;
    }
    int& flag = s_flag[DB ? (pass & 1) : 0];
    if (DB && S <= NT && C <= NT * QJ) {
      // ---- fast pass (one node per thread, 3 barriers).  The child counts
      // (chc, zeroed by the previous pass) were issued at the end of the
      // previous pass (or just below for the first); then per node in
      // reverse order (thread t = node S-1-t, the scan order of tmp1 in the
      // general pass) the packed count, its wave scan and the cross-wave
      // offsets straight from registers: no scan array, no second scan
      // barrier; then the children; then each key's new node, read from its
      // kept slot, and the next pass's counts in the same phase.
      if (!pre) qt_targets();
      __syncthreads();
      const int i = S - 1 - tid;
      int cn = 0, v = 0;
      if (i >= 0) {
        cn = cnt[i];
        int nch = 0;
        if (cn >= 2) nch = (chc[4 * i] > 0) + (chc[4 * i + 1] > 0) + (chc[4 * i + 2] > 0) + (chc[4 * i + 3] > 0);
        v = (nch << 16) | (cn == 1);
      }
      const int incl = wave_incl_scan(v);
      const int wave = tid >> 6;
      if ((tid & 63) == 63) wtmp[wave] = incl;
      // the next pass's counts (<= 4 children per node) and flag: their last
      // readers were before this pass's first barrier
      for (int j = tid; j < 4 * min(4 * S, smax); j += NT) chn[j] = 0;
      if (tid == 0) s_flag[(pass + 1) & 1] = 0;
      __syncthreads();
      int woff = 0, tot = 0;
#pragma unroll
      for (int w = 0; w < NT / 64; ++w) {
        const int x = wtmp[w];
        woff += w < wave ? x : 0;
        tot += x;
      }
      const int excl = woff + incl - v;
      const int totC = tot >> 16, totK = tot & 0xFFFF;
      newS = totC + totK;
      if (i >= 0) {
        if (cn >= 2) {
          int pos = excl >> 16;
          for (int q = 3; q >= 0; --q) {
            const int cc = chc[4 * i + q];
            if (cc > 0) {
              if (pos < smax) {
                int crx, cry;
                child_rect(rx[i], ry[i], q, &crx, &cry);
                nrx[pos] = crx;
                nry[pos] = cry;
                ncnt[pos] = cc;
              }
              if (cc >= 2) flag = 1;
              chc[4 * i + q] = pos++;
            } else {
              chc[4 * i + q] = -1;
            }
          }
        } else if (cn == 1) {
          const int pos = totC + totK - (excl & 0xFFFF) - 1;
          if (pos < smax) {
            nrx[pos] = rx[i];
            nry[pos] = ry[i];
            ncnt[pos] = 1;
          }
          chc[4 * i] = pos;
        }
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < QJ; ++j)
        if (NT * j < C) nr[j] = tq[j] >= 0 ? chc[tq[j]] : -1;
      const bool finish = (newS >= L.N) || (flag == 0);
      if (finish) {
        __syncthreads();  // the tail reuses chc's LDS
        break;
      }
      int* t = rx; rx = nrx; nrx = t;
      t = ry; ry = nry; nry = t;
      t = cnt; cnt = ncnt; ncnt = t;
      t = chc; chc = chn; chn = t;
      S = newS;
      // the next pass's counts right away (new node arrays written before
      // the barrier above; chc zeroed in this pass's second phase)
      pre = S <= NT;
      if (pre) qt_targets();
      continue;
    }
    int* const child = chc;  // the general pass (any S)
    for (int i = tid; i < 4 * S; i += NT) child[i] = 0;
    if (tid == 0) flag = 0;
    __syncthreads();
    for_keys([&](int, uint32_t key, int& n) {
      if (n >= 0 && cnt[n] >= 2) atomicAdd(&child[4 * n + quadrant(key, rx[n], ry[n], L.key_xs)], 1);
    });
    __syncthreads();
    for (int i = tid; i < S; i += NT) {
      const int cn = cnt[i];
      int nch = 0;
      if (cn >= 2) nch = (child[4 * i] > 0) + (child[4 * i + 1] > 0) + (child[4 * i + 2] > 0) + (child[4 * i + 3] > 0);
      // one scan for both counts (S < 2^16): children per parent in the high
      // half (reverse parent order), kept single-key nodes in the low half;
      // the forward exclusive count of the latter is totK - (reverse
      // exclusive + own)
      tmp1[S - 1 - i] = (nch << 16) | (cn == 1);
    }
    __syncthreads();
    const int tot = block_scan_excl<NT>(tmp1, S, wtmp);
    const int totC = tot >> 16, totK = tot & 0xFFFF;
    newS = totC + totK;
    for (int i = tid; i < S; i += NT) {
      const int cn = cnt[i];
      if (cn >= 2) {
        int pos = tmp1[S - 1 - i] >> 16;
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
            if (cc >= 2) flag = 1;
            child[4 * i + q] = pos++;
          } else {
            child[4 * i + q] = -1;
          }
        }
      } else if (cn == 1) {
        const int pos = totC + totK - (tmp1[S - 1 - i] & 0xFFFF) - 1;
        if (pos < smax) {
          nrx[pos] = rx[i];
          nry[pos] = ry[i];
          ncnt[pos] = 1;
        }
        child[4 * i] = pos;
      }
    }
    __syncthreads();
    for_keys([&](int, uint32_t key, int& n) {
      if (n >= 0) n = (cnt[n] >= 2) ? child[4 * n + quadrant(key, rx[n], ry[n], L.key_xs)] : child[4 * n];
    });
    const bool finish = (newS >= L.N) || (flag == 0);
    __syncthreads();
    if (finish) break;

    // ping-pong: the new node arrays become the current ones (every read of
    // the old ones is before the barrier above; the next pass writes the
    // other set only after its first barrier)
    int* t = rx; rx = nrx; nrx = t;
    t = ry; ry = nry; nry = t;
    t = cnt; cnt = ncnt; ncnt = t;
    S = newS;
  }
#if defined(QT_PROBE_STOP) && QT_PROBE_STOP == 2  // profiling only: gather + passes
  if (tid == 0) lcount[(size_t)f * nlevels + l] = 0;
  return;
#endif
  // per final node: first key with maximal response (:277-284)
  uint32_t* best = (uint32_t*)child;  // 4*smax >= newS
  if (newS > L.kcap) {
    if (tid == 0) atomicOr(err, ORBX_DEVERR_QTCAP);
    newS = 0;
  }
  for (int i = tid; i < newS; i += NT) best[i] = 0u;
  __syncthreads();
  for_keys([&](int k, uint32_t key, int& n) {
    if (n >= 0 && n < newS) atomicMax(&best[n], ((key & 0xFFu) << 24) | (0xFFFFFFu - (uint32_t)k));
  });
  __syncthreads();
  uint32_t* out = qout + (size_t)f * qout_stride + L.kout_off;
  for (int i = tid; i < newS; i += NT) {
    const uint32_t k = 0xFFFFFFu - (best[i] & 0xFFFFFFu);
    out[i] = keys[k];
  }
  // k_orient_brief's processing order: the winners by key index.  Keys are
  // cell-major (cell rows top to bottom, raster within a cell), so the
  // keypoints BRIEF works on at the same time lie in the same band of rows
  // and their patches share 128-B lines in L2 (the output order -- node
  // order, the reference's -- is unchanged).  rank = winners with a smaller
  // key index: a bitmap over the key indices and a scan of its popcounts.
  uint32_t* perm = qperm + (size_t)f * qout_stride + L.kout_off;
  const int nw = (C + 31) >> 5;
#ifdef OB_NO_PERM  // profiling variant: BRIEF in output order
  if (false) {
#else
  if (nw <= 3 * smax) {  // rx / ry / cnt hold the counts, nrx.. the bitmap (dead node arrays)
#endif
    uint32_t* bm = reinterpret_cast<uint32_t*>(nrx);
    int* pc = rx;
    for (int w = tid; w < nw; w += NT) bm[w] = 0u;
    __syncthreads();
    for (int i = tid; i < newS; i += NT) {
      const uint32_t k = 0xFFFFFFu - (best[i] & 0xFFFFFFu);
      atomicOr(&bm[k >> 5], 1u << (k & 31));
    }
    __syncthreads();
    for (int w = tid; w < nw; w += NT) pc[w] = __popc(bm[w]);
    __syncthreads();
    block_scan_excl<NT>(pc, nw, wtmp);
    for (int i = tid; i < newS; i += NT) {
      const uint32_t k = 0xFFFFFFu - (best[i] & 0xFFFFFFu);
      perm[pc[k >> 5] + __popc(bm[k >> 5] & ((1u << (k & 31)) - 1u))] = (uint32_t)i;
    }
  } else {
    for (int i = tid; i < newS; i += NT) perm[i] = (uint32_t)i;
  }
  if (tid == 0) lcount[(size_t)f * nlevels + l] = newS;
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void k_quadtree(QT_KERNEL_ARGS) {
  qt_body<8, 256>(QT_KERNEL_PASS);
}
// single-frame / small-batch calls (a grid of a few workgroups, the level-0
// one sets the latency): 1024 threads walk the keys and the node lists
__global__ __launch_bounds__(1024) void k_quadtree_wide(QT_KERNEL_ARGS) {
  qt_body<8, 1024>(QT_KERNEL_PASS);
}
#ifndef QT_JSMALL
#define QT_JSMALL 6 /* keys per thread in registers below 1 Mpx levels */
#endif
#ifndef QT_WPE_SMALL
#define QT_WPE_SMALL 8
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(QT_WPE_SMALL))) void k_quadtree_j6(QT_KERNEL_ARGS) {
  qt_body<QT_JSMALL, 256>(QT_KERNEL_PASS);
}

// ---------------------------------------------------------------------------
// cv::GaussianBlur(7x7, sigma 2, BORDER_REFLECT_101) on 8U (ORBextractor.cc:479)
// uses OpenCV's bit-exact fixed-point kernel [18,34,48,56,48,34,18]/256:
// H = sum k_i p (u16 exact), out = (sum k_j H_j + 32768) >> 16.  All integer,
// so it is evaluated only where BRIEF samples it (k_orient_brief).
// ---------------------------------------------------------------------------
__constant__ int c_gk[7] = {18, 34, 48, 56, 48, 34, 18};

__device__ __forceinline__ int reflect101(int p, int len) {
  p = p < 0 ? -p : p;
  return p >= len ? 2 * len - 2 - p : p;
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

// x is wave-uniform.  The exception keys live in two VGPRs per lane
// (entries lane and lane + 64, loaded once per wave), so the lookup is two
// compares and a ballot -- no chain of dependent scalar loads; the rare hit
// reads its (sin, cos) pair.
static_assert(ORBX_SINCOS_NEXC <= 128, "exception table fits two entries per lane");
__device__ __forceinline__ void brief_sincos(float x, uint32_t exk0, uint32_t exk1, float* s, float* c) {
  orbx_sincos_core(x, s, c);
  const uint32_t b = orbx_f2u(x);
  const uint64_t m0 = __ballot(exk0 == b), m1 = __ballot(exk1 == b);
  if (m0 | m1) {
    const int i = m0 ? __ffsll((unsigned long long)m0) - 1 : 64 + __ffsll((unsigned long long)m1) - 1;
    *s = orbx_u2f(ORBX_SINCOS_EXC[i][1]);
    *c = orbx_u2f(ORBX_SINCOS_EXC[i][2]);
  }
}

// 7-tap Gaussian (OpenCV 8U fixed point, sigma 2): [18,34,48,56,48,34,18]
__device__ constexpr uint32_t kb_tap(int i) {
  return i == 0 || i == 6 ? 18u : i == 1 || i == 5 ? 34u : i == 2 || i == 4 ? 48u : 56u;
}
// weight dword d (bytes 4d..4d+3 of a 12-byte window) with k0..k6 at bytes
// m+1..m+7: the horizontal pass's output column 4q+m over dwords q-1..q+1
__device__ constexpr uint32_t kb_w(int m, int d) {
  uint32_t w = 0;
  for (int b = 0; b < 4; ++b) {
    const int i = 4 * d + b - (m + 1);
    if (i >= 0 && i <= 6) w |= kb_tap(i) << (8 * b);
  }
  return w;
}
// H of window column m (0..3) of the 12 bytes d0|d1|d2: the dot4 of each dword
// with its tap weights, dwords whose weights are all 0 skipped (m = 0 never
// reaches d2, m = 3 never d0; the compiler does not fold a zero-weight dot4)
template <int M>
__device__ __forceinline__ uint32_t kb_hsum(uint32_t d0, uint32_t d1, uint32_t d2) {
  uint32_t h = 0u;
  if constexpr (kb_w(M, 0) != 0u) h = __builtin_amdgcn_udot4(d0, kb_w(M, 0), h, false);
  if constexpr (kb_w(M, 1) != 0u) h = __builtin_amdgcn_udot4(d1, kb_w(M, 1), h, false);
  if constexpr (kb_w(M, 2) != 0u) h = __builtin_amdgcn_udot4(d2, kb_w(M, 2), h, false);
  return h;
}
__device__ __forceinline__ uint32_t kb_hsum(int m, uint32_t d0, uint32_t d1, uint32_t d2) {
  return m == 0 ? kb_hsum<0>(d0, d1, d2) : m == 1 ? kb_hsum<1>(d0, d1, d2)
       : m == 2 ? kb_hsum<2>(d0, d1, d2) : kb_hsum<3>(d0, d1, d2);  // m is a compile-time index
}
// ---------------------------------------------------------------------------
// k_blur: GaussianBlur(clone(level), 7x7, 2, 2, BORDER_REFLECT_101)
// (ORBextractor.cc:478-479) of every unique level, materialised once per
// frame for the level-blur BRIEF (k_orient_brief_lb).  OpenCV's 8U
// fixed-point path: H = sum_i k_i p (exact u16), out =
// (sum_j k_j H_j + 32768) >> 16, reflect-101 in both passes.
// Column walk, no LDS: a wave owns 62 dword columns (lanes 1..62; lanes 0 /
// 63 only hold the neighbouring dwords) x LB_R rows.  Each lane loads its
// dword of the LB_R + 6 rows (one coalesced 256-B row segment per load, all
// in flight), takes the neighbours' dwords by DPP, forms the horizontal sums
// of its 4 pixels (3 v_dot4 each) and the vertical sums from row pairs
// packed as u16 x 2 (3 v_dot2 + 1 v_mad_u24 per pixel).  Dwords not wholly
// inside the level (its first and last columns, the halo) are assembled
// from reflected bytes.
// ---------------------------------------------------------------------------
#define KV_PAIR(a, b) ((uint32_t)(a) | ((uint32_t)(b) << 16))
#define LB_R 32                 /* output rows per wave */
#define LB_WC 62                /* dword columns per wave */
static_assert(ORBX_LB_TW == 4 * LB_WC && ORBX_LB_TH == 4 * LB_R,
              "tile = one wave's 62 dword columns x 4 waves of LB_R rows");
__global__ __launch_bounds__(256) void k_blur(const uint8_t* __restrict__ frames, size_t fstride,
                                              size_t rstride, const uint8_t* __restrict__ pyr,
                                              size_t pstride, uint8_t* __restrict__ blur, size_t bstride,
                                              const BlurArgs B) {
  const int t = (int)blockIdx.x, f = (int)blockIdx.y;
  const int lane = (int)threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6);
  int i = 0;
  while (i + 1 < B.nu && t >= B.tile_begin[i + 1]) ++i;  // wave-uniform
  const int W = B.w[i], H = B.h[i];
  const int lt = t - B.tile_begin[i];
  const int ty = lt / B.tiles_x[i], tx = lt - ty * B.tiles_x[i];
  const int y0 = ty * ORBX_LB_TH + wave * LB_R;
  if (y0 >= H) return;  // wave-uniform; no barrier in this kernel
  // dword columns gc0 .. gc0 + 61 (the last tile column is moved left so
  // that it ends at the level's last dword: its reflected bytes then always
  // come from lanes of this wave; columns two tiles share are computed twice,
  // identically)
  const int nd = (W + 3) >> 2;
  const int gc0 = min(tx * LB_WC, max(nd - LB_WC, 0));
  const int gc = gc0 + lane - 1;  // this lane's dword column (halo lanes 0 / 63)
  const int x = 4 * gc;
  const bool l0 = B.src_off[i] < 0;
  const uint8_t* src = l0 ? frames + (size_t)f * fstride : pyr + (size_t)f * pstride + B.src_off[i];
  const uint32_t sp = l0 ? (uint32_t)rstride : (uint32_t)B.pitch[i];
  // every lane loads a dword (all loads issued before the first use); a wave
  // with a lane not wholly inside the level (the first and last tile
  // columns) loads at clamped columns and then rebuilds every lane's dword
  // from reflected bytes taken from the lanes that hold them (ds_bpermute)
  const bool edge = gc0 == 0 || 4 * (gc0 + LB_WC) + 4 > W;  // wave-uniform
  const uint32_t lbx = (uint32_t)(edge ? min(max(x, 0), W - 4) : x);
  uint32_t V[LB_R + 6];
#pragma unroll
  for (int k = 0; k < LB_R + 6; ++k) {
    const int gy = reflect101(min(y0 - 3 + k, H + 2), H);
    V[k] = ld32u(src + (__umul24((uint32_t)gy, sp) + lbx));
  }
  if (edge) {
    // byte j of this lane's dword is level column xq = reflect101(x + j)
    // (clamped: lanes far past the level stay in range, their values feed no
    // stored pixel); it lives in lane xq / 4 - gc0 + 1 at byte xq & 3, or, in
    // the last (possibly partial) dword, in that dword's lane, which loaded
    // columns W-4 .. W-1
    int sl[4], sh[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int xq = reflect101(min(max(x + j, -4), W + 3), W);
      const bool last = xq >= 4 * (nd - 1);
      sl[j] = 4 * min(max((last ? nd - 1 : xq >> 2) - gc0 + 1, 0), 63);
      sh[j] = last ? 8 * (xq - (W - 4)) : 8 * (xq & 3);
    }
#pragma unroll
    for (int k = 0; k < LB_R + 6; ++k) {
      uint32_t v = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        v |= ((uint32_t)__builtin_amdgcn_ds_bpermute(sl[j], (int)V[k]) >> sh[j] & 0xFFu) << (8 * j);
      V[k] = v;
    }
  }
  uint8_t* dst = blur + (size_t)f * bstride + B.blur_off[i];
  const uint32_t bp = (uint32_t)B.bpitch[i];
  const bool store = lane >= 1 && lane <= LB_WC && x < W;
  uint32_t Hc[7][4];  // horizontal sums of the last 7 staged rows (fully unrolled: register renaming)
  uint32_t Pr[7][4];  // (H of row k-1, H of row k) as u16 x 2
#pragma unroll
  for (int k = 0; k < LB_R + 6; ++k) {
    const uint32_t w1 = V[k];
    const uint32_t w0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)w1, 0x138, 0xf, 0xf, true);  // wave_shr:1
    const uint32_t w2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)w1, 0x130, 0xf, 0xf, true);  // wave_shl:1
    const int s = k % 7;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const uint32_t h = kb_hsum(m, w0, w1, w2);
      if (k >= 1) Pr[s][m] = Hc[(k + 6) % 7][m] | (h << 16);
      Hc[s][m] = h;
    }
    if (k >= 6) {
      // output row o = k - 6 (staged rows o .. o + 6): pairs (o, o+1),
      // (o+2, o+3), (o+4, o+5) and row o + 6 alone
      const int o = k - 6, y = y0 + o;
      uint32_t q[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        uint32_t acc = __builtin_amdgcn_udot2(as_us2(Pr[(o + 1) % 7][m]), as_us2(KV_PAIR(18, 34)), 32768u, false);
        acc = __builtin_amdgcn_udot2(as_us2(Pr[(o + 3) % 7][m]), as_us2(KV_PAIR(48, 56)), acc, false);
        acc = __builtin_amdgcn_udot2(as_us2(Pr[(o + 5) % 7][m]), as_us2(KV_PAIR(48, 34)), acc, false);
        q[m] = acc + __umul24(18u, Hc[s][m]);  // out = q >> 16 (<= 255: the taps sum to 65536)
      }
      const uint32_t lo = __builtin_amdgcn_perm(q[1], q[0], 0x0c0c0602u);  // bytes 2 of q[0..3]
      const uint32_t hi = __builtin_amdgcn_perm(q[3], q[2], 0x06020c0cu);
      if (store && y < H) *reinterpret_cast<uint32_t*>(dst + (__umul24((uint32_t)y, bp) + (uint32_t)x)) = lo | hi;
    }
  }
}

// vertical pairs (lo = first row, hi = second row) for taps starting at the
// low half (E) or the high half (O) of the first row pair
#define KV_E0 KV_PAIR(18, 34)
#define KV_E1 KV_PAIR(48, 56)
#define KV_E2 KV_PAIR(48, 34)
#define KV_E3 KV_PAIR(18, 0)
#define KV_O0 KV_PAIR(0, 18)
#define KV_O1 KV_PAIR(34, 48)
#define KV_O2 KV_PAIR(56, 48)
#define KV_O3 KV_PAIR(34, 18)

// Keypoint patch: rows y-21..y+21, 48 columns from (x-21) & ~3 (a multiple of
// 4 in level coordinates; the row addresses need not be dword aligned);
// covers IC_Angle's radius-15 disk and every blur tap of the radius-18 samples.
#define KP_R 21
#define KP_ROWS 43
#define KP_COLS 48
#define KP_HCOLS 40  /* hblur columns: patch columns 4 qlo .. 4 qlo + 39 (samples use cc-18..cc+18) */
#define KP_HPAIRS 22 /* hblur row pairs: rows 0..43 (row 43 never weighted) */
#ifndef KP_HSTRIDE
#define KP_HSTRIDE 22 /* hblur column stride, dwords */
#endif
#define KP_PSTRIDE (KP_COLS / 4) /* patch row, dwords (+1 padding: no change measured) */
#ifndef OB_HPASS_GROUP
#define OB_HPASS_GROUP 1 /* MFMA blocks between scheduling barriers (A/B: 1, 3, 9) */
#endif
#define KP_PGUARD_LO 2
typedef short ob_s2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ ob_s2 as_s2(uint32_t x) { return __builtin_bit_cast(ob_s2, x); }
#define KP_PGUARD_HI (5 * KP_PSTRIDE + 2)

// One keypoint of the frame's level-major output list: where its level
// lives and where its patch starts (all wave-uniform).
struct BriefKp {
  int oi;  // output position (levels concatenated, node order within a level)
  int l, x, y, score, patch_size;
  float scale;
  const uint8_t* img;
  int pitch, UW, UH, px0, py0;
  bool inside;   // the whole patch lies in the level
  // level-blur mode: the blurred level and the blurred patch's first column
  const uint8_t* bimg;
  int bpitch, bx0;
};

// the patch is 43 rows x 12 dwords: lane (< 60) owns column lane % 12 of
// rows lane / 12 + 5u, u = 0..8 (row 43+ clamped).  The nine loads are issued
// together from one uniform base (saddr) + a 32-bit lane offset and held in
// registers (scalars in a struct: never spilled to scratch).
// Level-blur mode (LB, k_orient_brief_lb): 11 registers -- the unblurred
// disk rows y-15..y+15, patch dwords 1..10 (310 dwords: lane + 64u, u < 5)
// and the blurred patch rows y-18..y+18, 10 dwords from bx0 = (x-18) & ~3
// (370 dwords: lane + 64u, u < 6).
template <bool LB>
struct BriefRegs {
  uint32_t r[LB ? 11 : 9];
#if OB_HPASS == 0
  uint32_t ht;  // the keypoint's packed horizontal-pass tasks (c_htask), per-keypoint blur only
#endif
};

__device__ __forceinline__ void brief_issue(const BriefKp& k, BriefRegs<false>& R, int lane) {
  const int ln = min(lane, 59);
  const uint32_t c4 = (uint32_t)(ln % 12) * 4u, r0 = (uint32_t)(ln / 12);
#if OB_HPASS == 0
  R.ht = c_htask.v[k.x - k.px0 - 21][lane];  // cc = 21..24
#endif
  if (k.inside) {
    // wave-uniform; every row offset of a level fits 32 bits (levels >= 2
    // are orbx's own buffers; for level 0, the caller's frame,
    // orbx_plan_extract rejects rstride * H >= 2^32): 32-bit scalar offset
    // (a size_t product here was a quarter-rate v_mad_u64_u32 per keypoint)
    const uint8_t* b = k.img + ((uint32_t)k.py0 * (uint32_t)k.pitch + (uint32_t)k.px0);
#pragma unroll
    for (int u = 0; u < 9; ++u) {
      const uint32_t row = min(r0 + 5u * u, (uint32_t)(KP_ROWS - 1));
      R.r[u] = ld32u(b + (__umul24(row, (uint32_t)k.pitch) + c4));  // pitch < 2^24 (API check)
    }
  } else {
    // patch crosses the level border: reflect-101 rows, dword loads where the
    // four columns are inside, reflected bytes at the left/right edge only
    // 32-bit offsets from the wave-uniform level base (SGPR base + VGPR
    // offset loads): this rare path must not set the kernel's VGPR count
    const int cx = k.px0 + (int)c4;
    const bool cin = cx >= 0 && cx + 4 <= k.UW;
#pragma unroll
    for (int u = 0; u < 9; ++u) {
      const int r = min((int)r0 + 5 * u, KP_ROWS - 1);
      const int gy = reflect101(min(max(k.py0 + r, -3), k.UH + 2), k.UH);
      const uint32_t ro = __umul24((uint32_t)gy, (uint32_t)k.pitch);  // < 2^32: same API check
      if (cin) {
        R.r[u] = ld32u(k.img + (ro + (uint32_t)cx));
      } else {
        uint32_t w = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int gx = reflect101(min(max(cx + j, -3), k.UW + 2), k.UW);
          w |= (uint32_t)k.img[ro + (uint32_t)gx] << (8 * j);
        }
        R.r[u] = w;
      }
      __builtin_amdgcn_sched_barrier(0);  // one row's loads at a time
    }
  }
}

__device__ __forceinline__ void brief_commit(const BriefRegs<false>& R, uint32_t* P, int lane) {
  if (lane < 60) {
    const int c = lane % 12, r0 = lane / 12;
#pragma unroll
    for (int u = 0; u < 9; ++u) {
      const int row = r0 + 5 * u;
#if OB_HPASS == 1
      // stored signed (p - 128, the i8 MFMA's operand form): IC_Angle's sums
      // are unchanged (sec. ob_body), the pass's H is offset by -128 * 256
      if (row < KP_ROWS) P[row * KP_PSTRIDE + c] = R.r[u] ^ 0x80808080u;
#else
      if (row < KP_ROWS) P[row * KP_PSTRIDE + c] = R.r[u];
#endif
    }
  }
}

// Level-blur mode: every read lies inside its level (keypoints are >= 19 px
// from every border: FAST cells span [16, dim - 16) less cv::FAST's 3-px
// margin, ORBextractor.cc:316-331; the disk reaches 15 px, the blurred
// samples 18 px), so no reflection here -- k_blur applied it.  Bytes read
// past a row's last pixel (<= 3 of the unblurred rows, <= 2 of the blurred)
// belong to the next row or the pitch padding and are never used.
#define LB_DISK 310 /* 31 rows x 10 dwords */
#define LB_BP 370   /* 37 rows x 10 dwords */
__device__ __forceinline__ void brief_issue(const BriefKp& k, BriefRegs<true>& R, int lane) {
  const uint8_t* b = k.img + ((uint32_t)(k.y - 15) * (uint32_t)k.pitch + (uint32_t)(k.px0 + 4));
#pragma unroll
  for (int u = 0; u < 5; ++u) {
    const uint32_t e = (uint32_t)min(lane + 64 * u, LB_DISK - 1), row = e / 10u, dw = e - 10u * row;
    R.r[u] = ld32u(b + (__umul24(row, (uint32_t)k.pitch) + 4u * dw));  // pitch < 2^24 (API check)
  }
  const uint8_t* bb = k.bimg + ((uint32_t)(k.y - 18) * (uint32_t)k.bpitch + (uint32_t)k.bx0);
#pragma unroll
  for (int u = 0; u < 6; ++u) {
    const uint32_t e = (uint32_t)min(lane + 64 * u, LB_BP - 1), row = e / 10u, dw = e - 10u * row;
    R.r[5 + u] = *reinterpret_cast<const uint32_t*>(bb + (__umul24(row, (uint32_t)k.bpitch) + 4u * dw));
  }
}

__device__ __forceinline__ void brief_commit(const BriefRegs<true>& R, uint32_t* P, uint32_t* Bp, int lane) {
#pragma unroll
  for (int u = 0; u < 5; ++u) {
    const int e = lane + 64 * u, row = e / 10, dw = e - 10 * row;
    if (e < LB_DISK) P[row * KP_PSTRIDE + 1 + dw] = R.r[u];
  }
#pragma unroll
  for (int u = 0; u < 6; ++u) {
    const int e = lane + 64 * u;
    if (e < LB_BP) Bp[e] = R.r[5 + u];  // row-major, 10 dwords (40 bytes) per row
  }
}

#ifndef OB_WPE
#define OB_WPE 7
#endif
#ifndef OB_PROBE
#define OB_PROBE 0 /* profiling only: 1 / 2 / 3 skip the horizontal pass / IC_Angle sums / samples, 4 / 5 the fastAtan2 + sincos chain / sincos */
#endif
#define OB_KERNEL_ARGS                                                                             \
  const uint8_t *__restrict__ frames, size_t fstride, size_t rstride, const uint8_t *__restrict__ pyr, \
      size_t pstride, const BriefArgs A, const uint32_t *__restrict__ qout, size_t qout_stride,        \
      const int *__restrict__ lcount, orbx_keypoint *__restrict__ kps, uint8_t *__restrict__ desc,     \
      int *__restrict__ counts, const uint32_t *__restrict__ qperm, int dbg
#define OB_KERNEL_PASS frames, fstride, rstride, pyr, pstride, A, qout, qout_stride, lcount, kps, desc, counts, qperm, dbg
// LB = false: per-keypoint blur (the horizontal pass over the staged
// unblurred patch, the vertical taps at every sample); LB = true: samples
// read the level k_blur materialised (the planner picks per geometry,
// Plan::lb)
template <bool LB>
__device__ __forceinline__ void ob_body(OB_KERNEL_ARGS, const uint8_t* __restrict__ blur, size_t bstride) {
#if OB_HPASS == 1
  // guard dwords: the MFMA pass's windows start 2 dwords before a row and its
  // last row block reads 5 rows + 2 dwords past a patch (never weighted)
  __shared__ uint32_t patchbuf[KP_PGUARD_LO + 4 * KP_ROWS * KP_PSTRIDE + KP_PGUARD_HI];
#else
  __shared__ uint32_t patch[4][KP_ROWS][KP_PSTRIDE];
#endif
  // horizontally blurred patch, column-major: hblur[w][patch col][row pair]
  // = (H(row 2k), H(row 2k+1)) as u16 pair, H = sum_i k_i p (7 taps)
  __shared__ uint32_t hblur[4][KP_HCOLS][KP_HSTRIDE];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  int bx, f;
  frame_unit(bx, f);
  const int g = bx * 4 + wave;
  const int nlevels = A.nlevels, kcap = A.kcap;
  // per-level counts of this frame: one vector load + wave prefix
  const int lcv = lane < nlevels ? lcount[(size_t)f * nlevels + lane] : 0;
  const int incl = wave_incl_scan(lcv);
  const int total = lane_value(incl, 63);  // all lanes active here
  if (bx == 0 && threadIdx.x == 0) counts[f] = total;
  const int excl = incl - lcv;
  const uint32_t* Q = qout + (size_t)f * qout_stride;
  const uint32_t* QP = qperm + (size_t)f * qout_stride;
#if OB_HPASS == 1
  uint32_t(*P)[KP_PSTRIDE] = reinterpret_cast<uint32_t(*)[KP_PSTRIDE]>(patchbuf + KP_PGUARD_LO + wave * (KP_ROWS * KP_PSTRIDE));
  // B operand of the horizontal pass (lane = output column c of a 16-column
  // block, 8 k-bytes 8 (lane >> 4) + j = window columns): tap t = k - c - 5
  // of [18, 34, 48, 56, 48, 34, 18] (the window starts 8 columns left of the
  // block), 0 elsewhere -- one constant for every block and keypoint
  uint64_t hbw = 0;
  {
    const int c = lane & 15, k0 = 8 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int t = k0 + j - c - 5;
      if (t >= 0 && t <= 6) hbw |= (uint64_t)kb_tap(t) << (8 * j);
    }
  }
#else
  uint32_t(*P)[KP_PSTRIDE] = patch[wave];
#endif
  uint32_t* const Bp = &hblur[wave][0][0];  // LB: the blurred patch (37 x 40 bytes) in the hblur space
  const uint8_t* const Bpb = reinterpret_cast<const uint8_t*>(Bp);
  orbx_keypoint* const kpsf = kps + (size_t)f * kcap;  // this frame's outputs
  // IC_Angle weights, the lane's part (b0 = 24 for odd lanes, else 4)
  const uint32_t Wlane = (uint32_t)((lane & 1) ? 24 + 19 : 4 + 19) * 0x01010101u + 0x03020100u;
  uint8_t* const descf = desc + (size_t)f * kcap * 32;
  // sincos exception keys, entries lane and lane + 64 (brief_sincos)
  const uint32_t exk0 = ORBX_SINCOS_EXC[lane < ORBX_SINCOS_NEXC ? lane : 0][0];
  const uint32_t exk1 = lane + 64 < ORBX_SINCOS_NEXC ? ORBX_SINCOS_EXC[lane + 64][0] : 0xFFFFFFFFu;
  // this lane's pattern points (pairs lane + 64 rr) as floats, held for the
  // whole kernel (no per-keypoint byte extraction / conversion)
  float pfx[3][2], pfy[3][2];
#pragma unroll
  for (int rr = 0; rr < 3; ++rr) {
    const uint32_t pw = *reinterpret_cast<const uint32_t*>(ORBX_BRIEF_PATTERN[lane + 64 * rr]);
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      pfx[rr][e] = (float)(int)(int8_t)(pw >> (16 * e));
      pfy[rr][e] = (float)(int)(int8_t)(pw >> (16 * e + 8));
    }
  }
  __syncthreads();
  // output position o -> keypoint.  Everything is wave-uniform and forced
  // scalar (readfirstlane): the key and the level tables are s_loads, so the
  // only vector loads in flight while a keypoint is computed are the next
  // keypoint's patch (vmcnt stays exact; nothing waits on it early).
  auto locate = [&](int o) {
    const int l = __builtin_amdgcn_readfirstlane(__popcll(__ballot(lane < nlevels && incl <= o)));
    const int e = __builtin_amdgcn_readlane(excl, l);  // l is uniform
    // position o of the processing order (qperm, k_quadtree) -> winner i of
    // level l, written at output position e + i
    const int i = (int)__builtin_amdgcn_readfirstlane(QP[A.kout_off[l] + (o - e)]);
    const uint32_t key = __builtin_amdgcn_readfirstlane(Q[A.kout_off[l] + i]);
    BriefKp k;
    k.oi = e + i;
    k.l = l;
    k.x = orbx_key_x(key, A.key_xs) + ORBX_MINB;
    k.y = orbx_key_y(key, A.key_xs) + ORBX_MINB;
    k.score = (int)(key & 0xFF);
    k.scale = A.scale[l];
    k.patch_size = A.patch[l];
    const int u = A.unique[l];
    k.pitch = u == 0 ? (int)rstride : A.pitch[u];
    k.img = u == 0 ? frames + (size_t)f * fstride : pyr + (size_t)f * pstride + A.pyr_off[u];
    k.UW = A.w[u];
    k.UH = A.h[u];
    k.px0 = (k.x - KP_R) & ~3;
    k.py0 = k.y - KP_R;
    k.inside = k.px0 >= 0 && k.px0 + KP_COLS <= k.UW && k.py0 >= 0 && k.py0 + KP_ROWS <= k.UH;
    if constexpr (LB) {
      k.bimg = blur + (size_t)f * bstride + A.blur_off[u];
      k.bpitch = A.bpitch[u];
      k.bx0 = (k.x - 18) & ~3;
    }
    return k;
  };
  // output position o (levels concatenated, :455-494); waves stride over
  // the frame's keypoints, so the grid is sized by nfeatures, not capacity.
  // Software pipeline: keypoint o is computed while the patch of o+stride
  // is loading into registers.
  const int nwv = (int)gridDim.x * 4;
#ifdef OB_CONTIG  // profiling variant: each wave walks a contiguous run of the processing order
  const int per = (total + nwv - 1) / nwv;
  const int stride = 1;
  int o = g * per;
  const int oend = min(total, o + per);
#else
  const int stride = nwv;
  int o = g;
  const int oend = total;
#endif
  if (o >= oend) return;
  BriefKp cur = locate(o);
  BriefRegs<LB> R;
  brief_issue(cur, R, lane);
  for (; o < oend; o += stride) {  // wave-uniform
  // ---- stage this keypoint's patch (unblurred level), reflect-101 outside ----
  [[maybe_unused]] uint32_t hte = 0;  // OB_HPASS 0: the keypoint's task bytes
  if constexpr (LB) {
    brief_commit(R, &P[0][0], Bp, lane);
  } else {
    brief_commit(R, &P[0][0], lane);
#if OB_HPASS == 0
    hte = R.ht;  // before the next keypoint's issue overwrites R
#endif
  }
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  const BriefKp me = cur;
  if (o + stride < oend) {  // next keypoint: its patch loads stay in flight
    cur = locate(o + stride);
    brief_issue(cur, R, lane);
  }
  const int l = me.l, x = me.x, score = me.score, px0 = me.px0;
  // BRIEF (:57-73) on GaussianBlur(7x7, sigma 2): separable and exact,
  // out = (sum_j k_j H(r+j-3) + 32768) >> 16 with H = sum_i k_i p(c+i-3)
  // (OpenCV's fixed-point 8U path, [18,34,48,56,48,34,18]).  The horizontal
  // pass runs once per keypoint over the patch (hblur, column-major, row
  // pairs packed as 16-bit x 2: H - 32768 as i16 from the matrix cores, or H
  // as u16 from the v_dot4 tasks of OB_HPASS 0); each of the 364 live samples
  // is then 4 dword reads + 4 v_dot2 down its hblur column -- 64 LDS ops per
  // keypoint instead of 21 dword reads per sample (126).  It runs before
  // IC_Angle so its LDS writes drain while the angle and sin/cos are computed.
  // Matrix-core pass (round 5): 9 MFMAs + 18 v_perm per keypoint replace
  // ~130 VALU of v_dot4 tasks (BRIEF c4 0.456 -> 0.416 ms, c1 0.833 -> 0.738,
  // c2 0.434 -> 0.393)
#if OB_HPASS == 1
  if constexpr (!LB) {
    // one v_mfma_i32_16x16x32_i8 per 16 rows x 16 output columns: A = the
    // signed patch (lane: row r0 + (lane & 15), window bytes 8 (lane >> 4) ..
    // +7 -- one ds_read2_b32), B = hbw, D lane: rows 4 (lane >> 4) .. +3 of
    // column lane & 15 = H - 32768 (the taps sum to 256), packed as i16 row
    // pairs.  Blocks: rows 0..47 x hblur columns 0..47 (columns 4 qlo ..);
    // rows >= 44 and columns >= 40 are not stored, and every window byte
    // outside the patch or the block's taps has weight 0 (KP_PGUARD_*).
    const int cc = me.x - me.px0;
    const int qlo = (cc - 18) >> 2;
    typedef int v4i __attribute__((ext_vector_type(4)));
    const uint32_t* ab = &P[0][0] + (__mul24(lane & 15, KP_PSTRIDE) + 2 * (lane >> 4) - 2 + qlo);
    uint32_t* hb = &hblur[wave][0][0] + (__mul24(lane & 15, KP_HSTRIDE) + 2 * (lane >> 4));
#pragma unroll
    for (int rb = 0; rb < 3; ++rb) {
#pragma unroll
      for (int cb = 0; cb < 3; ++cb) {
        const uint32_t* a = ab + (16 * KP_PSTRIDE * rb + 4 * cb);
        const uint64_t av = (uint64_t)a[0] | ((uint64_t)a[1] << 32);
        const v4i h = __builtin_amdgcn_mfma_i32_16x16x32_i8((long)av, (long)hbw, (v4i){0, 0, 0, 0}, 0, 0, 0);
        const bool st = (cb < 2 || (lane & 15) < KP_HCOLS - 32) && (rb < 2 || (lane >> 4) < 3);
        if (st) {
          const uint32_t p01 = __builtin_amdgcn_perm((uint32_t)h[1], (uint32_t)h[0], 0x05040100u);
          const uint32_t p23 = __builtin_amdgcn_perm((uint32_t)h[3], (uint32_t)h[2], 0x05040100u);
          *reinterpret_cast<uint2*>(hb + (16 * KP_HSTRIDE * cb + 8 * rb)) = make_uint2(p01, p23);
        }
#if OB_HPASS_GROUP == 1
        __builtin_amdgcn_sched_barrier(0);  // one block's registers at a time (72 VGPRs)
#endif
      }
#if OB_HPASS_GROUP == 3
      __builtin_amdgcn_sched_barrier(0);
#endif
    }
  }
#else
  if constexpr (!LB) {
    // task = (row pair rp, 4-column group q): patch columns 4q..4q+3, rows
    // 2rp, 2rp+1; the 7-byte windows c-3..c+3 lie in dwords q-1..q+1
    // cc = x - px0 is 21..24, so the columns cc-18..cc+18 always span the 10
    // groups qlo..qlo+9 (qlo = 0 for cc = 21, else 1).  Of those 22 x 10
    // tasks only the ones under a rotated sample's taps are computed: the
    // live pattern points stay within a fixed radius at every angle
    // (tools/gen_brief_htasks.py), 189-190 tasks, 3 rounds of 64 lanes
    const int cc = me.x - me.px0;
    const int qlo = (cc - 18) >> 2;
    // this lane's task of round k: byte k of hte (loaded with the patch;
    // LDS holds patch + 40-column hblur only: 22.3 KB, 7 workgroups per CU)
#pragma unroll
    for (int k = 0; k < (OB_PROBE == 1 ? 0 : 3); ++k) {  // OB_PROBE 1: no horizontal pass (profiling only)
      const uint32_t e = (hte >> (8 * k)) & 0xFFu;
      if (e == 0xFFu) continue;
      // e / 10 (exact for e < 256); 24-bit multiplies throughout this loop
      // (v_mul_lo_u32 / v_mad_u64_u32 are quarter rate)
      const int rp = (int)(__umul24(e, 205u) >> 11), qi = (int)e - 10 * rp;
      const int q = qlo + qi;
      // the task's hblur column base (4 qi) * KP_HSTRIDE + rp as one
      // full-rate 24-bit multiply-add (left to the compiler, the product
      // was reassociated into a quarter-rate v_mul_lo_u32)
      uint32_t hcol;
      asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(hcol) : "v"(qi), "s"(4 * KP_HSTRIDE), "v"(rp));
      const int r0 = 2 * rp, r1 = min(2 * rp + 1, KP_ROWS - 1);
      const int d0 = max(q - 1, 0);  // q == 0: the weights of dword q-1 are 0 for the columns used
      const uint32_t a0 = P[r0][d0], a1 = P[r0][q], a2 = P[r0][q + 1];
      const uint32_t b0 = P[r1][d0], b1 = P[r1][q], b2 = P[r1][q + 1];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        // taps k0..k6 at window bytes m+1..m+7 of the 12 bytes a0|a1|a2
        const uint32_t h0 = kb_hsum(m, a0, a1, a2);
        const uint32_t h1 = kb_hsum(m, b0, b1, b2);
        (&hblur[wave][0][0])[hcol + m * KP_HSTRIDE] = h0 | (h1 << 16);  // column 4 q + m - 4 qlo
      }
    }
  }
#endif
  // IC_Angle (:21-48) on the unblurred level (integer sums: order-free).
  // Lane (< 62) = patch row v = lane/2 - 15, half = lane & 1: five dwords of
  // the row (columns 4..23 or 24..43; the disk spans cc-15..cc+15 <= 39).
  // The disk's byte mask (|u| <= umax[|v|]) comes from a 20-bit column mask,
  // four bits per dword spread to bytes by a multiply; sum I and
  // sum (u + 19) I are two v_dot4_u32_u8 per dword (weights u + 19 keep every
  // byte of a touched dword in 1..37: no borrow between bytes).
  const int cc = x - px0, cr = LB ? 15 : KP_R;  // LB: the staged disk rows start at y - 15
  const int hcc = cc - 4 * ((cc - 18) >> 2);  // hblur column of the keypoint (column 4 qlo is 0)
  const int bxc = 18 * 40 + (x - me.bx0);     // LB: the keypoint's byte in the blurred patch
  int m10 = 0, m01 = 0;
  if (OB_PROBE != 2 && lane < 62) {  // OB_PROBE 2: no IC_Angle sums (profiling only)
    const int v = (lane >> 1) - 15, av = v < 0 ? -v : v;
    const uint32_t uw = (av >> 2) == 0 ? A.umaxw[0] : (av >> 2) == 1 ? A.umaxw[1]
                      : (av >> 2) == 2 ? A.umaxw[2] : A.umaxw[3];
    const int um = (int)((uw >> (8 * (av & 3))) & 0xFFu);
    const int b0 = (lane & 1) ? 24 : 4;
    const int nhi = min(max(cc + um - b0 + 1, 0), 20), nlo = min(max(cc - um - b0, 0), 20);
    const uint32_t bits = ((1u << nhi) - 1u) & ~((1u << nlo) - 1u);
    const uint32_t* rowp = &P[cr + v][b0 >> 2];
    // W = (b0 - cc + 19) * 0x01010101 + 0x03020100 (mod 2^32: byte j of W +
    // 0x04040404 k is the weight u + 19 of column b0 + j + 4 k wherever the
    // disk mask keeps it) as the lane's loop-invariant part minus the
    // keypoint's scalar cc * 0x01010101: one VALU instead of a quarter-rate
    // v_mul_lo_u32 (a byte splat of the difference is not equivalent: the
    // carries of the whole-word form matter when b0 - cc + 19 < 0)
    const uint32_t W = Wlane - (uint32_t)cc * 0x01010101u;
    uint32_t s = 0, m = 0;
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const uint32_t ones = (__umul24((bits >> (4 * k)) & 0xFu, 0x00204081u)) & 0x01010101u;
      // 0x00 / 0xFF bytes: v_perm selector 0x0C gives 0x00, 0x0D gives 0xFF
      // (ones * 255 would be a quarter-rate v_mul_lo_u32)
      const uint32_t bmask = __builtin_amdgcn_perm(0u, 0u, 0x0C0C0C0Cu + ones);
      const uint32_t I = rowp[k];
#if OB_HPASS == 1
      if constexpr (!LB) {
        // signed patch bytes p - 128: each lane's sums move by -128 n and
        // -128 sum(u + 19); after the wave sums m10 and m01 move by
        // -128 sum u and -128 sum v over the disk, both 0 (it is symmetric)
        s = (uint32_t)__builtin_amdgcn_sdot4((int)I, (int)ones, (int)s, false);
        m = (uint32_t)__builtin_amdgcn_sdot4((int)I, (int)((W + 0x04040404u * k) & bmask), (int)m, false);
        continue;
      }
#endif
      s = __builtin_amdgcn_udot4(I, ones, s, false);
      m = __builtin_amdgcn_udot4(I, (W + 0x04040404u * k) & bmask, m, false);
    }
    m10 = (int)m - __mul24(19, (int)s);
    m01 = __mul24(v, (int)s);
  }
  // wave sums (uniform: scalar angle / sincos table) without LDS round trips
  m10 = wave_sum(m10);
  m01 = wave_sum(m01);
#if OB_PROBE == 4  // profiling only: no fastAtan2 / sincos chain (wrong descriptors)
  (void)exk0, (void)exk1;
  const float angle = (float)m01 * 1e-3f;
  float sn = (float)m10 * 1e-6f, cs = 1.0f - sn;
#elif OB_PROBE == 5  // profiling only: fastAtan2 but no sincos (wrong descriptors)
  (void)exk0, (void)exk1;
  const float angle = fast_atan2((float)m01, (float)m10);
  float sn = angle * 1e-3f, cs = 1.0f - sn;
#elif !defined(OB_FULL_WAVE_CHAIN)
  // the wave-uniform fastAtan2 + double-precision sin/cos chain runs on
  // lane 0 only and is broadcast (a VALU instruction whose upper 32 lanes
  // are all inactive costs one pass of the SIMD-32 instead of two: BRIEF
  // c4 0.496 -> 0.485 ms, c1 0.910 -> 0.887, round 5); the exception lookup
  // (brief_sincos's ballot) still needs every lane
  const float factorPI = (float)(3.1415926535897932384626433832795 / 180.f);
  float angle0 = 0.f, sn0 = 0.f, cs0 = 0.f;
  if (lane == 0) {
    angle0 = fast_atan2((float)m01, (float)m10);
    orbx_sincos_core(angle0 * factorPI, &sn0, &cs0);
  }
  const float angle = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, angle0)));
  float sn = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, sn0)));
  float cs = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, cs0)));
  {
    const uint32_t b = orbx_f2u(angle * factorPI);
    const uint64_t e0 = __ballot(exk0 == b), e1 = __ballot(exk1 == b);
    if (e0 | e1) {
      const int i = e0 ? __ffsll((unsigned long long)e0) - 1 : 64 + __ffsll((unsigned long long)e1) - 1;
      sn = orbx_u2f(ORBX_SINCOS_EXC[i][1]);
      cs = orbx_u2f(ORBX_SINCOS_EXC[i][2]);
    }
  }
#else
  const float angle = fast_atan2((float)m01, (float)m10);
  const float factorPI = (float)(3.1415926535897932384626433832795 / 180.f);
  float sn, cs;
  brief_sincos(angle * factorPI, exk0, exk1, &sn, &cs);
#endif
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  uint64_t words[4] = {0, 0, 0, 0};
#pragma unroll
  for (int rr = 0; rr < (OB_PROBE == 3 ? 0 : 3); ++rr) {  // OB_PROBE 3: no samples (profiling only)
    int t[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const float fx = pfx[rr][e], fy = pfy[rr][e];
      const float ya = fy * cs, yb = fy * sn;
#ifdef OB_RINT_CVT  // A/B: rint + conversion
      const int row = (int)__builtin_rintf(__builtin_fmaf(fx, sn, ya));
      const int col = (int)__builtin_rintf(__builtin_fmaf(fx, cs, -yb));
#else
      // cvRound = rint (round half to even): for |v| < 2^22, v + 1.5 * 2^23
      // is rounded (RNE) to an integer and its bits are 0x4B400000 + rint(v)
      // -- one add instead of v_rndne + v_cvt (|v| <= 18.4 here)
      const float kM = 12582912.0f;
      const int row = __builtin_bit_cast(int, __builtin_fmaf(fx, sn, ya) + kM) - 0x4B400000;
      const int col = __builtin_bit_cast(int, __builtin_fmaf(fx, cs, -yb) + kM) - 0x4B400000;
#endif
      if constexpr (LB) {
        t[e] = Bpb[bxc + __mul24(row, 40) + col];  // |row|, |col| <= 18
        continue;
      }
      const int rt = cr + row - 3;  // first vertical tap (patch row)
      const uint32_t* hc = &hblur[wave][0][0] + (__mul24(hcc + col, KP_HSTRIDE) + (rt >> 1));  // col may be < 0
      const uint32_t v0 = hc[0], v1 = hc[1], v2 = hc[2], v3 = hc[3];
      // row pairs (2k, 2k+1): taps rt..rt+6 start at the pair's low half
      // (rt even) or high half (rt odd)
      const bool odd = rt & 1;
      // the rounding 32768 rides in as the first dot2's accumulator (-1 VALU
      // per sample); <= 255 after the shift: the taps sum to 65536
#if OB_HPASS == 1
      // i16 H - 32768 (the MFMA pass): + 32768 * 256 restores sum k_j H_j
      int acc = __builtin_amdgcn_sdot2(as_s2(v0), as_s2(odd ? KV_O0 : KV_E0), 32768 + (32768 << 8), false);
      acc = __builtin_amdgcn_sdot2(as_s2(v1), as_s2(odd ? KV_O1 : KV_E1), acc, false);
      acc = __builtin_amdgcn_sdot2(as_s2(v2), as_s2(odd ? KV_O2 : KV_E2), acc, false);
      acc = __builtin_amdgcn_sdot2(as_s2(v3), as_s2(odd ? KV_O3 : KV_E3), acc, false);
      t[e] = (int)((uint32_t)acc >> 16);
#else
      uint32_t acc = __builtin_amdgcn_udot2(as_us2(v0), as_us2(odd ? KV_O0 : KV_E0), 32768u, false);
      acc = __builtin_amdgcn_udot2(as_us2(v1), as_us2(odd ? KV_O1 : KV_E1), acc, false);
      acc = __builtin_amdgcn_udot2(as_us2(v2), as_us2(odd ? KV_O2 : KV_E2), acc, false);
      acc = __builtin_amdgcn_udot2(as_us2(v3), as_us2(odd ? KV_O3 : KV_E3), acc, false);
      t[e] = (int)(acc >> 16);
#endif
    }
    words[rr] = __ballot(t[0] < t[1]);
  }
#ifdef OB_PROBE_NOSTORE  // profiling only: the outputs' stores never issue (wrong results)
  if (dbg == 0x5EED)
#endif
  if (lane < 4) {
    const uint64_t w = lane == 0 ? words[0] : lane == 1 ? words[1] : lane == 2 ? words[2] : words[3];
    reinterpret_cast<uint64_t*>(descf + (uint32_t)me.oi * 32u)[lane] = w;
  }
#ifdef OB_PROBE_NOSTORE
  if (dbg == 0x5EED)
#endif
  if (lane == 0) {
    orbx_keypoint kp;
    kp.x = (float)x;
    kp.y = (float)me.y;
    if (l != 0) {
      kp.x *= me.scale;
      kp.y *= me.scale;
    }
    kp.size = (float)me.patch_size;
    kp.angle = angle;
    kp.response = (float)score;
    kp.octave = l;
    kp.class_id = -1;
    *reinterpret_cast<orbx_keypoint*>(reinterpret_cast<uint8_t*>(kpsf) + (uint32_t)me.oi * (uint32_t)sizeof(orbx_keypoint)) = kp;
  }
  }
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OB_WPE))) void k_orient_brief(OB_KERNEL_ARGS) {
  ob_body<false>(OB_KERNEL_PASS, nullptr, 0);
}
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OB_WPE))) void k_orient_brief_lb(
    OB_KERNEL_ARGS, const uint8_t* __restrict__ blur, size_t bstride) {
  ob_body<true>(OB_KERNEL_PASS, blur, bstride);
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

#define ORBX_PAN_CLIP 16
#define ORBX_PAN_STEP 2
__global__ __launch_bounds__(256) void k_synth(uint8_t* __restrict__ frames, int W, int H,
                                               size_t fstride, int first_idx, int kind) {
  __shared__ int rect[96][5];
  const int f = blockIdx.y, tid = threadIdx.x;
  const int fidx = first_idx + f;
  const uint64_t seed = 0x5EED0000ull + (uint64_t)fidx;
  // kind 3 (pan): the rectangles of the clip's first frame (clips of
  // ORBX_PAN_CLIP frames) shifted right by ORBX_PAN_STEP px per frame
  const int phase = kind == 3 ? fidx % ORBX_PAN_CLIP : 0;
  const uint64_t rseed = seed - (uint64_t)phase;
  const int shift = ORBX_PAN_STEP * phase;
  if (kind == 0 || kind == 3) {
    for (int i = tid; i < 96 * 5; i += 256) {
      const uint64_t v = sm_at(rseed, (uint64_t)i);
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
        const int xa = min(rect[r][0], rect[r][1]) + shift, xb = max(rect[r][0], rect[r][1]) + shift;
        const int ya = min(rect[r][2], rect[r][3]), yb = max(rect[r][2], rect[r][3]);
        if (x >= xa && x <= xb && y >= ya && y <= yb) v = rect[r][4];
      }
      v += (int)(sm_at(seed, 480ull + (uint64_t)p) % 13ull) - 6;
      v = min(max(v, 0), 255);
    }
    out[(size_t)y * W + x] = (uint8_t)v;
  }
}

// ---------------------------------------------------------------------------
// k_selftest_sincos: brief_sincos exactly as k_orient_brief runs it (one
// wave per input, exception keys in two VGPRs per lane); orbx_selftest_sincos.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void k_selftest_sincos(const float* __restrict__ x, int n,
                                                        float* __restrict__ sc) {
  const int lane = threadIdx.x, i = blockIdx.x;
  if (i >= n) return;
  const uint32_t exk0 = ORBX_SINCOS_EXC[lane < ORBX_SINCOS_NEXC ? lane : 0][0];
  const uint32_t exk1 = lane + 64 < ORBX_SINCOS_NEXC ? ORBX_SINCOS_EXC[lane + 64][0] : 0xFFFFFFFFu;
  float s, c;  // x[i] is wave-uniform, as the BRIEF angle is
  brief_sincos(__uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(x[i]))), exk0, exk1, &s, &c);
  if (lane == 0) {
    sc[2 * i] = s;
    sc[2 * i + 1] = c;
  }
}

// k_selftest_sincos_range: the BRIEF sin/cos of consecutive float bit
// patterns, lane-parallel (orbx_sincos_core + the exception table, looked up
// by binary search -- the same table brief_sincos consults by ballot), for
// the exhaustive device check over every reachable angle
// (tests/test_sincos_gpu.py::test_device_sincos_exhaustive).
__global__ __launch_bounds__(256) void k_selftest_sincos_range(uint32_t first, int n,
                                                               float* __restrict__ sc) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint32_t b = first + (uint32_t)i;
  float s, c;
  orbx_sincos_core(orbx_u2f(b), &s, &c);
  int lo = 0, hi = ORBX_SINCOS_NEXC;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (ORBX_SINCOS_EXC[mid][0] < b) lo = mid + 1; else hi = mid;
  }
  if (lo < ORBX_SINCOS_NEXC && ORBX_SINCOS_EXC[lo][0] == b) {
    s = orbx_u2f(ORBX_SINCOS_EXC[lo][1]);
    c = orbx_u2f(ORBX_SINCOS_EXC[lo][2]);
  }
  reinterpret_cast<float2*>(sc)[i] = make_float2(s, c);
}

}  // namespace orbx

