// kernels_stream.hip -- row-streaming pyramid (ComputePyramid,
// src/ORBextractor.cc:497-515, cv::resize INTER_LINEAR) for batches of
// frames on gfx950.
//
// One workgroup per frame walks it top to bottom in ticks (planner:
// geometry.cpp plan_pyr_stream, layout: orbx_internal.h PyrStream):
//  * wave 0 is the loader: in tick k it brings level-0 rows [r0 k, r0 (k+1))
//    into level 0's LDS ring (plain loads, then ds_write);
//  * the other waves are workers: they take the tick's tasks in order by an
//    LDS ticket (a wave that draws a ticket of a later tick keeps it for that
//    tick) -- a task is (level j, chunk of 64 four-pixel groups, run of
//    destination rows) and computes those rows from level j-1's ring rows,
//    which earlier ticks wrote, into level j's ring and to HBM;
//  * one barrier per tick (LDS only: s_waitcnt lgkmcnt(0) + s_barrier).
// Every level pixel is computed once (the tile kernel recomputes 13.5 % of
// them in its halos), there is no per-level barrier, and a source row's
// horizontal pass is reused by consecutive destination rows of a task.
// Arithmetic: OpenCV 3.4 HResizeLinear / VResizeLinear<uchar> fixed point,
// the same instruction forms as k_pyramid (kernels_extract.hip):
//   D = S[sx]*a0 + S[sx1]*a1 (v_perm + v_dot2_u32_u16),
//   dst = (((b0*(D0>>4))>>16) + ((b1*(D1>>4))>>16) + 2) >> 2
// with ((b*(D>>4))>>16) == mulhi_u24(b << 12, D & ~15).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/orbx.h"
#include "fast_ops.h"
#include "orbx_internal.h"
#include "wave_ops.h"

namespace orbx {

typedef uint32_t ps_v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ us2 ps_as_us2(uint32_t x) { return as_us2(x); }

// tick barrier: this wave's LDS writes are done, then the workgroup barrier
// (no vmcnt wait: the level rows' HBM stores stay in flight across ticks)
__device__ __forceinline__ void ps_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// (b << 12) * (D & ~15) >> 32 for operands < 2^24: one v_mul_hi_u32_u24 (the
// compiler picks the quarter-rate v_mul_hi_u32 for the 64-bit form here)
__device__ __forceinline__ uint32_t ps_mulhi24(uint32_t bs, uint32_t d) {
  uint32_t r;
  asm("v_mul_hi_u32_u24 %0, %1, %2" : "=v"(r) : "s"(bs), "v"(d));
  return r;
}

__device__ __forceinline__ uint32_t ps_ld32u(const uint8_t* p) {
  uint32_t w;
  __builtin_memcpy(&w, p, 4);
  return w;
}

// horizontal pass of one source row for the lane's 4 destination columns:
// their source bytes lie in the 8-byte window at hbase + hsh (planner check)
__device__ __forceinline__ void ps_hpass(const uint8_t* row, int hsh, const uint32_t (&hsel)[4],
                                         const uint32_t (&hcoef)[4], uint32_t (&H)[4]) {
  const uint32_t* R = reinterpret_cast<const uint32_t*>(row);
  const uint32_t lo = __builtin_amdgcn_alignbyte(R[1], R[0], hsh);
  const uint32_t hi = __builtin_amdgcn_alignbyte(R[2], R[1], hsh);
#pragma unroll
  for (int k = 0; k < 4; ++k)
    H[k] = __builtin_amdgcn_udot2(ps_as_us2(__builtin_amdgcn_perm(hi, lo, hsel[k])), ps_as_us2(hcoef[k]), 0u,
                                  false) &
           0xFFFFF0u;
}

#define PS_LOAD_U 8 /* loader: loads in flight per lane */

#ifndef PS_PROBE  // profiling builds only (tools/variant.sh): 1 = the loader skips its loads
#define PS_PROBE 0
#endif
#ifndef PF_PROBE  // profiling builds only: skip 1 NMS, 2 FASTA, 4 resize, 8 stage C, 16 loads
#define PF_PROBE 0
#endif

template <int NT>
__device__ __forceinline__ void ps_loader(const uint8_t* __restrict__ src, size_t rstride, const PyrStream& S,
                                          uint8_t* __restrict__ lds, int lane, int aligned16) {
  const int W0 = S.w[0], H0 = S.h[0];
  uint8_t* ring = lds + S.roff[0];
  const int rp = S.rpitch[0], rr = S.rrows[0];
  const uint32_t rs = (uint32_t)rstride;
  for (int k = 0; k < S.nticks; ++k) {
    const int a = min(H0, S.r0 * k), b = PS_PROBE & 1 ? a : min(H0, S.r0 * (k + 1));
    if (aligned16) {
      const int nu = (W0 + 15) >> 4, total = (b - a) * nu;
      for (int i0 = 0; i0 < total; i0 += 64 * PS_LOAD_U) {
        ps_v4u v[PS_LOAD_U];
        int rr_[PS_LOAD_U], cc_[PS_LOAD_U];
#pragma unroll
        for (int u = 0; u < PS_LOAD_U; ++u) {
          const int idx = min(i0 + lane + 64 * u, total - 1);  // unconditional load, clamped index
          const int r = idx / nu, c = idx - r * nu;
          rr_[u] = r;
          cc_[u] = c;
          v[u] = *reinterpret_cast<const ps_v4u*>(src + ((size_t)(a + r) * rs + 16u * (uint32_t)c));
        }
#pragma unroll
        for (int u = 0; u < PS_LOAD_U; ++u)
          if (i0 + lane + 64 * u < total)
            *reinterpret_cast<ps_v4u*>(ring + ((a + rr_[u]) % rr) * rp + 16 * cc_[u]) = v[u];
      }
    } else {
      // dword units at any byte alignment; a row's last dword is loaded
      // ending at the row's last byte and shifted (nothing past the row read)
      const int nu = (W0 + 3) >> 2, total = (b - a) * nu;
      for (int i0 = 0; i0 < total; i0 += 64 * PS_LOAD_U) {
        uint32_t v[PS_LOAD_U];
        int rr_[PS_LOAD_U], cc_[PS_LOAD_U];
#pragma unroll
        for (int u = 0; u < PS_LOAD_U; ++u) {
          const int idx = min(i0 + lane + 64 * u, total - 1);
          const int r = idx / nu, c = idx - r * nu;
          rr_[u] = r;
          cc_[u] = c;
          const int cb = 4 * c, cl = min(cb, W0 - 4);
          v[u] = ps_ld32u(src + ((size_t)(a + r) * rs + (uint32_t)cl)) >> (8 * (cb - cl));
        }
#pragma unroll
        for (int u = 0; u < PS_LOAD_U; ++u)
          if (i0 + lane + 64 * u < total)
            *reinterpret_cast<uint32_t*>(ring + ((a + rr_[u]) % rr) * rp + 4 * cc_[u]) = v[u];
      }
    }
    ps_barrier();
  }
}

// one task: destination rows [y0, y0 + nr) of chain level j, groups
// [64 c, 64 c + 64) (lanes past the row repeat its last group, no stores)
__device__ __forceinline__ void ps_resize(const PyrStream& S, uint8_t* __restrict__ lds, uint8_t* __restrict__ fpyr,
                                          const uint2* __restrict__ ylut, uint32_t x, int y0, int lane) {
  const int j = (int)((x >> 4) & 31), c = (int)((x >> 9) & 127), nr = (int)((x >> 16) & 255);
  const int ng = S.ng[j];
  const int g = c * 64 + lane;
  const bool act = g < ng;
  const int gg = act ? g : ng - 1;
  // column LUT (build_blobs layout): column 0 holds s0 | (sx1 - s0) << 16,
  // columns 1..3 their v_perm selectors relative to s0; .y = a0 | a1 << 16
  const uint4* xl = reinterpret_cast<const uint4*>(lds + S.lut_lds) + (S.xl[j] >> 1) + 2 * gg;
  const uint4 q0 = xl[0], q1 = xl[1];
  const int s0 = (int)(q0.x & 0xFFFFu);
  const int hsh = s0 & 3;
  uint32_t hsel[4], hcoef[4];
  hsel[0] = (q0.x & 0xFFFF0000u) | 0x0C000C00u;
  hcoef[0] = q0.y;
  hsel[1] = q0.z;
  hcoef[1] = q0.w;
  hsel[2] = q1.x;
  hcoef[2] = q1.y;
  hsel[3] = q1.z;
  hcoef[3] = q1.w;
  const uint8_t* sring = lds + S.roff[j - 1] + (s0 & ~3);
  const int srp = S.rpitch[j - 1];
  uint8_t* dring = lds + S.roff[j] + 4 * gg;
  const int drp = S.rpitch[j];
  // HBM rows through a buffer resource: the row offset in an SGPR (soffset),
  // the lane's dword in a VGPR (no 64-bit address arithmetic per row)
  const __amdgpu_buffer_rsrc_t gres = __builtin_amdgcn_make_buffer_rsrc(fpyr + S.goff[j], (short)0, -1, 0x00020000);
  const int gp = S.gpitch[j];
  const uint2* yl = ylut + S.yl[j] + y0;
  int last = -1;  // ring slot whose horizontal pass Hp holds
  uint32_t Hp[4] = {0u, 0u, 0u, 0u};
  for (int r = 0; r < nr; ++r) {  // wave-uniform
    const uint2 e = yl[r];
    const int sa = (int)(e.x & 0xFF), sb = (int)((e.x >> 8) & 0xFF), sd = (int)((e.x >> 16) & 0xFF);
    uint32_t Ha[4], Hb[4];
    if (sa == last) {
#pragma unroll
      for (int k = 0; k < 4; ++k) Ha[k] = Hp[k];
    } else {
      ps_hpass(sring + sa * srp, hsh, hsel, hcoef, Ha);
    }
    if (sb == sa) {
#pragma unroll
      for (int k = 0; k < 4; ++k) Hb[k] = Ha[k];
    } else {
      ps_hpass(sring + sb * srp, hsh, hsel, hcoef, Hb);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) Hp[k] = Hb[k];
    last = sb;
    const uint32_t b0s = (e.y & 0xFFFu) << 12, b1s = ((e.y >> 16) & 0xFFFu) << 12;
    uint32_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = (ps_mulhi24(b0s, Ha[k]) + ps_mulhi24(b1s, Hb[k]) + 2u) >> 2;
    const uint32_t packed =
        __builtin_amdgcn_perm(v[1], v[0], 0x0C0C0400u) | __builtin_amdgcn_perm(v[3], v[2], 0x04000C0Cu);
    if (act) {
      *reinterpret_cast<uint32_t*>(dring + sd * drp) = packed;
      // the whole group (bytes past the level's last column land in the row
      // padding: level pitches are 16-B multiples)
      __builtin_amdgcn_raw_buffer_store_b32(packed, gres, 4 * gg, (y0 + r) * gp, 0);
    }
  }
}

template <int NT>
__device__ __forceinline__ void ps_body(const uint8_t* __restrict__ frames, size_t fstride, size_t rstride,
                                        uint8_t* __restrict__ pyr, size_t pstride, const PyrStream& S,
                                        const uint2* __restrict__ tasks, const int* __restrict__ tick_end,
                                        const uint4* __restrict__ xlut, const uint2* __restrict__ ylut,
                                        int aligned16) {
  extern __shared__ __align__(16) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int f = blockIdx.x;
  int* ticket = reinterpret_cast<int*>(lds + S.lds_bytes - 16);
  for (int i = tid; i < (S.lut_bytes >> 4); i += NT) reinterpret_cast<uint4*>(lds + S.lut_lds)[i] = xlut[i];
  if (tid == 0) *ticket = 0;
  __syncthreads();
  if (wave == 0) {
    ps_loader<NT>(frames + (size_t)f * fstride, rstride, S, lds, lane, aligned16);
    return;
  }
  uint8_t* fpyr = pyr + (size_t)f * pstride;
  int pending = -1;  // a ticket drawn past its tick's end, kept for a later tick
  for (int k = 0; k < S.nticks; ++k) {
    const int tend = tick_end[k];
    for (;;) {
      int t = pending;
      if (t < 0) {
        int v = 0;
        if (lane == 0) v = atomicAdd(ticket, 1);
        t = __builtin_amdgcn_readfirstlane(v);
      }
      if (t >= tend) {
        pending = t;
        break;
      }
      pending = -1;
      const uint2 d = tasks[t];
      ps_resize(S, lds, fpyr, ylut, d.x, (int)d.y, lane);
    }
    ps_barrier();
  }
}

#define PS_KERNEL_ARGS                                                                                   \
  const uint8_t *__restrict__ frames, size_t fstride, size_t rstride, uint8_t *__restrict__ pyr,       \
      size_t pstride, const PyrStream S, const uint2 *__restrict__ tasks, const int *__restrict__ tick_end, \
      const uint4 *__restrict__ xlut, const uint2 *__restrict__ ylut, int aligned16
#define PS_KERNEL_PASS frames, fstride, rstride, pyr, pstride, S, tasks, tick_end, xlut, ylut, aligned16

__global__ __launch_bounds__(1024) void k_pyr_stream_1024(PS_KERNEL_ARGS) { ps_body<1024>(PS_KERNEL_PASS); }
__global__ __launch_bounds__(512) void k_pyr_stream_512(PS_KERNEL_ARGS) { ps_body<512>(PS_KERNEL_PASS); }
__global__ __launch_bounds__(256) void k_pyr_stream_256(PS_KERNEL_ARGS) { ps_body<256>(PS_KERNEL_PASS); }


// ===========================================================================
// k_pyrfast: the pyramid and cell FAST in one streaming pass per level
// (ORBextractor.cc:497-515 ComputePyramid, :316-340 the cell loop with
// cv::FAST, cornerScore<16>, NMS and the minThFAST retry).  Planner:
// geometry.cpp plan_pyr_fast; layout: orbx_internal.h PyrFast.
//
// One workgroup per frame; wave 0 loads, waves 1.. work.  Pass p streams its
// source level through the level ring; each tick:
//  phase 1 (tasks by ticket, largest first):
//    * FASTA (rows, chunk of 62 groups): the cardinal test over ring rows in
//      a column walk (a lane's rows in registers, neighbours by DPP), the
//      strength row zero-filled, survivors appended to the wave's list L1;
//      every 64 entries the even-point test (stage B) appends its survivors
//      to the workgroup's list L2;
//    * RESIZE (rows, chunk) of the next level from two ring rows, to HBM;
//    * NMS (rows): one wave walks finished detection rows in order: the
//      row's corners from its bitmap in raster order, cv::FAST's strict 3x3
//      test within the cell's zone at iniThFAST and minThFAST, keys to the
//      cell's lists (slots: minThFAST set, slots_hi: iniThFAST set); at a
//      cell row's end the counts (ORBX_CC_HI: the cell keeps its iniThFAST
//      keys, else its minThFAST keys -- ORBextractor.cc:330-331);
//  phase 2: the full 16-point strength (stage C) of L2's entries, 64 per
//    ticket, into the strength ring and the corner bitmap.
// The level ring keeps 3 guard rows on each side (a row whose slot is within
// 3 of either end is also written past that end), so the 7-row window of any
// pixel is contiguous for stages B and C.
// ===========================================================================
struct PfLds {
  uint8_t* ring;      // level ring (rrows + 6 physical rows)
  uint8_t* aring;     // strength ring (arows rows)
  uint32_t* bmap;     // corner bitmaps (arows rows of bmw words)
  const uint4* lut;   // next level's column LUT, 2 x uint4 per group
  int* cellsoff;      // slot offsets of this level's cells
  int* cnt;           // minThFAST counts [0, ncv_max), iniThFAST counts [ncv_max, 2 ncv_max)
  uint32_t* l1;       // per-wave lists
  uint32_t* l2;       // even-test survivors of the tick
  uint16_t* nms;      // corner x list of the NMS wave
  int* misc;          // [0] task ticket, [1..2] L2 count, [3..4] stage-C ticket (tick parity)
};

__device__ __forceinline__ int pf_wrap_inc(int s, int n) { return s + 1 == n ? 0 : s + 1; }

// entries: col (bits 0-12) | physical ring row of the pixel (13-20) | strength ring row (21-28)
__device__ __forceinline__ void pf_stage_c(const PyrFastPass& Q, const PfLds& L, uint32_t e, bool act, int t_lo) {
  if (act) {
    const int col = (int)(e & 0x1FFFu), rp = (int)((e >> 13) & 0xFFu), as = (int)((e >> 21) & 0xFFu);
    const int a = fast_strength(L.ring + rp * Q.rpitch + col, Q.rpitch);
    if (a > t_lo) {
      L.aring[as * Q.rpitch + col] = (uint8_t)a;
      atomicOr(&L.bmap[as * Q.bmw + (col >> 5)], 1u << (col & 31));
    }
  }
}

__device__ __forceinline__ void pf_stage_b(const PyrFastPass& Q, const PfLds& L, uint32_t e, bool act, int t_lo,
                                           int lane, int par) {
  const int col = (int)(e & 0x1FFFu), rp = (int)((e >> 13) & 0xFFu);
  const bool keep = act && col >= Q.c0 && col < Q.c1 && fast_even_test_pk(L.ring + rp * Q.rpitch + col, Q.rpitch, t_lo);
  const unsigned long long bal = __ballot(keep);
  if (bal) {  // wave-uniform
    int base = 0;
    if (lane == 0) base = atomicAdd(&L.misc[1 + par], __popcll(bal));
    base = __builtin_amdgcn_readfirstlane(base);
    const int pos = base + lanes_below(bal);
    if (keep && pos < ORBX_PF_L2CAP) L.l2[pos] = e;
    // list full: this wave computes the strength now (phase 1 writes only
    // rows of this tick's detection rows, which no NMS of this tick reads)
    pf_stage_c(Q, L, e, keep && pos >= ORBX_PF_L2CAP, t_lo);
  }
}

#define PF_CW_RMAX 8 /* stage-A rows per task (registers hold PF_CW_RMAX + 6 ring rows) */

__device__ __forceinline__ void pf_fasta(const PyrFastPass& Q, const PfLds& L, uint32_t x, uint32_t yw, int lane,
                                         uint32_t* __restrict__ L1, int& n1, int t_lo, int par) {
  const int c = (int)((x >> 9) & 127), nr = (int)((x >> 16) & 255);
  const int ya = (int)(yw & 0x3FFFu);
  int sl = (int)((yw >> 14) & 0xFFu);  // logical ring slot of row ya - 3
  int as = (int)((yw >> 22) & 0xFFu);  // strength ring row of row ya
  const int g = Q.gs + 62 * c + lane - 1;
  const int gl = (Q.c1 - 1) >> 2;
  const bool lact = lane >= 1 && lane <= 62 && g <= gl;
  const int gc = min(max(g, 0), (Q.w - 1) >> 2);
  const uint32_t tt = (uint32_t)t_lo * 0x00010001u;
  const uint32_t tl = lact ? tt : 0xFF00FF00u;
  uint32_t V[PF_CW_RMAX + 6];
  int ph[PF_CW_RMAX + 6];  // physical ring rows (wave-uniform)
#pragma unroll
  for (int k = 0; k < PF_CW_RMAX + 6; ++k) {
    ph[k] = sl + 3;
    if (k < nr + 6) V[k] = *reinterpret_cast<const uint32_t*>(L.ring + ph[k] * Q.rpitch + 4 * gc);
    sl = pf_wrap_inc(sl, Q.rrows);
  }
  (void)ya;
#pragma unroll
  for (int k = 0; k < PF_CW_RMAX; ++k) {
    if (k < nr) {  // wave-uniform
      GroupWords q;
      q.up = V[k];
      q.w1 = V[k + 3];
      q.dn = V[k + 6];
      q.w0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)V[k + 3], 0x138, 0xf, 0xf, false);  // wave_shr:1
      q.w2 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)V[k + 3], 0x130, 0xf, 0xf, false);  // wave_shl:1
      uint32_t clo, chi;
      fast_cardinal(q, tl, clo, chi);
      if (lact) *reinterpret_cast<uint32_t*>(L.aring + as * Q.rpitch + 4 * g) = 0u;
      const uint32_t eb = (uint32_t)(4 * g) | ((uint32_t)ph[k + 3] << 13) | ((uint32_t)as << 21);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t xx = (j & 1) ? chi : clo;
        const bool kk = ((j & 2) ? (xx >> 16) : (xx & 0xFFFFu)) != 0;
        const unsigned long long bal = __ballot(kk);
        const int pos = lanes_below(bal);
        uint32_t* const L1n = L1 + __builtin_amdgcn_readfirstlane(n1);
        if (kk) L1n[pos] = eb + (uint32_t)j;
        n1 += __popcll(bal);
      }
      if (n1 >= 64) {  // wave-uniform
        wave_sync_lds();
        while (n1 >= 64) {
          n1 -= 64;
          pf_stage_b(Q, L, L1[n1 + lane], true, t_lo, lane, par);
        }
        wave_sync_lds();
      }
      as = pf_wrap_inc(as, Q.arows);
    }
  }
}

// next level rows [y0, y0 + nr), groups [64 c, 64 c + 64), from the ring to HBM
__device__ __forceinline__ void pf_resize(const PyrFastPass& Q, const PfLds& L, uint8_t* __restrict__ fpyr,
                                          const uint2* __restrict__ ylut, uint32_t x, int y0, int lane) {
  const int c = (int)((x >> 9) & 127), nr = (int)((x >> 16) & 255);
  const int g = c * 64 + lane;
  const bool act = g < Q.ng;
  const int gg = act ? g : Q.ng - 1;
  const uint4 q0 = L.lut[2 * gg], q1 = L.lut[2 * gg + 1];
  const int s0 = (int)(q0.x & 0xFFFFu);
  const int hsh = s0 & 3;
  uint32_t hsel[4], hcoef[4];
  hsel[0] = (q0.x & 0xFFFF0000u) | 0x0C000C00u;
  hcoef[0] = q0.y;
  hsel[1] = q0.z;
  hcoef[1] = q0.w;
  hsel[2] = q1.x;
  hcoef[2] = q1.y;
  hsel[3] = q1.z;
  hcoef[3] = q1.w;
  const uint8_t* sring = L.ring + 3 * Q.rpitch + (s0 & ~3);
  const int srp = Q.rpitch;
  const __amdgpu_buffer_rsrc_t gres = __builtin_amdgcn_make_buffer_rsrc(fpyr + Q.noff, (short)0, -1, 0x00020000);
  const uint2* yl = ylut + Q.yl + y0;
  int last = -1;
  uint32_t Hp[4] = {0u, 0u, 0u, 0u};
  for (int r = 0; r < nr; ++r) {
    const uint2 e = yl[r];
    const int sa = (int)(e.x & 0xFF), sb = (int)((e.x >> 8) & 0xFF);
    uint32_t Ha[4], Hb[4];
    if (sa == last) {
#pragma unroll
      for (int k = 0; k < 4; ++k) Ha[k] = Hp[k];
    } else {
      ps_hpass(sring + sa * srp, hsh, hsel, hcoef, Ha);
    }
    if (sb == sa) {
#pragma unroll
      for (int k = 0; k < 4; ++k) Hb[k] = Ha[k];
    } else {
      ps_hpass(sring + sb * srp, hsh, hsel, hcoef, Hb);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) Hp[k] = Hb[k];
    last = sb;
    const uint32_t b0s = (e.y & 0xFFFu) << 12, b1s = ((e.y >> 16) & 0xFFFu) << 12;
    uint32_t v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = (ps_mulhi24(b0s, Ha[k]) + ps_mulhi24(b1s, Hb[k]) + 2u) >> 2;
    const uint32_t packed =
        __builtin_amdgcn_perm(v[1], v[0], 0x0C0C0400u) | __builtin_amdgcn_perm(v[3], v[2], 0x04000C0Cu);
    if (act) __builtin_amdgcn_raw_buffer_store_b32(packed, gres, 4 * gg, (y0 + r) * Q.npitch, 0);
  }
}

// NMS + emit of detection rows [y0, y0 + nr) in order (one wave), for the
// cells of columns [jc0, jc1) (half 0: [0, ncv/2), half 1: [ncv/2, ncv); the
// two halves run side by side on two waves)
__device__ __forceinline__ void pf_nms(const PyrFast& F, const PyrFastPass& Q, const PfLds& L,
                                       uint32_t* __restrict__ fslots, uint32_t* __restrict__ fslots_hi,
                                       uint32_t* __restrict__ fccount, int y0, int nr, int as, int half,
                                       int lane) {
  const int ini = F.ini_th, mn = F.min_th;
  const float rw = __builtin_amdgcn_rcpf((float)Q.wcell);
  const int jc0 = half ? Q.ncv >> 1 : 0, jc1 = (half || Q.ncv == 1) ? Q.ncv : Q.ncv >> 1;
  const int xa = Q.c0 + jc0 * Q.wcell, xb = jc1 == Q.ncv ? Q.c1 : Q.c0 + jc1 * Q.wcell;
  const int wlo = xa >> 5, whi = (xb - 1) >> 5;  // bitmap words touching [xa, xb)
  uint16_t* const cl = L.nms + half * F.nms_cap;
  int ci = (y0 - Q.y0) / Q.hcell;
  int zy0 = Q.y0 + ci * Q.hcell, zy1 = ci == Q.nrv - 1 ? Q.y1 : zy0 + Q.hcell;
  const unsigned long long below = (1ull << lane) - 1ull;
  for (int r = 0; r < nr; ++r) {
    const int y = y0 + r;
    const int asm1 = as == 0 ? Q.arows - 1 : as - 1, asp1 = pf_wrap_inc(as, Q.arows);
    // the row's corners in raster order (bitmap words, cleared for the slot's next row)
    int nc = 0;
    for (int w0 = wlo; w0 <= whi; w0 += 64) {
      const int wi = w0 + lane;
      uint32_t m = 0;
      if (wi <= whi) {
        // this half's bits of the word; a word shared with the other half
        // loses only this half's bits (atomic and), an own word is cleared
        const int b0 = max(xa - 32 * wi, 0), b1 = min(xb - 32 * wi, 32);
        const uint32_t own = (b1 >= 32 ? 0xFFFFFFFFu : ((1u << b1) - 1u)) & ~((1u << b0) - 1u);
        uint32_t* wp = &L.bmap[as * Q.bmw + wi];
        m = *wp & own;
        if (own == 0xFFFFFFFFu) *wp = 0u;
        else atomicAnd(wp, ~own);
      }
      const int cn = __popc(m);
      const int incl = wave_incl_scan(cn);
      int off = nc + incl - cn;
      while (m) {
        const int b = __ffs((int)m) - 1;
        m &= m - 1u;
        cl[off++] = (uint16_t)(32 * wi + b);
      }
      nc += lane_value(incl, 63);
    }
    wave_sync_lds();
    const uint8_t* A0 = L.aring + as * Q.rpitch;
    const uint8_t* Am = L.aring + asm1 * Q.rpitch;
    const uint8_t* Ap = L.aring + asp1 * Q.rpitch;
    const bool up_in = y - 1 >= zy0, dn_in = y + 1 < zy1;
    const int crow = ci * Q.ncv;
    for (int q0 = 0; q0 < nc; q0 += 64) {  // wave-uniform
      const bool act = q0 + lane < nc;
      const int xx = act ? (int)cl[q0 + lane] : xa;
      const int jc = min((int)(((float)(xx - Q.c0) + 0.5f) * rw), Q.ncv - 1);
      const int zx0 = Q.c0 + jc * Q.wcell, zx1 = jc == Q.ncv - 1 ? Q.c1 : zx0 + Q.wcell;
      const int a = A0[xx];
      int nbi = 0, nbm = 0;
#pragma unroll
      for (int dy = -1; dy <= 1; ++dy)
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx) {
          if (!dx && !dy) continue;
          const uint8_t* row = dy < 0 ? Am : dy > 0 ? Ap : A0;
          const bool rin = dy < 0 ? up_in : dy > 0 ? dn_in : true;
          const int cc = xx + dx;
          const int aq = (rin && cc >= zx0 && cc < zx1) ? (int)row[cc] : 0;
          nbm = max(nbm, aq > mn ? aq - 1 : 0);
          nbi = max(nbi, aq > ini ? aq - 1 : 0);
        }
      const bool lo = act && a > mn && a - 1 > nbm;
      const bool hi = act && a > ini && a - 1 > nbi;
      const uint32_t key = orbx_pack_key((uint32_t)(xx - 16), (uint32_t)(y - 16), (uint32_t)a - 1u, F.key_xs);
      // lanes of one cell are consecutive (corners in raster order): a key's
      // position = the cell's count so far + the flagged lanes of its run
      // before it
      const int pj = __builtin_amdgcn_update_dpp(-1, jc, 0x138, 0xf, 0xf, false);  // wave_shr:1
      const unsigned long long sm = __ballot(lane == 0 || pj != jc);
      const int start = 63 - (int)__clzll(sm & (below | (1ull << lane)));
      const unsigned long long before = (1ull << start) - 1ull;
      const unsigned long long mlo = __ballot(lo), mhi = __ballot(hi);
      const int so = L.cellsoff[crow + jc];
      if (lo) {
        const int pos = L.cnt[jc] + __popcll(mlo & below) - __popcll(mlo & before);
        fslots[so + pos] = key;
      }
      if (hi) {
        const int pos = L.cnt[F.ncv_max + jc] + __popcll(mhi & below) - __popcll(mhi & before);
        fslots_hi[so + pos] = key;
      }
      if (lo) atomicAdd(&L.cnt[jc], 1);
      if (hi) atomicAdd(&L.cnt[F.ncv_max + jc], 1);
      wave_sync_lds();
    }
    if (y == zy1 - 1) {  // the cell row is complete
      for (int jc = jc0 + lane; jc < jc1; jc += 64) {
        const int clo = L.cnt[jc], chi = L.cnt[F.ncv_max + jc];
        fccount[Q.cell_begin + crow + jc] = chi > 0 ? ((uint32_t)chi | ORBX_CC_HI) : (uint32_t)clo;
        L.cnt[jc] = 0;
        L.cnt[F.ncv_max + jc] = 0;
      }
      wave_sync_lds();
      ++ci;
      zy0 = zy1;
      zy1 = ci == Q.nrv - 1 ? Q.y1 : zy0 + Q.hcell;
    }
    as = asp1;
  }
}

// loader: source rows [a, b) of pass Q into the ring (guard copies included)
__device__ __forceinline__ void pf_load(const PyrFastPass& Q, const uint8_t* __restrict__ src, uint32_t sp,
                                        uint8_t* __restrict__ ring, int a, int b, int lane, bool al16) {
  const int W = Q.w, rp = Q.rpitch, rr = Q.rrows;
  auto put = [&](int y, int cb, const uint8_t* vp, int nbytes) {
    const int s = y % rr;
    uint8_t* d0 = ring + (s + 3) * rp + cb;
    if (nbytes == 16) *reinterpret_cast<ps_v4u*>(d0) = *reinterpret_cast<const ps_v4u*>(vp);
    else *reinterpret_cast<uint32_t*>(d0) = *reinterpret_cast<const uint32_t*>(vp);
    if (s < 3 || s >= rr - 3) {
      uint8_t* d1 = ring + (s < 3 ? s + 3 + rr : s + 3 - rr) * rp + cb;
      if (nbytes == 16) *reinterpret_cast<ps_v4u*>(d1) = *reinterpret_cast<const ps_v4u*>(vp);
      else *reinterpret_cast<uint32_t*>(d1) = *reinterpret_cast<const uint32_t*>(vp);
    }
  };
  if (al16) {
    const int nu = (W + 15) >> 4, total = (b - a) * nu;
    for (int i0 = 0; i0 < total; i0 += 64 * PS_LOAD_U) {
      ps_v4u v[PS_LOAD_U];
      int rr_[PS_LOAD_U], cc_[PS_LOAD_U];
#pragma unroll
      for (int u = 0; u < PS_LOAD_U; ++u) {
        const int idx = min(i0 + lane + 64 * u, total - 1);
        const int r = idx / nu, cu = idx - r * nu;
        rr_[u] = r;
        cc_[u] = cu;
        v[u] = *reinterpret_cast<const ps_v4u*>(src + ((size_t)(a + r) * sp + 16u * (uint32_t)cu));
      }
#pragma unroll
      for (int u = 0; u < PS_LOAD_U; ++u)
        if (i0 + lane + 64 * u < total) put(a + rr_[u], 16 * cc_[u], reinterpret_cast<const uint8_t*>(&v[u]), 16);
    }
  } else {
    const int nu = (W + 3) >> 2, total = (b - a) * nu;
    for (int i0 = 0; i0 < total; i0 += 64 * PS_LOAD_U) {
      uint32_t v[PS_LOAD_U];
      int rr_[PS_LOAD_U], cc_[PS_LOAD_U];
#pragma unroll
      for (int u = 0; u < PS_LOAD_U; ++u) {
        const int idx = min(i0 + lane + 64 * u, total - 1);
        const int r = idx / nu, cu = idx - r * nu;
        rr_[u] = r;
        cc_[u] = cu;
        const int cb = 4 * cu, cl = min(cb, W - 4);
        v[u] = ps_ld32u(src + ((size_t)(a + r) * sp + (uint32_t)cl)) >> (8 * (cb - cl));
      }
#pragma unroll
      for (int u = 0; u < PS_LOAD_U; ++u)
        if (i0 + lane + 64 * u < total) put(a + rr_[u], 4 * cc_[u], reinterpret_cast<const uint8_t*>(&v[u]), 4);
    }
  }
}

#define PF_KERNEL_ARGS                                                                                       \
  const uint8_t *__restrict__ frames, size_t fstride, size_t rstride, uint8_t *__restrict__ pyr,           \
      size_t pstride, const PyrFast F, const uint2 *__restrict__ tasks, const int *__restrict__ tick_end,    \
      const uint4 *__restrict__ xlut, const uint2 *__restrict__ ylut, const CellInfo *__restrict__ cells,   \
      uint32_t *__restrict__ slots, uint32_t *__restrict__ slots_hi, size_t slot_stride,                    \
      uint32_t *__restrict__ ccount, int ncells_total, int aligned16

__global__ __launch_bounds__(1024) void k_pyrfast(PF_KERNEL_ARGS) {
  extern __shared__ __align__(16) uint8_t lds[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nw = (int)(blockDim.x >> 6);
  const int f = blockIdx.x;
  PfLds L;
  L.ring = lds + F.o_ring;
  L.aring = lds + F.o_aring;
  L.bmap = reinterpret_cast<uint32_t*>(lds + F.o_bmap);
  L.lut = reinterpret_cast<const uint4*>(lds + F.o_lut);
  L.cellsoff = reinterpret_cast<int*>(lds + F.o_cell);
  L.cnt = reinterpret_cast<int*>(lds + F.o_cnt);
  L.l1 = reinterpret_cast<uint32_t*>(lds + F.o_l1);
  L.l2 = reinterpret_cast<uint32_t*>(lds + F.o_l2);
  L.nms = reinterpret_cast<uint16_t*>(lds + F.o_nms);
  L.misc = reinterpret_cast<int*>(lds + F.o_misc);
  if (tid < 16) L.misc[tid] = 0;
  uint8_t* fpyr = pyr + (size_t)f * pstride;
  uint32_t* fslots = slots + (size_t)f * slot_stride;
  uint32_t* fslots_hi = slots_hi + (size_t)f * slot_stride;
  uint32_t* fccount = ccount + (size_t)f * ncells_total;
  const int t_lo = min(F.ini_th, F.min_th);
  uint32_t* L1 = L.l1 + (wave > 0 ? wave - 1 : 0) * ORBX_PF_L1CAP;
  int pending = -1;  // a task ticket drawn past its list's end, kept for a later list
  int T = 0;         // tick count over all passes (list parity)
  for (int p = 0; p < F.np; ++p) {
    const PyrFastPass& Q = F.p[p];
    int n1 = 0;
    // the tasks of one list (tick k, phase 1 or 2) by ticket, in list order
    auto run_tasks = [&](int tend) {
      for (;;) {
        int t = pending;
        if (t < 0) {
          int v = 0;
          if (lane == 0) v = atomicAdd(&L.misc[0], 1);
          t = __builtin_amdgcn_readfirstlane(v);
        }
        if (t >= tend) {
          pending = t;
          break;
        }
        pending = -1;
        const uint2 d = tasks[t];
        const int type = (int)(d.x & 15);
        if (type == ORBX_PF_FASTA) {
          if (!(PF_PROBE & 2)) pf_fasta(Q, L, d.x, d.y, lane, L1, n1, t_lo, T & 1);
        } else if (type == ORBX_PS_RESIZE) {
          if (!(PF_PROBE & 4)) pf_resize(Q, L, fpyr, ylut, d.x, (int)d.y, lane);
        } else if (!(PF_PROBE & 1)) {
          pf_nms(F, Q, L, fslots, fslots_hi, fccount, (int)(d.y & 0x3FFFu), (int)((d.x >> 16) & 255),
                 (int)((d.y >> 22) & 0xFFu), (int)((d.x >> 9) & 127), lane);
        }
      }
    };
    // pass setup: the next level's column LUT, this level's cell slot offsets,
    // zero counts and corner bitmaps
    if (Q.next) {
      const uint4* src = xlut + (Q.xl >> 1);
      for (int i = tid; i < 2 * Q.ng; i += (int)blockDim.x) const_cast<uint4*>(L.lut)[i] = src[i];
    }
    if (Q.fast) {
      const int nc = Q.ncv * Q.nrv;
      for (int i = tid; i < nc; i += (int)blockDim.x) L.cellsoff[i] = cells[Q.cell_begin + i].slot_off;
      for (int i = tid; i < 2 * F.ncv_max; i += (int)blockDim.x) L.cnt[i] = 0;
      for (int i = tid; i < Q.arows * Q.bmw; i += (int)blockDim.x) L.bmap[i] = 0u;
    }
    __syncthreads();
    const uint8_t* src = p == 0 ? frames + (size_t)f * fstride : fpyr + Q.soff;
    const uint32_t sp = p == 0 ? (uint32_t)rstride : (uint32_t)Q.spitch;
    const bool al16 = p > 0 || aligned16;
    for (int k = 0; k < Q.nticks; ++k, ++T) {
      const int par = T & 1;
      // ---- phase 1
      if (wave == 0) {
        pf_load(Q, src, sp, L.ring, min(Q.h, Q.R * k), (PF_PROBE & 16) ? min(Q.h, Q.R * k) : min(Q.h, Q.R * (k + 1)),
                lane, al16);
      } else {
        run_tasks(tick_end[2 * (Q.tick0 + k)]);
        // the wave's last even-test batch of the tick
        wave_sync_lds();
        if (n1 > 0) pf_stage_b(Q, L, lane < n1 ? L1[lane] : 0u, lane < n1, t_lo, lane, par);
        n1 = 0;
      }
      ps_barrier();
      // ---- phase 2: full strength of the tick's even-test survivors
      if (wave == 0) {
        if (lane == 0) {
          L.misc[1 + (par ^ 1)] = 0;
          L.misc[3 + (par ^ 1)] = 0;
        }
      } else {
        const int n2 = (PF_PROBE & 8) ? 0 : min(L.misc[1 + par], ORBX_PF_L2CAP);
        for (;;) {
          int v = 0;
          if (lane == 0) v = atomicAdd(&L.misc[3 + par], 1);
          const int q = 64 * __builtin_amdgcn_readfirstlane(v);
          if (q >= n2) break;
          const bool act = q + lane < n2;
          pf_stage_c(Q, L, act ? L.l2[q + lane] : 0u, act, t_lo);
        }
        // then the next level's rows (ring rows of earlier ticks -> HBM)
        run_tasks(tick_end[2 * (Q.tick0 + k) + 1]);
      }
      ps_barrier();
    }
    // the next pass reads the level this one wrote (HBM stores of this
    // workgroup, same CU: complete before the barrier)
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
  }
  (void)nw;
}

}  // namespace orbx
