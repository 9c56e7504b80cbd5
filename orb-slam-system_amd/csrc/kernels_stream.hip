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

#include "orbx_internal.h"

namespace orbx {

typedef uint32_t ps_v4u __attribute__((ext_vector_type(4)));
typedef unsigned short ps_us2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ ps_us2 ps_as_us2(uint32_t x) { return __builtin_bit_cast(ps_us2, x); }

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

template <int NT>
__device__ __forceinline__ void ps_loader(const uint8_t* __restrict__ src, size_t rstride, const PyrStream& S,
                                          uint8_t* __restrict__ lds, int lane, int aligned16) {
  const int W0 = S.w[0], H0 = S.h[0];
  uint8_t* ring = lds + S.roff[0];
  const int rp = S.rpitch[0], rr = S.rrows[0];
  const uint32_t rs = (uint32_t)rstride;
  for (int k = 0; k < S.nticks; ++k) {
    const int a = min(H0, S.r0 * k), b = min(H0, S.r0 * (k + 1));
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

}  // namespace orbx
