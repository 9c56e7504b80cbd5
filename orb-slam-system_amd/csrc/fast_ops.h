// fast_ops.h -- FAST-9/16 primitives of k_fast_strips
// (kernels_extract.hip): the strength
// A(p) = max(0, max_arc min_k I_k - p, p - min_arc max_k I_k) over the 16 arcs
// of 9 contiguous circle pixels (cv::FAST reports p at threshold t iff
// A(p) > t and cornerScore<16> returns A - 1; ORBextractor.cc:330-331), the
// packed even-point pre-test, and wave-level LDS ordering.
#ifndef ORBX_FAST_OPS_H
#define ORBX_FAST_OPS_H

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace orbx {

typedef unsigned short us2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ us2 as_us2(uint32_t x) { return __builtin_bit_cast(us2, x); }
__device__ __forceinline__ uint32_t as_u32(us2 x) { return __builtin_bit_cast(uint32_t, x); }

// FAST radius-3 circle (cv::makeOffsets, patternSize 16), as immediates
__device__ constexpr int8_t c_circle_dx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
__device__ constexpr int8_t c_circle_dy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};

__device__ __forceinline__ int min3i(int a, int b, int c) { return min(min(a, b), c); }
__device__ __forceinline__ int max3i(int a, int b, int c) { return max(max(a, b), c); }

__device__ __forceinline__ int fast_strength(const uint8_t* t, int tw) {
  int I[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) I[k] = t[c_circle_dy[k] * tw + c_circle_dx[k]];
  const int v = t[0];
  // the bright polarity, then the dark one: 16 + 16 values live at a time
  // instead of 16 + 32 (k_fast_pf keeps the next tile in registers beside it)
  int m3[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) m3[k] = min3i(I[k], I[(k + 1) & 15], I[(k + 2) & 15]);
  int Mb = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) Mb = max(Mb, min3i(m3[k], m3[(k + 3) & 15], m3[(k + 6) & 15]));
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int k = 0; k < 16; ++k) m3[k] = max3i(I[k], I[(k + 1) & 15], I[(k + 2) & 15]);
  int Md = 255;
#pragma unroll
  for (int k = 0; k < 16; ++k) Md = min(Md, max3i(m3[k], m3[(k + 3) & 15], m3[(k + 6) & 15]));
  return max3i(0, Mb - v, v - Md);
}

// 4 cyclically consecutive points of {0,2,..,14} all brighter (darker) than
// v +- t: necessary for a 9-arc (any 9 contiguous circle points contain 4
// consecutive even ones), i.e. for A > t.
// Packed form: E_i = circle point 2i; P_i = (E_i, E_{i+4}) as 16-bit lanes,
// so one packed min over four P's covers the windows starting at s and s+4:
// s = 0/4: P0..P3; 1/5: P1,P2,P3,rot(P0); 2/6: P2,P3,rot(P0),rot(P1);
// 3/7: P3,rot(P0),rot(P1),rot(P2) (rot swaps the halves).  Bright: some
// window's min > v + t; dark: some window's max < v - t.
__device__ __forceinline__ us2 rot16(us2 x) { return x.yx; }
__device__ __forceinline__ bool fast_even_test_pk(const uint8_t* t, int tw, int th) {
  us2 P0, P1, P2, P3;
  P0.x = t[3 * tw];           // point 0  (0, 3)
  P0.y = t[-3 * tw];          // point 8  (0, -3)
  P1.x = t[2 * tw + 2];       // point 2  (2, 2)
  P1.y = t[-2 * tw - 2];      // point 10 (-2, -2)
  P2.x = t[3];                // point 4  (3, 0)
  P2.y = t[-3];               // point 12 (-3, 0)
  P3.x = t[-2 * tw + 2];      // point 6  (2, -2)
  P3.y = t[2 * tw - 2];       // point 14 (-2, 2)
  const unsigned short v = t[0];
  const us2 s0 = rot16(P0), s1 = rot16(P1), s2 = rot16(P2);
  const us2 m23 = __builtin_elementwise_min(P2, P3), m123 = __builtin_elementwise_min(P1, m23);
  const us2 n01 = __builtin_elementwise_min(s0, s1);
  const us2 B = __builtin_elementwise_max(
      __builtin_elementwise_max(__builtin_elementwise_min(P0, m123), __builtin_elementwise_min(m123, s0)),
      __builtin_elementwise_max(__builtin_elementwise_min(m23, n01),
                                __builtin_elementwise_min(P3, __builtin_elementwise_min(n01, s2))));
  const us2 x23 = __builtin_elementwise_max(P2, P3), x123 = __builtin_elementwise_max(P1, x23);
  const us2 y01 = __builtin_elementwise_max(s0, s1);
  const us2 D = __builtin_elementwise_min(
      __builtin_elementwise_min(__builtin_elementwise_max(P0, x123), __builtin_elementwise_max(x123, s0)),
      __builtin_elementwise_min(__builtin_elementwise_max(x23, y01),
                                __builtin_elementwise_max(P3, __builtin_elementwise_max(y01, s2))));
  const us2 hh = (us2)(unsigned short)(v + th);
  const us2 vv = (us2)v, tt = (us2)(unsigned short)th;
  const us2 db = __builtin_elementwise_sub_sat(B, hh);
  const us2 dd = __builtin_elementwise_sub_sat(__builtin_elementwise_sub_sat(vv, D), tt);
  return (as_u32(db) | as_u32(dd)) != 0u;
}

__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct GroupWords {
  uint32_t w0, w1, w2, up, dn;
};

// The cardinal pre-test of one 4-pixel group (points 0/4/8/12: a 9-arc at
// threshold t holds two adjacent ones) in packed 16-bit lanes: w1 = the
// group's dword, w0 / w2 its left / right neighbours, up / dn the dwords 3
// rows above / below.  ttl = t * 0x10001 (0xFF00FF00 = no survivors).  clo /
// chi hold pixels 0, 2 / 1, 3 of the group, nonzero = survivor.
__device__ __forceinline__ void fast_cardinal(const GroupWords& q, uint32_t ttl, uint32_t& clo, uint32_t& chi) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t sel = h ? 0x0c030c01u : 0x0c020c00u;
    const us2 v = as_us2(__builtin_amdgcn_perm(0u, q.w1, sel));
    const us2 a0 = as_us2(__builtin_amdgcn_perm(0u, q.dn, sel));
    const us2 a8 = as_us2(__builtin_amdgcn_perm(0u, q.up, sel));
    const us2 a4 = as_us2(__builtin_amdgcn_perm(q.w2, q.w1, h ? 0x0c060c04u : 0x0c050c03u));
    const us2 a12 = as_us2(__builtin_amdgcn_perm(q.w1, q.w0, h ? 0x0c040c02u : 0x0c030c01u));
    const us2 t2 = as_us2(ttl);
    const us2 mb = __builtin_elementwise_min(__builtin_elementwise_max(a0, a8), __builtin_elementwise_max(a4, a12));
    const us2 md = __builtin_elementwise_max(__builtin_elementwise_min(a0, a8), __builtin_elementwise_min(a4, a12));
    const us2 db = __builtin_elementwise_sub_sat(mb, v + t2);
    const us2 dd = __builtin_elementwise_sub_sat(__builtin_elementwise_sub_sat(v, md), t2);
    const uint32_t x = as_u32(db) | as_u32(dd);
    if (h) chi = x; else clo = x;
  }
}

}  // namespace orbx

#endif
