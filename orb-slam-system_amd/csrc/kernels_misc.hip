// kernels_misc.hip -- gfx950 kernels of SURVEY.md §8f rank 4:
//   MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:222-271) -> k_distinctive
//   Frame::UndistortKeyPoints (src/Frame.cc:384-414, cv::undistortPoints) -> k_undistort
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/orbx.h"

namespace orbx {

__device__ __forceinline__ int hamming32(const uint8_t* a, const uint8_t* b) {
  const uint4* pa = reinterpret_cast<const uint4*>(a);
  const uint4* pb = reinterpret_cast<const uint4*>(b);
  const uint4 a0 = pa[0], a1 = pa[1], b0 = pb[0], b1 = pb[1];
  return __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) + __popc(a0.w ^ b0.w) +
         __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) + __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
}

// One wavefront per map point; lane = observation row i.  The median of row
// i (nth_element at N/2 over the N distances, d_ii = 0 included) is the
// smallest v with #{j : d_ij <= v} > N/2, found by a binary search over the
// distance range [0, 256]; the chosen row is the first minimum (strict '<').
__global__ __launch_bounds__(256) void k_distinctive(const uint8_t* __restrict__ desc,
                                                     const int32_t* __restrict__ off, int nmp,
                                                     int32_t* __restrict__ best) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= nmp) return;
  const int b = off[m], N = off[m + 1] - b;
  if (N <= 0) {
    if (lane == 0) best[m] = -1;
    return;
  }
  const uint8_t* D = desc + (size_t)b * 32;
  const int need = N / 2 + 1;
  uint32_t bk = 0xFFFFFFFFu;  // (median << 20) | i
  for (int i0 = 0; i0 < N; i0 += 64) {
    const int i = i0 + lane;
    if (i < N) {
      int lo = 0, hi = 256;  // count(hi) = N >= need
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        int c = 0;
        for (int j = 0; j < N; ++j) c += (j == i ? 0 : hamming32(D + (size_t)i * 32, D + (size_t)j * 32)) <= mid;
        if (c >= need) hi = mid; else lo = mid + 1;
      }
      bk = min(bk, ((uint32_t)lo << 20) | (uint32_t)i);
    }
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) bk = min(bk, (uint32_t)__shfl_xor((int)bk, d, 64));
  if (lane == 0) best[m] = (int32_t)(bk & 0xFFFFFu);
}

struct UndistortArgs {
  double fx, fy, cx, cy, ifx, ify;
  double k[14];
};

// cv::undistortPoints (OpenCV 3.4 undistort.cpp) in double, 5 iterations,
// R = I, P = K; operation order as written there (no contraction: the
// translation unit is built with -ffp-contract=off)
__global__ __launch_bounds__(256) void k_undistort(const orbx_keypoint* __restrict__ in, int n,
                                                   const UndistortArgs A,
                                                   orbx_keypoint* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  orbx_keypoint kp = in[i];
  double x = kp.x, y = kp.y;
  x = (x - A.cx) * A.ifx;
  y = (y - A.cy) * A.ify;
  const double x0 = x, y0 = y;
  const double* k = A.k;
  for (int j = 0; j < 5; j++) {
    const double r2 = x * x + y * y;
    const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) /
                          (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
    const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
    const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
    x = (x0 - deltaX) * icdist;
    y = (y0 - deltaY) * icdist;
  }
  const double xx = A.fx * x + 0. * y + A.cx;
  const double yy = 0. * x + A.fy * y + A.cy;
  const double ww = 1. / (0. * x + 0. * y + 1.);
  kp.x = (float)(xx * ww);
  kp.y = (float)(yy * ww);
  out[i] = kp;
}

// ---------------------------------------------------------------------------
// Multi-GPU boundary frame (orbx/dist.py): one frame's outputs
// (kcap keypoint rows, kcap descriptor rows, count) packed into / unpacked
// from one contiguous exchange record [kps | desc | count]: one launch each
// instead of six tensor copies (dword copies, 16 B per thread and pass; the
// region sizes 28 kcap, 32 kcap and 4 are dword multiples).  Rows beyond the
// frame's count are copied too (the record has a fixed size for the
// all-gather).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_boundary_copy(const uint8_t* __restrict__ a, size_t na,
                                                       const uint8_t* __restrict__ b, size_t nb,
                                                       const uint8_t* __restrict__ c, size_t nc,
                                                       uint8_t* __restrict__ out, int unpack,
                                                       uint8_t* __restrict__ oa,
                                                       uint8_t* __restrict__ ob,
                                                       uint8_t* __restrict__ oc) {
  // pack: out = a | b | c; unpack: a (= the record) -> oa | ob | oc
  const size_t n = na + nb + nc;
  for (size_t i = ((size_t)blockIdx.x * 256 + threadIdx.x) * 16; i < n; i += (size_t)gridDim.x * 256 * 16) {
    uint32_t w[4];
    const int m = (int)min((size_t)16, n - i) >> 2;
    for (int k = 0; k < m; ++k) {
      const size_t j = i + 4 * k;
      const uint8_t* src = unpack ? a + j : (j < na ? a + j : j < na + nb ? b + (j - na) : c + (j - na - nb));
      w[k] = *reinterpret_cast<const uint32_t*>(src);
    }
    for (int k = 0; k < m; ++k) {
      const size_t j = i + 4 * k;
      uint8_t* dst = !unpack ? out + j : (j < na ? oa + j : j < na + nb ? ob + (j - na) : oc + (j - na - nb));
      *reinterpret_cast<uint32_t*>(dst) = w[k];
    }
  }
}

// ---------------------------------------------------------------------------
// k_pack_results: the drop-in call's results straight into the caller-facing
// pinned staging (orbx_extract): {count, error word} and the frame's K
// keypoint rows and descriptor rows at their fixed offsets, written by the
// GPU over PCIe in one launch -- the exact K is known here, so no
// speculative prefix and no second copy, and no chain of small D2H copies
// (each a blit launch and a completion signal: 4 copies took ~37 us of a
// 1080p call, round 6).  16-B stores: the keypoint rows (28 B each) as one
// contiguous run of K * 28 bytes (the device buffer is 16-B aligned and
// sized for kcap rows, so the last 16-B chunk reads at most 12 bytes of
// the next row, never past the buffer), the descriptor rows at the 16-B
// aligned offset desc_q16 (in 16-B units).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_pack_results(const int* __restrict__ d_err,
                                                      const int* __restrict__ d_count,
                                                      const uint4* __restrict__ kps,
                                                      const uint4* __restrict__ desc, int kcap,
                                                      uint4* __restrict__ h_res, uint32_t desc_q16) {
  const int err = *d_err, cnt = *d_count;
  const int K = err ? 0 : min(max(cnt, 0), kcap);
  const int tid = (int)(blockIdx.x * 256 + threadIdx.x), nt = (int)(gridDim.x * 256);
  if (tid == 0) h_res[0] = make_uint4((uint32_t)cnt, (uint32_t)err, 0u, 0u);
  const int nk = (K * 28 + 15) >> 4, nd = K * 2;  // 16-B chunks: keypoint rows (7 dwords each), descriptors
  for (int i = tid; i < nk; i += nt) h_res[4 + i] = kps[i];
  for (int i = tid; i < nd; i += nt) h_res[desc_q16 + i] = desc[i];
}

}  // namespace orbx
