// kernels_stereo.hip -- gfx950 kernels of Frame::ComputeStereoMatches
// (/root/reference/src/Frame.cc:446-620) on device-resident left/right
// extractor outputs and pyramids.
//
//   vRowIndices (:456-473)                        -> k_stereo_rows   (per frame, LDS CSR)
//   descriptor search + SAD + parabola (:484-611) -> k_stereo_match  (one wavefront per left keypoint)
//   median outlier filter (:613-631)              -> k_stereo_filter (per frame, radix select)
//
// Integer work (rows, Hamming, SAD) is exact; the float work (row bounds,
// scaled coordinates, parabola, disparity, depth) is written
// operation-for-operation as the reference with -ffp-contract=off.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/orbx.h"
#include "orbx_internal.h"
#include "wave_ops.h"

namespace orbx {

#define SR_THREADS 1024

// exclusive scan of a[0..n) in place (1024 threads), returns the total
__device__ int stereo_block_scan(int* a, int n, int* wsum) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int chunk = (n + SR_THREADS - 1) / SR_THREADS;
  const int b = min(n, tid * chunk), e = min(n, b + chunk);
  int s = 0;
  for (int i = b; i < e; ++i) s += a[i];
  const int incl = orbx::wave_incl_scan(s);
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  if (tid == 0) {
    int run = 0;
    for (int w = 0; w < SR_THREADS / 64; ++w) {
      const int t = wsum[w];
      wsum[w] = run;
      run += t;
    }
    wsum[SR_THREADS / 64] = run;
  }
  __syncthreads();
  int run = wsum[wave] + incl - s;
  for (int i = b; i < e; ++i) {
    const int t = a[i];
    a[i] = run;
    run += t;
  }
  const int total = wsum[SR_THREADS / 64];
  __syncthreads();
  return total;
}

typedef unsigned short us2 __attribute__((ext_vector_type(2)));
typedef short s2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ us2 st_as_us2(uint32_t x) { return __builtin_bit_cast(us2, x); }
// dword load at any byte address (gfx950 global memory takes unaligned dwords)
__device__ __forceinline__ uint32_t st_ld32u(const uint8_t* p) {
  uint32_t v;
  __builtin_memcpy(&v, p, 4);
  return v;
}

__device__ __forceinline__ bool stereo_rows_of(const orbx_keypoint& k, const StereoArgs& A,
                                               int* minr, int* maxr) {
  if (k.octave < 0 || k.octave >= A.nlevels) return false;
  const float kpY = k.y;
  const float r = 2.0f * A.scale[k.octave];  // :465
  *maxr = (int)ceilf(kpY + r);               // :466
  *minr = (int)floorf(kpY - r);              // :467
  return *minr >= 0 && *maxr < A.nrows;      // vRowIndices[yi] in range
}

// vRowIndices as CSR: rowoff[f][0..nrows], rows[f][...] = the right
// keypoints of each row as {iR | octave << 16, x} (the search's gates read
// them from the entry: no dependent keypoint gather).  The order inside a row
// does not matter: the search takes the lexicographic minimum of (distance,
// iR), which is what the reference's ascending-iR scan with a strict '<'
// selects.
__global__ __launch_bounds__(SR_THREADS) void k_stereo_rows(const orbx_keypoint* __restrict__ kps_r,
                                                            const int* __restrict__ cnt_r,
                                                            const StereoArgs A,
                                                            int* __restrict__ rowoff,
                                                            uint2* __restrict__ rows,
                                                            int* __restrict__ err) {
  extern __shared__ int rc[];  // nrows
  __shared__ int wsum[SR_THREADS / 64 + 1];
  const int f = blockIdx.x, tid = threadIdx.x;
  const int n = cnt_r[f];
  const orbx_keypoint* K = kps_r + (size_t)f * A.kcap;
  for (int i = tid; i < A.nrows; i += SR_THREADS) rc[i] = 0;
  __syncthreads();
  bool bad = false;
  for (int iR = tid; iR < n; iR += SR_THREADS) {
    int lo, hi;
    if (!stereo_rows_of(K[iR], A, &lo, &hi)) {
      bad = true;
      continue;
    }
    for (int yi = lo; yi <= hi; ++yi) atomicAdd(&rc[yi], 1);
  }
  if (bad) atomicOr(err, ORBX_DEVERR_STEREO);
  __syncthreads();
  const int total = stereo_block_scan(rc, A.nrows, wsum);
  int* ro = rowoff + (size_t)f * (A.nrows + 1);
  for (int i = tid; i < A.nrows; i += SR_THREADS) ro[i] = rc[i];
  if (tid == 0) ro[A.nrows] = total;
  if (total > A.rcap) {  // cannot happen: rcap bounds the rows any keypoint spans
    if (tid == 0) atomicOr(err, ORBX_DEVERR_STEREO);
    return;
  }
  __syncthreads();
  uint2* R = rows + (size_t)f * A.rcap;
  for (int iR = tid; iR < n; iR += SR_THREADS) {
    const orbx_keypoint k = K[iR];
    int lo, hi;
    if (!stereo_rows_of(k, A, &lo, &hi)) continue;
    const uint2 e = make_uint2((uint32_t)iR | ((uint32_t)k.octave << 16), __float_as_uint(k.x));
    for (int yi = lo; yi <= hi; ++yi) R[atomicAdd(&rc[yi], 1)] = e;
  }
}

__device__ __forceinline__ const uint8_t* stereo_level(const uint8_t* frames, size_t fstride,
                                                       size_t rstride, const uint8_t* pyr,
                                                       size_t pstride, const StereoArgs& A, int f,
                                                       int l, int* pitch) {
  if (A.off[l] < 0) {
    *pitch = (int)rstride;
    return frames + (size_t)f * fstride;
  }
  *pitch = A.pitch[l];
  return pyr + (size_t)f * pstride + A.off[l];
}

// One wavefront per left keypoint iL (waves stride over the frame's count).
// Lanes split the row's candidates (octave and disparity gates, Hamming),
// then the 11 x 11 rows of the 11 sliding windows; lane 0 finishes the
// parabola fit.  Outputs per iL: uRight, depth, and the SAD used by the
// median filter (-1 = no stereo match).
__global__ __launch_bounds__(256) void k_stereo_match(
    const orbx_keypoint* __restrict__ kps_l, const uint8_t* __restrict__ desc_l,
    const int* __restrict__ cnt_l, const orbx_keypoint* __restrict__ kps_r,
    const uint8_t* __restrict__ desc_r, const uint8_t* __restrict__ frames_l,
    const uint8_t* __restrict__ frames_r, size_t fstride, size_t rstride,
    const uint8_t* __restrict__ pyr_l, const uint8_t* __restrict__ pyr_r, size_t pstride,
    const StereoArgs A, const int* __restrict__ rowoff, const uint2* __restrict__ rows,
    float* __restrict__ uright, float* __restrict__ depth, int* __restrict__ sad,
    int* __restrict__ err) {
  __shared__ int part[4][128];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int f = blockIdx.y;
  const int nl = cnt_l[f];
  const orbx_keypoint* KL = kps_l + (size_t)f * A.kcap;
  (void)kps_r;  // the right keypoints' gate fields come with the CSR entries
  const uint8_t* DL = desc_l + (size_t)f * A.kcap * 32;
  const uint8_t* DR = desc_r + (size_t)f * A.kcap * 32;
  const int* ro = rowoff + (size_t)f * (A.nrows + 1);
  const uint2* R = rows + (size_t)f * A.rcap;
  const float minD = 0;                // :477
  const float maxD = A.mbf / A.mb;     // :476-478 (minZ = mb)
  const int thOrbDist = (100 + 50) / 2;  // :451 (TH_HIGH + TH_LOW) / 2
  // the next left keypoint and its descriptor are loaded one keypoint ahead
  const int stride = gridDim.x * 4;
  int iL = blockIdx.x * 4 + wave;
  orbx_keypoint kpN;
  uint4 a0N, a1N;
  if (iL < nl) {
    kpN = KL[iL];
    a0N = reinterpret_cast<const uint4*>(DL + (size_t)iL * 32)[0];
    a1N = reinterpret_cast<const uint4*>(DL + (size_t)iL * 32)[1];
  }
  for (; iL < nl; iL += stride) {
    const orbx_keypoint kpL = kpN;
    const uint4 a0 = a0N, a1 = a1N;
    if (iL + stride < nl) {  // wave-uniform
      kpN = KL[iL + stride];
      a0N = reinterpret_cast<const uint4*>(DL + (size_t)(iL + stride) * 32)[0];
      a1N = reinterpret_cast<const uint4*>(DL + (size_t)(iL + stride) * 32)[1];
    }
    float ur = -1.0f, dp = -1.0f;
    int sv = -1;
    bool bad = false;
    const int levelL = kpL.octave;
    const float vL = kpL.y, uL = kpL.x;
    if (levelL < 0 || levelL >= A.nlevels || !(vL >= 0.0f) || (int)vL >= A.nrows) {
      bad = true;
    } else {
      const int row = (int)vL;  // vRowIndices[vL] (:492)
      const int cb = ro[row], ce = ro[row + 1];
      const float minU = uL - maxD, maxU = uL - minD;  // :497-498
      if (cb != ce && !(maxU < 0)) {
        uint32_t best = 0xFFFFFFFFu;
        float ubest = 0.0f;  // x of this lane's best candidate
        for (int c = cb + lane; c < ce; c += 64) {  // :507-529
          const uint2 e = R[c];
          const int iR = (int)(e.x & 0xFFFFu), oR = (int)(e.x >> 16);
          const float uR = __uint_as_float(e.y);
          if (oR >= levelL - 1 && oR <= levelL + 1 && uR >= minU && uR <= maxU) {
            const uint4* drp = reinterpret_cast<const uint4*>(DR + (size_t)iR * 32);
            const uint4 b0 = drp[0], b1 = drp[1];
            const int dist = __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) +
                             __popc(a0.w ^ b0.w) + __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) +
                             __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
            const uint32_t key = ((uint32_t)dist << 16) | (uint32_t)iR;
            if (dist < 100 && key < best) {
              best = key;
              ubest = uR;
            }
          }
        }
        const uint32_t mine = best;
        best = wave_min_u32(best);  // DPP, no LDS round trips
        const int bestDist = best == 0xFFFFFFFFu ? 100 : (int)(best >> 16);
        if (bestDist < thOrbDist) {  // :532
          // keys are unique (iR inside): the owner lane holds the winner's x
          const int owner = __ffsll((unsigned long long)__ballot(mine == best)) - 1;
          const float uR0 = __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(ubest), owner));
          const float scaleFactor = A.inv_scale[levelL];
          const float scaleduL = roundf(kpL.x * scaleFactor);
          const float scaledvL = roundf(kpL.y * scaleFactor);
          const float scaleduR0 = roundf(uR0 * scaleFactor);
          const int w = 5, L = 5;
          const int W = A.w[levelL], H = A.h[levelL];
          const int y0 = (int)scaledvL - w, xl0 = (int)scaleduL - w;
          const float iniu = scaleduR0 + L - w;        // :560
          const float endu = scaleduR0 + L + w + 1;    // :561
          const int xr0 = (int)scaleduR0 - L - w;
          if (y0 < 0 || y0 + 2 * w + 1 > H || xl0 < 0 || xl0 + 2 * w + 1 > W) {
            bad = true;  // IL rowRange/colRange assertion (:545)
          } else if (!(iniu < 0 || endu >= W)) {
            if (xr0 < 0 || xr0 + 2 * (L + w) + 1 > W) {
              bad = true;  // IR colRange assertion (:567)
            } else {
              int lp, rp;
              const uint8_t* Lb = stereo_level(frames_l, fstride, rstride, pyr_l, pstride, A, f, levelL, &lp);
              const uint8_t* Rb = stereo_level(frames_r, fstride, rstride, pyr_r, pstride, A, f, levelL, &rp);
              const uint8_t* IL = Lb + (size_t)y0 * lp + xl0;
              const uint8_t* IRb = Rb + (size_t)y0 * rp + xr0;
              const int cL = IL[w * lp + w];
              // 121 (incR, row) partial sums, two per lane: the row's 11
              // left / right bytes as three dword loads each (the last one
              // ending at byte 10: nothing past the window is read), then
              // |(l + cR) - (r + cL)| on byte pairs in packed 16-bit lanes
              const us2 cLL = (us2)(unsigned short)cL;
#pragma unroll
              for (int h2 = 0; h2 < 2; ++h2) {
                const int p = lane + 64 * h2;
                if (p < 121) {
                  const int k = p / 11, yy = p - 11 * (p / 11);  // k = incR + L
                  const uint8_t* lr = IL + yy * lp;
                  const uint8_t* rr = IRb + yy * rp + k;
                  const us2 cRR = (us2)(unsigned short)IRb[w * rp + k + w];
                  const uint32_t lw[3] = {st_ld32u(lr), st_ld32u(lr + 4), st_ld32u(lr + 7) >> 8};
                  const uint32_t rw[3] = {st_ld32u(rr), st_ld32u(rr + 4), st_ld32u(rr + 7) >> 8};
                  us2 acc = (us2)(unsigned short)0;
#pragma unroll
                  for (int q = 0; q < 3; ++q) {
#pragma unroll
                    for (int hh = 0; hh < 2; ++hh) {
                      const uint32_t sel = hh ? 0x0c030c01u : 0x0c020c00u;
                      const us2 A = st_as_us2(__builtin_amdgcn_perm(0u, lw[q], sel)) + cRR;
                      const us2 B = st_as_us2(__builtin_amdgcn_perm(0u, rw[q], sel)) + cLL;
                      const s2v D = __builtin_bit_cast(s2v, A) - __builtin_bit_cast(s2v, B);
                      us2 ad = __builtin_bit_cast(us2, __builtin_elementwise_abs(D));
                      if (q == 2 && hh == 1) ad.y = 0;  // byte 11 is not in the window
                      acc += ad;
                    }
                  }
                  part[wave][p] = (int)acc.x + (int)acc.y;
                }
              }
              __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
              __builtin_amdgcn_wave_barrier();
              __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
              // lane k < 11: vDists[k] (sum of its 11 rows); the first
              // minimum in k order is the least (SAD << 4 | k)
              int dk = 0;
              if (lane < 11) {
#pragma unroll
                for (int yy = 0; yy < 11; ++yy) dk += part[wave][lane * 11 + yy];
              }
              const uint32_t bk = wave_min_u32(lane < 11 ? ((uint32_t)dk << 4) | (uint32_t)lane : 0xFFFFFFFFu);
              const int bestSad = (int)(bk >> 4), bestincR = (int)(bk & 15u) - L;  // :552-578
              if (bestincR != -L && bestincR != L) {  // :580-581
                const float dist1 = (float)lane_value(dk, L + bestincR - 1);
                const float dist2 = (float)lane_value(dk, L + bestincR);
                const float dist3 = (float)lane_value(dk, L + bestincR + 1);
                const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
                if (!(deltaR < -1 || deltaR > 1)) {  // :590
                  float bestuR = A.scale[levelL] * ((float)scaleduR0 + (float)bestincR + deltaR);
                  float disparity = (uL - bestuR);
                  if (disparity >= minD && disparity < maxD) {  // :598
                    if (disparity <= 0) {
                      disparity = 0.01f;
                      bestuR = (float)((double)uL - 0.01);  // uL-0.01 in double (:603)
                    }
                    dp = A.mbf / disparity;
                    ur = bestuR;
                    sv = bestSad;
                  }
                }
              }
              __builtin_amdgcn_wave_barrier();
            }
          }
        }
      }
    }
    if (lane == 0) {
      const size_t o = (size_t)f * A.kcap + iL;
      uright[o] = ur;
      depth[o] = dp;
      sad[o] = sv;
      if (bad) atomicOr(err, ORBX_DEVERR_STEREO);
    }
  }
}

// :613-631: median of the kept SADs (vDistIdx[size/2].first after sorting)
// by a two-pass radix select over the 16-bit SAD values (max 121 * 510),
// then every match with SAD >= 1.5f * 1.4f * median is dropped.
__global__ __launch_bounds__(256) void k_stereo_filter(const int* __restrict__ cnt_l,
                                                       const StereoArgs A,
                                                       float* __restrict__ uright,
                                                       float* __restrict__ depth,
                                                       const int* __restrict__ sad,
                                                       int* __restrict__ nmatches) {
  __shared__ int hist[256];
  __shared__ int sh_nd, sh_bin, sh_k, sh_med, sh_rm;
  const int f = blockIdx.x, tid = threadIdx.x;
  const int n = cnt_l[f];
  const int* S = sad + (size_t)f * A.kcap;
  hist[tid] = 0;
  if (tid == 0) { sh_nd = 0; sh_rm = 0; }
  __syncthreads();
  int nd = 0;
  for (int i = tid; i < n; i += 256) {
    const int s = S[i];
    if (s >= 0) {
      ++nd;
      atomicAdd(&hist[s >> 8], 1);
    }
  }
  atomicAdd(&sh_nd, nd);
  __syncthreads();
  nd = sh_nd;
  if (nd == 0) {
    if (tid == 0) nmatches[f] = 0;
    return;
  }
  if (tid == 0) {
    int k = nd / 2, b = 0;
    while (k >= hist[b]) k -= hist[b++];
    sh_bin = b;
    sh_k = k;
  }
  __syncthreads();
  const int bin = sh_bin;
  hist[tid] = 0;
  __syncthreads();
  for (int i = tid; i < n; i += 256) {
    const int s = S[i];
    if (s >= 0 && (s >> 8) == bin) atomicAdd(&hist[s & 255], 1);
  }
  __syncthreads();
  if (tid == 0) {
    int k = sh_k, b = 0;
    while (k >= hist[b]) k -= hist[b++];
    sh_med = (bin << 8) | b;
  }
  __syncthreads();
  const float median = (float)sh_med;
  const float thDist = 1.5f * 1.4f * median;  // :616
  int rm = 0;
  for (int i = tid; i < n; i += 256) {
    const int s = S[i];
    if (s >= 0 && !((float)s < thDist)) {  // :618-629
      const size_t o = (size_t)f * A.kcap + i;
      uright[o] = -1;
      depth[o] = -1;
      ++rm;
    }
  }
  atomicAdd(&sh_rm, rm);
  __syncthreads();
  if (tid == 0) nmatches[f] = nd - sh_rm;
}

}  // namespace orbx
