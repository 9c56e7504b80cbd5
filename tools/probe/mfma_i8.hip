// Microbenchmark: cycles per v_mfma_i32_32x32x32_i8 on one SIMD, dependent
// chain vs 4 independent accumulators, 1..8 waves per SIMD (profiling tool).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

template <int NACC>
__global__ __launch_bounds__(256) void k(const v4i* a, v16i* out, int iters, long long* cyc) {
  v4i x = a[threadIdx.x & 63], y = a[(threadIdx.x + 7) & 63];
  v16i c[NACC];
  for (int j = 0; j < NACC; ++j) c[j] = v16i{};
  long long t0 = clock64();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int j = 0; j < NACC; ++j) c[j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(x, y, c[j], 0, 0, 0);
  }
  long long t1 = clock64();
  v16i s = c[0];
  for (int j = 1; j < NACC; ++j) s += c[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  v4i* a; v16i* o; long long* cyc;
  hipMalloc(&a, 64 * sizeof(v4i));
  hipMemset(a, 1, 64 * sizeof(v4i));
  const int maxb = 256 * 8;
  hipMalloc(&o, (size_t)maxb * 256 * sizeof(v16i));
  hipMalloc(&cyc, maxb * sizeof(long long));
  const int iters = 4096;
  for (int wps = 1; wps <= 8; wps *= 2) {
    for (int nacc = 1; nacc <= 4; nacc *= 4) {
      const int blocks = 256 * wps;  // 256 CUs x wps blocks of 4 waves (1 per SIMD)
      hipEvent_t e0, e1;
      hipEventCreate(&e0); hipEventCreate(&e1);
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        if (nacc == 1) hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, a, o, iters, cyc);
        else hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, a, o, iters, cyc);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
      }
      float ms; hipEventElapsedTime(&ms, e0, e1);
      long long c0; hipMemcpy(&c0, cyc, 8, hipMemcpyDeviceToHost);
      const double nmf = (double)iters * nacc;   // per wave
      // per SIMD: wps waves x nmf MFMAs in ms
      const double per_simd = nmf * wps;
      printf("waves/SIMD %d acc %d: %.3f ms, %.1f ns per MFMA per SIMD, wave clock64 %.1f per MFMA\n",
             wps, nacc, ms, ms * 1e6 / per_simd, (double)c0 / nmf);
    }
  }
  return 0;
}
