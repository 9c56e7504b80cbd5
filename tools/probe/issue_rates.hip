// Microbenchmark (profiling tool, not product code): per-CU issue rates of
// scalar and vector ALU instructions on gfx950, to settle what bounds
// k_fast_strips (is the CU's one scalar unit at one
// instruction per cycle the floor?).  Every kernel runs ITERS iterations of
// 8 independent instructions per wave (8 separate registers: no dependency
// chain inside an iteration), 1..8 waves per SIMD (256-thread blocks, one
// wave per SIMD, WPS blocks per CU).  Reports instructions per CU per
// nanosecond and, with the in-kernel clock (s_memtime / s_memrealtime),
// per cycle.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define ITERS 4096

__device__ __forceinline__ void stamp(long long* t, long long* rt) {
  *t = __builtin_amdgcn_s_memtime();
  *rt = __builtin_amdgcn_s_memrealtime();
}

// (the scalar adds declare their SCC clobber, else the loop branch reads it)
// MODE 0: 8 SALU; 1: 8 VALU; 2: 8 SALU + 8 VALU interleaved; 3: 8 dependent
// SALU (one chain); 4: the append skeleton of k_fast_strips (v_cmp to SGPRs,
// s_and_saveexec, s_cbranch_execz, v_mbcnt x2, ds_write_b16, s_or exec,
// s_bcnt1, s_add) x 4; 5: the same 4 appends with exec set straight from the
// compare (s_mov exec) and no branch
template <int MODE>
__global__ __launch_bounds__(256) void k(unsigned* out, long long* clk) {
  __shared__ unsigned short lst[4096];
  unsigned s0 = threadIdx.x >> 6, s1 = 1, s2 = 2, s3 = 3, s4 = 4, s5 = 5, s6 = 6, s7 = 7;
  unsigned v0 = threadIdx.x, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3, v4 = v0 + 4, v5 = v0 + 5, v6 = v0 + 6,
           v7 = v0 + 7;
  s0 = __builtin_amdgcn_readfirstlane(s0);
  long long t0, r0, t1, r1;
  stamp(&t0, &r0);
  unsigned n1 = 0;
  for (int i = 0; i < ITERS; ++i) {
    if (MODE == 0 || MODE == 2) {
      asm volatile(
          "s_add_u32 %0, %0, 1\n\ts_add_u32 %1, %1, 1\n\ts_add_u32 %2, %2, 1\n\ts_add_u32 %3, %3, 1\n\t"
          "s_add_u32 %4, %4, 1\n\ts_add_u32 %5, %5, 1\n\ts_add_u32 %6, %6, 1\n\ts_add_u32 %7, %7, 1"
          : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7)::"scc");
    }
    if (MODE == 1 || MODE == 2) {
      asm volatile(
          "v_add_u32 %0, 1, %0\n\tv_add_u32 %1, 1, %1\n\tv_add_u32 %2, 1, %2\n\tv_add_u32 %3, 1, %3\n\t"
          "v_add_u32 %4, 1, %4\n\tv_add_u32 %5, 1, %5\n\tv_add_u32 %6, 1, %6\n\tv_add_u32 %7, 1, %7"
          : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7));
    }
    if (MODE == 3) {
      asm volatile(
          "s_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\t"
          "s_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1\n\ts_add_u32 %0, %0, 1"
          : "+s"(s0)::"scc");
    }
    if (MODE == 4) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool k = ((v0 + (unsigned)i * 7u + (unsigned)j * 13u) & 7u) == 0u;  // ~1/8 survivors
        const unsigned long long bal = __ballot(k);
        const int pos = (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
        unsigned short* L = lst + (__builtin_amdgcn_readfirstlane(n1) & 2047);
        if (k) L[pos] = (unsigned short)(i + j);
        n1 += __popcll(bal);
      }
    }
    if (MODE == 5) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool k = ((v0 + (unsigned)i * 7u + (unsigned)j * 13u) & 7u) == 0u;
        const unsigned long long bal = __ballot(k);
        const unsigned base = (unsigned)__builtin_amdgcn_readfirstlane(n1) & 2047u;
        const unsigned pos = __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, base));
        const unsigned addr = (unsigned)(size_t)lst + 2u * pos;
        const unsigned val = (unsigned)(i + j);
        asm volatile("s_mov_b64 exec, %0\n\tds_write_b16 %1, %2\n\ts_mov_b64 exec, -1" ::"s"(bal), "v"(addr), "v"(val)
                     : "memory");
        n1 += __popcll(bal);
      }
    }
  }
  stamp(&t1, &r1);
  unsigned acc = s0 + s1 + s2 + s3 + s4 + s5 + s6 + s7 + v0 + v1 + v2 + v3 + v4 + v5 + v6 + v7 + n1;
  if (MODE >= 4) {
    __syncthreads();
    acc += lst[threadIdx.x];
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

template <int MODE>
void run(const char* name, int per_iter_salu, int per_iter_valu, unsigned* o, long long* clk) {
  for (int wps = 1; wps <= 8; wps *= 2) {
    const int blocks = 256 * wps;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float ms = 0;
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(k<MODE>, dim3(blocks), dim3(256), 0, 0, o, clk);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1);
    }
    static long long h[2 * 2048];
    hipMemcpy(h, clk, sizeof(long long) * 2 * blocks, hipMemcpyDeviceToHost);
    double ghz = 0;
    for (int b = 0; b < blocks; ++b) ghz += (double)h[2 * b] / ((double)h[2 * b + 1] * 10.0);  // memrealtime 100 MHz
    ghz /= blocks;
    const double waves_per_cu = 4.0 * wps;
    const double salu = waves_per_cu * ITERS * per_iter_salu, valu = waves_per_cu * ITERS * per_iter_valu;
    const double ns = ms * 1e6;
    printf("%-8s waves/SIMD %d: %.3f ms  clk %.2f GHz  SALU/CU/cycle %.3f  VALU/CU/cycle %.3f  CU cycles per wave-iteration %.2f\n",
           name, wps, ms, ghz, salu / (ns * ghz), valu / (ns * ghz), ns * ghz / (waves_per_cu * ITERS));
  }
}

int main(int argc, char** argv) {
  setvbuf(stdout, NULL, _IONBF, 0);
  const int only = argc > 1 ? atoi(argv[1]) : -1;
  unsigned* o;
  long long* clk;
  hipMalloc(&o, (size_t)2048 * 256 * 4);
  hipMalloc(&clk, (size_t)2 * 2048 * 8);
  printf("start\n");
  if (only < 0 || only == 0) run<0>("salu", 8, 0, o, clk);
  if (only < 0 || only == 1) run<1>("valu", 0, 8, o, clk);
  if (only < 0 || only == 2) run<2>("mix", 8, 8, o, clk);
  if (only < 0 || only == 3) run<3>("saludep", 8, 0, o, clk);
  if (only < 0 || only == 4) run<4>("append", 0, 0, o, clk);
  if (only < 0 || only == 5) run<5>("appexec", 0, 0, o, clk);
  return 0;
}
