// fetch_calib -- calibrates rocprofv3's FETCH_SIZE on gfx950 for the access
// shapes of the orbx kernels (profiling tool; MI355X_MICROARCH.md: FETCH_SIZE
// reads 1/2 of the bytes of wide coalesced streams, other widths are
// uncalibrated).  Every kernel reads a known set of bytes from a buffer far
// larger than the Infinity Cache, each byte once:
//   k_stream16  1 GiB, 16 B per lane, coalesced (the documented case)
//   k_stream4   1 GiB, 4 B per lane, coalesced
//   k_patch4    BRIEF's patch loads (k_orient_brief brief_issue): 43 rows x
//               48 B per patch at random byte x / row y, 12 lanes per row,
//               one unaligned dword per lane, patches far apart
//   k_tile16    FAST's strip staging (stage_region<v4u>): 37 rows x 288 B per
//               tile, 16-B aligned loads
// Run under `rocprofv3 --pmc FETCH_SIZE`; the program prints the bytes each
// kernel touches, counted in 64-B sectors and in 128-B lines, so the
// counter can be divided by both.
//   fetch_calib [patches]   (JSON on stdout)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <set>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_stream16(const v4u* __restrict__ p, size_t n, uint32_t* out) {
  uint32_t s = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const v4u v = p[i];
    s ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (s == 0x12345678u) out[0] = s;
}

__global__ __launch_bounds__(256) void k_stream4(const uint32_t* __restrict__ p, size_t n, uint32_t* out) {
  uint32_t s = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s ^= p[i];
  if (s == 0x12345678u) out[0] = s;
}

// one wave per patch; lane (< 60) = column dword lane % 12 of rows lane/12 + 5u
__global__ __launch_bounds__(256) void k_patch4(const uint8_t* __restrict__ img, uint32_t pitch,
                                                const uint2* __restrict__ pos, int n, uint32_t* out) {
  const int w = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (w >= n) return;
  const uint2 p = pos[w];
  const int ln = min(lane, 59);
  const uint32_t c4 = (uint32_t)(ln % 12) * 4u, r0 = (uint32_t)(ln / 12);
  const uint8_t* b = img + (size_t)p.y * pitch + p.x;
  uint32_t s = 0;
#pragma unroll
  for (int u = 0; u < 9; ++u) {
    const uint32_t row = min(r0 + 5u * u, 42u);
    uint32_t v;
    __builtin_memcpy(&v, b + (size_t)row * pitch + c4, 4);
    s ^= v;
  }
  if (s == 0x12345678u) out[0] = s;
}

// one workgroup per tile: 37 rows x 288 B, 16-B loads (18 per row)
__global__ __launch_bounds__(256) void k_tile16(const uint8_t* __restrict__ img, uint32_t pitch,
                                                const uint2* __restrict__ pos, int n, uint32_t* out) {
  const int t = blockIdx.x;
  if (t >= n) return;
  const uint2 p = pos[t];
  const uint8_t* b = img + (size_t)p.y * pitch + p.x;
  uint32_t s = 0;
  for (int i = threadIdx.x; i < 37 * 18; i += 256) {
    const int r = i / 18, c = i - r * 18;
    const v4u v = *reinterpret_cast<const v4u*>(b + (size_t)r * pitch + 16 * c);
    s ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (s == 0x12345678u) out[0] = s;
}

static void touched(std::set<uint64_t>& sec, std::set<uint64_t>& line, uint64_t a, uint64_t nbytes) {
  for (uint64_t x = a / 64; x <= (a + nbytes - 1) / 64; ++x) sec.insert(x);
  for (uint64_t x = a / 128; x <= (a + nbytes - 1) / 128; ++x) line.insert(x);
}

int main(int argc, char** argv) {
  const int np = argc > 1 ? atoi(argv[1]) : 200000;
  const size_t bytes = (size_t)3 << 30;  // 3 GiB >> the 256 MiB Infinity Cache
  uint8_t* d;
  uint32_t* o;
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&o, 64));
  CK(hipMemset(d, 1, bytes));
  const uint32_t pitch = 1920;
  const uint64_t rows = (bytes - 4096) / pitch;
  // patches: random y (row), x in [0, pitch - 48]; rows sorted apart so no
  // two patches share a line (y spaced by >= 43 rows via a shuffled grid)
  std::vector<uint2> pp(np), tp;
  std::set<uint64_t> s_sec, s_line;
  srand(12345);
  const uint64_t slots = rows / 48;
  for (int i = 0; i < np; ++i) {
    const uint64_t slot = ((uint64_t)rand() * 65536ull + (uint64_t)rand()) % slots;
    pp[i].y = (uint32_t)(slot * 48);
    pp[i].x = (uint32_t)(rand() % (int)(pitch - 48));
  }
  // distinct slots only (a repeated slot would be an L2 hit)
  {
    std::set<uint32_t> ys;
    std::vector<uint2> q;
    for (auto& p : pp)
      if (ys.insert(p.y).second) q.push_back(p);
    pp.swap(q);
  }
  for (auto& p : pp)
    for (int r = 0; r < 43; ++r) touched(s_sec, s_line, (uint64_t)(p.y + r) * pitch + p.x, 48);
  // tiles: 37 rows x 288 B at 16-B aligned x, distinct 40-row slots
  std::set<uint64_t> t_sec, t_line;
  {
    std::set<uint32_t> ys;
    for (int i = 0; i < np / 4; ++i) {
      const uint64_t slot = ((uint64_t)rand() * 65536ull + (uint64_t)rand()) % (rows / 40);
      if (!ys.insert((uint32_t)slot).second) continue;
      uint2 t;
      t.y = (uint32_t)(slot * 40);
      t.x = (uint32_t)((rand() % (int)((pitch - 288) / 16)) * 16);
      tp.push_back(t);
      for (int r = 0; r < 37; ++r) touched(t_sec, t_line, (uint64_t)(t.y + r) * pitch + t.x, 288);
    }
  }
  uint2 *dp, *dt;
  CK(hipMalloc(&dp, pp.size() * sizeof(uint2)));
  CK(hipMalloc(&dt, tp.size() * sizeof(uint2)));
  CK(hipMemcpy(dp, pp.data(), pp.size() * sizeof(uint2), hipMemcpyHostToDevice));
  CK(hipMemcpy(dt, tp.data(), tp.size() * sizeof(uint2), hipMemcpyHostToDevice));
  const size_t gib = (size_t)1 << 30;
  // each kernel reads a region the previous ones did not touch (no reuse
  // through the Infinity Cache): streams from the top of the buffer
  hipLaunchKernelGGL(k_stream16, dim3(4096), dim3(256), 0, 0, (const v4u*)(d + 2 * gib), gib / 16, o);
  hipLaunchKernelGGL(k_patch4, dim3((unsigned)((pp.size() + 3) / 4)), dim3(256), 0, 0, d, pitch, dp,
                     (int)pp.size(), o);
  hipLaunchKernelGGL(k_stream4, dim3(4096), dim3(256), 0, 0, (const uint32_t*)(d + gib), gib / 4, o);
  hipLaunchKernelGGL(k_tile16, dim3((unsigned)tp.size()), dim3(256), 0, 0, d, pitch, dt, (int)tp.size(), o);
  CK(hipDeviceSynchronize());
  printf("{\"k_stream16\": {\"bytes\": %zu}, \"k_stream4\": {\"bytes\": %zu}, "
         "\"k_patch4\": {\"patches\": %zu, \"sector64_bytes\": %zu, \"line128_bytes\": %zu, \"useful_bytes\": %zu}, "
         "\"k_tile16\": {\"tiles\": %zu, \"sector64_bytes\": %zu, \"line128_bytes\": %zu, \"useful_bytes\": %zu}}\n",
         gib, gib, pp.size(), s_sec.size() * 64, s_line.size() * 128, pp.size() * 43 * 48, tp.size(),
         t_sec.size() * 64, t_line.size() * 128, tp.size() * 37 * 288);
  return 0;
}
