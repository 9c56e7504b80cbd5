// Exhaustive device check of the rotated-BRIEF sin/cos:
// for EVERY float x in [0, f32(360 * factorPI)] -- every angle the reference
// feeds to sincosf at src/ORBextractor.cc:58-59 -- the device's (sin, cos)
// (orbx_selftest_sincos_range: orbx_sincos_core + the exception table, run
// on the GPU) must produce the same 364 live BRIEF sample positions
// (ORBextractor.cc:54, FMA form) as this host's glibc sincosf.  Also counts
// raw bitwise differences (expected: glibc is not correctly rounded) and
// exceptions hit.  Writes a one-line JSON summary; exit 1 on any
// position-changing difference.
//   sincos_exhaustive out.json [threads]
#include <gnu/libc-version.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <string>
#include <chrono>
#include <thread>
#include <vector>

#include "orbx.h"
#include "../../orb-slam-system_amd/csrc/orbx_sincos.h"
#define ORBX_BRIEF_STORAGE static const
#include "../../orb-slam-system_amd/csrc/brief_pattern.inc"
#define ORBX_SINCOS_STORAGE static const
#include "../../orb-slam-system_amd/csrc/sincos_exceptions.inc"

static int positions_differ(float s0, float c0, float s1, float c1) {
  for (int p = 0; p < 256; ++p)
    for (int e = 0; e < 2; ++e) {
      const float px = (float)ORBX_BRIEF_PATTERN[p][2 * e], py = (float)ORBX_BRIEF_PATTERN[p][2 * e + 1];
      const long r0 = lrintf(fmaf(px, s0, py * c0)), q0 = lrintf(fmaf(px, c0, -(py * s0)));
      const long r1 = lrintf(fmaf(px, s1, py * c1)), q1 = lrintf(fmaf(px, c1, -(py * s1)));
      if (r0 != r1 || q0 != q1) return 1;
    }
  return 0;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const int nth = argc > 2 ? atoi(argv[2]) : 16;
  const float factorPI = (float)(3.1415926535897932384626433832795 / 180.f);
  const uint32_t hi = orbx_f2u(360.0f * factorPI);
  const uint64_t total = (uint64_t)hi + 1;
  const int chunk = 1 << 25;
  std::vector<float> buf[2] = {std::vector<float>(2 * (size_t)chunk), std::vector<float>(2 * (size_t)chunk)};
  std::atomic<uint64_t> n_diff{0}, n_move{0};
  uint64_t first_move = UINT64_MAX;
  std::atomic<uint64_t> first_move_a{UINT64_MAX};
  const auto t0 = std::chrono::steady_clock::now();
  // GPU fills chunk k+1 while the host threads check chunk k
  auto fill = [&](uint64_t start, int b) {
    const int n = (int)std::min<uint64_t>(chunk, total - start);
    return orbx_selftest_sincos_range((uint32_t)start, n, buf[b].data(), 0);
  };
  int rc = fill(0, 0);
  if (rc) { fprintf(stderr, "orbx_selftest_sincos_range: %s\n", orbx_status_string(rc)); return 2; }
  int cur = 0;
  for (uint64_t start = 0; start < total; start += chunk, cur ^= 1) {
    const int n = (int)std::min<uint64_t>(chunk, total - start);
    int rc_next = ORBX_OK;
    std::thread gpu([&] {
      if (start + chunk < total) rc_next = fill(start + chunk, cur ^ 1);
    });
    std::vector<std::thread> th;
    for (int t = 0; t < nth; ++t)
      th.emplace_back([&, t] {
        uint64_t d = 0, m = 0;
        for (int i = t; i < n; i += nth) {
          const uint32_t b = (uint32_t)(start + i);
          float gs, gc;
          sincosf(orbx_u2f(b), &gs, &gc);
          const float ds = buf[cur][2 * (size_t)i], dc = buf[cur][2 * (size_t)i + 1];
          if (orbx_f2u(gs) == orbx_f2u(ds) && orbx_f2u(gc) == orbx_f2u(dc)) continue;
          ++d;
          if (positions_differ(gs, gc, ds, dc)) {
            ++m;
            uint64_t prev = first_move_a.load();
            while (b < prev && !first_move_a.compare_exchange_weak(prev, b)) {}
          }
        }
        n_diff += d;
        n_move += m;
      });
    for (auto& x : th) x.join();
    gpu.join();
    if (rc_next) { fprintf(stderr, "orbx_selftest_sincos_range: %s\n", orbx_status_string(rc_next)); return 2; }
  }
  first_move = first_move_a.load();
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  FILE* f = fopen(argv[1], "w");
  fprintf(f,
          "{\"glibc\": \"%s\", \"inputs\": %llu, \"x_max_bits\": \"0x%08x\", "
          "\"bitwise_differences\": %llu, \"position_changing\": %llu, \"first_bad\": %s, "
          "\"exceptions_in_table\": %d, \"threads\": %d, \"seconds\": %.1f}\n",
          gnu_get_libc_version(), (unsigned long long)total, hi, (unsigned long long)n_diff.load(),
          (unsigned long long)n_move.load(),
          first_move == UINT64_MAX ? "null" : std::to_string(first_move).c_str(), ORBX_SINCOS_NEXC,
          nth, secs);
  fclose(f);
  printf("sincos exhaustive: %llu inputs, %llu bitwise differences, %llu position-changing, %.1f s\n",
         (unsigned long long)total, (unsigned long long)n_diff.load(), (unsigned long long)n_move.load(),
         secs);
  return n_move.load() ? 1 : 0;
}
