// fast_traffic_model -- byte model of k_fast_strips' staging (profiling aid).
// For every FAST strip of the plan: the algorithmic bytes (the strip's share
// of its level's pixels: scan band + 3-px rings counted once per level), the
// bytes the strip stages (tile rows x 16-B-aligned width, rings included),
// and the bytes of the 64-B / 128-B memory lines those rows touch.  Printed
// per 1080p frame; compare with profiles/traffic_c4.json (FETCH_SIZE x 2).
//   g++ -O1 -std=c++17 -I orb-slam-system_amd/csrc -I include tools/fast_traffic_model.cpp \
//       orb-slam-system_amd/csrc/geometry.cpp -o /tmp/ftm && /tmp/ftm [W H nfeatures]
#include <stdio.h>
#include <stdlib.h>

#include "geometry.h"

using namespace orbx;

int main(int argc, char** argv) {
  const int W = argc > 1 ? atoi(argv[1]) : 1920, H = argc > 2 ? atoi(argv[2]) : 1080;
  const int nf = argc > 3 ? atoi(argv[3]) : 2000;
  orbx_params p = {nf, 1.2f, 8, 20, 7, 1};
  Plan P;
  if (plan_geometry(p, W, H, P)) return 1;
  long long alg = 0, staged = 0, l64 = 0, l128 = 0, rows_staged = 0, rows_alg = 0;
  for (const LevelInfo& lv : P.levels)
    if (&lv - &P.levels[0] == lv.unique) alg += (long long)lv.w * lv.h;
  for (const StripInfo& st : P.strips) {
    const LevelInfo& lv = P.levels[st.level];
    const long long pitch = st.level == 0 ? W : lv.pitch;
    const int x0 = st.x & ~15, x1 = (st.x + st.w + 15) & ~15;  // aligned16 staging
    staged += (long long)st.h * (x1 - x0);
    rows_staged += st.h;
    rows_alg += st.h - 6;
    for (int r = 0; r < st.h; ++r) {
      const long long a = (st.y + r) * pitch + x0, b = (st.y + r) * pitch + x1;  // [a, b) bytes
      l64 += ((b + 63) / 64 - a / 64) * 64;
      l128 += ((b + 127) / 128 - a / 128) * 128;
    }
  }
  printf("{\"W\": %d, \"H\": %d, \"strips\": %zu, \"algorithmic_bytes\": %lld, \"staged_bytes\": %lld, "
         "\"line64_bytes\": %lld, \"line128_bytes\": %lld, \"row_ring_factor\": %.4f, "
         "\"staged_over_alg\": %.4f, \"line128_over_alg\": %.4f}\n",
         W, H, P.strips.size(), alg, staged, l64, l128, (double)rows_staged / rows_alg,
         (double)staged / alg, (double)l128 / alg);
  return 0;
}
