// Host-side ASan/UBSan run of the C ABI's host code: geometry
// planning (geometry.cpp) over many sizes / parameter sets, the constant
// tables, the resize LUTs, and the argument validation of the matcher,
// vocabulary, stereo, projection and extractor entry points with malformed
// inputs.  Runs without a GPU (device entry points must fail cleanly with
// ORBX_ERR_NO_DEVICE after validating).  Built by `make sanitize`.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "orbx.h"

static int fails = 0;
#define EXPECT(cond)                                            \
  do {                                                          \
    if (!(cond)) {                                              \
      fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++fails;                                                  \
    }                                                           \
  } while (0)

int main() {
  // 1. geometry + tables + LUTs over a sweep of sizes and parameter sets
  const int sizes[][2] = {{640, 480}, {752, 480}, {1241, 376}, {1226, 370}, {1280, 720},
                          {1920, 1080}, {320, 240}, {97, 77}, {2048, 64}, {64, 2048}, {4000, 3000}};
  const float scales[] = {1.2f, 1.3f, 1.1f, 1.5f, 1.9f};
  long long ok = 0, rejected = 0;
  for (auto& s : sizes)
    for (float sc : scales)
      for (int L = 1; L <= 12; L += 3)
        for (int guard = 0; guard < 2; ++guard) {
          orbx_params p = {1000 + 100 * L, sc, L, 20, 7, guard};
          orbx_geometry g;
          const int rc = orbx_geometry_compute(&p, s[0], s[1], &g);
          if (rc != ORBX_OK) {
            ++rejected;
            continue;
          }
          ++ok;
          std::vector<float> a(L), b(L), c(L), d(L);
          std::vector<int> f(L);
          int umax[16];
          EXPECT(orbx_tables(&p, a.data(), b.data(), c.data(), d.data(), f.data(), umax) == ORBX_OK);
          for (int l = 1; l < L; ++l) {
            if (g.alias[l] != l) continue;
            std::vector<int32_t> xo(g.width[l]), yo(g.height[l]);
            std::vector<int16_t> al(2 * g.width[l]), be(2 * g.height[l]);
            EXPECT(orbx_resize_tables(&p, s[0], s[1], l, xo.data(), al.data(), yo.data(), be.data()) ==
                   ORBX_OK);
          }
        }
  EXPECT(ok > 50);
  // 2. argument validation (no device needed)
  orbx_params bad = {1000, 0.5f, 8, 20, 7, 0};
  orbx_geometry g;
  EXPECT(orbx_geometry_compute(&bad, 640, 480, &g) != ORBX_OK);
  EXPECT(orbx_geometry_compute(nullptr, 640, 480, &g) == ORBX_ERR_ARG);
  EXPECT(orbx_tables(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) == ORBX_ERR_ARG);
  uint8_t desc[4 * 32] = {0};
  float ang[4] = {0};
  uint32_t ids_unsorted[2] = {5, 3}, off[3] = {0, 2, 4}, feat[4] = {0, 1, 2, 3};
  uint32_t ids[2] = {3, 5}, feat_bad[4] = {0, 1, 2, 9};
  orbx_bow_frame f1 = {4, desc, ang, nullptr, 2, ids_unsorted, off, feat};
  orbx_bow_frame f2 = {4, desc, ang, nullptr, 2, ids, off, feat_bad};
  orbx_bow_frame f3 = {4, desc, ang, nullptr, 2, ids, off, feat};
  int32_t m12[4];
  int nm = 0;
  EXPECT(orbm_search_by_bow(&f1, &f3, 0.6f, 1, 0, m12, &nm) == ORBX_ERR_ARG);  // std::map key order
  EXPECT(orbm_search_by_bow(&f3, &f2, 0.6f, 1, 0, m12, &nm) == ORBX_ERR_ARG);  // feature index range
  EXPECT(orbm_search_by_bow(&f3, &f3, 0.6f, 1, 0, nullptr, &nm) == ORBX_ERR_ARG);
  const int rc_ok = orbm_search_by_bow(&f3, &f3, 0.6f, 1, 0, m12, &nm);
  EXPECT(rc_ok == ORBX_ERR_NO_DEVICE || rc_ok == ORBX_OK);
  int32_t ia[2] = {0, 7}, ib[2] = {0, 1}, dist[2];
  EXPECT(orbm_descriptor_distance_batch(desc, 4, desc, 4, ia, ib, 2, 0, dist) == ORBX_ERR_ARG);
  EXPECT(orbx_stereo_match(nullptr, nullptr, nullptr, nullptr, 0, nullptr, nullptr, 0, 0, 0, nullptr,
                           nullptr, nullptr) == ORBX_ERR_ARG);
  EXPECT(orbm_search_by_projection(4, nullptr, nullptr, nullptr, 0, 0.6f, 100, 1, 0, nullptr, &nm) ==
         ORBX_ERR_ARG);
  int32_t off_bad[3] = {0, 5, 3}, best[2];
  EXPECT(orbm_compute_distinctive_descriptors(desc, off_bad, 2, 0, best) == ORBX_ERR_ARG);
  orbx_keypoint kp[2];
  memset(kp, 0, sizeof(kp));
  float K[9] = {500, 0, 320, 0, 500, 240, 0, 0, 1}, D[5] = {0, 0, 0, 0, 0};
  orbx_keypoint kout[2];
  EXPECT(orbx_undistort_keypoints(kp, 2, K, D, 5, 0, kout) == ORBX_OK);  // k1 == 0: host copy
  EXPECT(orbx_undistort_keypoints(kp, 2, K, D, 15, 0, kout) == ORBX_ERR_ARG);
  EXPECT(orbx_extract(nullptr, nullptr, 0, 0, 0, nullptr, 0, nullptr, nullptr) == ORBX_ERR_ARG);
  orbv_vocab* v = nullptr;
  EXPECT(orbv_vocab_load_text("/nonexistent/voc.txt", 0, &v) != ORBX_OK);
  int32_t parent[2] = {0, 7};
  int32_t leaf[2] = {1, 1};
  double w[2] = {1, 1};
  EXPECT(orbv_vocab_create(10, 6, 0, 0, 2, parent, leaf, desc, w, 0, &v) != ORBX_OK);
  for (int s = -2; s < 12; ++s) EXPECT(orbx_status_string(s) != nullptr);
  printf("sanitize: %lld geometries planned, %lld rejected, %d failures\n", ok, rejected, fails);
  return fails ? 1 : 0;
}
