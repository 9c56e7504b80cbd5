// Exercise the C++ host mirror (orb-slam-system_amd/cpp/orbx.hpp) the way the
// reference's Frame/LoopClosing call sites do.  Used by tests/test_cpp_adapter.py.
//   adapter_main img1.raw img2.raw W H nfeatures nlevels cell_guard out.bin
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "orbx.hpp"

static std::vector<uint8_t> load(const char* p, size_t n) {
  std::vector<uint8_t> v(n);
  FILE* f = fopen(p, "rb");
  if (!f || fread(v.data(), 1, n, f) != n) { fprintf(stderr, "read %s\n", p); exit(2); }
  fclose(f);
  return v;
}

int main(int argc, char** argv) {
  if (argc != 9) return 2;
  const int W = atoi(argv[3]), H = atoi(argv[4]);
  auto a = load(argv[1], (size_t)W * H), b = load(argv[2], (size_t)W * H);
  orbx::ORBextractor ex(atoi(argv[5]), 1.2f, atoi(argv[6]), 20, 7, atoi(argv[7]));
  std::vector<orbx::KeyPoint> k1, k2;
  std::vector<uint8_t> d1, d2;
  orbx::ImageView none;
  ex(orbx::ImageView{a.data(), W, H, (size_t)W}, none, k1, d1);
  orbx::Image lvl = ex.ImagePyramid(ex.GetLevels() - 1);
  ex(orbx::ImageView{b.data(), W, H, (size_t)W}, none, k2, d2);
  // SearchByBoW with one vocabulary node holding every feature (brute force)
  orbx::FeatureVector f1, f2;
  for (uint32_t i = 0; i < k1.size(); ++i) f1.addFeature(7, i);
  for (uint32_t i = 0; i < k2.size(); ++i) f2.addFeature(7, i);
  std::vector<float> a1, a2;
  for (auto& k : k1) a1.push_back(k.angle);
  for (auto& k : k2) a2.push_back(k.angle);
  orbx::ORBmatcher m(0.75f, true);
  std::vector<int32_t> m12;
  int nm = m.SearchByBoW({d1.data(), a1.data(), nullptr, (int)k1.size(), &f1},
                         {d2.data(), a2.data(), nullptr, (int)k2.size(), &f2}, m12);
  int dist01 = k1.size() && k2.size() ? m.DescriptorDistance(d1.data(), d2.data()) : -1;
  FILE* o = fopen(argv[8], "wb");
  int hdr[6] = {(int)k1.size(), (int)k2.size(), nm, dist01, lvl.cols, lvl.rows};
  fwrite(hdr, sizeof(int), 6, o);
  fwrite(k1.data(), sizeof(orbx::KeyPoint), k1.size(), o);
  fwrite(d1.data(), 1, d1.size(), o);
  fwrite(m12.data(), sizeof(int32_t), m12.size(), o);
  fwrite(lvl.pixels.data(), 1, lvl.pixels.size(), o);
  fclose(o);
  std::vector<float> s = ex.GetScaleFactors();
  printf("adapter ok: K1=%zu K2=%zu matches=%d scale[1]=%g\n", k1.size(), k2.size(), nm, s.size() > 1 ? s[1] : 0.f);
  return 0;
}
