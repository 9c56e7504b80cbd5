// Drive orbx::ORBVocabulary the way Frame::ComputeBoW / LoopClosing do:
// load ORBvoc-format text, transform two frames' descriptors (levelsup 4),
// SearchByBoW on the resulting FeatureVectors.  Used by tests/test_cpp_adapter.py.
//   vocab_main voc.txt a.raw b.raw W H out.bin
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
  if (argc != 7) return 2;
  const int W = atoi(argv[4]), H = atoi(argv[5]);
  auto a = load(argv[2], (size_t)W * H), b = load(argv[3], (size_t)W * H);
  orbx::ORBVocabulary voc;
  if (!voc.loadFromTextFile(argv[1]) || voc.empty()) { fprintf(stderr, "vocab\n"); return 3; }
  orbx::ORBextractor ex(2000, 1.2f, 8, 20, 7);
  std::vector<orbx::KeyPoint> k1, k2;
  std::vector<uint8_t> d1, d2;
  orbx::ImageView none;
  ex(orbx::ImageView{a.data(), W, H, (size_t)W}, none, k1, d1);
  ex(orbx::ImageView{b.data(), W, H, (size_t)W}, none, k2, d2);
  orbx::BowVector bv1, bv2;
  orbx::FeatureVector f1, f2;
  voc.transform(d1.data(), (int)k1.size(), bv1, f1, 4);
  voc.transform(d2.data(), (int)k2.size(), bv2, f2, 4);
  std::vector<float> a1, a2;
  for (auto& k : k1) a1.push_back(k.angle);
  for (auto& k : k2) a2.push_back(k.angle);
  orbx::ORBmatcher m(0.75f, true);
  std::vector<int32_t> m12;
  int nm = m.SearchByBoW({d1.data(), a1.data(), nullptr, (int)k1.size(), &f1},
                         {d2.data(), a2.data(), nullptr, (int)k2.size(), &f2}, m12);
  FILE* o = fopen(argv[6], "wb");
  int hdr[4] = {(int)k1.size(), (int)bv1.word.size(), (int)f1.node_id.size(), nm};
  fwrite(hdr, sizeof(int), 4, o);
  fwrite(bv1.word.data(), 4, bv1.word.size(), o);
  fwrite(bv1.value.data(), 8, bv1.value.size(), o);
  fwrite(f1.node_id.data(), 4, f1.node_id.size(), o);
  fwrite(f1.node_off.data(), 4, f1.node_off.size(), o);
  fwrite(f1.feat.data(), 4, f1.feat.size(), o);
  fwrite(m12.data(), 4, m12.size(), o);
  fclose(o);
  printf("vocab ok: K1=%zu words=%zu nodes=%zu matches=%d\n", k1.size(), bv1.word.size(),
         f1.node_id.size(), nm);
  return 0;
}
