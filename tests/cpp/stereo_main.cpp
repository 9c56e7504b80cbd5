// Drive orbx::ComputeStereoMatches the way Frame's stereo constructor does
// (src/Frame.cc:58-70): two extractors, one per image, then the stereo search.
// Used by tests/test_cpp_adapter.py.
//   stereo_main left.raw right.raw W H nfeatures fx bf out.bin
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
  const int W = atoi(argv[3]), H = atoi(argv[4]), nf = atoi(argv[5]);
  const float fx = (float)atof(argv[6]), bf = (float)atof(argv[7]);
  auto l = load(argv[1], (size_t)W * H), r = load(argv[2], (size_t)W * H);
  orbx::ORBextractor left(nf, 1.2f, 8, 20, 7), right(nf, 1.2f, 8, 20, 7);
  std::vector<orbx::KeyPoint> kl, kr;
  std::vector<uint8_t> dl, dr;
  orbx::ImageView none;
  left(orbx::ImageView{l.data(), W, H, (size_t)W}, none, kl, dl);
  right(orbx::ImageView{r.data(), W, H, (size_t)W}, none, kr, dr);
  std::vector<float> ur, depth;
  const float mb = bf / fx;  // Frame.cc:94
  int n = orbx::ComputeStereoMatches(left, right, kl, dl, kr, dr, mb, bf, ur, depth);
  FILE* o = fopen(argv[8], "wb");
  int hdr[3] = {(int)kl.size(), (int)kr.size(), n};
  fwrite(hdr, sizeof(int), 3, o);
  fwrite(ur.data(), sizeof(float), ur.size(), o);
  fwrite(depth.data(), sizeof(float), depth.size(), o);
  fclose(o);
  printf("stereo ok: NL=%zu NR=%zu kept=%d\n", kl.size(), kr.size(), n);
  return 0;
}
