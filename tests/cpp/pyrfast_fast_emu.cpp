// Functional emulation of k_pyrfast's FAST half (kernels_stream.hip) on the
// planner's tables (geometry.cpp plan_pyr_fast): the strength A of every
// detection pixel, the corner bitmap (A > min(ini, min) thresholds), the NMS
// of each row in the two cell-column halves (cv::FAST's strict 3x3 test
// within the cell's zone, at iniThFAST and minThFAST), the raster-order emit
// into the per-cell minThFAST / iniThFAST lists with running counts, and the
// per-cell choice at each cell row's end (ORBX_CC_HI).  The concatenated cell
// lists of every level must equal the oracle's vToDistributeKeys
// (ORBextractor.cc:305-340, oo_level_candidates) key for key, and no list may
// pass its cell's slot capacity.
// usage: pyrfast_fast_emu in.raw W H nfeatures nlevels scale ini min
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "geometry.h"
extern "C" {
#include "orb_oracle.h"
}

using namespace orbx;

static void fail(const char* m, int a, int b, int c) {
  fprintf(stderr, "FAIL %s %d %d %d\n", m, a, b, c);
  exit(2);
}

static int strength(const uint8_t* img, int pitch, int x, int y) {
  static const int dx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
  static const int dy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
  int I[16];
  for (int k = 0; k < 16; ++k) I[k] = img[(y + dy[k]) * pitch + x + dx[k]];
  const int v = img[y * pitch + x];
  int Mb = 0, Md = 255;
  for (int s = 0; s < 16; ++s) {
    int mn = 255, mx = 0;
    for (int k = 0; k < 9; ++k) {
      mn = std::min(mn, I[(s + k) & 15]);
      mx = std::max(mx, I[(s + k) & 15]);
    }
    Mb = std::max(Mb, mn);
    Md = std::min(Md, mx);
  }
  return std::max(0, std::max(Mb - v, v - Md));
}

int main(int argc, char** argv) {
  if (argc < 9) return 1;
  const int W = atoi(argv[2]), H = atoi(argv[3]), ini = atoi(argv[7]), mn = atoi(argv[8]);
  orbx_params prm = {atoi(argv[4]), (float)atof(argv[6]), atoi(argv[5]), ini, mn, 1};
  std::vector<uint8_t> img((size_t)W * H);
  FILE* f = fopen(argv[1], "rb");
  if (!f || fread(img.data(), 1, img.size(), f) != img.size()) return 1;
  fclose(f);
  Plan P;
  if (plan_geometry(prm, W, H, P)) return 3;
  if (!P.pf_ok) { printf("no fused plan\n"); return 4; }
  oo_extractor* e = oo_create(prm.nfeatures, prm.scale_factor, prm.nlevels, ini, mn, 1);
  int n = 0;
  std::vector<oo_keypoint> kp(P.kcap + 16);
  std::vector<uint8_t> desc(32 * (P.kcap + 16));
  if (oo_extract(e, img.data(), W, H, W, kp.data(), (int)kp.size(), desc.data(), &n)) return 5;
  const PyrFast& F = P.pf;
  const int t_lo = std::min(P.ini_th, P.min_th);
  long long total = 0;
  for (int p = 0; p < F.np; ++p) {
    const PyrFastPass& Q = F.p[p];
    if (!Q.fast) continue;
    int lw, lh;
    oo_level_size(e, Q.lev, &lw, &lh);
    if (lw != Q.w || lh != Q.h) fail("level size", p, lw, lh);
    const uint8_t* L = oo_level_pixels(e, Q.lev);
    std::vector<int> A((size_t)Q.w * Q.h, 0);
    for (int y = Q.y0; y < Q.y1; ++y)
      for (int x = Q.c0; x < Q.c1; ++x) {
        const int a = strength(L, Q.w, x, y);
        A[(size_t)y * Q.w + x] = a > t_lo ? a : 0;
      }
    const int ncell = Q.ncv * Q.nrv;
    std::vector<std::vector<uint32_t>> lo(ncell), hi(ncell);
    std::vector<uint32_t> cc(ncell, 0xFFFFFFFFu);
    for (int half = 0; half < (Q.ncv > 1 ? 2 : 1); ++half) {
      const int jc0 = half ? Q.ncv >> 1 : 0, jc1 = (half || Q.ncv == 1) ? Q.ncv : Q.ncv >> 1;
      const int xa = Q.c0 + jc0 * Q.wcell, xb = jc1 == Q.ncv ? Q.c1 : Q.c0 + jc1 * Q.wcell;
      for (int y = Q.y0; y < Q.y1; ++y) {
        const int ci = (y - Q.y0) / Q.hcell;
        const int zy0 = Q.y0 + ci * Q.hcell, zy1 = ci == Q.nrv - 1 ? Q.y1 : zy0 + Q.hcell;
        for (int x = xa; x < xb; ++x) {
          const int a = A[(size_t)y * Q.w + x];
          if (!a) continue;
          const int jc = std::min((int)(((float)(x - Q.c0) + 0.5f) * (1.0f / (float)Q.wcell)), Q.ncv - 1);
          if (jc < jc0 || jc >= jc1) fail("corner outside its half", x, y, jc);
          const int zx0 = Q.c0 + jc * Q.wcell, zx1 = jc == Q.ncv - 1 ? Q.c1 : zx0 + Q.wcell;
          if (x < zx0 || x >= zx1) fail("cell of corner", x, y, jc);
          int nbi = 0, nbm = 0;
          for (int ddy = -1; ddy <= 1; ++ddy)
            for (int ddx = -1; ddx <= 1; ++ddx) {
              if (!ddx && !ddy) continue;
              const int yy = y + ddy, xx = x + ddx;
              const int aq = (yy >= zy0 && yy < zy1 && xx >= zx0 && xx < zx1) ? A[(size_t)yy * Q.w + xx] : 0;
              nbm = std::max(nbm, aq > mn ? aq - 1 : 0);
              nbi = std::max(nbi, aq > ini ? aq - 1 : 0);
            }
          const uint32_t key = orbx_pack_key((uint32_t)(x - 16), (uint32_t)(y - 16), (uint32_t)a - 1u, F.key_xs);
          if (a > mn && a - 1 > nbm) lo[ci * Q.ncv + jc].push_back(key);
          if (a > ini && a - 1 > nbi) hi[ci * Q.ncv + jc].push_back(key);
        }
        if (y == zy1 - 1)
          for (int jc = jc0; jc < jc1; ++jc) {
            const int c = ci * Q.ncv + jc;
            cc[c] = hi[c].size() ? ((uint32_t)hi[c].size() | ORBX_CC_HI) : (uint32_t)lo[c].size();
          }
      }
    }
    std::vector<uint32_t> got;
    for (int c = 0; c < ncell; ++c) {
      if (cc[c] == 0xFFFFFFFFu) fail("cell count never written", p, c, 0);
      const std::vector<uint32_t>& v = (cc[c] & ORBX_CC_HI) ? hi[c] : lo[c];
      if ((int)lo[c].size() > P.cells[Q.cell_begin + c].slot_cap || (int)hi[c].size() > P.cells[Q.cell_begin + c].slot_cap)
        fail("slot capacity", p, c, (int)lo[c].size());
      got.insert(got.end(), v.begin(), v.end());
    }
    const int nref = oo_level_candidates(e, Q.lev, nullptr, 0);
    std::vector<oo_keypoint> ref(nref + 1);
    oo_level_candidates(e, Q.lev, ref.data(), nref);
    if ((int)got.size() != nref) fail("candidate count", p, (int)got.size(), nref);
    for (int i = 0; i < nref; ++i) {
      const uint32_t k = got[i];
      if (orbx_key_x(k, F.key_xs) != (int)ref[i].x || orbx_key_y(k, F.key_xs) != (int)ref[i].y ||
          (int)(k & 0xFF) != (int)ref[i].response)
        fail("candidate", p, i, orbx_key_x(k, F.key_xs));
    }
    total += nref;
  }
  printf("ok candidates %lld\n", total);
  oo_destroy(e);
  return 0;
}
