// CPU emulation of k_pyramid's tiling (kernels_extract.hip) on the host
// planner's tables (geometry.cpp): every tile of every segment is computed
// from its LDS regions only, exactly as the kernel indexes them, with
// out-of-region reads trapped.  Writes the unique levels to argv[7] for the
// oracle comparison in tests/test_host.py.
// usage: pyramid_emu in.raw W H nfeatures nlevels scale out.bin
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "geometry.h"

using namespace orbx;

static int fail(const char* m, int a, int b) {
  fprintf(stderr, "FAIL %s %d %d\n", m, a, b);
  exit(2);
}

int main(int argc, char** argv) {
  if (argc < 8) return 1;
  const int W = atoi(argv[2]), H = atoi(argv[3]);
  orbx_params prm = {atoi(argv[4]), (float)atof(argv[6]), atoi(argv[5]), 20, 7, 1};
  std::vector<uint8_t> img((size_t)W * H);
  FILE* f = fopen(argv[1], "rb");
  if (!f || fread(img.data(), 1, img.size(), f) != img.size()) return 1;
  fclose(f);
  Plan P;
  int rc = plan_geometry(prm, W, H, P);
  if (rc) { printf("rc %d\n", rc); return 3; }
  std::vector<uint8_t> pyr(P.pyr_bytes + 16, 0xCD);
  std::vector<uint8_t> owner(P.pyr_bytes + 16, 0);
  std::vector<std::pair<size_t, uint8_t>> shadow;  // non-owned bytes of edge dwords
  for (const PyrSeg& g : P.segs) {
    if (g.area) {  // k_pyr_area2: one exact-2x level, (a + b + c + d + 2) >> 2
      auto src = [&](int y, int x) {
        return g.off[0] < 0 ? (int)img[(size_t)y * W + x] : (int)pyr[g.off[0] + (size_t)y * g.pitch[0] + x];
      };
      for (int y = 0; y < g.h[1]; ++y)
        for (int x = 0; x < g.w[1]; ++x) {
          const size_t o = g.off[1] + (size_t)y * g.pitch[1] + x;
          pyr[o] = (uint8_t)((src(2 * y, 2 * x) + src(2 * y, 2 * x + 1) + src(2 * y + 1, 2 * x) +
                              src(2 * y + 1, 2 * x + 1) + 2) >> 2);
          owner[o] = 1;
        }
      continue;
    }
    if (g.lds_a + g.lds_b + g.lds_xl + g.lds_yl > ORBX_PYR_LDS_MAX) fail("lds total", 0, 0);
    for (int ty = 0; ty < g.nty; ++ty)
      for (int tx = 0; tx < g.ntx; ++tx) {
        const int xb = P.pyr_bo[g.xbo_off + tx], yb = P.pyr_bo[g.ybo_off + ty];
        if ((P.pyr_bo[g.xbo_off + tx + 1] - xb) * 8 > g.lds_xl) fail("xblob", tx, 0);
        if ((P.pyr_bo[g.ybo_off + ty + 1] - yb) * 8 > g.lds_yl) fail("yblob", ty, 0);
        if ((xb | yb) & 1) fail("blob align", xb, yb);
        int xo = 0, yo = 0;
        // staged source region (only [clo,chi) x rows valid; other bytes poisoned)
        const int* X = &P.pyr_xs[4 * (g.xs_off + tx)];
        const int* Y = &P.pyr_ys[4 * (g.ys_off + ty)];
        int cax = X[0] & ~15, cay = Y[0], cpitch = ((X[1] + 15) & ~15) - cax;
        int cx0 = X[0], cx1 = X[1], cy0 = Y[0], cy1 = Y[1];
        if ((long long)cpitch * (cy1 - cy0) > g.lds_a) fail("lds_a", tx, ty);
        if (cpitch > g.lpitch[0]) fail("lpitch 0", tx, cpitch);
        if ((long long)g.lpitch[0] * (cy1 - cy0) > g.lds_a) fail("lds_a (uniform pitch)", tx, ty);
        std::vector<int> cur((size_t)cpitch * (cy1 - cy0), -1);
        for (int r = cy0; r < cy1; ++r)
          for (int c = cx0; c < cx1; ++c) {
            int v = g.off[0] < 0 ? img[(size_t)r * W + c] : pyr[g.off[0] + (size_t)r * g.pitch[0] + c];
            cur[(size_t)(r - cay) * cpitch + c - cax] = v;
          }
        for (int s = 1; s <= g.nl; ++s) {
          X = &P.pyr_xs[4 * (g.xs_off + s * g.ntx + tx)];
          Y = &P.pyr_ys[4 * (g.ys_off + s * g.nty + ty)];
          const int dax = X[0] & ~3, ncg = (X[1] - dax + 3) >> 2, nrows = Y[1] - Y[0];
          const int dpitch = 4 * ncg;
          if ((long long)dpitch * nrows > ((s & 1) ? g.lds_b : g.lds_a)) fail("lds", s, tx);
          if (dpitch > g.lpitch[s] || (long long)g.lpitch[s] * nrows > ((s & 1) ? g.lds_b : g.lds_a))
            fail("lds (uniform pitch)", s, tx);
          if (ncg > 256) fail("ncg", ncg, s);
          std::vector<int> nxt((size_t)std::max(dpitch * nrows, 1), -1);
          const LevelInfo& lv = P.levels[g.lev[s]];
          for (int r = 0; r < nrows; ++r) {
            const int y = Y[0] + r;
            const uint32_t* ye = &P.pyr_blob[2 * (yb + yo + r)];
            // row entries: LDS byte offsets of the two source rows in level
            // s-1's buffer (k_pyramid's uniform pitch g.lpitch[s-1])
            const int lbase = ((s - 1) & 1) ? g.lds_a : 0, lp = g.lpitch[s - 1];
            const int o0 = (int)(ye[0] & 0xFFFF) - lbase, o1 = (int)(ye[0] >> 16) - lbase;
            if (lp <= 0 || o0 < 0 || o1 < 0 || o0 % lp || o1 % lp) fail("yblob offset", s, y);
            const int ry0 = o0 / lp, ry1 = o1 / lp;
            const int b0 = (int16_t)(ye[1] & 0xFFFF), b1 = (int16_t)(ye[1] >> 16);
            {  // blob vs the LUTs it packs
              const int sy = P.yofs[g.lut_y[s] + y], shm1 = g.h[s - 1] - 1;
              if (ry0 != std::min(std::max(sy, 0), shm1) - cay || ry1 != std::min(std::max(sy + 1, 0), shm1) - cay ||
                  b0 != P.beta[2 * (g.lut_y[s] + y)] || b1 != P.beta[2 * (g.lut_y[s] + y) + 1])
                fail("yblob entry", s, y);
            }
            for (int c = dax; c < dax + dpitch; ++c) {
              const uint32_t* xe = &P.pyr_blob[2 * (xb + xo + c - dax)];
              // x entries per 4-column group: column 0 = s0 | (sx1 - s0) << 16,
              // columns 1..3 = v_perm selectors (bytes 0 / 2) relative to s0
              const uint32_t g0 = P.pyr_blob[2 * (xb + xo + ((c - dax) & ~3))];
              const int s0 = g0 & 0xFFFF;
              const int sx = ((c - dax) & 3) ? s0 + (int)(xe[0] & 0xFF) : s0;
              const int sx1 = ((c - dax) & 3) ? s0 + (int)((xe[0] >> 16) & 0xFF) : s0 + (int)(xe[0] >> 16);
              const int a0 = (int16_t)(xe[1] & 0xFFFF), a1 = (int16_t)(xe[1] >> 16);
              auto rd = [&](int rr, int cc) {
                if (rr < 0 || rr >= cy1 - cay || cc < 0 || cc >= cpitch) fail("oob", rr, cc);
                int v = cur[(size_t)rr * cpitch + cc];
                if (v < 0) fail("uninit", rr + cay, cc + cax);
                return v;
              };
              const int gx0 = c & ~3;  // k_pyramid stores a group with an owned pixel as one dword
              const bool any_x = gx0 + 4 > X[2] && gx0 < X[3];
              if (c < X[0] || c >= X[1]) {  // pad columns: garbage in the kernel
                if (any_x && c < g.w[s]) fail("unsafe dword", y, c);
                continue;
              }
              const int d0 = rd(ry0, sx) * a0 + rd(ry0, sx1) * a1;
              const int d1 = rd(ry1, sx) * a0 + rd(ry1, sx1) * a1;
              const int v = (((b0 * (d0 >> 4)) >> 16) + ((b1 * (d1 >> 4)) >> 16) + 2) >> 2;
              nxt[(size_t)r * dpitch + c - dax] = v & 0xFF;
              if (y >= Y[2] && y < Y[3] && c >= X[2] && c < X[3]) {
                const size_t o = g.off[s] + (size_t)y * g.pitch[s] + c;
                if (owner[o]) fail("double write", y, c);
                owner[o] = 1;
                pyr[o] = (uint8_t)v;
              } else if (any_x && c < g.w[s]) {
                // a byte k_pyramid stores that this tile does not own (edge
                // group, or a computed row of another tile): must equal its owner's
                shadow.push_back({g.off[s] + (size_t)y * g.pitch[s] + c, (uint8_t)v});
              }
            }
          }
          (void)lv;
          xo += dpitch;
          yo += nrows;
          cur.swap(nxt);
          cax = dax; cay = Y[0]; cpitch = dpitch;
          cx0 = X[0]; cx1 = X[1]; cy0 = Y[0]; cy1 = Y[1];
        }
      }
  }
  for (const auto& sw : shadow)
    if (pyr[sw.first] != sw.second) fail("edge dword byte differs from its owner", (int)(sw.first >> 16), (int)(sw.first & 0xFFFF));
  FILE* o = fopen(argv[7], "wb");
  for (int l = 1; l < prm.nlevels; ++l) {
    const LevelInfo& lv = P.levels[l];
    if (lv.unique != l) continue;
    for (int y = 0; y < lv.h; ++y)
      for (int x = 0; x < lv.w; ++x)
        if (!owner[lv.pyr_off + (size_t)y * lv.pitch + x]) fail("unwritten", l, y * 100000 + x);
    for (int y = 0; y < lv.h; ++y) fwrite(&pyr[lv.pyr_off + (size_t)y * lv.pitch], 1, lv.w, o);
  }
  fclose(o);
  int nt = 0;
  for (const PyrSeg& g : P.segs) nt += g.ntx * g.nty;
  printf("segs %zu tiles %d lds %d+%d\n", P.segs.size(), nt, P.segs.empty() ? 0 : P.segs[0].lds_a,
         P.segs.empty() ? 0 : P.segs[0].lds_b);
  return 0;
}
