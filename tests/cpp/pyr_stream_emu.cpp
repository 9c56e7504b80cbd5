// CPU emulation of k_pyr_stream (kernels_stream.hip) on the host planner's
// tables (geometry.cpp plan_pyr_stream): tick by tick, every task reads its
// source rows from the LDS rings exactly as the kernel indexes them (column
// LUT entries, ring slots of the row LUT), and every ring slot carries the
// (row, tick) it was written in.  Trapped: a read of a slot that does not hold
// the expected row, a read of a row written in the same tick (no barrier
// between them), a slot written twice in one tick or written while read in
// the same tick, a level row computed twice or never.  Writes the unique
// levels to argv[7] for the oracle comparison in tests/test_host.py.
// usage: pyr_stream_emu in.raw W H nfeatures nlevels scale out.bin [r0 rpt]
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "geometry.h"

using namespace orbx;

static void fail(const char* m, int a, int b, int c) {
  fprintf(stderr, "FAIL %s %d %d %d\n", m, a, b, c);
  exit(2);
}

struct Slot {
  int row = -1, tick = -1;
  int rtick = -1;  // last tick it was read in
};

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
  if (argc >= 10 && !plan_pyr_stream(P, atoi(argv[8]), atoi(argv[9]))) { printf("no stream plan\n"); return 4; }
  if (!P.ps_ok) { printf("no stream plan\n"); return 4; }
  const PyrStream& S = P.ps;
  if (S.lds_bytes > ORBX_PS_LDS_MAX) fail("lds", S.lds_bytes, 0, 0);
  const int n = S.nl;
  // LDS image: rings as bytes plus per-slot tags
  std::vector<std::vector<uint8_t>> ring(n);
  std::vector<std::vector<Slot>> tag(n);
  for (int j = 0; j < n; ++j) {
    ring[j].assign((size_t)S.rrows[j] * S.rpitch[j] + 16, 0xCD);
    tag[j].assign(S.rrows[j], Slot());
  }
  std::vector<uint8_t> pyr(P.pyr_bytes + 16, 0xCD);
  std::vector<std::vector<int>> done(n);
  for (int j = 0; j < n; ++j) done[j].assign(S.h[j], 0);
  const uint32_t* xl = P.ps_xlut.data();
  const uint32_t* yl = P.ps_ylut.data();
  auto rd_slot = [&](int j, int slot, int want_row, int k) {
    Slot& s = tag[j][slot];
    if (s.row != want_row) fail("slot holds another row", j, slot, want_row);
    if (s.tick >= k) fail("row read in the tick it was written", j, want_row, k);
    s.rtick = k;
  };
  auto wr_slot = [&](int j, int slot, int row, int k) {
    Slot& s = tag[j][slot];
    if (s.tick == k && s.row != row) fail("slot written twice in a tick", j, slot, k);
    if (s.rtick == k) fail("slot written in a tick that reads it", j, slot, k);
    s.row = row;
    s.tick = k;
  };
  int t0 = 0;
  for (int k = 0; k < S.nticks; ++k) {
    // workers: the tick's tasks (the kernel runs them concurrently; every read
    // is checked against rows of earlier ticks, every write against this
    // tick's reads -- reads first, then writes, then re-check the writes)
    struct Wr { int j, slot, row; };
    std::vector<Wr> writes;
    const int t1 = P.ps_tick_end[k];
    for (int t = t0; t < t1; ++t) {
      const uint32_t x = P.ps_tasks[2 * t], y0 = P.ps_tasks[2 * t + 1];
      if ((x & 15) != ORBX_PS_RESIZE) fail("task type", t, 0, 0);
      const int j = (x >> 4) & 31, c = (x >> 9) & 127, nr = (x >> 16) & 255;
      if (j < 1 || j >= n) fail("task level", t, j, 0);
      const LevelInfo& lv = P.levels[S.lev[j]];
      const int sh = S.h[j - 1];
      for (int r = 0; r < nr; ++r) {
        const int y = (int)y0 + r;
        if (y >= S.h[j]) fail("row past level", j, y, 0);
        const uint32_t ex = yl[2 * (S.yl[j] + y)], ey = yl[2 * (S.yl[j] + y) + 1];
        const int sa = ex & 0xFF, sb = (ex >> 8) & 0xFF, sd = (ex >> 16) & 0xFF;
        const int sy = P.yofs[lv.lut_y + y];
        const int s0 = std::min(std::max(sy, 0), sh - 1), s1 = std::min(std::max(sy + 1, 0), sh - 1);
        if (sa != s0 % S.rrows[j - 1] || sb != s1 % S.rrows[j - 1] || sd != y % S.rrows[j]) fail("row lut", j, y, 0);
        rd_slot(j - 1, sa, s0, k);
        rd_slot(j - 1, sb, s1, k);
        const int b0 = ey & 0xFFF, b1 = (ey >> 16) & 0xFFF;
        for (int l = 0; l < 64; ++l) {
          const int g = c * 64 + l;
          if (g >= S.ng[j]) break;
          const uint32_t* e = xl + 2 * (S.xl[j] + 4 * g);
          const int g0 = e[0] & 0xFFFF;
          uint8_t out[4];
          for (int q = 0; q < 4; ++q) {
            int lo, hi;
            if (q == 0) { lo = g0; hi = g0 + (int)(e[0] >> 16); }
            else { lo = g0 + (int)(e[2 * q] & 0xFF); hi = g0 + (int)((e[2 * q] >> 16) & 0xFF); }
            const uint32_t cf = e[2 * q + 1];
            const int a0 = cf & 0xFFFF, a1 = cf >> 16;
            if (lo >= S.w[j - 1] || hi >= S.w[j - 1]) fail("column past source row", j, g, q);
            if (lo < g0 || lo - g0 > 7 || hi < g0 || hi - g0 > 7) fail("8-byte window", j, g, q);
            const uint8_t* R0 = &ring[j - 1][(size_t)sa * S.rpitch[j - 1]];
            const uint8_t* R1 = &ring[j - 1][(size_t)sb * S.rpitch[j - 1]];
            const int D0 = (R0[lo] * a0 + R0[hi] * a1) & 0xFFFFF0, D1 = (R1[lo] * a0 + R1[hi] * a1) & 0xFFFFF0;
            const int v = (int)((((long long)(b0 << 12) * D0) >> 32) + (((long long)(b1 << 12) * D1) >> 32) + 2) >> 2;
            out[q] = (uint8_t)v;
          }
          memcpy(&ring[j][(size_t)sd * S.rpitch[j] + 4 * g], out, 4);
          for (int q = 0; q < 4; ++q) {
            const int xx = 4 * g + q;
            if (xx < S.w[j]) pyr[lv.pyr_off + (size_t)y * lv.pitch + xx] = out[q];
            else if (xx >= lv.pitch) fail("store past pitch", j, y, xx);
          }
        }
        if (c == 0) {
          if (done[j][y]) fail("row computed twice", j, y, 0);
          done[j][y] = 1;
        }
        writes.push_back({j, sd, y});
      }
    }
    // loader: level-0 rows of this tick
    const int a = std::min(S.h[0], S.r0 * k), b = std::min(S.h[0], S.r0 * (k + 1));
    for (int y = a; y < b; ++y) {
      memcpy(&ring[0][(size_t)(y % S.rrows[0]) * S.rpitch[0]], &img[(size_t)y * W], W);
      writes.push_back({0, y % S.rrows[0], y});
      done[0][y] = 1;
    }
    for (const Wr& w : writes) wr_slot(w.j, w.slot, w.row, k);
    t0 = t1;
  }
  if (t0 != (int)(P.ps_tasks.size() / 2)) fail("tasks after the last tick", t0, 0, 0);
  for (int j = 0; j < n; ++j)
    for (int y = 0; y < S.h[j]; ++y)
      if (!done[j][y]) fail("row never computed", j, y, 0);
  FILE* o = fopen(argv[7], "wb");
  for (int j = 1; j < n; ++j) {
    const LevelInfo& lv = P.levels[S.lev[j]];
    for (int y = 0; y < lv.h; ++y) fwrite(&pyr[lv.pyr_off + (size_t)y * lv.pitch], 1, lv.w, o);
  }
  fclose(o);
  printf("ok ticks %d tasks %zu lds %d r0 %d rings", S.nticks, P.ps_tasks.size() / 2, S.lds_bytes, S.r0);
  for (int j = 0; j < n; ++j) printf(" %d", S.rrows[j]);
  printf("\n");
  return 0;
}
