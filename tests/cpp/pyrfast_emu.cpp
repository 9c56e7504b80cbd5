// Schedule check of k_pyrfast (kernels_stream.hip) on the host planner's
// tables (geometry.cpp plan_pyr_fast): tick by tick and phase by phase,
// every read of the level ring (stage A windows, resize source rows, stage C
// windows in phase 2), of the strength ring and of the corner bitmaps (NMS)
// must find the row it expects, written in an earlier tick (strength rows:
// zero-filled and completed by stage C in earlier ticks), and no slot may be
// written in a phase that reads it.  Every detection row is tested once and
// NMS'd once after its neighbours, every next-level row resized once.
// usage: pyrfast_emu W H nfeatures nlevels scale
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "geometry.h"

using namespace orbx;

static void fail(const char* m, int a, int b, int c) {
  fprintf(stderr, "FAIL %s %d %d %d\n", m, a, b, c);
  exit(2);
}

struct Tag {
  int row = -1, tick = -1, phase = -1;  // last write
  int rtick = -1, rphase = -1;          // last read
};

int main(int argc, char** argv) {
  if (argc < 6) return 1;
  orbx_params prm = {atoi(argv[3]), (float)atof(argv[5]), atoi(argv[4]), 20, 7, 1};
  Plan P;
  if (plan_geometry(prm, atoi(argv[1]), atoi(argv[2]), P)) return 3;
  if (!P.pf_ok) { printf("no fused plan\n"); return 4; }
  const PyrFast& F = P.pf;
  if (F.lds_bytes > ORBX_PF_LDS_MAX) fail("lds", F.lds_bytes, 0, 0);
  int t0 = 0;
  for (int p = 0; p < F.np; ++p) {
    const PyrFastPass& Q = F.p[p];
    if (Q.tick0 != (p ? F.p[p - 1].tick0 + F.p[p - 1].nticks : 0)) fail("tick0", p, Q.tick0, 0);
    if ((long long)(Q.rrows + 6) * Q.rpitch > F.o_aring - F.o_ring) fail("ring bytes", p, 0, 0);
    if ((long long)Q.arows * Q.rpitch > F.o_bmap - F.o_aring) fail("strength ring bytes", p, 0, 0);
    if ((long long)Q.arows * Q.bmw * 4 > F.o_lut - F.o_bmap) fail("bitmap bytes", p, 0, 0);
    if (Q.next && (long long)Q.ng * 32 > F.o_cell - F.o_lut) fail("lut bytes", p, 0, 0);
    std::vector<Tag> ring(Q.rrows + 6), aring(Q.arows);
    std::vector<int> stA(Q.h, 0), stN(Q.h, 0), stR(Q.next ? Q.nh : 1, 0), aDone(Q.h, -1);
    const LevelInfo* nv = Q.next ? &P.levels[F.p[p + 1].lev] : nullptr;
    auto rd = [&](std::vector<Tag>& v, int slot, int row, int k, int ph, const char* what) {
      if (slot < 0 || slot >= (int)v.size()) fail(what, slot, row, k);
      Tag& t = v[slot];
      if (t.row != row) fail(what, slot, row, k);
      if (t.tick == k && t.phase == ph) fail("read of a slot written in the same phase", slot, row, k);
      t.rtick = k;
      t.rphase = ph;
    };
    struct W { std::vector<Tag>* v; int slot, row; };
    auto apply = [&](std::vector<W>& ws, int k, int ph) {
      for (W& w : ws) {
        Tag& t = (*w.v)[w.slot];
        if (t.rtick == k && t.rphase == ph && t.row != w.row) fail("slot written while read", w.slot, w.row, k);
        if (t.tick == k && t.phase == ph && t.row != w.row) fail("slot written twice", w.slot, w.row, k);
        t.row = w.row;
        t.tick = k;
        t.phase = ph;
      }
      ws.clear();
    };
    auto ring_rows = [&](int y, std::vector<int>& phys) {  // physical rows holding row y
      const int s = y % Q.rrows;
      phys.assign(1, s + 3);
      if (s < 3) phys.push_back(s + 3 + Q.rrows);
      if (s >= Q.rrows - 3) phys.push_back(s + 3 - Q.rrows);
    };
    std::vector<int> phys;
    for (int k = 0; k < Q.nticks; ++k) {
      const int T = Q.tick0 + k;
      std::vector<W> ws;
      std::vector<int> tickA;  // detection rows stage-A'd this tick
      const int t1 = P.pf_tick_end[2 * T], t2 = P.pf_tick_end[2 * T + 1];
      for (int t = t0; t < t2; ++t) {
        const int phase = t < t1 ? 1 : 2;
        const uint32_t x = P.pf_tasks[2 * t], yw = P.pf_tasks[2 * t + 1];
        const int type = x & 15, pp = (x >> 4) & 31, c = (x >> 9) & 127, nr = (x >> 16) & 255;
        if (pp != p) fail("task pass", t, pp, p);
        if ((type == ORBX_PS_RESIZE) != (phase == 2)) fail("task in the wrong phase", t, type, phase);
        if (type == ORBX_PF_FASTA) {
          const int ya = yw & 0x3FFF, sl = (yw >> 14) & 0xFF, as = (yw >> 22) & 0xFF;
          if (nr > 8 || c >= Q.nchunk) fail("fasta task", t, nr, c);
          if (sl != (ya - 3) % Q.rrows || as != ya % Q.arows) fail("fasta slots", t, ya, 0);
          for (int y = ya - 3; y < ya + nr + 3; ++y) {
            // column walk reads the primary copy; stages B / C read the
            // center's primary row +-3 (guard copies), in both phases
            rd(ring, y % Q.rrows + 3, y, k, 1, "stage A ring row");
          }
          for (int y = ya; y < ya + nr; ++y) {
            const int pc = y % Q.rrows + 3;
            for (int d = -3; d <= 3; ++d) rd(ring, pc + d, y + d, k, 1, "stage B window");
            if (c == 0) {
              if (y < Q.y0 || y >= Q.y1 || stA[y]) fail("stage A row", y, stA[y], k);
              stA[y] = 1;
              tickA.push_back(y);
            }
            ws.push_back({&aring, y % Q.arows, y});  // zero-fill
          }
        } else if (type == ORBX_PS_RESIZE) {
          if (!Q.next) fail("resize without next", t, 0, 0);
          const int y0 = (int)yw;
          for (int y = y0; y < y0 + nr; ++y) {
            if (y >= Q.nh) fail("resize row", y, 0, 0);
            const int sy = P.yofs[nv->lut_y + y];
            const int s0 = std::min(std::max(sy, 0), Q.h - 1), s1 = std::min(std::max(sy + 1, 0), Q.h - 1);
            const uint32_t e = P.pf_ylut[2 * (Q.yl + y)];
            if ((int)(e & 0xFF) != s0 % Q.rrows || (int)((e >> 8) & 0xFF) != s1 % Q.rrows) fail("row lut", y, 0, 0);
            rd(ring, s0 % Q.rrows + 3, s0, k, 2, "resize source");
            rd(ring, s1 % Q.rrows + 3, s1, k, 2, "resize source");
            if (c == 0) {
              if (stR[y]) fail("row resized twice", y, 0, 0);
              stR[y] = 1;
            }
          }
        } else if (type == ORBX_PF_NMS) {
          const int y0 = yw & 0x3FFF, as = (yw >> 22) & 0xFF;
          if (as != y0 % Q.arows) fail("nms slot", y0, as, 0);
          if (c > 1 || (Q.ncv == 1 && c)) fail("nms half", c, Q.ncv, 0);
          for (int y = y0; y < y0 + nr; ++y) {
            if (y < Q.y0 || y >= Q.y1 || (stN[y] >> c) & 1) fail("nms row", y, c, k);
            if (y > Q.y0 && !((stN[y - 1] >> c) & 1)) fail("nms out of order", y, c, k);
            stN[y] |= 1 << c;
            for (int d = -1; d <= 1; ++d) {
              const int yy = y + d;
              if (yy < Q.y0 || yy >= Q.y1) continue;
              if (aDone[yy] < 0 || aDone[yy] >= k) fail("strength row not final", yy, y, k);
              rd(aring, yy % Q.arows, yy, k, 1, "nms strength row");
            }
          }
        } else {
          fail("task type", t, type, 0);
        }
      }
      t0 = t2;
      apply(ws, k, 1);
      // phase 2: stage C on this tick's rows (windows and strength rows), loader rows
      for (int y : tickA) {
        const int pc = y % Q.rrows + 3;
        for (int d = -3; d <= 3; ++d) rd(ring, pc + d, y + d, k, 2, "stage C window");
        aDone[y] = k;
      }
      const int a = std::min(Q.h, Q.R * k), b = std::min(Q.h, Q.R * (k + 1));
      for (int y = a; y < b; ++y) {
        ring_rows(y, phys);
        // the loader writes during phase 1 (and is done before its end): its
        // slots must be read neither in phase 1 nor in phase 2 of this tick
        for (int s : phys) {
          Tag& t = ring[s];
          if (t.rtick == k) fail("loader overwrites a row read this tick", s, y, k);
          ws.push_back({&ring, s, y});
        }
      }
      apply(ws, k, 0);
    }
    const int halves = Q.ncv > 1 ? 3 : 1;
    for (int y = Q.y0; Q.fast && y < Q.y1; ++y)
      if (!stA[y] || stN[y] != halves) fail("detection row not processed", p, y, stA[y] * 4 + stN[y]);
    for (int y = 0; Q.next && y < Q.nh; ++y)
      if (!stR[y]) fail("next-level row not resized", p, y, 0);
  }
  if (t0 != (int)(P.pf_tasks.size() / 2)) fail("tasks left", t0, 0, 0);
  printf("ok passes %d ticks %zu tasks %zu lds %d\n", F.np, P.pf_tick_end.size() / 2, P.pf_tasks.size() / 2,
         F.lds_bytes);
  return 0;
}
