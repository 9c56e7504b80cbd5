/* geometry.cpp -- host planner.  Pure host C++ (no HIP calls); compiled into
 * liborbx.so so the CPU test-suite can check it without a GPU.
 *
 * Floating-point expressions are written with the same operand types and
 * evaluation order as the reference so the float/double roundings match
 * (build flag -ffp-contract=off). */
#include "geometry.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

namespace orbx {

static int round_f(float v) { return (int)lrintf(v); } /* cvRound(float), half-even */
static int round_d(double v) { return (int)lrint(v); }
static short sat_s16(int v) { return (short)std::min(32767, std::max(-32768, v)); }

int compute_tables(const orbx_params& p, Tables& t) {
  if (p.nlevels < 1 || p.nlevels > ORBX_MAX_LEVELS || p.nfeatures < 0 || !(p.scale_factor > 0.f))
    return ORBX_ERR_ARG;
  const int n = p.nlevels;
  t.nlevels = n;
  t.scaleFactor = (double)p.scale_factor; /* ORBextractor.h:78 double member */
  t.scale.assign(n, 1.0f);
  /* src/ORBextractor.cc:123-124: std::partial_sum(begin, end-1, begin+1, op)
   * writes d_first[0] = first[0] first, so scale[1] = scale[0] = 1 and
   * scale[i] = f32(scale[i-1] * (double)scaleFactor) for i >= 2. */
  if (n >= 2) {
    float acc = t.scale[0];
    t.scale[1] = acc;
    for (int i = 2; i < n; ++i) {
      acc = (float)((double)acc * t.scaleFactor);
      t.scale[i] = acc;
    }
  }
  t.sigma2.resize(n);
  t.inv_scale.resize(n);
  t.inv_sigma2.resize(n);
  for (int i = 0; i < n; ++i) {
    t.sigma2[i] = t.scale[i] * t.scale[i];
    t.inv_scale[i] = 1.0f / t.scale[i];
    t.inv_sigma2[i] = 1.0f / t.sigma2[i];
  }
  /* :141-151 features per level */
  t.features.assign(n, 0);
  const float factor = (float)(1.0f / t.scaleFactor);
  float desired = (float)((float)(p.nfeatures * (1 - factor)) / (1 - pow((double)factor, n)));
  int sum = 0;
  for (int l = 0; l < n - 1; ++l) {
    int cur = round_f(desired);
    sum += cur;
    desired *= factor;
    t.features[l] = cur;
  }
  t.features[n - 1] = std::max(p.nfeatures - sum, 0);
  /* :155-169 umax */
  const int half = 15;
  int vmax = (int)floorf(half * sqrtf(2.f) / 2 + 1);
  int vmin = (int)ceilf(half * sqrtf(2.f) / 2);
  const double hp2 = half * half;
  for (int v = 0; v <= vmax; ++v) t.umax[v] = round_d(sqrt(hp2 - v * v));
  for (int v = half, v0 = 0; v >= vmin; --v) {
    while (t.umax[v0] == t.umax[v0 + 1]) ++v0;
    t.umax[v] = v0;
    ++v0;
  }
  return ORBX_OK;
}

static int pitch_of(int w) { return (w + 15) & ~15; }

/* cv::resize INTER_LINEAR coefficient tables (OpenCV 3.4 resize():
 * scale = 1/((double)dsize/ssize); f = (float)((d+0.5)*scale-0.5); s =
 * cvFloor(f); f -= s; coefficients saturate_cast<short>((1-f)*2048), f*2048). */
static void resize_lut(int sw, int sh, int dw, int dh, std::vector<int32_t>& xofs,
                       std::vector<int32_t>& xofs1, std::vector<int16_t>& alpha,
                       std::vector<int32_t>& yofs, std::vector<int16_t>& beta) {
  const double scale_x = 1. / ((double)dw / sw), scale_y = 1. / ((double)dh / sh);
  int xmax = dw;
  const size_t x0 = xofs.size();
  for (int dx = 0; dx < dw; ++dx) {
    float fx = (float)((dx + 0.5) * scale_x - 0.5);
    int sx = (int)floorf(fx);
    fx -= sx;
    if (sx < 0) fx = 0, sx = 0;
    if (sx + 1 >= sw) {
      xmax = std::min(xmax, dx);
      if (sx >= sw - 1) fx = 0, sx = sw - 1;
    }
    xofs.push_back(sx);
    xofs1.push_back(std::min(sx + 1, sw - 1));
    alpha.push_back(sat_s16(round_f((1.f - fx) * 2048)));
    alpha.push_back(sat_s16(round_f(fx * 2048)));
  }
  /* columns at or beyond xmax use S[sx]*2048 (HResizeLinear tail loop) */
  for (int dx = xmax; dx < dw; ++dx) {
    alpha[2 * (x0 + dx)] = 2048;
    alpha[2 * (x0 + dx) + 1] = 0;
    xofs1[x0 + dx] = xofs[x0 + dx];
  }
  for (int dy = 0; dy < dh; ++dy) {
    float fy = (float)((dy + 0.5) * scale_y - 0.5);
    int sy = (int)floorf(fy);
    fy -= sy;
    yofs.push_back(sy);
    beta.push_back(sat_s16(round_f((1.f - fy) * 2048)));
    beta.push_back(sat_s16(round_f(fy * 2048)));
  }
}

static bool area_fast_2x(int sw, int sh, int dw, int dh) {
  double sx = 1. / ((double)dw / sw), sy = 1. / ((double)dh / sh);
  int ix = round_d(sx), iy = round_d(sy);
  return fabs(sx - ix) < 2.220446049250313e-16 && fabs(sy - iy) < 2.220446049250313e-16 &&
         ix == 2 && iy == 2;
}

/* ---- fused pyramid tiling (k_pyramid) ----------------------------------
 * 1-D chain for one axis of segment levels lev[0..ns-1] (lev[0] = source).
 * The last level is cut into tiles of T; each coarser level's owned
 * intervals are the source positions of the finer level's tile starts, so
 * they partition the level.  Computed intervals are built from the last
 * level back: C(s-1) = hull(footprint of C(s), owned(s-1)). */
struct Iv { int clo, chi, plo, phi; };

static void src_span(const Plan& P, int l, bool isx, int d, int& lo, int& hi) {
  const LevelInfo& lv = P.levels[l];
  const LevelInfo& sv = P.levels[lv.src_level];
  if (isx) {
    lo = P.xofs[lv.lut_x + d];
    hi = P.xofs1[lv.lut_x + d];
  } else {
    const int sy = P.yofs[lv.lut_y + d];
    lo = std::min(std::max(sy, 0), sv.h - 1);
    hi = std::min(std::max(sy + 1, 0), sv.h - 1);
  }
}

static int chain_1d(const Plan& P, const std::vector<int>& lev, bool isx, int T,
                    std::vector<Iv>& out) {
  const int ns = (int)lev.size();
  auto size = [&](int s) { return isx ? P.levels[lev[s]].w : P.levels[lev[s]].h; };
  const int nt = (size(ns - 1) + T - 1) / T;
  out.assign((size_t)ns * nt, Iv{0, 0, 0, 0});
  std::vector<int> X(nt + 1);
  for (int t = 0; t <= nt; ++t) X[t] = std::min(t * T, size(ns - 1));
  for (int s = ns - 1; s >= 1; --s) {
    for (int t = 0; t < nt; ++t) {
      out[(size_t)s * nt + t].plo = X[t];
      out[(size_t)s * nt + t].phi = X[t + 1];
    }
    std::vector<int> Xn(nt + 1);
    Xn[0] = 0;
    Xn[nt] = size(s - 1);
    for (int t = 1; t < nt; ++t) {
      int lo = size(s - 1), hi;
      if (X[t] < size(s)) src_span(P, lev[s], isx, X[t], lo, hi);
      Xn[t] = std::min(std::max(lo, Xn[t - 1]), size(s - 1));
    }
    X.swap(Xn);
  }
  for (int t = 0; t < nt; ++t) {
    int clo = out[(size_t)(ns - 1) * nt + t].plo, chi = out[(size_t)(ns - 1) * nt + t].phi;
    for (int s = ns - 1; s >= 1; --s) {
      if (isx) {
        /* every 4-pixel group holding an owned pixel is computed whole (or
         * ends past the level's last column): k_pyramid stores such groups as
         * one dword, the bytes it does not own carrying the same values the
         * owner writes (the LDS pitch is unchanged: clo & ~3 and the rounded
         * chi stay; only the footprint in level s-1 grows) */
        const Iv& o = out[(size_t)s * nt + t];
        if (o.phi > o.plo) {
          clo = std::min(clo, o.plo & ~3);
          chi = std::max(chi, std::min((o.phi + 3) & ~3, size(s)));
        }
      }
      out[(size_t)s * nt + t].clo = clo;
      out[(size_t)s * nt + t].chi = chi;
      int flo = 1 << 30, fhi = -1;
      for (int d = clo; d < chi; ++d) { /* footprint (LUTs are monotone; scan to be safe) */
        int lo, hi;
        src_span(P, lev[s], isx, d, lo, hi);
        flo = std::min(flo, lo);
        fhi = std::max(fhi, hi);
      }
      if (s - 1 >= 1) {
        const Iv& o = out[(size_t)(s - 1) * nt + t];
        if (o.phi > o.plo) { flo = std::min(flo, o.plo); fhi = std::max(fhi, o.phi - 1); }
      }
      if (fhi < flo) { clo = chi = 0; } else { clo = flo; chi = fhi + 1; }
    }
    out[t].clo = clo;
    out[t].chi = chi;
    out[t].plo = out[t].phi = 0;
  }
  return nt;
}

/* LDS bytes of level s's region (formulas shared with k_pyramid) */
static long long region_bytes(const Iv& x, const Iv& y, int s) {
  if (x.chi <= x.clo || y.chi <= y.clo) return 0;
  long long pitch;
  if (s == 0) pitch = ((x.chi + 15) & ~15) - (x.clo & ~15);
  else pitch = (long long)((x.chi - (x.clo & ~3) + 3) >> 2) * 4;
  return pitch * (y.chi - y.clo);
}

static bool try_segment(Plan& P, const std::vector<int>& lev, int TW, int TH, PyrSeg& g,
                        std::vector<Iv>& xs, std::vector<Iv>& ys) {
  const int ns = (int)lev.size();
  const int ntx = chain_1d(P, lev, true, TW, xs);
  const int nty = chain_1d(P, lev, false, TH, ys);
  long long a = 0, b = 0;
  for (int s = 0; s < ns; ++s) {
    long long m = 0;
    for (int tx = 0; tx < ntx; ++tx) {
      const Iv& x = xs[(size_t)s * ntx + tx];
      if (s > 0 && ((x.chi - (x.clo & ~3) + 3) >> 2) > 256) return false;
      for (int ty = 0; ty < nty; ++ty) m = std::max(m, region_bytes(x, ys[(size_t)s * nty + ty], s));
    }
    if (s % 2 == 0) a = std::max(a, m); else b = std::max(b, m);
  }
  a = (a + 15) & ~15LL;
  b = (b + 15) & ~15LL;
  if (a + b > ORBX_PYR_LDS_BUDGET) return false;
  long long bx = 0, by = 0; /* LUT blob entries (build_blobs layout) */
  for (int tx = 0; tx < ntx; ++tx) {
    long long n = 0;
    for (int s = 1; s < ns; ++s) {
      const Iv& x = xs[(size_t)s * ntx + tx];
      if (x.chi > x.clo) n += 4 * ((x.chi - (x.clo & ~3) + 3) >> 2);
    }
    bx = std::max(bx, (n + 1) & ~1LL);
  }
  for (int ty = 0; ty < nty; ++ty) {
    long long n = 0;
    for (int s = 1; s < ns; ++s) n += std::max(0, ys[(size_t)s * nty + ty].chi - ys[(size_t)s * nty + ty].clo);
    by = std::max(by, (n + 1) & ~1LL);
  }
  if (a + b + 8 * (bx + by) > ORBX_PYR_LDS_MAX) return false;
  memset(&g, 0, sizeof(g));
  /* one LDS pitch per level for every tile (the widest tile column's): the
   * row LUT then holds final LDS offsets, shared by all tile columns; the
   * buffers above were sized with it (max pitch x max rows) */
  for (int s = 0; s < ns; ++s) {
    long long m = 0;
    for (int tx = 0; tx < ntx; ++tx) {
      const Iv& x = xs[(size_t)s * ntx + tx];
      if (x.chi <= x.clo) continue;
      m = std::max(m, s == 0 ? (long long)(((x.chi + 15) & ~15) - (x.clo & ~15))
                             : (long long)((x.chi - (x.clo & ~3) + 3) >> 2) * 4);
    }
    g.lpitch[s] = (int)m;
  }
  g.nl = ns - 1;
  g.ntx = ntx;
  g.nty = nty;
  g.lds_a = (int)a;
  g.lds_b = (int)b;
  for (int s = 0; s < ns; ++s) {
    const LevelInfo& lv = P.levels[lev[s]];
    g.lev[s] = lev[s];
    g.w[s] = lv.w;
    g.h[s] = lv.h;
    g.pitch[s] = lv.pitch;
    g.off[s] = lev[s] == 0 ? -1 : lv.pyr_off;
    g.lut_x[s] = s ? lv.lut_x : 0;
    g.lut_y[s] = s ? lv.lut_y : 0;
  }
  return true;
}

/* per tile column / row LUT blobs (layout: orbx_internal.h) */
/* returns false when k_pyramid's packed arithmetic does not apply: the 4
 * columns of a thread must read bytes within 8 of the first one's sx, and
 * every coefficient must lie in [0, 4095] (INTER_LINEAR downscale: [0, 2048]) */
static bool build_blobs(Plan& P, const std::vector<int>& lev, PyrSeg& g, const std::vector<Iv>& xs,
                        const std::vector<Iv>& ys) {
  const int ns = (int)lev.size();
  for (int axis = 0; axis < 2; ++axis) {
    const bool isx = axis == 0;
    const int nt = isx ? g.ntx : g.nty;
    const std::vector<Iv>& v = isx ? xs : ys;
    (isx ? g.xbo_off : g.ybo_off) = (int)P.pyr_bo.size();
    int maxn = 0;
    for (int t = 0; t < nt; ++t) {
      P.pyr_bo.push_back((int)(P.pyr_blob.size() / 2));
      int n = 0;
      for (int s = 1; s < ns; ++s) {
        const Iv& c = v[(size_t)s * nt + t];
        const Iv& pc = v[(size_t)(s - 1) * nt + t];
        const int origin = isx ? (s - 1 == 0 ? (pc.clo & ~15) : (pc.clo & ~3)) : pc.clo;
        const LevelInfo& lv = P.levels[lev[s]];
        int b, e;
        if (isx) {
          b = c.clo & ~3;
          e = b + 4 * ((c.chi - b + 3) >> 2);
        } else {
          b = c.clo;
          e = c.chi;
        }
        if (c.chi <= c.clo) e = b;
        int glo = 0;
        for (int d = b; d < e; ++d) {
          const int dd = std::min(std::max(d, c.clo), c.chi - 1);
          int lo, hi;
          src_span(P, lev[s], isx, dd, lo, hi);
          const int16_t* cf = isx ? &P.alpha[2 * (lv.lut_x + dd)] : &P.beta[2 * (lv.lut_y + dd)];
          if (cf[0] < 0 || cf[0] > 4095 || cf[1] < 0 || cf[1] > 4095) return false;
          if (isx && ((d - b) & 3) == 0) glo = lo;
          if (isx && hi - glo > 7) return false;
          if (!isx) { /* LDS byte offsets of the two source rows (< 64 KiB) */
            const uint32_t base = ((s - 1) & 1) ? (uint32_t)g.lds_a : 0u;
            const uint32_t o0 = base + (uint32_t)(lo - origin) * (uint32_t)g.lpitch[s - 1];
            const uint32_t o1 = base + (uint32_t)(hi - origin) * (uint32_t)g.lpitch[s - 1];
            if (o0 > 0xFFFF || o1 > 0xFFFF) return false;
            P.pyr_blob.push_back(o0 | (o1 << 16));
          }
          else if (((d - b) & 3) == 0) /* group column 0: s0 | (sx1 - s0) << 16 */
            P.pyr_blob.push_back((uint32_t)(lo - origin) | ((uint32_t)(hi - lo) << 16));
          else /* columns 1..3: k_pyramid's v_perm selector, bytes relative to s0 */
            P.pyr_blob.push_back((uint32_t)(lo - glo) | 0x0C00u | ((uint32_t)(hi - glo) << 16) | 0x0C000000u);
          P.pyr_blob.push_back((uint32_t)(uint16_t)cf[0] | ((uint32_t)(uint16_t)cf[1] << 16));
          ++n;
        }
      }
      while (n & 1) { P.pyr_blob.push_back(0); P.pyr_blob.push_back(0); ++n; } /* 16-B pad */
      maxn = std::max(maxn, n);
    }
    P.pyr_bo.push_back((int)(P.pyr_blob.size() / 2));
    (isx ? g.lds_xl : g.lds_yl) = 8 * maxn;
  }
  return true;
}

/* greedy: longest run of unique levels from `first` that fits a tile of at
 * least 32x16 at its last level (smaller tiles only for a single level) */
static int plan_pyramid(Plan& P) {
  P.segs.clear();
  P.pyr_xs.clear();
  P.pyr_ys.clear();
  P.pyr_blob.clear();
  P.pyr_bo.clear();
  std::vector<int> uniq;
  for (int l = 0; l < (int)P.levels.size(); ++l)
    if (P.levels[l].unique == l) uniq.push_back(l);
  static const int tiles[][2] = {{64, 16}, {128, 16}, {128, 8}, {64, 8}, {64, 32}, {32, 16},
                                 {16, 16}, {16, 8}, {8, 8}};
  int k0 = 0; /* ORBX_DEBUG_PYR_TILE=k: start the tile search at tiles[k] (profiling only) */
  size_t maxseg = 1 << 20; /* ORBX_DEBUG_PYR_MAXSEG=n: at most n levels per segment, source included (profiling only) */
#ifdef ORBX_PROFILING
  if (const char* e = getenv("ORBX_DEBUG_PYR_TILE")) k0 = std::min(std::max(atoi(e), 0), 8);
  if (const char* e = getenv("ORBX_DEBUG_PYR_MAXSEG")) maxseg = (size_t)std::max(atoi(e), 2);
#endif
  size_t i = 1;
  while (i < uniq.size()) {
    if (P.area2[uniq[i]]) {  /* exact 2x: its own launch of k_pyr_area2 */
      PyrSeg g{};
      memset(&g, 0, sizeof(g));
      g.nl = 1;
      g.area = 1;
      for (int s = 0; s < 2; ++s) {
        const LevelInfo& lv = P.levels[uniq[i - 1 + s]];
        g.lev[s] = uniq[i - 1 + s];
        g.w[s] = lv.w;
        g.h[s] = lv.h;
        g.pitch[s] = lv.pitch;
        g.off[s] = g.lev[s] == 0 ? -1 : lv.pyr_off;
      }
      P.segs.push_back(g);
      ++i;
      continue;
    }
    size_t lim = i; /* the linear chain stops before the next 2x level */
    while (lim < uniq.size() && !P.area2[uniq[lim]]) ++lim;
    bool done = false;
    for (size_t j = std::min(lim, i - 1 + maxseg); j > i && !done; --j) {
      std::vector<int> lev(uniq.begin() + (i - 1), uniq.begin() + j);
      const int ntile = (j == i + 1) ? 9 : 6;
      for (int k = std::min(k0, ntile - 1); k < ntile && !done; ++k) {
        PyrSeg g{};
        std::vector<Iv> xs, ys;
        if (!try_segment(P, lev, tiles[k][0], tiles[k][1], g, xs, ys)) continue;
        g.xs_off = (int)(P.pyr_xs.size() / 4);
        g.ys_off = (int)(P.pyr_ys.size() / 4);
        for (const Iv& v : xs) P.pyr_xs.insert(P.pyr_xs.end(), {v.clo, v.chi, v.plo, v.phi});
        for (const Iv& v : ys) P.pyr_ys.insert(P.pyr_ys.end(), {v.clo, v.chi, v.plo, v.phi});
        if (!build_blobs(P, lev, g, xs, ys)) return ORBX_ERR_UNSUPPORTED;
        P.segs.push_back(g);
        i = j;
        done = true;
      }
    }
    if (!done) return ORBX_ERR_UNSUPPORTED; /* level ratio too large for one tile */
  }
  return ORBX_OK;
}

int plan_geometry(const orbx_params& p, int width, int height, Plan& P) {
  int rc = compute_tables(p, P.tables);
  if (rc) return rc;
  if (width <= 0 || height <= 0) return ORBX_ERR_ARG;
  P.params = p;
  P.W = width;
  P.H = height;
  P.ini_th = std::min(std::max(p.ini_th_fast, 0), 255);
  P.min_th = std::min(std::max(p.min_th_fast, 0), 255);
  const int L = p.nlevels;
  P.levels.assign(L, LevelInfo());
  P.area2.assign(L, 0);
  P.cells.clear();
  P.strips.clear();
  P.strip_max_w = P.strip_max_h = P.strip_max_cells = 0;
  P.nstrips_l0 = 0;
  P.xofs.clear(); P.xofs1.clear(); P.alpha.clear(); P.yofs.clear(); P.beta.clear();
  memset(&P.geo, 0, sizeof(P.geo));
  P.geo.nlevels = L;

  /* ComputePyramid sizes (:501-502) and storage */
  long long pyr = 0, blur = 0;
  int key_xs = 20;
  for (int l = 0; l < L; ++l) {
    LevelInfo& lv = P.levels[l];
    float s = P.tables.inv_scale[l];
    lv.w = round_f((float)width * s);
    lv.h = round_f((float)height * s);
    if (lv.h <= 32 || lv.w < 32) return ORBX_ERR_LEVEL_SIZE;
    if (l == 0) { /* FAST key packing (orbx_pack_key): coordinate bits for level 0 */
      const int xw = lv.w - 32, yh = lv.h - 32;
      if (xw <= 4095 && yh <= 4095) key_xs = 20;
      else if (xw <= 8191 && yh <= 2047) key_xs = 19;
      else if (xw <= 2047 && yh <= 8191) key_xs = 21;
      else return ORBX_ERR_UNSUPPORTED;
    }
    lv.key_xs = key_xs;
    if (l > 0 && lv.w == P.levels[l - 1].w && lv.h == P.levels[l - 1].h) {
      lv.unique = P.levels[l - 1].unique; /* cv::resize: dsize == ssize -> copyTo */
    } else {
      lv.unique = l;
      /* cv::resize switches to its INTER_AREA fast path for exact 2x ratios */
      if (l > 0 && area_fast_2x(P.levels[l - 1].w, P.levels[l - 1].h, lv.w, lv.h)) P.area2[l] = 1;
    }
    if (lv.unique == l) {
      lv.pitch = (l == 0) ? 0 /* caller's row stride */ : pitch_of(lv.w);
      lv.pyr_off = (l == 0) ? -1 : pyr;
      if (l > 0) pyr += (long long)pitch_of(lv.w) * lv.h;
      lv.blur_off = blur;
      lv.bpitch = pitch_of(lv.w);
      blur += (long long)pitch_of(lv.w) * lv.h;
    } else {
      const LevelInfo& u = P.levels[lv.unique];
      lv.pitch = u.pitch;
      lv.pyr_off = u.pyr_off;
      lv.blur_off = u.blur_off;
      lv.bpitch = u.bpitch;
    }
    lv.scale = P.tables.scale[l];
    lv.patch_size = (int)(31 * P.tables.scale[l]); /* :345 int scaledPatchSize = 31 * float */
    P.geo.width[l] = lv.w;
    P.geo.height[l] = lv.h;
    P.geo.alias[l] = lv.unique;
    P.geo.features[l] = P.tables.features[l];
  }
  P.pyr_bytes = pyr;
  P.blur_bytes = blur;

  /* resize LUTs for unique levels >= 1 */
  for (int l = 1; l < L; ++l) {
    LevelInfo& lv = P.levels[l];
    if (lv.unique != l) continue;
    const LevelInfo& src = P.levels[l - 1];
    lv.src_level = src.unique;
    lv.lut_x = (int)P.xofs.size();
    lv.lut_y = (int)P.yofs.size();
    resize_lut(src.w, src.h, lv.w, lv.h, P.xofs, P.xofs1, P.alpha, P.yofs, P.beta);
  }
  rc = plan_pyramid(P);
  if (rc) return rc;

  /* FAST cell grid (ComputeKeyPointsOctTree :298-340) for unique levels */
  long long slots = 0;
  /* k_fast_strips' column walk only pays on wide levels */
  int cw_minw = ORBX_FS_COLWALK_MINW;
#ifdef ORBX_PROFILING
  if (const char* e = getenv("ORBX_DEBUG_CW_MINW")) cw_minw = atoi(e);
#endif
  for (int l = 0; l < L; ++l) {
    LevelInfo& lv = P.levels[l];
    const int minB = ORBX_MINB, maxBX = lv.w - ORBX_EDGE + 3, maxBY = lv.h - ORBX_EDGE + 3;
    const float width_f = (float)(maxBX - minB), height_f = (float)(maxBY - minB);
    const int nCols = (int)(width_f / 30.f), nRows = (int)(height_f / 30.f);
    const int wCell = nCols > 0 ? (int)ceilf(width_f / nCols) : 0;
    const int hCell = nRows > 0 ? (int)ceilf(height_f / nRows) : 0;
    P.geo.ncols[l] = nCols; P.geo.nrows[l] = nRows;
    P.geo.wcell[l] = wCell; P.geo.hcell[l] = hCell;
    /* DistributeOctTree (:230-231) */
    lv.Wr = maxBX - minB;
    lv.Hr = maxBY - minB;
    lv.nini = lv.Wr / lv.Hr;
    lv.hX = (float)lv.Wr / (float)(lv.nini > 0 ? lv.nini : 1);
    lv.N = P.tables.features[l];
    P.geo.nini[l] = lv.nini;
    if (lv.unique != l) {
      const LevelInfo& u = P.levels[lv.unique];
      lv.cell_begin = u.cell_begin; lv.ncells = u.ncells;
      lv.slot_begin = u.slot_begin; lv.nslots = u.nslots;
      P.geo.ncells_bad[l] = P.geo.ncells_bad[lv.unique];
      continue;
    }
    lv.cell_begin = (int)P.cells.size();
    lv.slot_begin = slots;
    lv.wcell = wCell;
    int bad = 0;
    for (int i = 0; i < nRows; ++i) {
      const int row_first = (int)P.cells.size();
      const float iniY = (float)(minB + i * hCell);
      const float maxY = std::min(iniY + hCell + 6, (float)maxBY);
      for (int j = 0; j < nCols; ++j) {
        const float iniX = (float)(minB + j * wCell);
        const float maxX = std::min(iniX + wCell + 6, (float)maxBX);
        const int rx = (int)iniX, ry = (int)iniY, rw = (int)(maxX - iniX), rh = (int)(maxY - iniY);
        if (rw < 0 || rh < 0) { ++bad; continue; } /* cv::Mat(m, Rect) assertion */
        if (rw < 7 || rh < 7) continue;            /* FAST scans nothing */
        if (rw > ORBX_CELL_MAX || rh > ORBX_CELL_MAX) return ORBX_ERR_UNSUPPORTED;
        CellInfo c;
        c.level = l; c.x = rx; c.y = ry; c.w = rw; c.h = rh;
        const int bw = rw - 6, bh = rh - 6;
        c.slot_cap = ((bw + 1) / 2) * ((bh + 1) / 2); /* strict 3x3 NMS: independent set */
        c.slot_off = (int)slots;
        c.pad = 0;
        slots += c.slot_cap;
        P.cells.push_back(c);
      }
      /* valid cells of a row are a prefix (only the last columns can be
       * negative / narrower than 7); group them into strips */
      const int nvalid = (int)P.cells.size() - row_first;
      const int per = std::max(1, ORBX_STRIP_MAXW / std::max(wCell, 1));
      for (int j0 = 0; j0 < nvalid; j0 += per) {
        const int j1 = std::min(nvalid, j0 + per);
        const CellInfo& a = P.cells[row_first + j0];
        const CellInfo& b = P.cells[row_first + j1 - 1];
        StripInfo st;
        st.level = l; st.x = a.x; st.y = a.y; st.w = b.x + b.w - a.x; st.h = a.h;
        st.cell_begin = row_first + j0; st.ncells = j1 - j0; st.wcell = wCell;
        st.colwalk = lv.w >= cw_minw;
        st.pitch = 0;  /* set by the plan (api_extract.hip) */
        st.off = 0;
        P.strips.push_back(st);
        P.strip_max_w = std::max(P.strip_max_w, st.w);
        P.strip_max_h = std::max(P.strip_max_h, st.h);
        P.strip_max_cells = std::max(P.strip_max_cells, st.ncells);
        if (st.ncells > ORBX_STRIP_MAXCELLS) return ORBX_ERR_UNSUPPORTED;
      }
    }
    lv.ncells = (int)P.cells.size() - lv.cell_begin;
    lv.nslots = slots - lv.slot_begin;
    P.geo.ncells_bad[l] = bad;
    if (bad && !p.cell_guard) return ORBX_ERR_CELL_ROI;
  }
  P.nslots = slots;
  P.ncells = (int)P.cells.size();
  P.nstrips_l0 = 0;
  while (P.nstrips_l0 < (int)P.strips.size() && P.strips[P.nstrips_l0].level == 0) ++P.nstrips_l0;
  int bt = 0;
  for (int l = 0; l < L; ++l) {
    LevelInfo& lv = P.levels[l];
    if (lv.unique != l) { lv.blur_tile_begin = -1; lv.blur_tiles_x = 0; continue; }
    lv.blur_tile_begin = bt;
    lv.blur_tiles_x = (lv.w + ORBX_BLUR_TW - 1) / ORBX_BLUR_TW;
    bt += lv.blur_tiles_x * ((lv.h + ORBX_BLUR_TH - 1) / ORBX_BLUR_TH);
  }
  P.blur_tiles = bt;

  /* quadtree capacities */
  int kout = 0, smax = 1, maxc = 1;
  long long qk = 0;
  for (int l = 0; l < L; ++l) {
    LevelInfo& lv = P.levels[l];
    long long cap = 4LL * std::max(lv.N - 1, lv.nini);
    cap = std::min(cap, lv.nslots);
    lv.kcap = (int)std::max(0LL, cap);
    lv.kout_off = kout;
    kout += lv.kcap;
    lv.qk_off = qk;
    qk += lv.nslots;
    smax = std::max(smax, std::max(lv.N - 1, lv.nini));
    maxc = std::max(maxc, lv.ncells);
    P.geo.kcap_level[l] = lv.kcap;
  }
  P.kcap = kout;
  P.qk_elems = qk;
  P.qt_smax = smax;
  P.qt_max_cells = maxc;
  P.geo.kcap = kout;

  /* algorithmic bytes of pyramid + FAST per frame: every unique level is
   * written once by the resize that reads its source level, and read once
   * by FAST (SURVEY §8d formula restricted to unique levels). */
  long long px = 0, bytes = 0;
  for (int l = 0; l < L; ++l) {
    const LevelInfo& lv = P.levels[l];
    if (lv.unique != l) continue;
    long long P_l = (long long)lv.w * lv.h;
    px += P_l;
    bytes += P_l; /* FAST read */
    if (l > 0) bytes += P_l + (long long)P.levels[lv.src_level].w * P.levels[lv.src_level].h;
  }
  P.geo.pixels = px;
  P.geo.bytes_pyr_fast = bytes;
  return ORBX_OK;
}

}  // namespace orbx
