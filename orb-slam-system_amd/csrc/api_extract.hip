// api_extract.hip -- C ABI of the extractor (include/orbx.h): plan
// creation, batched launches, the ORBextractor::operator() drop-in, stage
// timing and synthetic frames.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <vector>

#include "../../include/orbx.h"
#include "api_common.h"
#include "geometry.h"
#include "plan_internal.h"

namespace orbx {
__global__ void k_pyramid(const uint8_t*, size_t, size_t, uint8_t*, size_t, const PyrSeg,
                          const int4*, const int4*, const uint4*, const int*, int);
__global__ void k_pyr_area2(const uint8_t*, size_t, size_t, uint8_t*, size_t, const PyrSeg);
__global__ void k_fast_strips(const uint8_t*, size_t, size_t, const uint8_t*, size_t,
                              const LevelArgs, const CellInfo*, const StripInfo*, uint32_t*,
                              size_t, uint32_t*, int, int, int, int, int, int, int, int*, int, int);
__global__ void k_fast_strips_p288(const uint8_t*, size_t, size_t, const uint8_t*, size_t,
                              const LevelArgs, const CellInfo*, const StripInfo*, uint32_t*,
                              size_t, uint32_t*, int, int, int, int, int, int, int, int*, int, int);
__global__ void k_quadtree(const LevelInfo*, const CellInfo*, const uint32_t*, size_t,
                           const uint32_t*, int, uint32_t*, int32_t*, size_t, uint32_t*, size_t,
                           int*, int, int, int, int*, uint32_t*);
__global__ void k_quadtree_j6(const LevelInfo*, const CellInfo*, const uint32_t*, size_t,
                              const uint32_t*, int, uint32_t*, int32_t*, size_t, uint32_t*, size_t,
                              int*, int, int, int, int*, uint32_t*);
__global__ void k_pack_results(const int*, const int*, const uint4*, const uint4*, int, uint4*, uint32_t);
static_assert(sizeof(orbx_keypoint) == 28, "k_pack_results copies 7-dword keypoint rows");
__global__ void k_quadtree_wide(const LevelInfo*, const CellInfo*, const uint32_t*, size_t,
                                const uint32_t*, int, uint32_t*, int32_t*, size_t, uint32_t*, size_t,
                                int*, int, int, int, int*, uint32_t*);
__global__ void k_orient_brief(const uint8_t*, size_t, size_t, const uint8_t*, size_t,
                               const BriefArgs, const uint32_t*, size_t, const int*,
                               orbx_keypoint*, uint8_t*, int*, const uint32_t*, int);
__global__ void k_orient_brief_lb(const uint8_t*, size_t, size_t, const uint8_t*, size_t,
                                  const BriefArgs, const uint32_t*, size_t, const int*,
                                  orbx_keypoint*, uint8_t*, int*, const uint32_t*, int,
                                  const uint8_t*, size_t);
__global__ void k_blur(const uint8_t*, size_t, size_t, const uint8_t*, size_t, uint8_t*, size_t, const BlurArgs);
__global__ void k_synth(uint8_t*, int, int, size_t, int, int);
__global__ void k_selftest_sincos(const float*, int, float*);
__global__ void k_selftest_sincos_range(uint32_t, int, float*);
}  // namespace orbx

using namespace orbx;

static const char* kStageNames[ORBX_NSTAGES] = {
    "resize", "fast_cells", "quadtree", "blur", "orient_brief",
    "match_select", "match_candidates", "match_resolve", "match_finalize",
    "stereo_rows", "stereo_match", "stereo_filter"};

extern "C" int orbx_abi_version(void) { return ORBX_ABI_VERSION; }

extern "C" const char* orbx_status_string(int s) {
  switch (s) {
    case ORBX_OK: return "ok";
    case ORBX_ERR_ARG: return "invalid argument";
    case ORBX_ERR_CELL_ROI: return "negative-extent FAST cell (reference throws cv::Exception)";
    case ORBX_ERR_LEVEL_SIZE: return "pyramid level too small";
    case ORBX_ERR_QUADTREE: return "DistributeOctTree does not terminate";
    case ORBX_ERR_CAPACITY: return "output capacity too small";
    case ORBX_ERR_UNSUPPORTED: return "unsupported configuration";
    case ORBX_ERR_HIP: return "HIP runtime error";
    case ORBX_ERR_NO_DEVICE: return "no gfx950 device";
    default: return "unknown status";
  }
}

extern "C" int orbx_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

extern "C" int orbx_stage_count(void) { return ORBX_NSTAGES; }
extern "C" const char* orbx_stage_name(int s) {
  return (s >= 0 && s < ORBX_NSTAGES) ? kStageNames[s] : "";
}

extern "C" int orbx_tables(const orbx_params* p, float* scale, float* inv_scale, float* sigma2,
                           float* inv_sigma2, int* fpl, int* umax16) {
  if (!p) return ORBX_ERR_ARG;
  Tables t;
  int rc = compute_tables(*p, t);
  if (rc) return rc;
  for (int l = 0; l < t.nlevels; ++l) {
    if (scale) scale[l] = t.scale[l];
    if (inv_scale) inv_scale[l] = t.inv_scale[l];
    if (sigma2) sigma2[l] = t.sigma2[l];
    if (inv_sigma2) inv_sigma2[l] = t.inv_sigma2[l];
    if (fpl) fpl[l] = t.features[l];
  }
  if (umax16) memcpy(umax16, t.umax, sizeof(t.umax));
  return ORBX_OK;
}

extern "C" int orbx_geometry_compute(const orbx_params* p, int width, int height,
                                     orbx_geometry* g) {
  if (!p || !g) return ORBX_ERR_ARG;
  Plan P;
  int rc = plan_geometry(*p, width, height, P);
  if (rc) return rc;
  *g = P.geo;
  return ORBX_OK;
}

extern "C" int orbx_resize_tables(const orbx_params* p, int width, int height, int level,
                                  int32_t* xofs, int16_t* alpha, int32_t* yofs, int16_t* beta) {
  if (!p) return ORBX_ERR_ARG;
  Plan P;
  int rc = plan_geometry(*p, width, height, P);
  if (rc) return rc;
  if (level < 1 || level >= p->nlevels || P.levels[level].unique != level) return ORBX_ERR_ARG;
  const LevelInfo& L = P.levels[level];
  for (int x = 0; x < L.w; ++x) {
    if (xofs) xofs[x] = P.xofs[L.lut_x + x];
    if (alpha) { alpha[2 * x] = P.alpha[2 * (L.lut_x + x)]; alpha[2 * x + 1] = P.alpha[2 * (L.lut_x + x) + 1]; }
  }
  for (int y = 0; y < L.h; ++y) {
    if (yofs) yofs[y] = P.yofs[L.lut_y + y];
    if (beta) { beta[2 * y] = P.beta[2 * (L.lut_y + y)]; beta[2 * y + 1] = P.beta[2 * (L.lut_y + y) + 1]; }
  }
  return ORBX_OK;
}

// ---------------------------------------------------------------------------
// orbx_plan
// ---------------------------------------------------------------------------

static size_t round_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

static void plan_free(orbx_plan* p) {
  if (!p) return;
  hipSetDevice(p->device);
  void* bufs[] = {p->d_lv, p->d_cells, p->d_strips, p->d_xofs, p->d_xofs1, p->d_yofs, p->d_alpha, p->d_beta,
                  p->d_pyr, p->d_blur, p->d_slots, p->d_ccount, p->d_qkeys, p->d_qout, p->d_qperm,
                  p->d_qnode, p->d_lcount, p->d_err, p->d_pyr_xs, p->d_pyr_ys, p->d_pyr_bo, p->d_pyr_blob};
  for (void* b : bufs)
    if (b) hipFree(b);
  p->timer.release();
  if (p->h_err) hipHostFree(p->h_err);
  if (p->stream) hipStreamDestroy(p->stream);
  if (p->s_aux) hipStreamDestroy(p->s_aux);
  if (p->ev_aux0) hipEventDestroy(p->ev_aux0);
  if (p->ev_aux1) hipEventDestroy(p->ev_aux1);
  delete p;
}

// stream-ordered upload (the host vectors outlive the plan_create call,
// which ends with a synchronisation of this stream only)
template <typename T>
static int upload(T** dst, const std::vector<T>& v, hipStream_t s) {
  size_t n = v.size() ? v.size() : 1;
  if (hipMalloc((void**)dst, n * sizeof(T)) != hipSuccess) return ORBX_ERR_HIP;
  if (v.size() && hipMemcpyAsync(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s) != hipSuccess)
    return ORBX_ERR_HIP;
  return ORBX_OK;
}

static int dev_alloc(void** p, size_t bytes) {
  if (hipMalloc(p, bytes ? bytes : 16) != hipSuccess) return ORBX_ERR_HIP;
  return ORBX_OK;
}

static std::atomic<int> g_debug_ccap{-1};

extern "C" int orbx_debug_set_fast_ccap(int ccap) {
  if (ccap > FS_CCAP) return ORBX_ERR_ARG;
  g_debug_ccap.store(ccap < 0 ? -1 : ccap);
  return ORBX_OK;
}

extern "C" int orbx_plan_create(const orbx_params* prm, int width, int height, int max_batch,
                                int device, orbx_plan** out) {
  if (!prm || !out || max_batch < 1) return ORBX_ERR_ARG;
  *out = nullptr;
  int ndev = orbx_device_count();
  if (device < 0 || device >= ndev) return ORBX_ERR_NO_DEVICE;
  orbx_plan* p = new orbx_plan();
#ifdef ORBX_PROFILING
  /* profiling builds only (tools/variant.sh): kernel phase early exits, grid
   * divisors, chunked passes; a release library never reads these (an
   * inherited environment cannot change its results) */
  if (const char* e = getenv("ORBX_DEBUG_STOP")) p->dbg = atoi(e);
  if (const char* e = getenv("ORBX_DEBUG_OBDIV")) p->ob_div = atoi(e);
  if (const char* e = getenv("ORBX_DEBUG_LDSPAD")) sscanf(e, "%d,%d,%d", &p->pad_pyr, &p->pad_fast, &p->pad_brief);
  if (const char* e = getenv("ORBX_CHUNK")) p->chunk = atoi(e);
  if (const char* e = getenv("ORBX_DEBUG_OVERLAP")) p->overlap = atoi(e); /* FAST level 0 beside the pyramid */
#endif
  p->fs_ccap = FS_CCAP;
  /* testing only: a smaller FAST corner list, so the overflow path runs
   * (one launch group, this list length), set through
   * orbx_debug_set_fast_ccap -- not the environment, which an inherited
   * variable could set for a release process */
  if (const int c = g_debug_ccap.load(); c >= 0) {
    p->fs_ccap = std::max(0, std::min(FS_CCAP, c));
    p->ccap_fixed_dbg = true;
  }
  int rc = plan_geometry(*prm, width, height, p->P);
  if (rc) { delete p; return rc; }
  const Plan& P = p->P;
  p->device = device;
  p->max_batch = max_batch;
  ORBX_TRY(hipSetDevice(device));
  // quadtree LDS: cell offsets + slot offsets, then (reusing them) 11 int arrays of qt_smax
  p->qt_lds = sizeof(int) * std::max(2 * (size_t)P.qt_max_cells + 1, 11 * (size_t)P.qt_smax);
  if (p->qt_lds > 150 * 1024) { plan_free(p); return ORBX_ERR_UNSUPPORTED; }
  // the wide single-frame form adds a second child array (4 smax ints)
  p->qt_lds_wide = sizeof(int) * std::max(2 * (size_t)P.qt_max_cells + 1, 15 * (size_t)P.qt_smax);
  if (set_max_dynamic_lds((const void*)k_quadtree, device) ||
      set_max_dynamic_lds((const void*)k_quadtree_j6, device) ||
      set_max_dynamic_lds((const void*)k_quadtree_wide, device) ||
      set_max_dynamic_lds((const void*)k_fast_strips, device) ||
      set_max_dynamic_lds((const void*)k_fast_strips_p288, device) ||
      set_max_dynamic_lds((const void*)k_pyramid, device)) { plan_free(p); return ORBX_ERR_HIP; }
  if (p->overlap && (hipStreamCreateWithFlags(&p->s_aux, hipStreamNonBlocking) != hipSuccess ||
                     hipEventCreateWithFlags(&p->ev_aux0, hipEventDisableTiming) != hipSuccess ||
                     hipEventCreateWithFlags(&p->ev_aux1, hipEventDisableTiming) != hipSuccess)) {
    plan_free(p);
    return ORBX_ERR_HIP;
  }
  if (hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking) != hipSuccess ||
      hipHostMalloc((void**)&p->h_err, 64, hipHostMallocDefault) != hipSuccess) { plan_free(p); return ORBX_ERR_HIP; }
  memset(&p->bargs, 0, sizeof(p->bargs));
  // IC_Angle row extents (ORBextractor.cc:28-45): the centre row spans
  // [-15, 15], row v spans [-umax[|v|], umax[|v|]]
  for (int v = 0; v < 16; ++v) {
    const uint32_t um = (v == 0) ? 15u : (uint32_t)P.tables.umax[v];
    p->bargs.umaxw[v >> 2] |= um << (8 * (v & 3));
  }
  memset(&p->largs, 0, sizeof(p->largs));
  for (int l = 0; l < P.params.nlevels; ++l) {
    const LevelInfo& u = P.levels[P.levels[l].unique];
    p->largs.pyr_off[l] = u.pyr_off;
    p->largs.pitch[l] = u.pitch;
  }
  p->largs.key_xs = P.levels[0].key_xs;
  // each FAST strip carries its level's pitch and pyramid offset: the kernel
  // reads them with the strip record instead of indexing the by-value level
  // tables (two dependent scalar loads per workgroup)
  for (StripInfo& si : p->P.strips) {
    si.pitch = si.level == 0 ? 0 : p->largs.pitch[si.level];
    si.off = si.level == 0 ? 0 : p->largs.pyr_off[si.level];
    // the kernel's staging decisions for a 16-B-aligned base, made here
    // once (fs_kernel's general branch makes the same test at run time)
    si.lead16 = si.x & 15;
    const int cg0 = (si.lead16 + 3) >> 2, cg1 = (si.lead16 + si.w) >> 2;
    const int cgb = cg0 - (((si.lead16 + 3) & 3) != 3 ? 1 : 0);
    si.cw16 = si.colwalk && si.h - 6 <= (FS_NT / 64) * FS_CW_RMAX && cg1 - cgb <= 63;
    si.soff16 = si.level == 0 ? 0 : si.off + (long long)si.y * si.pitch + (si.x - si.lead16);
  }
  // plans with a pyramid run its waves and FAST's at a raised issue
  // priority (ORBX_EX_PRIO): measured in the pipelined step, c4 +1.4-2.3 %,
  // c1 +0.5-0.7 %, c5 neutral; a single level (c2) lost 2.3 %, the matcher
  // then being a larger share of its step
  p->largs.prio = (ORBX_EX_PRIO && P.params.nlevels > 1) ? 1 : 0;
  p->bargs.key_xs = P.levels[0].key_xs;
  p->bargs.nlevels = P.params.nlevels;
  p->bargs.kcap = P.kcap;
  for (int l = 0; l < P.params.nlevels; ++l) {
    const LevelInfo& lv = P.levels[l];
    p->bargs.kout_off[l] = lv.kout_off;
    p->bargs.lcap[l] = lv.kcap;
    p->bargs.unique[l] = lv.unique;
    p->bargs.w[l] = lv.w;
    p->bargs.h[l] = lv.h;
    p->bargs.pitch[l] = lv.pitch;
    p->bargs.pyr_off[l] = lv.pyr_off;
    p->bargs.scale[l] = lv.scale;
    p->bargs.patch[l] = lv.patch_size;
    p->bargs.bpitch[l] = lv.bpitch;
    p->bargs.blur_off[l] = lv.blur_off;
  }
  // level-blur mode (k_blur + k_orient_brief_lb): blur every unique level
  // once when the keypoints' per-keypoint patches (43 x 48 px each) would
  // cover clearly more pixels than the levels hold (c1 /
  // c2 / c5 blur their levels, c4's 1080p levels keep the per-keypoint blur)
  {
    memset(&p->blargs, 0, sizeof(p->blargs));
    int nt = 0;
    for (int l = 0; l < P.params.nlevels; ++l) {
      const LevelInfo& lv = P.levels[l];
      if (lv.unique != l) continue;
      const int i = p->blargs.nu++;
      p->blargs.tile_begin[i] = nt;
      p->blargs.tiles_x[i] = (lv.w + ORBX_LB_TW - 1) / ORBX_LB_TW;
      nt += p->blargs.tiles_x[i] * ((lv.h + ORBX_LB_TH - 1) / ORBX_LB_TH);
      p->blargs.w[i] = lv.w;
      p->blargs.h[i] = lv.h;
      p->blargs.pitch[i] = lv.pitch;
      p->blargs.src_off[i] = l == 0 ? -1 : lv.pyr_off;
      p->blargs.bpitch[i] = lv.bpitch;
      p->blargs.blur_off[i] = lv.blur_off;
    }
    p->blargs.tile_begin[p->blargs.nu] = nt;
    const double patch_px = (double)P.params.nfeatures * (KP_PATCH_ROWS * KP_PATCH_COLS);
    p->lb_auto = patch_px > ORBX_LB_RATIO * (double)P.geo.pixels ? 1 : 0;
  }
  // FAST strip LDS: tile + strength map + row masks + counts + cell slots +
  // corner list, per launch group
  {
    p->fs_tpitch = (15 + P.strip_max_w + 8 + 15) & ~15; /* lead <= 15, row reads up to +8 */
    hipFuncAttributes fa;
    const size_t st = hipFuncGetAttributes(&fa, (const void*)k_fast_strips_p288) == hipSuccess ? fa.sharedSizeBytes : 4096;
    /* dynamic LDS of a workgroup (the NMS masks reuse the tile when they fit,
     * k_fast_strips), and the workgroups per CU it leaves: up to the 6 that
     * k_fast_strips' 75 VGPRs allow, LDS counted in 1-KB steps (conservative)
     * with the kernel's static LDS */
    const auto lds_for = [&](int tmaxh, int mcells, int ccap) {
      const size_t tile = (size_t)p->fs_tpitch * tmaxh;
      const size_t masks = 16 * (size_t)mcells * (tmaxh - 6);
      return tile + (size_t)p->fs_tpitch * (tmaxh - 6) + 8 * (size_t)((mcells + 3) & ~3) +
             (masks <= tile ? 0 : masks) + 2 * (size_t)((ccap + 3) & ~3);
    };
    const auto wgs = [&](size_t lds) { return std::min<size_t>(6, 163840 / (((lds + st) + 1023) & ~(size_t)1023)); };
    const int mcells = std::max(P.strip_max_cells, 1);
    /* When the tallest strip keeps even a shortened corner list below 6
     * workgroups per CU, the strips no taller than hA (6 workgroups with the
     * whole list) go first and the taller ones (a few small levels with
     * taller cells: KITTI levels 5-6 have 44-46-row strips, 37-39 elsewhere)
     * behind them, in a second launch: they no longer set every strip's LDS
     * (round 5: c5 FAST 0.649 -> 0.616 ms).  Where a shortened list reaches
     * 6 for all strips, one launch stays (640x480: a second launch for its
     * ten 40-row strips measured +3.5 %).  Strip order changes no result:
     * each strip writes its own cells. */
    int hA = 0;
    for (const StripInfo& si : P.strips)
      if (wgs(lds_for(std::max(si.h, 7), mcells, FS_CCAP)) >= 6) hA = std::max(hA, si.h);
    Plan& PM = p->P;
    const int tallest = std::max(P.strip_max_h, 7);
    const bool one_fits = wgs(lds_for(tallest, mcells, FS_CCAP_MIN)) >= 6;
    if (hA > 0 && hA < P.strip_max_h && !one_fits && !p->ccap_fixed_dbg) {
      std::stable_partition(PM.strips.begin(), PM.strips.end(), [&](const StripInfo& si) { return si.h <= hA; });
      int na = 0;
      while (na < (int)PM.strips.size() && PM.strips[na].h <= hA) ++na;
      PM.nstrips_l0 = 0;
      while (PM.nstrips_l0 < na && PM.strips[PM.nstrips_l0].level == 0) ++PM.nstrips_l0;
      p->fs_ngrp = 2;
      p->fs_grp[0].begin = 0;
      p->fs_grp[0].end = na;
      p->fs_grp[0].tmaxh = std::max(hA, 7);
      p->fs_grp[1].begin = na;
      p->fs_grp[1].end = (int)PM.strips.size();
      p->fs_grp[1].tmaxh = tallest;
    } else {
      p->fs_ngrp = 1;
      p->fs_grp[0].begin = 0;
      p->fs_grp[0].end = (int)PM.strips.size();
      p->fs_grp[0].tmaxh = tallest;
    }
    for (int g = 0; g < p->fs_ngrp; ++g) {
      orbx_plan::FsGroup& G = p->fs_grp[g];
      G.mcells = 1;
      for (int k = G.begin; k < G.end; ++k) G.mcells = std::max(G.mcells, PM.strips[k].ncells);
      G.ccap = p->fs_ccap;
      if (!p->ccap_fixed_dbg) {
        /* the corner list (FS_CCAP entries, ~60 used per strip at 1080p) is
         * shortened, down to FS_CCAP_MIN, when that fits one more workgroup
         * per CU: 640x480 x 8 levels (40-row strips) 5 -> 6 workgroups, 830
         * entries, FAST -8 %, no strip over the list on the bench frames; a
         * strip over it takes the strength-map scan (round 5) */
        const size_t w0 = wgs(lds_for(G.tmaxh, G.mcells, FS_CCAP));
        if (w0 < 6)
          for (int c = FS_CCAP - 2; c >= FS_CCAP_MIN; c -= 2)
            if (wgs(lds_for(G.tmaxh, G.mcells, c)) > w0) { G.ccap = c; break; }
      }
      G.lds = lds_for(G.tmaxh, G.mcells, G.ccap);
#ifdef FS_LDS_PAD  // profiling variant: occupancy sensitivity of k_fast_strips
      G.lds += FS_LDS_PAD;
#endif
      if (G.lds > 150 * 1024) { plan_free(p); return ORBX_ERR_UNSUPPORTED; }
    }
  }
  hipStream_t us = p->stream;
  if (upload(&p->d_lv, P.levels, us) || upload(&p->d_cells, P.cells, us) ||
      upload(&p->d_strips, P.strips, us) || upload(&p->d_xofs, P.xofs, us) ||
      upload(&p->d_xofs1, P.xofs1, us) || upload(&p->d_yofs, P.yofs, us) ||
      upload(&p->d_alpha, P.alpha, us) || upload(&p->d_beta, P.beta, us) ||
      upload(&p->d_pyr_xs, P.pyr_xs, us) || upload(&p->d_pyr_ys, P.pyr_ys, us) ||
      upload(&p->d_pyr_bo, P.pyr_bo, us) || upload(&p->d_pyr_blob, P.pyr_blob, us)) {
    plan_free(p);
    return ORBX_ERR_HIP;
  }
  p->pyr_stride = round_up((size_t)P.pyr_bytes, 256);
  p->blur_stride = round_up((size_t)P.blur_bytes, 256);
  if (p->lb_auto && dev_alloc((void**)&p->d_blur, (size_t)max_batch * p->blur_stride)) {
    plan_free(p);
    return ORBX_ERR_HIP;
  }
  p->slot_stride = round_up((size_t)P.nslots, 64);
  p->qk_stride = round_up((size_t)P.qk_elems, 64);
  p->qout_stride = round_up((size_t)P.kcap, 64);
  const size_t B = (size_t)max_batch;
  if (dev_alloc((void**)&p->d_pyr, B * p->pyr_stride) ||
      dev_alloc((void**)&p->d_slots, B * p->slot_stride * 4) ||
      dev_alloc((void**)&p->d_ccount, B * (size_t)(P.ncells ? P.ncells : 1) * 4) ||
      dev_alloc((void**)&p->d_qkeys, B * p->qk_stride * 4) ||
      dev_alloc((void**)&p->d_qnode, B * p->qk_stride * 4) ||
      dev_alloc((void**)&p->d_qout, B * p->qout_stride * 4) ||
      dev_alloc((void**)&p->d_qperm, B * p->qout_stride * 4) ||
      dev_alloc((void**)&p->d_lcount, B * (size_t)P.params.nlevels * 4) ||
      dev_alloc((void**)&p->d_err, 16)) {
    plan_free(p);
    return ORBX_ERR_HIP;
  }
  // stream-ordered: no device-wide synchronisation (other extractors and
  // the matcher may be running on this device from other threads)
  if (hipMemsetAsync(p->d_err, 0, 16, us) != hipSuccess ||
      hipMemsetAsync(p->d_ccount, 0, B * (size_t)(P.ncells ? P.ncells : 1) * 4, us) != hipSuccess ||
      hipStreamSynchronize(us) != hipSuccess) { plan_free(p); return ORBX_ERR_HIP; }
  *out = p;
  return ORBX_OK;
}

extern "C" int orbx_plan_destroy(orbx_plan* p) {
  plan_free(p);
  return ORBX_OK;
}

extern "C" int orbx_plan_geometry(const orbx_plan* p, orbx_geometry* g) {
  if (!p || !g) return ORBX_ERR_ARG;
  *g = p->P.geo;
  return ORBX_OK;
}

extern "C" int orbx_plan_set_timing(orbx_plan* p, int enable) {
  if (!p) return ORBX_ERR_ARG;
  hipSetDevice(p->device);
  p->timer.reset(enable != 0);
  return ORBX_OK;
}

extern "C" int orbx_plan_stage_times(orbx_plan* p, double* ms, int* launches, int n) {
  if (!p) return ORBX_ERR_ARG;
  hipSetDevice(p->device);
  return p->timer.collect(ms, launches, n);
}

// one extraction pass over frames [0, n) of the given (already offset) buffers
static int extract_pass(orbx_plan* p, const uint8_t* frames, int n, size_t fstride, size_t rstride,
                        orbx_keypoint* kps, uint8_t* desc, int* counts, hipStream_t s, size_t f0) {
  const Plan& P = p->P;
  const int L = P.params.nlevels;
  uint8_t* const d_pyr = p->d_pyr + f0 * p->pyr_stride;
  uint32_t* const d_slots = p->d_slots + f0 * p->slot_stride;
  uint32_t* const d_ccount = p->d_ccount + f0 * (size_t)P.ncells;
  uint32_t* const d_qkeys = p->d_qkeys + f0 * p->qk_stride;
  int32_t* const d_qnode = p->d_qnode + f0 * p->qk_stride;
  uint32_t* const d_qout = p->d_qout + f0 * p->qout_stride;
  int* const d_lcount = p->d_lcount + f0 * (size_t)L;
  // strips [strip0, strip1) of launch group g
  // the call's level-0 alignment (k_fast_strips takes the planner's staging
  // decisions when the frames are 16-B aligned)
  LevelArgs la = p->largs;
  la.l0al16 = ((reinterpret_cast<uintptr_t>(frames) | (uintptr_t)fstride | (uintptr_t)rstride) & 15) == 0;
  auto fast_launch = [&](int g, int strip0, int strip1, hipStream_t st) {
    if (strip1 <= strip0) return;
    const orbx_plan::FsGroup& G = p->fs_grp[g];
    hipLaunchKernelGGL(p->fs_tpitch == 288 ? k_fast_strips_p288 : k_fast_strips, dim3((unsigned)(strip1 - strip0), n), dim3(FS_NT), G.lds + p->pad_fast, st,
                       frames, fstride, rstride, d_pyr, p->pyr_stride, la, p->d_cells,
                       p->d_strips, d_slots, p->slot_stride, d_ccount, P.ncells, P.ini_th,
                       P.min_th, p->fs_tpitch, G.tmaxh, G.mcells, G.ccap,
                       p->d_err + ORBX_ERRW_FAST_OVF, strip0, p->dbg);
  };
  const bool overlap = p->overlap && p->s_aux && P.nstrips_l0 > 0;
  if (overlap) {
    // FAST on level 0 (which needs no pyramid) runs on the auxiliary stream
    // beside the pyramid kernel; the other levels' strips follow the pyramid
    if (hipEventRecord(p->ev_aux0, s) != hipSuccess || hipStreamWaitEvent(p->s_aux, p->ev_aux0, 0) != hipSuccess)
      return ORBX_ERR_HIP;
    fast_launch(0, 0, P.nstrips_l0, p->s_aux);  // level 0's strips lead group 0
    if (hipEventRecord(p->ev_aux1, p->s_aux) != hipSuccess) return ORBX_ERR_HIP;
  }
  // K1 pyramid: the tile chain (many small workgroups per frame; the
  // row-streaming and fused kernels of round 4 measured slower and were
  // retired)
  p->timer.begin(ORBX_STAGE_RESIZE, s);
  for (const PyrSeg& g : P.segs) {
    if (g.area) {
      hipLaunchKernelGGL(k_pyr_area2, dim3((unsigned)((g.w[1] + 1023) / 1024), (unsigned)g.h[1], (unsigned)n),
                         dim3(256), 0, s, frames, fstride, rstride, d_pyr, p->pyr_stride, g);
      continue;
    }
    PyrSeg gp = g;
    gp.prio = p->largs.prio;
    hipLaunchKernelGGL(k_pyramid, dim3(g.ntx * g.nty, n), dim3(256),
                       g.lds_a + g.lds_b + g.lds_yl + p->pad_pyr, s, frames, fstride, rstride,
                       d_pyr, p->pyr_stride, gp, reinterpret_cast<const int4*>(p->d_pyr_xs),
                       reinterpret_cast<const int4*>(p->d_pyr_ys),
                       reinterpret_cast<const uint4*>(p->d_pyr_blob), p->d_pyr_bo, p->dbg);
  }
  p->timer.end(ORBX_STAGE_RESIZE, s);
  if (p->ev_after_pyr && hipEventRecord(p->ev_after_pyr, s) != hipSuccess) return ORBX_ERR_HIP;
  // K2 FAST cells
  p->timer.begin(ORBX_STAGE_FAST, s);
  for (int g = 0; g < p->fs_ngrp; ++g)
    fast_launch(g, overlap && g == 0 ? P.nstrips_l0 : p->fs_grp[g].begin, p->fs_grp[g].end, s);
  if (overlap && hipStreamWaitEvent(s, p->ev_aux1, 0) != hipSuccess) return ORBX_ERR_HIP;
  p->timer.end(ORBX_STAGE_FAST, s);
  if (p->dbg && p->dbg < 20) return ORBX_OK; /* phase probe: later stages would read partial results */
  // level-blur mode: the 7x7 Gaussian of every unique level (the stage runs
  // beside nothing: it reads the levels the pyramid wrote and the BRIEF
  // kernel reads its output)
  uint8_t* const d_blur = p->uses_lb() ? p->d_blur + f0 * p->blur_stride : nullptr;
  if (d_blur) {
    p->timer.begin(ORBX_STAGE_BLUR, s);
    hipLaunchKernelGGL(k_blur, dim3((unsigned)p->blargs.tile_begin[p->blargs.nu], n), dim3(256), 0, s, frames,
                       fstride, rstride, d_pyr, p->pyr_stride, d_blur, p->blur_stride, p->blargs);
    p->timer.end(ORBX_STAGE_BLUR, s);
  }
  // K3 DistributeOctTree
  p->timer.begin(ORBX_STAGE_QUADTREE, s);
  // keys per thread in registers: 8 for 1080p-class level 0, else 6
  // (qt_body); a call of a few frames (the drop-in's one frame per
  // Frame::ExtractORB) leaves the chip mostly idle and the level-0 workgroup
  // sets the latency: 1024-thread workgroups there
  bool qt_wide = (long long)n * L <= 64 && p->qt_lds_wide <= 150 * 1024;
#ifdef ORBX_PROFILING
  if (const char* e = getenv("ORBX_DEBUG_QT_WIDE")) qt_wide = atoi(e) != 0 && p->qt_lds_wide <= 150 * 1024;  // A/B (profiling only)
#endif
  hipLaunchKernelGGL(qt_wide ? k_quadtree_wide : P.levels[0].w * P.levels[0].h >= (1 << 20) ? k_quadtree : k_quadtree_j6,
                     dim3(n, L), dim3(qt_wide ? 1024 : 256), qt_wide ? p->qt_lds_wide : p->qt_lds, s, p->d_lv, p->d_cells,
                     d_slots, p->slot_stride, d_ccount, P.ncells, d_qkeys, d_qnode,
                     p->qk_stride, d_qout, p->qout_stride, d_lcount, L, P.qt_smax,
                     P.qt_max_cells, p->d_err, p->d_qperm + f0 * p->qout_stride);
  p->timer.end(ORBX_STAGE_QUADTREE, s);
  // K4+K5+K6+K7 orientation, blur-at-sample descriptors, assembly
  p->timer.begin(ORBX_STAGE_BRIEF, s);
  // waves stride over each frame's keypoints (about nfeatures of them)
  // (about 12 keypoints per wave once the batch alone fills the chip: the
  // next patch's loads overlap the current keypoint and the per-wave setup
  // -- pattern registers, exception keys, level scan -- is amortised; 4 / 8
  // / 12 / 16 / 24 per wave measured 0.535 / 0.522 / 0.521 / 0.531 / 0.538 ms
  // at c4, 1.004 / 0.961 / 0.947 / 0.946 / 0.956 at c1).  Frames of 1 Mpx
  // and more take about 6: the frames of an XCD are dispatched one after
  // the other (frame_unit), so more waves per frame means fewer frames'
  // patch bands resident in its L2 at once and more of the patches' line
  // overlap caught there -- c4 HBM reads 1726 -> 1311 MB per launch (1.58x
  // -> 1.20x the algorithmic bytes) for +1.2 % BRIEF time
  // (tools/obdiv_fetch.sh: ~12 / 6 / 3 / 2 / 1 per wave read 1726 / 1311 /
  // 1091 / 1119 / 1003 MB in 0.544 / 0.551 / 0.576 / 0.599 / 0.653 ms)
  const int ob_full = std::max(4, std::min(P.kcap, P.params.nfeatures + 256));
  const int ob_kpw = (long long)P.levels[0].w * P.levels[0].h >= (1 << 20) ? 6 : 12;
  int ob_waves = std::min(ob_full, std::max((ob_full + ob_kpw - 1) / ob_kpw, (16384 + n - 1) / n));
  if (p->ob_div > 0) ob_waves = std::max(4, ob_full / p->ob_div); /* profiling only */
  if (p->uses_lb()) {
    hipLaunchKernelGGL(k_orient_brief_lb, dim3((ob_waves + 3) / 4, n),
                       dim3(256), p->pad_brief, s, frames, fstride, rstride, d_pyr, p->pyr_stride, p->bargs,
                       d_qout, p->qout_stride, d_lcount, kps, desc,
                       counts, p->d_qperm + f0 * p->qout_stride, p->dbg, d_blur, p->blur_stride);
  } else {
    hipLaunchKernelGGL(k_orient_brief, dim3((ob_waves + 3) / 4, n),
                       dim3(256), p->pad_brief, s, frames, fstride, rstride, d_pyr, p->pyr_stride, p->bargs,
                       d_qout, p->qout_stride, d_lcount, kps, desc,
                       counts, p->d_qperm + f0 * p->qout_stride, p->dbg);
  }
  p->timer.end(ORBX_STAGE_BRIEF, s);
  if (hipGetLastError() != hipSuccess) return ORBX_ERR_HIP;
  return ORBX_OK;
}

extern "C" int orbx_plan_extract(orbx_plan* p, const uint8_t* frames, int nframes,
                                 size_t fstride, size_t rstride, orbx_keypoint* kps,
                                 uint8_t* desc, int* counts, void* stream) {
  if (!p || !frames || !kps || !desc || !counts || nframes < 1 || nframes > p->max_batch)
    return ORBX_ERR_ARG;
  const Plan& P = p->P;
  if (rstride < (size_t)P.W || fstride < rstride * (size_t)P.H) return ORBX_ERR_ARG;
  /* the kernels form row offsets with 24-bit multiplies (__umul24) and the
   * BRIEF patch base of level 0 (the caller's frame) as a 32-bit product of
   * row and stride: every row offset of a frame must fit 32 bits */
  if (rstride >= ((size_t)1 << 24) || rstride * (size_t)P.H >= ((size_t)1 << 32))
    return ORBX_ERR_UNSUPPORTED;
  ORBX_TRY(hipSetDevice(p->device));
  hipStream_t s = (hipStream_t)stream; /* NULL = the default stream */
  // frames in passes of p->chunk: one pass's pyramid levels stay in the
  // Infinity Cache for its FAST and BRIEF reads
  const int ck = p->chunk > 0 ? p->chunk : nframes;
  const size_t kc = (size_t)P.kcap;
  p->nextracted = 0;
  for (int c = 0; c < nframes; c += ck) {
    const int rc = extract_pass(p, frames + (size_t)c * fstride, std::min(ck, nframes - c), fstride, rstride,
                                kps + (size_t)c * kc, desc + (size_t)c * kc * 32, counts + c, s, (size_t)c);
    if (rc) return rc;
  }
  p->nextracted = nframes;
  return ORBX_OK;
}

extern "C" int orbx_plan_check(orbx_plan* p, void* stream) {
  if (!p) return ORBX_ERR_ARG;
  ORBX_TRY(hipSetDevice(p->device));
  hipStream_t s = (hipStream_t)stream; /* NULL = the default stream */
  ORBX_TRY(hipMemcpyAsync(p->h_err, p->d_err, sizeof(int), hipMemcpyDeviceToHost, s));
  ORBX_TRY(hipStreamSynchronize(s));
  const int err = *p->h_err;
  if (err) {
    ORBX_TRY(hipMemsetAsync(p->d_err, 0, sizeof(int), s));
    ORBX_TRY(hipStreamSynchronize(s));
    if (err & ORBX_DEVERR_QUADTREE) return ORBX_ERR_QUADTREE;
    return ORBX_ERR_CAPACITY;
  }
  return ORBX_OK;
}

extern "C" int orbx_plan_set_options(orbx_plan* p, int flags) {
  if (!p || (flags & ~(ORBX_PLAN_PYR_TILES | ORBX_PLAN_BRIEF_PATCH | ORBX_PLAN_BRIEF_LEVEL)) ||
      (flags & (ORBX_PLAN_BRIEF_PATCH | ORBX_PLAN_BRIEF_LEVEL)) == (ORBX_PLAN_BRIEF_PATCH | ORBX_PLAN_BRIEF_LEVEL))
    return ORBX_ERR_ARG;
  if ((flags & ORBX_PLAN_BRIEF_LEVEL) && !p->d_blur) {
    ORBX_TRY(hipSetDevice(p->device));
    ORBX_TRY(hipStreamSynchronize(p->stream));
    if (dev_alloc((void**)&p->d_blur, (size_t)p->max_batch * p->blur_stride)) return ORBX_ERR_HIP;
  }
  p->options = flags;
  return ORBX_OK;
}

extern "C" int orbx_plan_level(orbx_plan* p, int frame, int level, uint8_t* dst, size_t dst_stride, int* width,
                               int* height, void* stream) {
  if (!p || frame < 0 || frame >= p->max_batch || level < 0 || level >= p->P.params.nlevels) return ORBX_ERR_ARG;
  const LevelInfo& L = p->P.levels[level];
  if (width) *width = L.w;
  if (height) *height = L.h;
  if (L.unique == 0) return ORBX_ERR_ARG;
  if (!dst) return ORBX_OK;
  if (frame >= p->nextracted) return ORBX_ERR_ARG; /* frames the last extraction wrote */
  if (dst_stride < (size_t)L.w) return ORBX_ERR_ARG;
  ORBX_TRY(hipSetDevice(p->device));
  hipStream_t s = (hipStream_t)stream;
  const uint8_t* src = p->d_pyr + (size_t)frame * p->pyr_stride + p->P.levels[L.unique].pyr_off;
  ORBX_TRY(hipMemcpy2DAsync(dst, dst_stride, src, (size_t)L.pitch, (size_t)L.w, (size_t)L.h,
                            hipMemcpyDeviceToHost, s));
  ORBX_TRY(hipStreamSynchronize(s));
  return ORBX_OK;
}

extern "C" int orbx_plan_debug_counters(orbx_plan* p, int* fast_overflow_strips) {
  if (!p || !fast_overflow_strips) return ORBX_ERR_ARG;
  ORBX_TRY(hipSetDevice(p->device));
  int v = 0;
  ORBX_TRY(hipMemcpyAsync(&p->h_err[ORBX_ERRW_FAST_OVF], p->d_err + ORBX_ERRW_FAST_OVF, sizeof(int),
                          hipMemcpyDeviceToHost, p->stream));
  ORBX_TRY(hipStreamSynchronize(p->stream));
  v = p->h_err[ORBX_ERRW_FAST_OVF];
  ORBX_TRY(hipMemsetAsync(p->d_err + ORBX_ERRW_FAST_OVF, 0, sizeof(int), p->stream));
  ORBX_TRY(hipStreamSynchronize(p->stream));
  *fast_overflow_strips = v;
  return ORBX_OK;
}

extern "C" int orbx_synth_frames(uint8_t* d_frames, int W, int H, size_t fstride, int nframes,
                                 int first_idx, int kind, void* stream) {
  if (!d_frames || W <= 0 || H <= 0 || nframes < 1 || kind < 0 || kind > 3 ||
      fstride < (size_t)W * H)
    return ORBX_ERR_ARG;
  const long long npx = (long long)W * H;
  dim3 grid((unsigned)((npx + 4095) / 4096), nframes);
  hipLaunchKernelGGL(k_synth, grid, dim3(256), 0, (hipStream_t)stream, d_frames, W, H, fstride,
                     first_idx, kind);
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_ERR_HIP;
}

extern "C" int orbx_selftest_sincos(const float* d_x, int n, float* d_sc, void* stream) {
  if (n < 0 || (n > 0 && (!d_x || !d_sc))) return ORBX_ERR_ARG;
  if (n == 0) return ORBX_OK;
  hipLaunchKernelGGL(k_selftest_sincos, dim3(n), dim3(64), 0, (hipStream_t)stream, d_x, n, d_sc);
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_ERR_HIP;
}

extern "C" int orbx_selftest_sincos_range(uint32_t first_bits, int n, float* sc, int device) {
  if (n < 0 || (n > 0 && !sc)) return ORBX_ERR_ARG;
  if (n == 0) return ORBX_OK;
  if (device < 0 || device >= orbx_device_count()) return ORBX_ERR_NO_DEVICE;
  ORBX_TRY(hipSetDevice(device));
  WsLease L(device);
  CallWs* w = L.w;
  if (!w) return ORBX_ERR_HIP;
  const size_t bytes = (size_t)n * 8;
  int rc = w->reserve(bytes, 0);
  if (rc) return rc;
  hipLaunchKernelGGL(k_selftest_sincos_range, dim3((n + 255) / 256), dim3(256), 0, w->stream,
                     first_bits, n, reinterpret_cast<float*>(w->d));
  if (hipGetLastError() != hipSuccess) return ORBX_ERR_HIP;
  ORBX_TRY(hipMemcpyAsync(sc, w->d, bytes, hipMemcpyDeviceToHost, w->stream));
  ORBX_TRY(hipStreamSynchronize(w->stream));
  return ORBX_OK;
}

// ---------------------------------------------------------------------------
// orbx_extractor: the ORBextractor::operator() drop-in (host buffers).
// ---------------------------------------------------------------------------

static void extractor_release_plan(orbx_extractor* e) {
  hipSetDevice(e->device);
  orbx_stereo_release(e);
  if (e->plan) orbx_plan_destroy(e->plan);
  if (e->d_img) hipFree(e->d_img);
  if (e->d_kps) hipFree(e->d_kps);
  if (e->d_desc) hipFree(e->d_desc);
  if (e->d_count) hipFree(e->d_count);
  if (e->h_res) hipHostFree(e->h_res);
  if (e->h_img) hipHostFree(e->h_img);
  if (e->h_pyr) hipHostFree(e->h_pyr);
  if (e->ev_pyr) hipEventDestroy(e->ev_pyr);
  if (e->s_copy) hipStreamDestroy(e->s_copy);
  e->plan = nullptr; e->d_img = nullptr; e->d_kps = nullptr; e->d_desc = nullptr;
  e->d_count = nullptr; e->h_res = nullptr; e->d_res = nullptr; e->W = e->H = 0; e->have_frame = false;
  e->h_img = nullptr; e->h_pyr = nullptr; e->ev_pyr = nullptr; e->s_copy = nullptr;
  e->pyr_bytes = 0; e->host_pyr = false;
}

static int extractor_prepare(orbx_extractor* e, int W, int H) {
  if (e->plan && e->W == W && e->H == H) return ORBX_OK;
  extractor_release_plan(e);
  int rc = orbx_plan_create(&e->params, W, H, 1, e->device, &e->plan);
  if (rc) return rc;
  const size_t kcap = (size_t)std::max(e->plan->P.kcap, 1);
  if (dev_alloc((void**)&e->d_img, (size_t)W * H) ||
      dev_alloc((void**)&e->d_kps, sizeof(orbx_keypoint) * kcap + 16) ||  /* + k_pack_results' last 16-B chunk */
      dev_alloc((void**)&e->d_desc, 32 * kcap) ||
      dev_alloc((void**)&e->d_count, sizeof(int)) ||
      hipHostMalloc((void**)&e->h_res, 64 + 16 + (sizeof(orbx_keypoint) + 32) * kcap,
                    hipHostMallocDefault) != hipSuccess ||
      hipHostGetDevicePointer((void**)&e->d_res, e->h_res, 0) != hipSuccess ||
      hipHostMalloc((void**)&e->h_img, (size_t)W * H, hipHostMallocDefault) != hipSuccess) {
    extractor_release_plan(e);
    return ORBX_ERR_HIP;
  }
  e->pyr_bytes = (size_t)e->plan->P.pyr_bytes;
  if ((e->pyr_bytes && hipHostMalloc((void**)&e->h_pyr, e->pyr_bytes, hipHostMallocDefault) != hipSuccess) ||
      hipStreamCreateWithFlags(&e->s_copy, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&e->ev_pyr, hipEventDisableTiming) != hipSuccess) {
    extractor_release_plan(e);
    return ORBX_ERR_HIP;
  }
  e->last_k = 0;
  e->W = W;
  e->H = H;
  return ORBX_OK;
}

extern "C" int orbx_extractor_create(const orbx_params* p, int device, orbx_extractor** out) {
  if (!p || !out) return ORBX_ERR_ARG;
  *out = nullptr;
  Tables t;
  int rc = compute_tables(*p, t);
  if (rc) return rc;
  if (device < 0 || device >= orbx_device_count()) return ORBX_ERR_NO_DEVICE;
  orbx_extractor* e = new orbx_extractor();
  e->params = *p;
  e->device = device;
  *out = e;
  return ORBX_OK;
}

extern "C" int orbx_extractor_destroy(orbx_extractor* e) {
  if (!e) return ORBX_OK;
  extractor_release_plan(e);
  delete e;
  return ORBX_OK;
}

extern "C" int orbx_extractor_capacity(orbx_extractor* e, int W, int H, int* kcap) {
  if (!e || !kcap) return ORBX_ERR_ARG;
  if (e->plan && e->W == W && e->H == H) {  // every call of the drop-in asks: no re-planning
    *kcap = e->plan->P.kcap;
    return ORBX_OK;
  }
  Plan P;
  int rc = plan_geometry(e->params, W, H, P);
  if (rc) return rc;
  *kcap = P.kcap;
  return ORBX_OK;
}

extern "C" int orbx_extract(orbx_extractor* e, const uint8_t* img, int W, int H, size_t stride,
                            orbx_keypoint* kps, int cap, uint8_t* desc, int* n) {
  if (!e || !n) return ORBX_ERR_ARG;
  *n = 0;
  if (!img || W <= 0 || H <= 0) return ORBX_OK; /* _image.empty(): return (:444-445) */
  if (stride < (size_t)W) return ORBX_ERR_ARG;
  int rc = extractor_prepare(e, W, H);
  if (rc) return rc;
  ORBX_TRY(hipSetDevice(e->device));
  orbx_plan* p = e->plan;
  hipStream_t s = p->stream;
  e->host_pyr = false;
  ++e->n_calls;
  const bool to_host = (e->flags & ORBX_EXTRACTOR_PYRAMID_TO_HOST) != 0;
  if (!(e->flags & ORBX_EXTRACTOR_PINNED_H2D)) {
    // straight from the caller's (pageable) rows: the runtime's own staging
    // measured faster than a host copy into pinned memory (176 vs 257 us per
    // 1080p call, bench latency leg)
    // (a 1D copy for contiguous rows measured no faster: p50 180 vs 174-229 us)
    ORBX_TRY(hipMemcpy2DAsync(e->d_img, (size_t)W, img, stride, (size_t)W, (size_t)H,
                              hipMemcpyHostToDevice, s));
  } else {
    // through the pinned staging buffer in row chunks of ~256 KB: the host
    // copy of chunk c+1 runs while chunk c is DMA'd (measurement option)
    const int rows_per = std::max(1, (256 << 10) / W);
    for (int r0 = 0; r0 < H; r0 += rows_per) {
      const int nr = std::min(rows_per, H - r0);
      uint8_t* h = e->h_img + (size_t)r0 * W;
      if (stride == (size_t)W) {
        memcpy(h, img + (size_t)r0 * W, (size_t)nr * W);
      } else {
        for (int r = 0; r < nr; ++r) memcpy(h + (size_t)r * W, img + (size_t)(r0 + r) * stride, (size_t)W);
      }
      ORBX_TRY(hipMemcpyAsync(e->d_img + (size_t)r0 * W, h, (size_t)nr * W, hipMemcpyHostToDevice, s));
    }
  }
  // one launch writes the count, the error word and exactly the frame's
  // rows into the pinned staging (k_pack_results, over PCIe)
  const int kcap = std::max(p->P.kcap, 1);
  const int* h_hdr = reinterpret_cast<const int*>(e->h_res);  // {count, error word}
  orbx_keypoint* h_kps = reinterpret_cast<orbx_keypoint*>(e->h_res + 64);
  // descriptor rows at a 16-B boundary (k_pack_results copies 16 B per lane)
  const size_t desc_off = (64 + sizeof(orbx_keypoint) * (size_t)kcap + 15) & ~(size_t)15;
  uint8_t* h_desc = e->h_res + desc_off;
  auto chain = [&]() -> int {
    const int r = orbx_plan_extract(p, e->d_img, 1, (size_t)W * H, (size_t)W, e->d_kps, e->d_desc,
                                    e->d_count, s);
    if (r) return r;
    hipLaunchKernelGGL(k_pack_results, dim3(std::min((kcap * 8 + 255) / 256, 64)), dim3(256), 0, s,
                       p->d_err, e->d_count, reinterpret_cast<const uint4*>(e->d_kps),
                       reinterpret_cast<const uint4*>(e->d_desc), kcap, reinterpret_cast<uint4*>(e->d_res),
                       (uint32_t)(desc_off / 16));
    return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_ERR_HIP;
  };
  // (the chain captured once as a HIP graph and replayed was measured: no
  // change in the call's latency, p50 174-176 us either way in the probe --
  // the gap after the upload is the pageable copy's completion, not the
  // host's launches; not kept)
  p->ev_after_pyr = to_host ? e->ev_pyr : nullptr;
  rc = chain();
  p->ev_after_pyr = nullptr;
  if (rc) return rc;
  if (to_host && e->pyr_bytes) {
    // the level buffer (levels >= 2) comes back on the copy stream while
    // FAST, the quadtree and BRIEF run, once the pyramid kernel is done
    ORBX_TRY(hipStreamWaitEvent(e->s_copy, e->ev_pyr, 0));
    ORBX_TRY(hipMemcpyAsync(e->h_pyr, p->d_pyr, e->pyr_bytes, hipMemcpyDeviceToHost, e->s_copy));
  }

  if (to_host && !(e->flags & ORBX_EXTRACTOR_PINNED_H2D)) {
    // level 0 (= level 1) of the host pyramid: a host copy of the caller's
    // rows made while the GPU works (the thread would only wait), instead of
    // a D2H of the uploaded image on the copy stream ahead of the levels
    if (stride == (size_t)W) {
      memcpy(e->h_img, img, (size_t)W * H);
    } else {
      for (int r = 0; r < H; ++r) memcpy(e->h_img + (size_t)r * W, img + (size_t)r * stride, (size_t)W);
    }
  }
  ORBX_TRY(stream_wait(s));
  if (to_host) ORBX_TRY(stream_wait(e->s_copy));
  if (h_hdr[1]) {
    rc = orbx_plan_check(p, s); /* resets the device error word */
    e->have_frame = false;
    return rc ? rc : ORBX_ERR_CAPACITY;
  }
  e->have_frame = true;
  e->host_pyr = to_host;
  const int K = h_hdr[0];
  *n = K;
  if (K == 0) return ORBX_OK; /* keypoints untouched, descriptors released (:460-463) */
  if (K > cap || !kps || !desc) return ORBX_ERR_CAPACITY;
  e->last_k = K;
  memcpy(kps, h_kps, sizeof(orbx_keypoint) * (size_t)K);
  memcpy(desc, h_desc, 32 * (size_t)K);
  return ORBX_OK;
}

extern "C" int orbx_extractor_set_options(orbx_extractor* e, int flags) {
  if (!e || (flags & ~(ORBX_EXTRACTOR_PYRAMID_TO_HOST | ORBX_EXTRACTOR_PINNED_H2D))) return ORBX_ERR_ARG;
  e->flags = flags;
  return ORBX_OK;
}

extern "C" int orbx_extractor_stats(orbx_extractor* e, long long* calls, long long* refetches) {
  if (!e) return ORBX_ERR_ARG;
  if (calls) *calls = e->n_calls;
  if (refetches) *refetches = e->n_refetch;
  return ORBX_OK;
}

extern "C" int orbx_extractor_level_host(orbx_extractor* e, int level, const uint8_t** data,
                                         size_t* stride, int* width, int* height) {
  if (!e || !e->plan || !e->have_frame || !e->host_pyr || level < 0 || level >= e->params.nlevels)
    return ORBX_ERR_ARG;
  const LevelInfo& L = e->plan->P.levels[level];
  if (width) *width = L.w;
  if (height) *height = L.h;
  if (L.unique == 0) {
    if (data) *data = e->h_img;
    if (stride) *stride = (size_t)e->W;
  } else {
    if (data) *data = e->h_pyr + e->plan->P.levels[L.unique].pyr_off;
    if (stride) *stride = (size_t)L.pitch;
  }
  return ORBX_OK;
}

extern "C" int orbx_extractor_level(orbx_extractor* e, int level, uint8_t* dst, size_t dst_stride,
                                    int* width, int* height) {
  if (!e || !e->plan || !e->have_frame || level < 0 || level >= e->params.nlevels)
    return ORBX_ERR_ARG;
  const LevelInfo& L = e->plan->P.levels[level];
  if (width) *width = L.w;
  if (height) *height = L.h;
  if (!dst) return ORBX_OK;
  if (dst_stride < (size_t)L.w) return ORBX_ERR_ARG;
  ORBX_TRY(hipSetDevice(e->device));
  const uint8_t* src;
  size_t pitch;
  if (L.unique == 0) {
    src = e->d_img;
    pitch = (size_t)e->W;
  } else {
    src = e->plan->d_pyr + e->plan->P.levels[L.unique].pyr_off;
    pitch = (size_t)L.pitch;
  }
  ORBX_TRY(hipMemcpy2DAsync(dst, dst_stride, src, pitch, (size_t)L.w, (size_t)L.h,
                            hipMemcpyDeviceToHost, e->plan->stream));
  ORBX_TRY(hipStreamSynchronize(e->plan->stream));
  return ORBX_OK;
}
