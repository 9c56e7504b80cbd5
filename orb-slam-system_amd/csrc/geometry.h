/* geometry.h -- host-side planning of a (params, width, height) extraction:
 * constant tables, pyramid sizes, resize LUTs, FAST cell grid, quadtree
 * parameters and the per-frame HBM layout (orbx_internal.h). */
#ifndef ORBX_GEOMETRY_H
#define ORBX_GEOMETRY_H

#include <stdint.h>

#include <vector>

#include "../../include/orbx.h"
#include "orbx_internal.h"

namespace orbx {

struct Tables {
  int nlevels = 0;
  double scaleFactor = 0;
  std::vector<float> scale, inv_scale, sigma2, inv_sigma2;
  std::vector<int> features;
  int umax[16];
};

/* ORBextractor::ORBextractor (src/ORBextractor.cc:116-170) */
int compute_tables(const orbx_params& p, Tables& t);

struct Plan {
  orbx_params params;
  Tables tables;
  int W = 0, H = 0;
  int ini_th = 0, min_th = 0; /* clamped to [0,255] as cv::FAST does */
  std::vector<LevelInfo> levels;
  std::vector<CellInfo> cells;
  std::vector<StripInfo> strips;
  int strip_max_w = 0, strip_max_h = 0, strip_max_cells = 0;
  int nstrips_l0 = 0;  /* strips of level 0 (strips are level-major) */
  std::vector<char> area2; /* per level: resized from the previous one by OpenCV's 2x INTER_AREA path */
  int blur_tiles = 0;
  std::vector<int32_t> xofs;   /* concatenated per unique level >= 1 */
  std::vector<int16_t> alpha;  /* 2 per x */
  std::vector<int32_t> xofs1;  /* second tap column (clamped) */
  std::vector<int32_t> yofs;
  std::vector<int16_t> beta;
  std::vector<PyrSeg> segs;      /* fused pyramid launches, in dependency order */
  std::vector<int32_t> pyr_xs;   /* {clo, chi, plo, phi} quads */
  std::vector<int32_t> pyr_ys;
  std::vector<uint32_t> pyr_blob; /* LUT blobs (pairs of u32 = uint2 entries) */
  std::vector<int32_t> pyr_bo;    /* blob start offsets (uint2 units), per segment ntx+1, nty+1 */
  /* row-streaming pyramid (k_pyr_stream; orbx_internal.h); ps_ok = false when
   * the chain has an exact-2x level or does not fit the LDS budget */
  bool ps_ok = false;
  PyrStream ps;
  std::vector<uint32_t> ps_tasks;    /* uint2 {x, y} per task, ticks in order */
  std::vector<int32_t> ps_tick_end;  /* cumulative task count after each tick */
  std::vector<uint32_t> ps_xlut;     /* uint2 per column, 4 per group, groups of every level */
  std::vector<uint32_t> ps_ylut;     /* uint2 per destination row: ring slots | coefficients */
  /* fused pyramid + FAST (k_pyrfast; orbx_internal.h PyrFast) */
  bool pf_ok = false;
  PyrFast pf;
  std::vector<uint32_t> pf_tasks;    /* uint2 {x, y} per task, ticks of all passes in order */
  std::vector<int32_t> pf_tick_end;  /* cumulative task count after each tick */
  std::vector<uint32_t> pf_xlut;     /* column LUTs (uint2 per column, 4 per group) */
  std::vector<uint32_t> pf_ylut;     /* row LUTs: source ring slots | coefficients */
  long long pyr_bytes = 0, blur_bytes = 0, nslots = 0, qk_elems = 0;
  int ncells = 0, kcap = 0;
  int qt_smax = 0;     /* max DistributeOctTree splittable list length */
  int qt_max_cells = 0;
  orbx_geometry geo;
};

/* returns ORBX_OK or an ORBX_ERR_* code */
int plan_geometry(const orbx_params& p, int width, int height, Plan& plan);

/* k_pyr_stream schedule for rows_per_tick level-0 rows per tick and at most
 * rows_per_task destination rows per task (plan_geometry calls it with the
 * largest tick that fits ORBX_PS_LDS_MAX); false when not applicable */
bool plan_pyr_stream(Plan& P, int rows_per_tick, int rows_per_task);

/* k_pyrfast schedule: pass p uses ticks of about rows0 * w0 / w_p source
 * rows (at least 4), stage-A / resize tasks of at most rows_per_task rows;
 * false when not applicable (exact-2x level, LDS budget, cell geometry) */
bool plan_pyr_fast(Plan& P, int rows0, int rows_per_task);

}  // namespace orbx

#endif
