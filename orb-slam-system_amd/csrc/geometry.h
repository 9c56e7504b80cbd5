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
  long long pyr_bytes = 0, blur_bytes = 0, nslots = 0, qk_elems = 0;
  int ncells = 0, kcap = 0;
  int qt_smax = 0;     /* max DistributeOctTree splittable list length */
  int qt_max_cells = 0;
  orbx_geometry geo;
};

/* returns ORBX_OK or an ORBX_ERR_* code */
int plan_geometry(const orbx_params& p, int width, int height, Plan& plan);

}  // namespace orbx

#endif
