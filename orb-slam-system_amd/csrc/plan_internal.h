// plan_internal.h -- host-side state of an extraction plan and of the
// ORBextractor drop-in, shared by the C-ABI translation units (the stereo
// matcher reads the device pyramid the extractor left behind).
#ifndef ORBX_PLAN_INTERNAL_H
#define ORBX_PLAN_INTERNAL_H

#include <hip/hip_runtime.h>

#include "../../include/orbx.h"
#include "api_common.h"
#include "geometry.h"

struct orbx_plan {
  orbx::Plan P;
  int device = 0, max_batch = 0;
  hipStream_t stream = nullptr;
  LevelInfo* d_lv = nullptr;
  CellInfo* d_cells = nullptr;
  StripInfo* d_strips = nullptr;
  int fs_tpitch = 0;
  /* k_fast_strips launches: strips [begin, end) of the (height-partitioned)
   * strip table with their tile rows, cells, corner-list entries and LDS */
  struct FsGroup {
    int begin = 0, end = 0, tmaxh = 7, mcells = 1, ccap = 0;
    size_t lds = 0;
  };
  FsGroup fs_grp[2];
  int fs_ngrp = 1;
  int32_t *d_xofs = nullptr, *d_xofs1 = nullptr, *d_yofs = nullptr;
  int32_t *d_pyr_xs = nullptr, *d_pyr_ys = nullptr, *d_pyr_bo = nullptr;
  uint32_t* d_pyr_blob = nullptr;
  int16_t *d_alpha = nullptr, *d_beta = nullptr;
  uint8_t *d_pyr = nullptr, *d_blur = nullptr;
  uint32_t *d_slots = nullptr, *d_ccount = nullptr, *d_qkeys = nullptr, *d_qout = nullptr;
  uint32_t* d_qperm = nullptr; /* per level: k_orient_brief's processing order (k_quadtree) */
  int32_t* d_qnode = nullptr;
  int *d_lcount = nullptr, *d_err = nullptr;
  int* h_err = nullptr; /* pinned: orbx_plan_check reads the error word without a blocking copy */
  size_t pyr_stride = 0, blur_stride = 0, slot_stride = 0, qk_stride = 0, qout_stride = 0;
  size_t qt_lds = 0;
  size_t qt_lds_wide = 0; /* k_quadtree_wide (single-frame calls): + a second child array */
  BriefArgs bargs;
  BlurArgs blargs;  /* level-blur mode: k_blur's tiles */
  int lb_auto = 0;  /* the planner's BRIEF blur choice: 1 = level blur (k_blur + k_orient_brief_lb) */
  LevelArgs largs;
  orbx::StageTimer timer;
  int dbg = 0; /* ORBX_DEBUG_STOP: kernel phase early-exit for profiling only */
  int ob_div = 0; /* ORBX_DEBUG_OBDIV: k_orient_brief grid divisor, profiling only */
  /* ORBX_DEBUG_LDSPAD=pyr,fast,brief: extra dynamic LDS per workgroup
   * (occupancy probes: room for other streams' kernels), profiling only */
  int pad_pyr = 0, pad_fast = 0, pad_brief = 0;
  int fs_ccap = 0; /* FAST per-strip corner list entries (FS_CCAP; orbx_debug_set_fast_ccap fixes a lower one) */
  bool ccap_fixed_dbg = false; /* orbx_debug_set_fast_ccap: one launch group, that list length */
  int chunk = 0;  /* frames per extraction pass (0 = the whole batch in one pass) */
  hipEvent_t ev_after_pyr = nullptr; /* recorded after the pyramid launch when set (orbx_extract) */
  int overlap = 0; /* FAST on level 0 beside the pyramid on s_aux */
  hipStream_t s_aux = nullptr;
  hipEvent_t ev_aux0 = nullptr, ev_aux1 = nullptr;
  int options = 0; /* ORBX_PLAN_* (include/orbx.h) */
  int nextracted = 0; /* frames of the last orbx_plan_extract (orbx_plan_level bound) */
  int uses_lb() const {
    return (options & ORBX_PLAN_BRIEF_LEVEL) ? 1 : (options & ORBX_PLAN_BRIEF_PATCH) ? 0 : lb_auto;
  }
};

struct orbx_extractor {
  orbx_params params;
  int device = 0;
  orbx_plan* plan = nullptr;
  int W = 0, H = 0;
  uint8_t* d_img = nullptr;
  orbx_keypoint* d_kps = nullptr;
  uint8_t* d_desc = nullptr;
  int* d_count = nullptr;
  /* pinned result staging: [count, error word | kps rows | desc rows] (64-B
   * header, kcap rows each), written by k_pack_results through d_res */
  uint8_t* h_res = nullptr;
  uint8_t* d_res = nullptr;  /* h_res's device address */
  int last_k = 0; /* keypoints of the previous call */
  bool have_frame = false;
  int flags = 0;             /* ORBX_EXTRACTOR_* */
  uint8_t* h_img = nullptr;  /* pinned staging of the caller's image (= host level 0) */
  uint8_t* h_pyr = nullptr;  /* pinned host copy of the level buffer (PYRAMID_TO_HOST) */
  size_t pyr_bytes = 0;
  hipStream_t s_copy = nullptr; /* pyramid D2H, overlapped with FAST .. BRIEF */
  hipEvent_t ev_pyr = nullptr;
  bool host_pyr = false;     /* the last call filled h_img / h_pyr */
  long long n_calls = 0, n_refetch = 0; /* n_refetch: always 0 (k_pack_results writes exactly K rows) */
  void* stereo = nullptr; /* orbs_plan of orbx_stereo_match (api_stereo.hip) */
};

/* frees the stereo scratch an extractor owns (api_stereo.hip) */
void orbx_stereo_release(orbx_extractor* e);

#endif
