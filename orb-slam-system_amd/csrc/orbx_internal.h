/* orbx_internal.h -- layouts shared by the host planner and the HIP kernels.
 *
 * HBM layout per frame:
 *   level 0            = the caller's frame (no copy)
 *   pyr  [pyr_bytes]   = unique levels >= 1, row pitch = pitch (16-B multiple)
 *   blur [blur_bytes]  = 7x7 Gaussian of every unique level (same pitches)
 *   slots[nslots] u32  = per-cell FAST keypoint lists, packed (x<<20|y<<8|score)
 *   ccount[ncells] u32 = per-cell keypoint counts
 *   qkeys/qnode        = DistributeOctTree scratch (per level)
 *   qout [kcap] u32    = per-level selected keys, packed like slots
 *   lcount[nlevels]    = per-level selected counts
 * "unique" levels: level l shares level l-1's pixels when their sizes are
 * equal (cv::resize copies when dsize == ssize); with the reference's
 * std::partial_sum scale table this is always true for l == 1.
 */
#ifndef ORBX_INTERNAL_H
#define ORBX_INTERNAL_H

#include <stdint.h>

#define ORBX_MAX_LEVELS 32
#define ORBX_EDGE 19
#define ORBX_MINB 16          /* EDGE_THRESHOLD - 3 */
#define ORBX_CELL_MAX 72      /* max FAST cell tile edge handled by the cell kernel */
#define ORBX_QT_MAX_PASSES 64 /* DistributeOctTree pass bound (termination guard) */

/* device error flags (latched in plan->d_err) */
#define ORBX_DEVERR_QUADTREE 1
#define ORBX_DEVERR_QTCAP 2

struct LevelInfo {
  int w, h, pitch;     /* pixels and row pitch of this level's storage          */
  int unique;          /* level whose storage holds these pixels                */
  long long pyr_off;   /* offset in the per-frame pyramid buffer (unique >= 1)  */
  long long blur_off;  /* offset in the per-frame blur buffer (unique levels)   */
  /* resize from level l-1 (unique levels >= 1) */
  int lut_x, lut_y;    /* offsets into the xofs/alpha and yofs/beta LUTs         */
  int src_level;       /* unique level the resize reads                          */
  /* FAST cells (unique levels) */
  int cell_begin, ncells;
  long long slot_begin, nslots;
  /* DistributeOctTree (all levels) */
  int N, nini;
  float hX;
  int Wr, Hr;
  int kcap, kout_off;
  long long qk_off;    /* offset of this level's key scratch (per frame)        */
  float scale;
  int patch_size;
  int blur_tile_begin; /* first blur tile of this unique level (ORBX_BLUR_TW x ORBX_BLUR_TH) */
  int blur_tiles_x;
  int wcell;
  int pad;
};

#define ORBX_BLUR_TW 128
#define ORBX_BLUR_TH 32
#define ORBX_STRIP_MAXW 256 /* FAST strip: band width budget per workgroup */

struct CellInfo {
  int level; /* unique level */
  int x, y, w, h;
  int slot_off; /* relative to the frame's slot base */
  int slot_cap;
  int pad;
};

/* FAST strip = consecutive valid cells of one cell row, processed by one
 * workgroup; all its cells share y/h and their scan bands are contiguous. */
struct StripInfo {
  int level;      /* unique level */
  int x, y, w, h; /* tile = [x, x+w) x [y, y+h) */
  int cell_begin; /* first cell (index into the CellInfo table) */
  int ncells;
  int wcell;
};

#if defined(__HIPCC__)
#define ORBX_HDI __host__ __device__ inline
#else
#define ORBX_HDI inline
#endif

static ORBX_HDI uint32_t orbx_pack_key(uint32_t x, uint32_t y, uint32_t score) {
  return (x << 20) | (y << 8) | score;
}

#endif
