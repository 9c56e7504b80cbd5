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
  int bpitch;          /* its row pitch (16-B multiple)                          */
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
  int key_xs;          /* FAST key packing shift (orbx_pack_key)                 */
};

#define ORBX_BLUR_TW 128
#define ORBX_BLUR_TH 32
#define ORBX_STRIP_MAXW 256 /* FAST strip: band width budget per workgroup */
#ifndef ORBX_FS_COLWALK_MINW
#define ORBX_FS_COLWALK_MINW 400 /* narrowest level whose strips take the column walk */
#endif

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
  int colwalk;    /* planner's choice of k_fast_strips' column walk (when it applies) */
  int pitch;      /* row pitch of the level's storage; 0 = level 0 (the call's row stride) */
  long long off;  /* byte offset of the level in the per-frame pyramid buffer (level > 0) */
  /* k_fast_strips' staging for a 16-B-aligned level base (every pyramid
   * level; level 0 when the call's frames are, LevelArgs::l0al16), set by
   * the planner so the kernel skips its alignment and column-walk tests:
   * the tile's lead columns (x & 15), the column-walk decision, and the
   * tile's first byte in the per-frame pyramid buffer (level > 0) */
  int lead16, cw16;
  long long soff16;
};

/* per-level storage of the pyramid, passed by value to kernels that only
 * need to locate a level (no dependent LevelInfo loads) */
/* s_setprio of the pyramid and FAST waves when a plan sets prio: in the
 * pipelined step they then win their SIMDs' issue arbitration over the
 * matcher's co-resident waves (the matcher fills the slots they leave).
 * Plans with a pyramid set it (orbx_plan_create); 0 disables */
#ifndef ORBX_EX_PRIO
#define ORBX_EX_PRIO 2
#endif
struct LevelArgs {
  long long pyr_off[ORBX_MAX_LEVELS];
  int pitch[ORBX_MAX_LEVELS];
  int key_xs; /* orbx_pack_key shift */
  int prio;   /* 1: FAST waves at ORBX_EX_PRIO */
  int l0al16; /* per launch: the call's frames, frame and row strides are 16-B aligned */
};
#define ORBX_STRIP_MAXCELLS 64 /* cells per FAST strip (>= 256 / min cell width) */

/* per-level constants of the stereo matcher (Frame::ComputeStereoMatches),
 * passed by value.  Left and right plans share the geometry: the storage of
 * level l is the caller's frame when off[l] < 0, else pyr + off[l]. */
struct StereoArgs {
  int nlevels, nrows, kcap, rcap; /* nrows = level-0 height; rcap = row-list entries per frame */
  long long off[ORBX_MAX_LEVELS];
  int pitch[ORBX_MAX_LEVELS], w[ORBX_MAX_LEVELS], h[ORBX_MAX_LEVELS];
  float scale[ORBX_MAX_LEVELS], inv_scale[ORBX_MAX_LEVELS];
  float mb, mbf;
};
#ifndef FS_NT
#define FS_NT 256 /* threads per k_fast_strips workgroup (one strip) */
#endif
#ifndef FS_CW_RMAX
#define FS_CW_RMAX 8 /* column walk: band rows per wave (registers hold FS_CW_RMAX + 6 rows) */
#endif
#ifndef FS_CCAP
#define FS_CCAP 1024 /* per-strip corner list (overflow falls back to a map scan); the plan may take
                        * fewer entries (>= FS_CCAP_MIN) where that buys a workgroup per CU */
#ifndef FS_CCAP_MIN
#define FS_CCAP_MIN 384
#endif
#endif
/* d_err[ORBX_ERRW_FAST_OVF]: strips whose corner list overflowed (debug counter) */
#define ORBX_ERRW_FAST_OVF 1
#define ORBX_DEVERR_STEREO 4 /* the reference would index out of range / throw */
#define ORBX_STEREO_MAXROWS 8192

/* per-level constants of k_orient_brief, passed by value (kernel arguments
 * live in SGPRs: no dependent global loads to find a keypoint's level) */
/* level-blur mode (k_blur + k_orient_brief_lb, Plan::lb): the 7x7 Gaussian of
 * every unique level materialised once per frame in the blur buffer (row
 * pitch bpitch = pitch_of(w), offset blur_off), tiles of ORBX_LB_TW x
 * ORBX_LB_TH, unique level i owning tiles [tile_begin[i], tile_begin[i+1]) */
#define ORBX_LB_TW 248 /* k_blur tile: 62 dword columns (+ 2 halo lanes) x 4 waves of 32 rows */
#define ORBX_LB_TH 128
#define KP_PATCH_ROWS 43 /* the per-keypoint blur's staged patch (k_orient_brief) */
#define KP_PATCH_COLS 48
#ifndef ORBX_LB_RATIO
/* level blur when nfeatures x patch > ratio x unique level pixels.  Measured
 * (DESIGN §4 round 5): the blur pass costs more than the per-keypoint blur it
 * saves at c1 (ratio 2.2), c5 (2.9) and c4 (0.66); c2 (6.7) is break-even. */
#define ORBX_LB_RATIO 8.0
#endif
struct BlurArgs {
  int nu;                                  /* unique levels */
  int tile_begin[ORBX_MAX_LEVELS + 1];     /* cumulative tile counts */
  int tiles_x[ORBX_MAX_LEVELS];
  int w[ORBX_MAX_LEVELS], h[ORBX_MAX_LEVELS];
  int pitch[ORBX_MAX_LEVELS];              /* source pitch (unique level 0: the caller's rstride) */
  long long src_off[ORBX_MAX_LEVELS];      /* pyr offset, -1 = the caller's frame */
  int bpitch[ORBX_MAX_LEVELS];
  long long blur_off[ORBX_MAX_LEVELS];
};

struct BriefArgs {
  int nlevels, kcap;
  int kout_off[ORBX_MAX_LEVELS], lcap[ORBX_MAX_LEVELS];
  int unique[ORBX_MAX_LEVELS], w[ORBX_MAX_LEVELS], h[ORBX_MAX_LEVELS], pitch[ORBX_MAX_LEVELS];
  int bpitch[ORBX_MAX_LEVELS];             /* level-blur mode: blurred level pitch / offset */
  long long blur_off[ORBX_MAX_LEVELS];
  long long pyr_off[ORBX_MAX_LEVELS];
  float scale[ORBX_MAX_LEVELS];
  int patch[ORBX_MAX_LEVELS];
  uint32_t umaxw[4]; /* IC_Angle umax[0..15], one byte each */
  int key_xs;        /* orbx_pack_key shift */
};

/* fused pyramid segment: destination levels lev[1..nl] computed in one
 * launch from source level lev[0] (read from HBM).  Workgroup = one tile of
 * the last level; per tile and level s the region tables hold
 * {clo, chi, plo, phi}: the computed interval (everything level s+1 of this
 * tile reads) and the owned interval (written to HBM; the owned intervals of
 * a level partition it).  Row and column tables are separate (ys / xs). */
#define ORBX_PYR_LDS_BUDGET 40960 /* level buffers */
#define ORBX_PYR_LDS_MAX 61440    /* + LUT blobs (below the 64 KiB default limit) */
/* per tile column (row) a LUT blob of uint2 {src0 | src1 << 16, coef pair}
 * for every level s = 1..nl and every computed column c in [dax, dax+4*ncg)
 * (row in [clo, chi)); column sources relative to the LDS origin of level
 * s-1's region, row sources as LDS byte offsets of the two source rows
 * (ping-pong buffer + row * lpitch[s-1]); blobs are padded to 16 B */
struct PyrSeg {
  int nl;
  int area;           /* 1: one exact-2x level by INTER_AREA (k_pyr_area2; nl = 1, no tiling) */
  int ntx, nty;
  int xs_off, ys_off; /* in quads; table index (s * ntx + tx) / (s * nty + ty) */
  int lds_a, lds_b;   /* ping-pong buffer bytes (source staged in A) */
  int lds_xl, lds_yl; /* LUT blob bytes (max over tile columns / rows) */
  int xbo_off, ybo_off; /* into the blob offset tables (ntx+1 / nty+1 entries) */
  int lev[ORBX_MAX_LEVELS], w[ORBX_MAX_LEVELS], h[ORBX_MAX_LEVELS], pitch[ORBX_MAX_LEVELS];
  int lut_x[ORBX_MAX_LEVELS], lut_y[ORBX_MAX_LEVELS];
  int lpitch[ORBX_MAX_LEVELS];     /* LDS row pitch of level s's region, the same for every tile (max over tile columns) */
  long long off[ORBX_MAX_LEVELS]; /* pyr offset; -1 = the caller's frame (level 0) */
  int prio;                       /* 1: pyramid waves at ORBX_EX_PRIO (set at launch) */
};


#if defined(__HIPCC__)
#define ORBX_HDI __host__ __device__ inline
#else
#define ORBX_HDI inline
#endif

/* FAST keys: (x - 16) << xs | (y - 16) << 8 | score.  xs = 20 (12 + 12
 * coordinate bits) unless the frame is wider or taller than 4127 px: then 19
 * (13-bit x, 11-bit y) or 21 (11-bit x, 13-bit y), chosen by the planner */
static ORBX_HDI uint32_t orbx_pack_key(uint32_t x, uint32_t y, uint32_t score, int xs) {
  return (x << xs) | (y << 8) | score;
}
static ORBX_HDI int orbx_key_x(uint32_t key, int xs) { return (int)(key >> xs); }
static ORBX_HDI int orbx_key_y(uint32_t key, int xs) { return (int)((key >> 8) & ((1u << (xs - 8)) - 1u)); }

#endif
