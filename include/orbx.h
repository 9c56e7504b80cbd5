/* orbx.h -- C ABI of the MI355X-native ORB front end (liborbx.so).
 *
 * Drop-in boundary for the reference's hot path:
 *   ORB_SLAM2::ORBextractor   /root/reference/include/ORBextractor.h:25-91
 *   ORB_SLAM2::ORBmatcher     /root/reference/include/ORBmatcher.h:16-81
 * Plain C: POD structs, raw pointers, explicit sizes, int status codes, no
 * exceptions across the boundary, no torch types.  Every compute entry point
 * runs hand-written HIP kernels on a gfx950 device; there is no CPU path.
 *
 * Threading: an orbx_extractor / orbx_plan owns its own HIP stream and
 * scratch and may be used from one thread at a time; distinct instances may
 * run concurrently (the reference runs left/right extractors on two threads,
 * /root/reference/src/Frame.cc:58-61).  Matcher calls are re-entrant.
 */
#ifndef ORBX_H
#define ORBX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2 (round 6): plan option flags 2 and 4 retired (ORBX_ERR_ARG), flags 8 / 16,
 * orbx_proj_problem and the orbm_proj_plan_* / orbm_search_by_bow_kf_frame
 * entry points added (round 5) */
#define ORBX_ABI_VERSION 2

/* status codes */
enum {
  ORBX_OK = 0,
  ORBX_ERR_ARG = -1,         /* bad argument / image type                               */
  ORBX_ERR_CELL_ROI = -2,    /* strict cell guard: a FAST cell has negative extent; the
                                reference throws cv::Exception from cv::Mat(m, Rect) at
                                src/ORBextractor.cc:328 (1920x1080)      */
  ORBX_ERR_LEVEL_SIZE = -3,  /* a pyramid level has <= 32 rows (reference divides by 0 at
                                src/ORBextractor.cc:230) or < 32 cols                     */
  ORBX_ERR_QUADTREE = -4,    /* DistributeOctTree would never terminate */
  ORBX_ERR_CAPACITY = -5,    /* caller buffer too small (*n holds the required count)     */
  ORBX_ERR_UNSUPPORTED = -6, /* a configuration beyond the kernels' static limits: a level
                                ratio > ~2.3 other than exactly 2, or a level-0 size
                                outside the FAST key packing -- supported are
                                (w-32 <= 4095 and h-32 <= 4095), (w-32 <= 8191 and
                                h-32 <= 2047) or (w-32 <= 2047 and h-32 <= 8191), so
                                e.g. 4200x2100 is refused; ...                        */
  ORBX_ERR_HIP = -7,         /* HIP runtime error                                         */
  ORBX_ERR_NO_DEVICE = -8,   /* no gfx950 device / bad device ordinal                     */
};

/* ORBextractor constructor arguments (ORBextractor.h:31-32) + switches. */
typedef struct {
  int nfeatures;
  float scale_factor;
  int nlevels;
  int ini_th_fast;
  int min_th_fast;
  int cell_guard; /* 0 = strict (reference: throw on negative-extent FAST cells),
                     1 = empty (such cells yield no corners; == upstream ORB-SLAM2 guards) */
} orbx_params;

/* Layout-identical to cv::KeyPoint (28 bytes): pt.x, pt.y, size, angle,
 * response, octave, class_id. */
typedef struct {
  float x, y, size, angle, response;
  int32_t octave, class_id;
} orbx_keypoint;

int orbx_abi_version(void);
const char* orbx_status_string(int status);
/* number of visible gfx950 devices (0 on a host without GPU) */
int orbx_device_count(void);

/* ---------------------------------------------------------------------------
 * Level geometry and constant tables (host-only, no device needed).
 * Mirrors ORBextractor::ORBextractor (src/ORBextractor.cc:116-170),
 * GetScaleFactors() & co. (ORBextractor.h:43-63) and ComputePyramid sizes
 * (src/ORBextractor.cc:501-502).
 * ------------------------------------------------------------------------- */
int orbx_tables(const orbx_params* p, float* scale, float* inv_scale, float* sigma2,
                float* inv_sigma2, int* features_per_level, int* umax16);

typedef struct {
  int nlevels;
  int width[32], height[32];
  int alias[32];          /* level whose pixels this level shares (level 1 == level 0:
                             mvScaleFactor[1] == 1)                    */
  int ncols[32], nrows[32], wcell[32], hcell[32]; /* FAST cell grid (:308-314)        */
  int ncells_bad[32];     /* cells with negative extent (strict guard -> error)       */
  int features[32];       /* mnFeaturesPerLevel                                        */
  int nini[32];           /* DistributeOctTree initial nodes (:230)                    */
  int kcap_level[32];     /* max keypoints a level can emit                            */
  int kcap;               /* max keypoints per frame (sum of kcap_level)               */
  long long pixels;       /* sum of level pixel counts                                 */
  long long bytes_pyr_fast; /* algorithmic bytes of pyramid + FAST per frame */
} orbx_geometry;

int orbx_geometry_compute(const orbx_params* p, int width, int height, orbx_geometry* g);

/* Resize coefficient tables for level l (l >= 1, non-alias): xofs[w_l],
 * alpha[2*w_l], yofs[h_l], beta[2*h_l] (INTER_RESIZE_COEF_BITS = 11). */
int orbx_resize_tables(const orbx_params* p, int width, int height, int level, int32_t* xofs,
                       int16_t* alpha, int32_t* yofs, int16_t* beta);

/* ---------------------------------------------------------------------------
 * ORBextractor drop-in: host image in, host keypoints/descriptors out.
 * Replaces ORBextractor::operator() (src/ORBextractor.cc:442-495).
 * ------------------------------------------------------------------------- */
typedef struct orbx_extractor orbx_extractor;

int orbx_extractor_create(const orbx_params* p, int device, orbx_extractor** out);
int orbx_extractor_destroy(orbx_extractor* e);

/* Capacity needed for a w x h image (upper bound of the keypoint count). */
int orbx_extractor_capacity(orbx_extractor* e, int width, int height, int* kcap);

/* operator()(image, mask, keypoints, descriptors): img is CV_8UC1 rows of
 * `stride` bytes.  On success *n = K; kps[0..K) and desc[0..K*32) hold the
 * level-major keypoints (level coordinates * mvScaleFactor) and descriptors.
 * K == 0 leaves kps/desc untouched (reference :460-463).  cap < K returns
 * ORBX_ERR_CAPACITY with *n = K.  Synchronous. */
int orbx_extract(orbx_extractor* e, const uint8_t* img, int width, int height, size_t stride,
                 orbx_keypoint* kps, int cap, uint8_t* desc, int* n);

/* mvImagePyramid[level] of the last orbx_extract (copied D2H on demand). */
int orbx_extractor_level(orbx_extractor* e, int level, uint8_t* dst, size_t dst_stride,
                         int* width, int* height);

/* Options of an extractor (default 0; persistent across calls):
 * ORBX_EXTRACTOR_PYRAMID_TO_HOST  every orbx_extract also brings the whole
 *     pyramid back (the reference refills mvImagePyramid on each call,
 *     src/ORBextractor.cc:497-515, read by Frame::ComputeStereoMatches): one
 *     D2H of the level buffer on a second stream, overlapped with the rest
 *     of the extraction; read it with orbx_extractor_level_host;
 * ORBX_EXTRACTOR_PINNED_H2D  upload the caller's image through the
 *     extractor's pinned staging buffer (host copy in row chunks overlapped
 *     with the DMA) instead of straight from its pageable rows (measurement
 *     option: slower at 1080p). */
#define ORBX_EXTRACTOR_PYRAMID_TO_HOST 1
#define ORBX_EXTRACTOR_PINNED_H2D 2
int orbx_extractor_set_options(orbx_extractor* e, int flags);

/* Host view of mvImagePyramid[level] after an orbx_extract with
 * ORBX_EXTRACTOR_PYRAMID_TO_HOST: *data / *stride point into extractor-owned
 * pinned memory, valid until the next orbx_extract or destroy of `e` (levels
 * whose size equals the previous level's -- level 1 with the reference's
 * scale table -- share its pixels, as cv::resize copies them). */
int orbx_extractor_level_host(orbx_extractor* e, int level, const uint8_t** data, size_t* stride,
                              int* width, int* height);

/* Call statistics of an extractor since creation: calls of orbx_extract and
 * the calls that needed a second D2H round trip for their results (always 0
 * since round 6: one kernel writes exactly the frame's rows into the pinned
 * staging; kept for ABI compatibility). */
int orbx_extractor_stats(orbx_extractor* e, long long* calls, long long* refetches);

/* ---------------------------------------------------------------------------
 * Batched device-resident extraction (the throughput path; bench.py).
 * ------------------------------------------------------------------------- */
typedef struct orbx_plan orbx_plan;

int orbx_plan_create(const orbx_params* p, int width, int height, int max_batch, int device,
                     orbx_plan** out);
int orbx_plan_destroy(orbx_plan* plan);
int orbx_plan_geometry(const orbx_plan* plan, orbx_geometry* g);

/* d_frames: nframes images, frame i at d_frames + i*frame_stride, rows of
 * row_stride bytes (device memory; any byte alignment -- 16-B aligned rows
 * take the fastest staging path; no byte outside a frame's row_stride x
 * height bytes is read; row_stride < 2^24, else ORBX_ERR_UNSUPPORTED: the
 * kernels form row offsets with 24-bit multiplies).  Outputs (device memory):
 *   d_kps  [nframes][kcap], d_desc [nframes][kcap][32], d_counts [nframes].
 * Asynchronous on `stream` (a hipStream_t; NULL = the default stream).
 * Device-side failures (quadtree stuck) are latched; read them with
 * orbx_plan_check(). */
int orbx_plan_extract(orbx_plan* plan, const uint8_t* d_frames, int nframes, size_t frame_stride,
                      size_t row_stride, orbx_keypoint* d_kps, uint8_t* d_desc, int* d_counts,
                      void* stream);
/* synchronises `stream`, returns and clears the latched device error */
int orbx_plan_check(orbx_plan* plan, void* stream);
/* Debug counters since the last call (then reset; synchronises the plan's
 * stream): FAST strips whose corner list overflowed into the strength-map
 * scan (see orbx_debug_set_fast_ccap). */
int orbx_plan_debug_counters(orbx_plan* plan, int* fast_overflow_strips);
/* Testing only: plans created after this call give the FAST kernels a
 * corner list of `ccap` entries (<= 1024) in one launch group, so the
 * strength-map overflow path runs on ordinary frames; ccap < 0 restores the
 * planner's own length.  Process-global; results are unchanged either way. */
int orbx_debug_set_fast_ccap(int ccap);

/* Kernel-path options of a plan (default 0 = automatic; persistent).  Every
 * path gives bit-identical results; they differ in speed only.
 *   ORBX_PLAN_PYR_TILES    the pyramid by k_pyramid (2-D tiles of the level
 *                          chain, halo recompute) -- the one pyramid path;
 *   ORBX_PLAN_BRIEF_PATCH  descriptors blur each keypoint's 43 x 48 patch
 *                          (k_orient_brief);
 *   ORBX_PLAN_BRIEF_LEVEL  every unique level is blurred once (k_blur) and
 *                          the descriptors sample it (k_orient_brief_lb).
 * Automatic (0): the tile pyramid, and the level blur when nfeatures x 43 x
 * 48 exceeds ORBX_LB_RATIO x the unique level pixels.
 * The round-4 row-streaming pyramid and fused pyramid + FAST kernels (flags
 * 2 and 4) measured 1.1x / 2.6x the tile path's time and were retired; their
 * flags, like any other unknown bit or both BRIEF flags at once, return
 * ORBX_ERR_ARG (options unchanged). */
#define ORBX_PLAN_PYR_TILES 1
#define ORBX_PLAN_BRIEF_PATCH 8
#define ORBX_PLAN_BRIEF_LEVEL 16
int orbx_plan_set_options(orbx_plan* plan, int flags);

/* mvImagePyramid[level] of frame `frame` of the last orbx_plan_extract on
 * this plan, copied to host rows of dst_stride bytes (synchronises `stream`,
 * which must be the stream of that extraction or ordered after it; NULL =
 * the default stream).  Level 0 (and levels aliasing it) are the caller's
 * frame and are not held by the plan: ORBX_ERR_ARG.  With dst != NULL,
 * `frame` must be below the frame count of the plan's last orbx_plan_extract
 * (ORBX_ERR_ARG before any extraction); dst == NULL only reports the size. */
int orbx_plan_level(orbx_plan* plan, int frame, int level, uint8_t* dst, size_t dst_stride,
                    int* width, int* height, void* stream);

/* Per-stage device timing (HIP events around every launch of a stage). */
int orbx_stage_count(void);
const char* orbx_stage_name(int stage);
int orbx_plan_set_timing(orbx_plan* plan, int enable); /* also resets the accumulators   */
/* after the stream is synchronised: total ms and launch count per stage */
int orbx_plan_stage_times(orbx_plan* plan, double* ms, int* launches, int nstages);

/* Device synthetic frames (same bytes as orbx/synth.py): kind 0 rects, 3 pan,
 * 1 noise, 2 flat; frame i gets seed 0x5EED0000 + first_idx + i. */
int orbx_synth_frames(uint8_t* d_frames, int width, int height, size_t frame_stride, int nframes,
                      int first_idx, int kind, void* stream);

/* Self-test of the rotated-BRIEF sin/cos (device memory): sc[2i], sc[2i+1] =
 * the (sin, cos) k_orient_brief uses for angle x[i] -- glibc sincosf
 * (ORBextractor.cc:58-59) wherever it moves a BRIEF sample (orbx_sincos.h). */
int orbx_selftest_sincos(const float* d_x, int n, float* d_sc, void* stream);
/* Same (sin, cos) for the n consecutive float bit patterns first_bits ..
 * first_bits + n - 1, lane-parallel, into host memory sc[2n] (synchronous):
 * the exhaustive device check of every reachable BRIEF angle. */
int orbx_selftest_sincos_range(uint32_t first_bits, int n, float* sc, int device);

/* ---------------------------------------------------------------------------
 * ORBmatcher drop-in.
 * ------------------------------------------------------------------------- */
/* One KeyFrame's matcher inputs.  DBoW2::FeatureVector
 * (Thirdparty/DBoW2/DBoW2/FeatureVector.h:21-22) flattened: node_id[nnodes]
 * ascending & unique, node j holds feat[node_off[j] .. node_off[j+1]).
 * valid[i] != 0 <=> GetMapPointMatches()[i] && !isBad() (NULL = all valid).
 * angle[i] = mvKeysUn[i].angle. */
typedef struct {
  int n;
  const uint8_t* desc; /* n x 32 */
  const float* angle;  /* n */
  const uint8_t* valid;
  int nnodes;
  const uint32_t* node_id;
  const uint32_t* node_off; /* nnodes + 1 */
  const uint32_t* feat;
} orbx_bow_frame;

/* ORBmatcher::SearchByBoW(KeyFrame*, KeyFrame*, vector<MapPoint*>&)
 * (src/ORBmatcher.cc:278-366).  Host inputs; match12[n1] = matched index in
 * kf2 (vpMatches12[i] = vpMapPoints2[match12[i]]), -1 where the reference
 * never writes vpMatches12[i] (it only resize()s the caller's vector, :289),
 * or -2 where it matched and the rotation check reset it to nullptr (:359).
 * Synchronous. */
int orbm_search_by_bow(const orbx_bow_frame* kf1, const orbx_bow_frame* kf2, float nnratio,
                       int check_ori, int device, int32_t* match12, int* nmatches);

/* SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&) in upstream ORB-SLAM2's
 * form (SURVEY.md §5 switch bow_kf_frame=full; this reference ships only the
 * stub of src/ORBmatcher.cc:88-119, which the compat header keeps as the
 * default).  kf: the KeyFrame (valid[i] = its MapPoint i is non-null and not
 * bad, angles of mvKeysUn); frame: the Frame (mvKeys angles; its valid is
 * ignored: every Frame feature is a candidate).  Per KF row in node order:
 * best / second over the node's unclaimed Frame features, accepted when
 * best <= TH_LOW (50) and best < nnratio * second; the rotation check as the
 * KF-KF form.  match_f[frame->n] = the KF feature whose MapPoint the Frame
 * feature received (vpMapPointMatches[i] = vpMapPointsKF[match_f[i]]), -1 for
 * none (vpMapPointMatches starts as F.N nulls).  Synchronous.
 * ORBX_ERR_UNSUPPORTED for nnratio <= 50/256 (no second-best could pass). */
int orbm_search_by_bow_kf_frame(const orbx_bow_frame* kf, const orbx_bow_frame* frame, float nnratio,
                                int check_ori, int device, int32_t* match_f, int* nmatches);

/* ORBmatcher::DescriptorDistance (src/ORBmatcher.cc:896-908), batched on the
 * device: dist[i] = Hamming(a + 32*ia[i], b + 32*ib[i]); host pointers. */
int orbm_descriptor_distance_batch(const uint8_t* a, int na, const uint8_t* b, int nb,
                                   const int32_t* ia, const int32_t* ib, int npairs, int device,
                                   int32_t* dist);

/* Batched device matcher over extractor outputs (bench "extract+match",
 * BASELINE config 4): pair p matches frame A_p against frame B_p, each
 * reduced to its top `topn` keypoints by (response desc, index asc) and
 * placed in ONE vocabulary node in ascending index order (brute force).
 * match12 rows are indexed by keypoint index of frame A (cap kcap), value =
 * keypoint index in frame B, -1 for no match, or -2 where a match was found
 * and the rotation check (check_ori) reset it (as orbm_search_by_bow; test
 * `< 0` for "no match").  Frame p of side A is d_kps_a + p*kcap,
 * d_desc_a + p*kcap*32, d_count_a[p] (side B likewise), i.e. the layout of
 * orbx_plan_extract outputs; d_match12 is [npairs][kcap], d_nmatches
 * [npairs].  Asynchronous on `stream`.  Descriptors are arbitrary 32-byte
 * rows unless the caller opts in to ORBM_PLAN_ZERO_TAIL. */
typedef struct orbm_plan orbm_plan;
int orbm_plan_create(int max_pairs, int kcap, int topn, int device, orbm_plan** out);
int orbm_plan_destroy(orbm_plan* mp);
int orbm_plan_match_frames(orbm_plan* mp, int npairs, const orbx_keypoint* d_kps_a,
                           const uint8_t* d_desc_a, const int* d_count_a,
                           const orbx_keypoint* d_kps_b, const uint8_t* d_desc_b,
                           const int* d_count_b, float nnratio, int check_ori,
                           int32_t* d_match12, int* d_nmatches, void* stream);
int orbm_plan_set_timing(orbm_plan* mp, int enable);
int orbm_plan_stage_times(orbm_plan* mp, double* ms, int* launches, int nstages);
/* Options of orbm_plan_match_frames (default 0):
 * ORBM_PLAN_ZERO_TAIL  the caller guarantees bytes 24..31 of every descriptor
 *                      are zero -- true of orbx_plan_extract outputs (the
 *                      reference's 728-entry BRIEF pattern leaves them 0) --
 *                      so the distance kernels skip those two dwords;
 * ORBM_PLAN_VALU       distances by xor/popcount on the VALU instead of the
 *                      i8 MFMA formulation (same results; for testing). */
#define ORBM_PLAN_ZERO_TAIL 1
#define ORBM_PLAN_VALU 2
int orbm_plan_set_options(orbm_plan* mp, int flags);

/* ---------------------------------------------------------------------------
 * Stereo matcher: Frame::ComputeStereoMatches (src/Frame.cc:446-620), the
 * consumer of the extractors' mvImagePyramid.
 * ------------------------------------------------------------------------- */
/* Drop-in on host keypoints: kps_l/desc_l (mvKeys / mDescriptors) and
 * kps_r/desc_r (mvKeysRight / mDescriptorsRight) of a rectified pair whose
 * images were the last orbx_extract of `left` and `right` (their pyramids are
 * read on the device).  mb = baseline, mbf = baseline * fx (the reference
 * reads the member mb before assigning it at Frame.cc:94; callers pass
 * mbf / fx).  Outputs uright[nl] (mvuRight) and depth[nl] (mvDepth), -1 =
 * no match; *nmatches = stereo matches kept by the median filter.
 * ORBX_ERR_ARG where the reference would index out of range or throw. */
int orbx_stereo_match(orbx_extractor* left, orbx_extractor* right, const orbx_keypoint* kps_l,
                      const uint8_t* desc_l, int nl, const orbx_keypoint* kps_r,
                      const uint8_t* desc_r, int nr, float mb, float mbf, float* uright,
                      float* depth, int* nmatches);

/* Batched device path: nframes rectified pairs.  `left` / `right` are the
 * plans whose last orbx_plan_extract consumed d_frames_l / d_frames_r (their
 * device pyramids are read); keypoint arrays are the orbx_plan_extract
 * outputs ([nframes][kcap], counts [nframes]).  d_uright / d_depth are
 * [nframes][kcap], d_nmatches [nframes].  Asynchronous on `stream`;
 * orbs_plan_check() synchronises and reports latched range errors. */
typedef struct orbs_plan orbs_plan;
int orbs_plan_create(const orbx_plan* geometry, int max_batch, orbs_plan** out);
int orbs_plan_destroy(orbs_plan* sp);
int orbs_plan_match(orbs_plan* sp, int nframes, const orbx_plan* left, const orbx_plan* right,
                    const uint8_t* d_frames_l, const uint8_t* d_frames_r, size_t frame_stride,
                    size_t row_stride, const orbx_keypoint* d_kps_l, const uint8_t* d_desc_l,
                    const int* d_count_l, const orbx_keypoint* d_kps_r, const uint8_t* d_desc_r,
                    const int* d_count_r, float mb, float mbf, float* d_uright, float* d_depth,
                    int* d_nmatches, void* stream);
int orbs_plan_check(orbs_plan* sp, void* stream);
int orbs_plan_set_timing(orbs_plan* sp, int enable);
int orbs_plan_stage_times(orbs_plan* sp, double* ms, int* launches, int nstages);

/* ---------------------------------------------------------------------------
 * DBoW2 vocabulary transform: the producer of the
 * FeatureVectors SearchByBoW consumes (Frame::ComputeBoW / KeyFrame::ComputeBoW,
 * src/Frame.cc:375-382, src/KeyFrame.cc:39-48, levelsup = 4).
 *   TemplatedVocabulary<FORB::TDescriptor, FORB>
 *     loadFromTextFile     Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1338-1424
 *     transform(features, BowVector&, FeatureVector&, levelsup)          :1126-1191
 *     transform(feature, word, weight, nid, levelsup)                    :1222-1259
 * ------------------------------------------------------------------------- */
typedef struct orbv_vocab orbv_vocab;
/* Text vocabulary (ORBvoc.txt format): "k L scoring weighting" then one node
 * per line "parent isLeaf d0..d31 weight".  ORBX_ERR_ARG for a rejected
 * header (:1356-1360) or a parent that does not precede its child. */
int orbv_vocab_load_text(const char* path, int device, orbv_vocab** out);
/* The same from node records (record r = node r+1 in file order). */
int orbv_vocab_create(int k, int L, int scoring, int weighting, int nrec, const int32_t* parent,
                      const int32_t* is_leaf, const uint8_t* desc, const double* weight,
                      int device, orbv_vocab** out);
int orbv_vocab_destroy(orbv_vocab* v);
int orbv_vocab_info(const orbv_vocab* v, int* k, int* L, int* scoring, int* weighting,
                    int* nnodes, int* nwords);
/* transform(features, BowVector&, FeatureVector&, levelsup) on host
 * descriptors desc[n][32].  BowVector: bow_word[nbow] ascending with
 * bow_value[nbow] (WordValue = double, normalised as the scoring requires);
 * FeatureVector (DBoW2::FeatureVector, FeatureVector.h:21-22) as CSR:
 * fv_node[nfv] ascending, features fv_feat[fv_off[j] .. fv_off[j+1]) in
 * ascending index order -- exactly the orbx_bow_frame layout.  Outputs hold
 * n entries (fv_off n + 1).  ORBX_ERR_ARG where the reference would read an
 * uninitialised NodeId (a leaf above the levelsup level); at most 8192
 * descriptors per call (ORBX_ERR_UNSUPPORTED beyond). */
int orbv_transform(orbv_vocab* v, const uint8_t* desc, int n, int levelsup, uint32_t* bow_word,
                   double* bow_value, int* nbow, uint32_t* fv_node, uint32_t* fv_off,
                   uint32_t* fv_feat, int* nfv);
/* Batched device form over orbx_plan_extract outputs: d_desc [nframes][kcap][32],
 * d_counts [nframes]; outputs [nframes][kcap] (d_fv_off [nframes][kcap+1]) and
 * counts [nframes].  Asynchronous on `stream`; orbv_check() synchronises and
 * reports the latched unset-NodeId error. */
int orbv_transform_batch(orbv_vocab* v, int nframes, const uint8_t* d_desc, const int* d_counts,
                         int kcap, int levelsup, uint32_t* d_bow_word, double* d_bow_value,
                         int* d_nbow, uint32_t* d_fv_node, uint32_t* d_fv_off, uint32_t* d_fv_feat,
                         int* d_nfv, void* stream);
int orbv_check(orbv_vocab* v, void* stream);

/* ---------------------------------------------------------------------------
 * Projection matchers: the frame grid
 * (Frame::AssignFeaturesToGrid / PosInGrid / GetFeaturesInArea,
 * src/Frame.cc:210-225,307-371, 64 x 48 cells) and the windowed Hamming
 * search of ORBmatcher::SearchByProjection.  Query form: the caller projects
 * (the cv::Mat pose arithmetic and MapPoint::PredictScale stay with the
 * caller) and passes per query the arguments the reference hands to
 * GetFeaturesInArea plus the gates' inputs.
 * ------------------------------------------------------------------------- */
typedef struct {
  float x, y;                    /* mTrackProjX/Y (mode 1) or the projection u, v       */
  float radius;                  /* the r argument of GetFeaturesInArea (already scaled)  */
  int32_t min_level, max_level;  /* its level bounds (-1 = the defaults)                 */
  float xr;                      /* mode 1: mTrackProjXR (stereo gate, :39-43)           */
  float angle;                   /* modes 2/3: angle of the source keypoint             */
} orbx_query_proj;

typedef struct {
  int n;
  const orbx_keypoint* keys;  /* mvKeysUn                                              */
  const uint8_t* desc;        /* mDescriptors, n x 32                                   */
  const float* uright;        /* mvuRight (mode 1 stereo gate), NULL = monocular        */
  const uint8_t* occupied;    /* mode 1: mvpMapPoints[i] && Observations() > 0;
                                 modes 2/3: mvpMapPoints[i] != NULL; NULL = none        */
  float min_x, min_y;         /* mnMinX, mnMinY                                         */
  float grid_w_inv, grid_h_inv; /* mfGridElementWidthInv / HeightInv                    */
} orbx_proj_frame;

/* mode 1: SearchByProjection(Frame&, const vector<MapPoint*>&, th) (src/ORBmatcher.cc:19-61):
 *         best/second over unoccupied candidates, accept best <= TH_HIGH and
 *         best <= nnratio * second (th_dist and check_ori unused).
 * mode 2: SearchByProjection(Frame& Current, const Frame& Last, th, bMono) (:732-818):
 *         accept best <= th_dist (TH_HIGH); rotation check if check_ori.
 * mode 3: SearchByProjection(Frame&, KeyFrame*, set<MapPoint*>&, th, ORBdist) (:820-894):
 *         accept best <= th_dist (ORBdist); rotation check if check_ori.
 * Queries are walked in order (each takes its best unoccupied candidate,
 * later queries skip it).  match[i] = the query that took feature i, or -1.
 * At most 8192 features.  Synchronous; host buffers. */
int orbm_search_by_projection(int mode, const orbx_proj_frame* frame, const orbx_query_proj* q,
                              const uint8_t* qdesc, int nq, float nnratio, int th_dist,
                              int check_ori, int device, int32_t* match, int* nmatches);

/* Batched device form of orbm_search_by_projection: nprob independent
 * problems (e.g. the current frames of many streams, each with its projected
 * map points) searched in one set of launches -- the grid of every frame, a
 * wavefront per (query, problem), the greedy walk of every problem in
 * parallel.  Every pointer of a problem is DEVICE memory (frame.keys / desc
 * / uright / occupied, q, qdesc; outputs match[frame.n] and *nmatches);
 * asynchronous on `stream`.  Same results as orbm_search_by_projection on
 * each problem.  A plan holds the scratch for max_problems problems of at
 * most max_n features (<= 8192) and max_nq queries; one host thread calls a
 * plan at a time (the problem table is staged in pinned memory; a call
 * waits on the host for the previous call's table upload, not for its
 * kernels).  Calls may use different streams: each call's stream waits on
 * the device for the previous call's kernels before it reuses the plan's
 * scratch. */
typedef struct {
  orbx_proj_frame frame;
  const orbx_query_proj* q;
  const uint8_t* qdesc;
  int nq;
  int32_t* match;
  int* nmatches;
} orbx_proj_problem;
typedef struct orbm_proj_plan orbm_proj_plan;
int orbm_proj_plan_create(int max_problems, int max_n, int max_nq, int device, orbm_proj_plan** out);
int orbm_proj_plan_destroy(orbm_proj_plan* plan);
int orbm_proj_plan_search(orbm_proj_plan* plan, int mode, int nprob, const orbx_proj_problem* probs,
                          float nnratio, int th_dist, int check_ori, void* stream);

/* ---------------------------------------------------------------------------
 * SURVEY.md §8f rank 4.
 * ------------------------------------------------------------------------- */
/* MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:222-271), batched
 * over map points: map point m's observation descriptors (mObservations order,
 * non-bad keyframes) are rows off[m] .. off[m+1]) of desc; best[m] = the row
 * (relative to off[m]) with the smallest median distance, the first on ties,
 * -1 for no observation. */
int orbm_compute_distinctive_descriptors(const uint8_t* desc, const int32_t* off, int nmp,
                                         int device, int32_t* best);
/* Frame::UndistortKeyPoints (src/Frame.cc:384-414): K = mK (3x3 row-major,
 * CV_32F), dist = mDistCoef (ndist = 4 or 5: k1 k2 p1 p2 [k3]).  k1 == 0
 * copies the keypoints (:386-390); otherwise cv::undistortPoints(.., K, D,
 * noArray(), K) (OpenCV 3.4: double, 5 iterations).  out may equal kps. */
int orbx_undistort_keypoints(const orbx_keypoint* kps, int n, const float* K, const float* dist,
                             int ndist, int device, orbx_keypoint* out);

/* Multi-GPU boundary frame (bench/orbx.dist): one frame of
 * orbx_plan_extract outputs (kcap keypoint rows, kcap descriptor rows, the
 * count) as one contiguous record of orbx_boundary_record_bytes(kcap) bytes
 * [kps | desc | count | pad], the unit of the RCCL all-gather.  Device
 * pointers (kps/desc 4-B aligned), asynchronous on `stream`, one launch. */
size_t orbx_boundary_record_bytes(int kcap);
int orbx_boundary_pack(const orbx_keypoint* d_kps, const uint8_t* d_desc, const int* d_count,
                       int kcap, uint8_t* d_record, void* stream);
int orbx_boundary_unpack(const uint8_t* d_record, int kcap, orbx_keypoint* d_kps, uint8_t* d_desc,
                         int* d_count, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ORBX_H */
