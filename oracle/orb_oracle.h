/* orb_oracle.h -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference
 * ORB front end (WangHewei16/ORB-SLAM-System), used as the parity checker.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library.  The product (liborbx.so) never links or calls it.
 *
 * PARITY STATUS: "parity unpinned" against the reference binary.
 *   - The reference cannot be built here (needs OpenCV 3.4, Eigen, Pangolin;
 *     none exist in the image) and it ships no golden vectors, fixtures or
 *     tests for this path.
 *   - This file restates /root/reference/src/ORBextractor.cc and
 *     /root/reference/src/ORBmatcher.cc line by line (citations inline), and
 *     the OpenCV 3.4 primitives they call (cv::resize INTER_LINEAR,
 *     cv::FAST, cv::GaussianBlur, cv::fastAtan2) from OpenCV's published
 *     algorithm.
 *   - Partial pins: constant tables (umax, features per level, scale tables,
 *     the BRIEF pattern parsed from the reference source) are checked against
 *     known answers in tests/test_oracle.py.
 */
#ifndef ORB_ORACLE_H
#define ORB_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* cv::KeyPoint layout (28 bytes) */
typedef struct {
  float x, y, size, angle, response;
  int octave, class_id;
} oo_keypoint;

#define OO_MAX_LEVELS 32

enum {
  OO_OK = 0,
  OO_ERR_ARG = -1,
  OO_ERR_CELL_ROI = -2,     /* reference: cv::Mat(m, Rect) assertion -> cv::Exception */
  OO_ERR_LEVEL_SIZE = -3,   /* reference: division by zero / bad alloc on tiny levels */
  OO_ERR_QUADTREE = -4,     /* reference: DistributeOctTree never terminates */
  OO_ERR_CAPACITY = -5,
  OO_ERR_UNSUPPORTED = -6,  /* exact 2x level ratio: OpenCV switches to INTER_AREA */
};

typedef struct oo_extractor oo_extractor;

oo_extractor* oo_create(int nfeatures, float scaleFactor, int nlevels, int iniThFAST,
                        int minThFAST, int cell_guard /*0 strict, 1 empty*/);
void oo_destroy(oo_extractor* e);

/* tables (ORBextractor.cc:116-170) */
int oo_get_tables(const oo_extractor* e, float* scale, float* inv_scale, float* sigma2,
                  float* inv_sigma2, int* features_per_level, int* umax16);

/* ORBextractor::operator() (ORBextractor.cc:442-495).  Returns OO_OK or an
 * error; *n = keypoint count (0 => kps/desc untouched, as the reference). */
int oo_extract(oo_extractor* e, const uint8_t* img, int w, int h, int stride, oo_keypoint* kps,
               int cap, uint8_t* desc, int* n);

/* stage outputs of the last oo_extract call, for per-stage parity */
int oo_level_size(const oo_extractor* e, int level, int* w, int* h);
const uint8_t* oo_level_pixels(const oo_extractor* e, int level); /* tight rows */
/* vToDistributeKeys of a level (ORBextractor.cc:305-340): x,y relative to 16,16 */
int oo_level_candidates(const oo_extractor* e, int level, oo_keypoint* out, int cap);
/* DistributeOctTree output (+16 offset, octave, size; angle set) before rescale */
int oo_level_keys(const oo_extractor* e, int level, oo_keypoint* out, int cap);

/* individual primitives (for known-answer tests) */
float oo_fast_atan2(float y, float x);
int oo_fast_detect(const uint8_t* img, int w, int h, int stride, int threshold, int nonmax,
                   oo_keypoint* out, int cap);
void oo_resize_linear(const uint8_t* src, int sw, int sh, int sstride, uint8_t* dst, int dw,
                      int dh, int dstride);
/* exact 2x downscale: OpenCV's INTER_AREA fast path that resize(INTER_LINEAR)
 * switches to when both ratios are exactly 2 */
void oo_resize_area2(const uint8_t* src, int sw, int sh, int sstride, uint8_t* dst, int dw, int dh,
                     int dstride);
void oo_gaussian_blur7(const uint8_t* src, int w, int h, int stride, uint8_t* dst, int dstride);
void oo_gaussian_kernel7(int raw[7]);
void oo_brief_descriptor(const uint8_t* blurred, int stride, int cx, int cy, float angle_deg,
                         uint8_t* desc32);

/* ORBmatcher (ORBmatcher.cc) */
int oo_descriptor_distance(const uint8_t* a, const uint8_t* b);
/* SearchByBoW(KeyFrame*, KeyFrame*) (ORBmatcher.cc:278-366).
 * FeatureVector k: nodes ids node_id[k][0..nnode), ascending & unique; node j
 * holds features feat[k][off[k][j] .. off[k][j+1]).  valid[k][i] = MapPoint
 * present and !isBad (NULL => all valid).  match12[i] = idx2 or -1. */
int oo_search_by_bow(int n1, const uint8_t* desc1, const float* angle1, const uint8_t* valid1,
                     int nnode1, const uint32_t* node_id1, const uint32_t* off1,
                     const uint32_t* feat1, int n2, const uint8_t* desc2, const float* angle2,
                     const uint8_t* valid2, int nnode2, const uint32_t* node_id2,
                     const uint32_t* off2, const uint32_t* feat2, float nnratio, int check_ori,
                     int32_t* match12);
/* upstream ORB-SLAM2's SearchByBoW(KeyFrame*, Frame&) (the reference ships a
 * stub, src/ORBmatcher.cc:88-119); match_f[nf]: KF index or -1 */
int oo_search_by_bow_kf_frame(int nk, const uint8_t* desc_k, const float* angle_k,
                              const uint8_t* valid_k, int nnode_k, const uint32_t* node_id_k,
                              const uint32_t* off_k, const uint32_t* feat_k, int nf,
                              const uint8_t* desc_f, const float* angle_f, int nnode_f,
                              const uint32_t* node_id_f, const uint32_t* off_f, const uint32_t* feat_f,
                              float nnratio, int check_ori, int32_t* match_f);

/* Frame::ComputeStereoMatches (src/Frame.cc:446-620).  Left/right keypoints
 * and descriptors of one rectified pair; lpyr/rpyr[l] = mvImagePyramid[l] of
 * the left/right extractor (both of size lw[l] x lh[l], rows lstride[l]);
 * scale/inv_scale = mvScaleFactors / mvInvScaleFactors; mb and mbf as the
 * Frame members (the reference reads mb before assigning it, Frame.cc:70 vs
 * :94 -- callers pass mbf/fx).  Outputs mvuRight/mvDepth (-1 = none).
 * Returns the number of stereo matches kept, or OO_ERR_ARG where the
 * reference would index out of range or throw (cv::Mat range asserts). */
int oo_compute_stereo_matches(int nl, const oo_keypoint* kl, const uint8_t* dl, int nr,
                              const oo_keypoint* kr, const uint8_t* dr, int nlevels,
                              const float* scale, const float* inv_scale,
                              const uint8_t* const* lpyr, const uint8_t* const* rpyr,
                              const int* lw, const int* lh, const int* lstride, float mb,
                              float mbf, float* uright, float* depth);

/* DBoW2 vocabulary (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h).  Node
 * records in loadFromTextFile order (:1378-1422): record r is node r+1 with
 * parent[r], is_leaf[r] (nIsLeaf), desc[r] (32 B), weight[r].  NULL if the
 * header is rejected (:1356-1360) or a parent does not exist yet. */
typedef struct oo_vocab oo_vocab;
oo_vocab* oo_vocab_from_records(int k, int L, int scoring, int weighting, int nrec,
                                const int* parent, const int* is_leaf, const uint8_t* desc,
                                const double* weight);
void oo_vocab_destroy(oo_vocab* v);
int oo_vocab_info(const oo_vocab* v, int* k, int* L, int* scoring, int* weighting, int* nnodes,
                  int* nwords);
/* transform(features, BowVector&, FeatureVector&, levelsup) (:1126-1191) */
int oo_vocab_transform(const oo_vocab* v, const uint8_t* desc, int n, int levelsup,
                       uint32_t* bow_word, double* bow_value, int* nbow, uint32_t* fv_node,
                       uint32_t* fv_off, uint32_t* fv_feat, int* nfv);

/* Frame grid (src/Frame.cc:210-225,307-371, 64 x 48 cells) and
 * ORBmatcher::SearchByProjection in query form: the caller projects (pose
 * math on cv::Mat) and passes per query the position, the radius handed to
 * GetFeaturesInArea, its level bounds, mTrackProjXR (mode 1 stereo gate)
 * and the source keypoint angle (modes 2/3 rotation check). */
typedef struct {
  float x, y, radius;
  int min_level, max_level;
  float xr;
  float angle;
} oo_proj_query;
int oo_features_in_area(int n, const oo_keypoint* keys, float minX, float minY, float wInv,
                        float hInv, float x, float y, float r, int minLevel, int maxLevel,
                        int* out);
int oo_search_by_projection(int mode, int n, const oo_keypoint* keys, const uint8_t* desc,
                            const float* uright, const uint8_t* occupied, float minX, float minY,
                            float wInv, float hInv, int nq, const oo_proj_query* q,
                            const uint8_t* qdesc, float nnratio, int th_dist, int check_ori,
                            int32_t* match);

/* MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:222-271) */
int oo_distinctive_descriptor(const uint8_t* desc, int N);
/* Frame::UndistortKeyPoints (src/Frame.cc:384-414) with cv::undistortPoints */
void oo_undistort_keypoints(const oo_keypoint* in, int n, const float* K9, const float* dist,
                            int ndist, oo_keypoint* out);

#ifdef __cplusplus
}
#endif
#endif
