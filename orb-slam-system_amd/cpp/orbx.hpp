// orbx.hpp -- C++ host mirror of the reference's ORBextractor / ORBmatcher
// class surface, implemented over the C ABI (include/orbx.h).
//
//   orbx::ORBextractor  <->  ORB_SLAM2::ORBextractor  (reference include/ORBextractor.h:25-91)
//   orbx::ORBmatcher    <->  ORB_SLAM2::ORBmatcher    (reference include/ORBmatcher.h:16-81)
//   orbx::ComputeStereoMatches <-> Frame::ComputeStereoMatches (reference src/Frame.cc:446-620)
//   orbx::ORBVocabulary <-> DBoW2::TemplatedVocabulary<FORB> (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h)
//   orbx::UndistortKeyPoints / ComputeDistinctiveDescriptor <-> Frame.cc:384-414 / MapPoint.cc:222-271
//
// Same constructor arguments, same getters, same operator() contract
// (keypoints cleared and refilled level-major; untouched when no keypoint
// is found; descriptors K x 32; the pyramid readable after the call), same
// error behaviour (the reference throws cv::Exception where OpenCV asserts:
// here orbx::Error).  Types are layout-compatible stand-ins for cv::KeyPoint
// and a CV_8UC1 cv::Mat view, so INTEGRATION.md's glue can hand the
// reference's own std::vector<cv::KeyPoint> storage straight through.
#ifndef ORBX_HPP
#define ORBX_HPP

#include <stdint.h>
#include <string.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/orbx.h"

namespace orbx {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& what)
      : std::runtime_error(what + ": " + orbx_status_string(c)), code(c) {}
};

inline void check(int rc, const char* what) {
  if (rc != ORBX_OK) throw Error(rc, what);
}

// cv::KeyPoint layout: Point2f pt; float size, angle, response; int octave, class_id
struct KeyPoint {
  struct {
    float x, y;
  } pt;
  float size, angle, response;
  int octave, class_id;
};
static_assert(sizeof(KeyPoint) == sizeof(orbx_keypoint), "cv::KeyPoint layout");

// CV_8UC1 image view (cv::Mat: data, cols, rows, step)
struct ImageView {
  const uint8_t* data = nullptr;
  int cols = 0, rows = 0;
  size_t step = 0;
  bool empty() const { return !data || cols <= 0 || rows <= 0; }
};

struct Image {
  int cols = 0, rows = 0;
  std::vector<uint8_t> pixels;  // tight rows
  ImageView view() const { return ImageView{pixels.data(), cols, rows, (size_t)cols}; }
};

class ORBextractor {
 public:
  enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

  // cell_guard: 0 = the reference's behaviour (throw on negative-extent FAST
  // cells, e.g. 1920x1080), 1 = treat them as empty (upstream ORB-SLAM2 guard).
  ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST,
               int cell_guard = 0, int device = 0) {
    prm_ = {nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, cell_guard};
    scale_.resize(nlevels);
    inv_.resize(nlevels);
    s2_.resize(nlevels);
    inv2_.resize(nlevels);
    fpl_.resize(nlevels);
    check(orbx_tables(&prm_, scale_.data(), inv_.data(), s2_.data(), inv2_.data(), fpl_.data(),
                      umax_),
          "ORBextractor tables");
    check(orbx_extractor_create(&prm_, device, &h_), "orbx_extractor_create");
  }
  ~ORBextractor() { orbx_extractor_destroy(h_); }
  ORBextractor(const ORBextractor&) = delete;
  ORBextractor& operator=(const ORBextractor&) = delete;

  // operator()(image, mask, keypoints, descriptors); mask ignored as in the reference
  void operator()(const ImageView& image, const ImageView& /*mask*/, std::vector<KeyPoint>& keypoints,
                  std::vector<uint8_t>& descriptors) {
    if (image.empty()) return;  // reference :444-445
    int cap = 0;
    check(orbx_extractor_capacity(h_, image.cols, image.rows, &cap), "capacity");
    std::vector<KeyPoint> kps(cap > 0 ? cap : 1);
    std::vector<uint8_t> desc((size_t)(cap > 0 ? cap : 1) * 32);
    int n = 0;
    check(orbx_extract(h_, image.data, image.cols, image.rows, image.step,
                       reinterpret_cast<orbx_keypoint*>(kps.data()), cap, desc.data(), &n),
          "ORBextractor::operator()");
    if (n == 0) {  // reference :460-463: descriptors released, keypoints untouched
      descriptors.clear();
      return;
    }
    keypoints.assign(kps.begin(), kps.begin() + n);
    descriptors.assign(desc.begin(), desc.begin() + (size_t)n * 32);
  }

  int GetLevels() { return prm_.nlevels; }
  float GetScaleFactor() { return prm_.scale_factor; }
  std::vector<float> GetScaleFactors() { return scale_; }
  std::vector<float> GetInverseScaleFactors() { return inv_; }
  std::vector<float> GetScaleSigmaSquares() { return s2_; }
  std::vector<float> GetInverseScaleSigmaSquares() { return inv2_; }

  // mvImagePyramid[level] of the last call (device -> host on demand)
  Image ImagePyramid(int level) {
    Image im;
    check(orbx_extractor_level(h_, level, nullptr, 0, &im.cols, &im.rows), "pyramid level");
    im.pixels.resize((size_t)im.cols * im.rows);
    check(orbx_extractor_level(h_, level, im.pixels.data(), (size_t)im.cols, nullptr, nullptr),
          "pyramid level");
    return im;
  }

  orbx_extractor* handle() const { return h_; }

 private:
  orbx_params prm_;
  orbx_extractor* h_ = nullptr;
  std::vector<float> scale_, inv_, s2_, inv2_;
  std::vector<int> fpl_;
  int umax_[16];
};

// DBoW2::FeatureVector (std::map<NodeId, std::vector<unsigned>>) flattened
struct FeatureVector {
  std::vector<uint32_t> node_id, node_off{0}, feat;
  void addFeature(uint32_t id, uint32_t i_feature) {  // FeatureVector.cpp:31-45 order
    size_t j = 0;
    while (j < node_id.size() && node_id[j] < id) ++j;
    if (j == node_id.size() || node_id[j] != id) {
      node_id.insert(node_id.begin() + j, id);
      node_off.insert(node_off.begin() + j + 1, node_off[j]);
    }
    feat.insert(feat.begin() + node_off[j + 1], i_feature);
    for (size_t k = j + 1; k < node_off.size(); ++k) node_off[k]++;
  }
};

// What SearchByBoW reads from a KeyFrame: descriptors, mvKeysUn angles,
// GetMapPointMatches() validity (non-null and !isBad) and mFeatVec.
struct KeyFrameView {
  const uint8_t* descriptors = nullptr;  // N x 32
  const float* angles = nullptr;         // N
  const uint8_t* valid = nullptr;        // N, nullptr = all valid
  int N = 0;
  const FeatureVector* featvec = nullptr;
};

class ORBmatcher {
 public:
  static const int TH_LOW = 50, TH_HIGH = 100, HISTO_LENGTH = 30;  // ORBmatcher.cc:13-15

  explicit ORBmatcher(float nnratio = 0.6f, bool checkOri = true, int device = 0)
      : mfNNratio(nnratio), mbCheckOrientation(checkOri), device_(device) {}

  // DescriptorDistance (ORBmatcher.cc:896-908): exact host popcount of the
  // 8 dwords -- the reference calls it per pair inside CPU loops
  // (Frame.cc:521, MapPoint.cc:252), where a device round trip per pair
  // would cost more than it saves.  Bulk callers use DescriptorDistances().
  static int DescriptorDistance(const uint8_t* a, const uint8_t* b) {
    int dist = 0;
    for (int i = 0; i < 8; ++i) {
      uint32_t va, vb;
      memcpy(&va, a + 4 * i, 4);
      memcpy(&vb, b + 4 * i, 4);
      dist += __builtin_popcount(va ^ vb);
    }
    return dist;
  }
  std::vector<int32_t> DescriptorDistances(const uint8_t* a, int na, const uint8_t* b, int nb,
                                           const std::vector<int32_t>& ia,
                                           const std::vector<int32_t>& ib) const {
    std::vector<int32_t> d(ia.size());
    check(orbm_descriptor_distance_batch(a, na, b, nb, ia.data(), ib.data(), (int)ia.size(),
                                         device_, d.data()),
          "DescriptorDistances");
    return d;
  }

  // SearchByBoW(KeyFrame*, KeyFrame*, vector<MapPoint*>&) (ORBmatcher.cc:278-366):
  // vpMatches12[i] = vpMapPoints2[matches12[i]] for matches12[i] >= 0.
  int SearchByBoW(const KeyFrameView& kf1, const KeyFrameView& kf2,
                  std::vector<int32_t>& matches12) const {
    orbx_bow_frame a = frame(kf1), b = frame(kf2);
    matches12.assign(kf1.N, -1);
    int n = 0;
    check(orbm_search_by_bow(&a, &b, mfNNratio, mbCheckOrientation ? 1 : 0, device_,
                             matches12.data(), &n),
          "SearchByBoW");
    return n;
  }

  // SearchByProjection (ORBmatcher.cc:19-61 / 732-818 / 820-894) in query
  // form: the caller projects and fills one orbx_query_proj per map point (see
  // include/orbx.h); matches[i] = the query that took frame feature i, or -1.
  //   mode 1: (Frame&, vector<MapPoint*>, th)        -- ratio test mfNNratio
  //   mode 2: (Frame& Current, const Frame& Last)    -- th_dist = TH_HIGH
  //   mode 3: (Frame& Current, KeyFrame*, set, ...)  -- th_dist = ORBdist
  int SearchByProjection(int mode, const orbx_proj_frame& frame,
                         const std::vector<orbx_query_proj>& queries,
                         const std::vector<uint8_t>& query_desc, int th_dist,
                         std::vector<int32_t>& matches) const {
    matches.assign(frame.n, -1);
    int n = 0;
    check(orbm_search_by_projection(mode, &frame, queries.data(), query_desc.data(),
                                    (int)queries.size(), mfNNratio, th_dist,
                                    mbCheckOrientation ? 1 : 0, device_, matches.data(), &n),
          "SearchByProjection");
    return n;
  }

  // SearchByBoW(KeyFrame*, Frame&, ...) in the reference is a stub that
  // returns 0 and leaves every match null (ORBmatcher.cc:88-119); kept as is.
  int SearchByBoWFrame(const KeyFrameView&, int frameN, std::vector<int32_t>& matches) const {
    matches.assign(frameN, -1);
    return 0;
  }

 private:
  static orbx_bow_frame frame(const KeyFrameView& k) {
    orbx_bow_frame f;
    f.n = k.N;
    f.desc = k.descriptors;
    f.angle = k.angles;
    f.valid = k.valid;
    f.nnodes = k.featvec ? (int)k.featvec->node_id.size() : 0;
    f.node_id = k.featvec ? k.featvec->node_id.data() : nullptr;
    f.node_off = k.featvec ? k.featvec->node_off.data() : nullptr;
    f.feat = k.featvec ? k.featvec->feat.data() : nullptr;
    return f;
  }
  float mfNNratio;
  bool mbCheckOrientation;
  int device_;
};

// DBoW2 vocabulary (ORBVocabulary) on the device: loadFromTextFile and
// transform(features, BowVector&, FeatureVector&, levelsup).
struct BowVector {
  std::vector<uint32_t> word;  // ascending (std::map order)
  std::vector<double> value;
};

class ORBVocabulary {
 public:
  explicit ORBVocabulary(int device = 0) : device_(device) {}
  ~ORBVocabulary() { orbv_vocab_destroy(v_); }
  ORBVocabulary(const ORBVocabulary&) = delete;
  ORBVocabulary& operator=(const ORBVocabulary&) = delete;

  bool loadFromTextFile(const std::string& filename) {
    orbv_vocab* v = nullptr;
    if (orbv_vocab_load_text(filename.c_str(), device_, &v) != ORBX_OK) return false;
    orbv_vocab_destroy(v_);
    v_ = v;
    return true;
  }
  bool empty() const {
    int nwords = 0;
    return !v_ || orbv_vocab_info(v_, nullptr, nullptr, nullptr, nullptr, nullptr, &nwords) ||
           nwords == 0;
  }
  // descriptors: n x 32 (mDescriptors); Frame::ComputeBoW uses levelsup = 4
  void transform(const uint8_t* descriptors, int n, BowVector& bow, FeatureVector& fv,
                 int levelsup) const {
    bow.word.assign(n, 0);
    bow.value.assign(n, 0.0);
    fv.node_id.assign(n, 0);
    fv.node_off.assign(n + 1, 0);
    fv.feat.assign(n, 0);
    int nb = 0, nf = 0;
    check(orbv_transform(v_, descriptors, n, levelsup, bow.word.data(), bow.value.data(), &nb,
                         fv.node_id.data(), fv.node_off.data(), fv.feat.data(), &nf),
          "ORBVocabulary::transform");
    bow.word.resize(nb);
    bow.value.resize(nb);
    fv.node_id.resize(nf);
    fv.node_off.resize(nf + 1);
    fv.feat.resize(fv.node_off[nf]);
  }

 private:
  orbv_vocab* v_ = nullptr;
  int device_;
};

// Frame::UndistortKeyPoints (src/Frame.cc:384-414): mvKeysUn from mvKeys,
// K = mK (row-major 3x3), dist = mDistCoef (k1 k2 p1 p2 [k3]).
inline std::vector<KeyPoint> UndistortKeyPoints(const std::vector<KeyPoint>& keys,
                                                const float K[9], const std::vector<float>& dist,
                                                int device = 0) {
  std::vector<KeyPoint> out(keys.size());
  check(orbx_undistort_keypoints(reinterpret_cast<const orbx_keypoint*>(keys.data()),
                                 (int)keys.size(), K, dist.data(), (int)dist.size(), device,
                                 reinterpret_cast<orbx_keypoint*>(out.data())),
        "UndistortKeyPoints");
  return out;
}

// MapPoint::ComputeDistinctiveDescriptors (src/MapPoint.cc:222-271): the row
// of the observation descriptors (n x 32, mObservations order) to keep.
inline int ComputeDistinctiveDescriptor(const uint8_t* descriptors, int n, int device = 0) {
  const int32_t off[2] = {0, n};
  int32_t best = -1;
  check(orbm_compute_distinctive_descriptors(descriptors, off, 1, device, &best),
        "ComputeDistinctiveDescriptors");
  return best;
}

// Frame::ComputeStereoMatches (src/Frame.cc:446-620) for a rectified pair
// whose images were the last operator() calls of `left` and `right` (the
// pyramids they left on the device are read there).  mb = baseline,
// mbf = baseline * fx.  Fills mvuRight / mvDepth (-1 = no match) and returns
// the number of stereo matches the median filter kept.
inline int ComputeStereoMatches(ORBextractor& left, ORBextractor& right,
                                const std::vector<KeyPoint>& keysL,
                                const std::vector<uint8_t>& descL,
                                const std::vector<KeyPoint>& keysR,
                                const std::vector<uint8_t>& descR, float mb, float mbf,
                                std::vector<float>& uRight, std::vector<float>& depth) {
  uRight.assign(keysL.size(), -1.0f);  // :448-449
  depth.assign(keysL.size(), -1.0f);
  int n = 0;
  check(orbx_stereo_match(left.handle(), right.handle(),
                          reinterpret_cast<const orbx_keypoint*>(keysL.data()), descL.data(),
                          (int)keysL.size(), reinterpret_cast<const orbx_keypoint*>(keysR.data()),
                          descR.data(), (int)keysR.size(), mb, mbf, uRight.data(), depth.data(),
                          &n),
        "ComputeStereoMatches");
  return n;
}

}  // namespace orbx

#endif
