// orbx.hpp -- C++ host mirror of the reference's ORBextractor / ORBmatcher
// class surface, implemented over the C ABI (include/orbx.h).
//
//   orbx::ORBextractor  <->  ORB_SLAM2::ORBextractor  (reference include/ORBextractor.h:25-91)
//   orbx::ORBmatcher    <->  ORB_SLAM2::ORBmatcher    (reference include/ORBmatcher.h:16-81)
//   orbx::ComputeStereoMatches <-> Frame::ComputeStereoMatches (reference src/Frame.cc:446-620)
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

  // DescriptorDistance (ORBmatcher.cc:896-908), evaluated on the device.
  // Bulk callers should use DescriptorDistances().
  int DescriptorDistance(const uint8_t* a, const uint8_t* b) const {
    int32_t z = 0, d = 0;
    check(orbm_descriptor_distance_batch(a, 1, b, 1, &z, &z, 1, device_, &d),
          "DescriptorDistance");
    return d;
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
