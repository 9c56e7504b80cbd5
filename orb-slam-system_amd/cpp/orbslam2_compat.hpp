// orbslam2_compat.hpp -- the reference's own class surface for the hot path,
// over liborbx, for code bases without OpenCV.
//
// The reference's call sites (Frame::ExtractORB, src/Frame.cc:227-233; the
// Frame ctors' scale getters, :49-55,107-113,162-168; Tracking's extractor
// construction, src/Tracking.cc:76-82; LoopClosing::ComputeSim3 ->
// SearchByBoW(KF, KF), src/LoopClosing.cc:149; DescriptorDistance callers,
// src/Frame.cc:521, src/MapPoint.cc:252) compile unchanged against this
// header:
//   * namespace cv: the subset of OpenCV 3.4 types those signatures use
//     (Mat for CV_8UC1 data, InputArray / OutputArray, KeyPoint, Point_),
//     with OpenCV's value semantics (Mat headers share a ref-counted buffer);
//   * ORB_SLAM2::ORBextractor with the public surface of the reference's
//     include/ORBextractor.h:25-91 (constructor, operator(), the six getters,
//     public mvImagePyramid);
//   * ORB_SLAM2::ORBmatcher with ORBmatcher.h's DescriptorDistance and the
//     two SearchByBoW overloads (include/ORBmatcher.h:20-45) as templates
//     over the caller's KeyFrame / MapPoint / Frame classes, reading exactly
//     the members the reference reads (GetMapPointMatches, isBad, mvKeysUn,
//     mFeatVec, mDescriptors, N).
// A project that has OpenCV keeps its cv:: and uses INTEGRATION.md's glue
// instead; define ORBX_COMPAT_NO_CV to take cv:: from OpenCV headers.
#ifndef ORBX_ORBSLAM2_COMPAT_HPP
#define ORBX_ORBSLAM2_COMPAT_HPP

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/orbx.h"

#ifndef ORBX_COMPAT_NO_CV
#ifndef CV_8U
#define CV_8U 0
#endif
#ifndef CV_8UC1
#define CV_8UC1 0
#endif

namespace cv {

template <typename T>
struct Point_ {
  T x = 0, y = 0;
  Point_() {}
  Point_(T x_, T y_) : x(x_), y(y_) {}
};
typedef Point_<float> Point2f;
typedef Point_<int> Point2i;
typedef Point2i Point;

// cv::KeyPoint: 28 bytes, the field order orbx_keypoint mirrors
struct KeyPoint {
  Point2f pt;
  float size = 0, angle = -1, response = 0;
  int octave = 0, class_id = -1;
  KeyPoint() {}
  KeyPoint(float x, float y, float size_, float angle_ = -1, float response_ = 0, int octave_ = 0,
           int class_id_ = -1)
      : pt(x, y), size(size_), angle(angle_), response(response_), octave(octave_), class_id(class_id_) {}
};

class Exception : public std::runtime_error {
 public:
  int code;
  Exception(int c, const std::string& msg) : std::runtime_error(msg), code(c) {}
};

// 2-D CV_8UC1 matrix header over a shared byte buffer (OpenCV value semantics:
// copies share data, create() reallocates only when the shape changes)
class Mat {
 public:
  int rows = 0, cols = 0;
  uint8_t* data = nullptr;
  size_t step = 0;

  Mat() {}
  Mat(int r, int c, int type) { create(r, c, type); }
  // wraps external data (not owned), like cv::Mat(rows, cols, type, data, step)
  Mat(int r, int c, int type, void* d, size_t st = 0)
      : rows(r), cols(c), data(static_cast<uint8_t*>(d)), step(st ? st : (size_t)c), type_(type) {}

  void create(int r, int c, int type) {
    if (buf_ && r == rows && c == cols && type == type_ && step == (size_t)c) return;
    buf_ = std::make_shared<std::vector<uint8_t>>((size_t)r * c);
    rows = r;
    cols = c;
    step = (size_t)c;
    type_ = type;
    data = buf_->data();
  }
  void release() {
    buf_.reset();
    data = nullptr;
    rows = cols = 0;
    step = 0;
  }
  bool empty() const { return data == nullptr || rows == 0 || cols == 0; }
  int type() const { return type_; }
  bool isContinuous() const { return step == (size_t)cols; }
  template <typename T>
  T* ptr(int r = 0) { return reinterpret_cast<T*>(data + (size_t)r * step); }
  template <typename T>
  const T* ptr(int r = 0) const { return reinterpret_cast<const T*>(data + (size_t)r * step); }
  uint8_t* ptr(int r = 0) { return data + (size_t)r * step; }
  const uint8_t* ptr(int r = 0) const { return data + (size_t)r * step; }
  template <typename T>
  T& at(int r, int c) { return ptr<T>(r)[c]; }
  template <typename T>
  const T& at(int r, int c) const { return ptr<T>(r)[c]; }
  Mat row(int r) const { return rowRange(r, r + 1); }
  Mat rowRange(int r0, int r1) const {
    Mat m(*this);
    m.rows = r1 - r0;
    m.data = data + (size_t)r0 * step;
    return m;
  }
  Mat clone() const {
    Mat m(rows, cols, type_);
    for (int r = 0; r < rows; ++r) memcpy(m.ptr(r), ptr(r), (size_t)cols);
    return m;
  }
  void copyTo(Mat& dst) const {
    if (dst.data == data && dst.rows == rows && dst.cols == cols) return;
    Mat src(*this);  // keeps the source alive if dst aliases it
    dst.create(rows, cols, type_);
    for (int r = 0; r < rows; ++r) memcpy(dst.ptr(r), src.ptr(r), (size_t)cols);
  }

 private:
  std::shared_ptr<std::vector<uint8_t>> buf_;
  int type_ = CV_8UC1;
};

class _InputArray {
 public:
  _InputArray(const Mat& m) : m_(&m) {}
  Mat getMat() const { return *m_; }
  bool empty() const { return m_->empty(); }
  int type() const { return m_->type(); }

 private:
  const Mat* m_;
};
typedef const _InputArray& InputArray;

class _OutputArray {
 public:
  _OutputArray(Mat& m) : m_(&m) {}
  void create(int r, int c, int type) const { m_->create(r, c, type); }
  void release() const { m_->release(); }
  Mat& getMatRef() const { return *m_; }
  Mat getMat() const { return *m_; }

 private:
  Mat* m_;
};
typedef const _OutputArray& OutputArray;

}  // namespace cv
#endif  // ORBX_COMPAT_NO_CV

namespace ORB_SLAM2 {

inline void orbx_throw(int rc, const char* what) {
  if (rc != ORBX_OK) throw cv::Exception(rc, std::string(what) + ": " + orbx_status_string(rc));
}

static_assert(sizeof(cv::KeyPoint) == sizeof(orbx_keypoint), "cv::KeyPoint layout");

// ORB_SLAM2::ORBextractor (reference include/ORBextractor.h:25-91) over
// orbx_extractor: one liborbx extractor (own HIP stream and scratch) per
// instance, so the stereo threads of Frame::Frame (src/Frame.cc:58-61) run
// two instances concurrently as before.
class ORBextractor {
 public:
  enum { HARRIS_SCORE = 0, FAST_SCORE = 1 };

  ORBextractor(int nfeatures_, float scaleFactor_, int nlevels_, int iniThFAST_, int minThFAST_)
      : nfeatures(nfeatures_), scaleFactor(scaleFactor_), nlevels(nlevels_),
        iniThFAST(iniThFAST_), minThFAST(minThFAST_) {
    // cell_guard: 0 reproduces the reference (throws on negative-extent FAST
    // cells, e.g. at 1920x1080); ORBX_CELL_GUARD=1 in the environment selects
    // upstream ORB-SLAM2's skip
    const char* g = getenv("ORBX_CELL_GUARD");
    orbx_params p = {nfeatures_, scaleFactor_, nlevels_, iniThFAST_, minThFAST_, g && *g == '1'};
    mvScaleFactor.resize(nlevels);
    mvInvScaleFactor.resize(nlevels);
    mvLevelSigma2.resize(nlevels);
    mvInvLevelSigma2.resize(nlevels);
    mnFeaturesPerLevel.resize(nlevels);
    umax.resize(16);
    orbx_throw(orbx_tables(&p, mvScaleFactor.data(), mvInvScaleFactor.data(), mvLevelSigma2.data(),
                           mvInvLevelSigma2.data(), mnFeaturesPerLevel.data(), umax.data()),
               "ORBextractor");
    orbx_throw(orbx_extractor_create(&p, 0, &h_), "ORBextractor");
    orbx_throw(orbx_extractor_set_options(h_, ORBX_EXTRACTOR_PYRAMID_TO_HOST), "ORBextractor");
    mvImagePyramid.resize(nlevels);
  }
  ~ORBextractor() { orbx_extractor_destroy(h_); }
  ORBextractor(const ORBextractor&) = delete;
  ORBextractor& operator=(const ORBextractor&) = delete;

  // operator() (src/ORBextractor.cc:442-495); the mask is ignored there too
  void operator()(cv::InputArray _image, cv::InputArray /*_mask*/,
                  std::vector<cv::KeyPoint>& _keypoints, cv::OutputArray _descriptors) {
    if (_image.empty()) return;  // :444-445
    cv::Mat image = _image.getMat();
    if (image.type() != CV_8UC1) orbx_throw(ORBX_ERR_ARG, "ORBextractor: CV_8UC1 expected");  // :448
    int cap = 0, n = 0;
    orbx_throw(orbx_extractor_capacity(h_, image.cols, image.rows, &cap), "ORBextractor");
    kbuf_.resize(cap > 0 ? cap : 1);
    dbuf_.resize((size_t)(cap > 0 ? cap : 1) * 32);
    orbx_throw(orbx_extract(h_, image.data, image.cols, image.rows, image.step,
                            reinterpret_cast<orbx_keypoint*>(kbuf_.data()), cap, dbuf_.data(), &n),
               "ORBextractor::operator()");
    if (pyramid_to_host_) fill_pyramid();
    if (n == 0) {  // :460-463: descriptors released, keypoints untouched
      _descriptors.release();
      return;
    }
    _keypoints.assign(kbuf_.begin(), kbuf_.begin() + n);
    _descriptors.create(n, 32, CV_8U);
    cv::Mat& d = _descriptors.getMatRef();
    for (int r = 0; r < n; ++r) memcpy(d.ptr(r), dbuf_.data() + (size_t)r * 32, 32);
  }

  int inline GetLevels() { return nlevels; }
  float inline GetScaleFactor() { return (float)scaleFactor; }
  std::vector<float> inline GetScaleFactors() { return mvScaleFactor; }
  std::vector<float> inline GetInverseScaleFactors() { return mvInvScaleFactor; }
  std::vector<float> inline GetScaleSigmaSquares() { return mvLevelSigma2; }
  std::vector<float> inline GetInverseScaleSigmaSquares() { return mvInvLevelSigma2; }

  // the reference fills this on every call (read by Frame::ComputeStereoMatches,
  // src/Frame.cc:453,543,555,560).  The pyramid comes back with the call (one
  // D2H of the level buffer overlapped with FAST .. BRIEF; level 0 is the
  // staged copy of the image) and the headers point into the extractor's
  // pinned buffers, which the next operator() call overwrites -- the
  // reference's call sites read it before extracting again.  Monocular
  // callers may turn it off.
  std::vector<cv::Mat> mvImagePyramid;
  void SetPyramidToHost(bool on) {
    pyramid_to_host_ = on;
    orbx_throw(orbx_extractor_set_options(h_, on ? ORBX_EXTRACTOR_PYRAMID_TO_HOST : 0), "ORBextractor");
  }
  orbx_extractor* Orbx() const { return h_; }

 protected:
  void fill_pyramid() {
    for (int l = 0; l < nlevels; ++l) {
      const uint8_t* d = nullptr;
      size_t st = 0;
      int w = 0, h = 0;
      orbx_throw(orbx_extractor_level_host(h_, l, &d, &st, &w, &h), "mvImagePyramid");
      mvImagePyramid[l] = cv::Mat(h, w, CV_8U, const_cast<uint8_t*>(d), st);
    }
  }

  int nfeatures;
  double scaleFactor;
  int nlevels;
  int iniThFAST;
  int minThFAST;
  std::vector<int> mnFeaturesPerLevel;
  std::vector<int> umax;
  std::vector<float> mvScaleFactor;
  std::vector<float> mvInvScaleFactor;
  std::vector<float> mvLevelSigma2;
  std::vector<float> mvInvLevelSigma2;

 private:
  orbx_extractor* h_ = nullptr;
  bool pyramid_to_host_ = true;
  std::vector<cv::KeyPoint> kbuf_;
  std::vector<uint8_t> dbuf_;
};

// ORB_SLAM2::ORBmatcher: DescriptorDistance and SearchByBoW
// (include/ORBmatcher.h:20-45; src/ORBmatcher.cc:88-119,278-366,896-908).
class ORBmatcher {
 public:
  static const int TH_LOW = 50, TH_HIGH = 100, HISTO_LENGTH = 30;  // ORBmatcher.cc:13-15

  ORBmatcher(float nnratio = 0.6, bool checkOri = true) : mfNNratio(nnratio), mbCheckOrientation(checkOri) {}

  // Hamming distance of two 32-byte rows (ORBmatcher.cc:896-908): an exact
  // host popcount -- the per-pair callers (stereo search, projection search,
  // MapPoint::ComputeDistinctiveDescriptors) sit in CPU loops, where a
  // device round trip per pair would cost far more than the 8 popcounts
  static int DescriptorDistance(const cv::Mat& a, const cv::Mat& b) {
    const uint8_t* pa = a.ptr(0);
    const uint8_t* pb = b.ptr(0);
    int dist = 0;
    for (int i = 0; i < 8; ++i) {
      uint32_t va, vb;
      memcpy(&va, pa + 4 * i, 4);
      memcpy(&vb, pb + 4 * i, 4);
      dist += __builtin_popcount(va ^ vb);
    }
    return dist;
  }

  // SearchByBoW(KeyFrame*, KeyFrame*, vector<MapPoint*>&) (:278-366) on the
  // device.  KF: the reference's KeyFrame (GetMapPointMatches(), mvKeysUn,
  // mFeatVec, mDescriptors); MP: its MapPoint (isBad()).
  template <class KF, class MP>
  int SearchByBoW(KF* pKF1, KF* pKF2, std::vector<MP*>& vpMatches12) {
    const std::vector<MP*> vpMapPoints1 = pKF1->GetMapPointMatches();
    const std::vector<MP*> vpMapPoints2 = pKF2->GetMapPointMatches();
    Flat f1, f2;
    flatten(pKF1, vpMapPoints1, f1);
    flatten(pKF2, vpMapPoints2, f2);
    std::vector<int32_t> m12(vpMapPoints1.size(), -1);
    int n = 0;
    orbx_throw(orbm_search_by_bow(&f1.f, &f2.f, mfNNratio, mbCheckOrientation ? 1 : 0, 0,
                                  m12.data(), &n),
               "SearchByBoW");
    // as the reference (:289, :330, :359): the caller's entries survive the
    // resize; matched ones are overwritten, rotation-rejected ones reset
    vpMatches12.resize(vpMapPoints1.size(), static_cast<MP*>(nullptr));
    for (size_t i = 0; i < m12.size(); ++i) {
      if (m12[i] >= 0) vpMatches12[i] = vpMapPoints2[m12[i]];
      else if (m12[i] == -2) vpMatches12[i] = static_cast<MP*>(nullptr);
    }
    return n;
  }

  // SearchByBoW(KeyFrame*, Frame&, vector<MapPoint*>&) (:88-119) is a stub
  // in the reference: F.N null matches, returns 0.  That stays the default
  // (SURVEY.md §5 switch bow_kf_frame=stub); SetBowKFFrame(BowKFFrame::Full)
  // selects upstream ORB-SLAM2's search on the device
  // (orbm_search_by_bow_kf_frame): KF MapPoints matched to the Frame's
  // features over common vocabulary nodes.  FR: the reference's Frame (N,
  // mvKeys, mFeatVec after ComputeBoW, mDescriptors).
  enum class BowKFFrame { Stub, Full };
  void SetBowKFFrame(BowKFFrame m) { mBowKFFrame = m; }
  template <class KF, class FR, class MP>
  int SearchByBoW(KF* pKF, FR& F, std::vector<MP*>& vpMapPointMatches) {
    if (mBowKFFrame == BowKFFrame::Stub) {
      vpMapPointMatches.resize(F.N, static_cast<MP*>(nullptr));  // :90
      return 0;
    }
    const std::vector<MP*> vpMapPointsKF = pKF->GetMapPointMatches();
    Flat fk, ff;
    flatten(pKF, vpMapPointsKF, fk);
    flatten_frame(F, ff);
    std::vector<int32_t> mf(F.N > 0 ? (size_t)F.N : 1, -1);
    int n = 0;
    orbx_throw(orbm_search_by_bow_kf_frame(&fk.f, &ff.f, mfNNratio, mbCheckOrientation ? 1 : 0, 0, mf.data(), &n),
               "SearchByBoW");
    vpMapPointMatches.assign(F.N, static_cast<MP*>(nullptr));  // upstream: vector<MapPoint*>(F.N, NULL)
    for (int i = 0; i < F.N; ++i)
      if (mf[i] >= 0) vpMapPointMatches[i] = vpMapPointsKF[mf[i]];
    return n;
  }

 protected:
  struct Flat {
    orbx_bow_frame f;
    std::vector<uint8_t> valid;
    std::vector<float> angle;
    std::vector<uint32_t> ids, off, feat;
  };
  template <class KF, class MP>
  static void flatten(KF* kf, const std::vector<MP*>& mps, Flat& o) {
    o.valid.resize(mps.size());
    for (size_t i = 0; i < mps.size(); ++i) o.valid[i] = mps[i] && !mps[i]->isBad();
    o.angle.resize(kf->mvKeysUn.size());
    for (size_t i = 0; i < kf->mvKeysUn.size(); ++i) o.angle[i] = kf->mvKeysUn[i].angle;
    o.off.push_back(0);
    for (const auto& node : kf->mFeatVec) {  // std::map: ascending NodeId
      o.ids.push_back(node.first);
      o.feat.insert(o.feat.end(), node.second.begin(), node.second.end());
      o.off.push_back((uint32_t)o.feat.size());
    }
    o.f.n = (int)mps.size();
    o.f.desc = kf->mDescriptors.data;
    o.f.angle = o.angle.data();
    o.f.valid = o.valid.data();
    o.f.nnodes = (int)o.ids.size();
    o.f.node_id = o.ids.data();
    o.f.node_off = o.off.data();
    o.f.feat = o.feat.data();
  }

  template <class FR>
  static void flatten_frame(FR& F, Flat& o) {
    o.angle.resize(F.mvKeys.size());
    for (size_t i = 0; i < F.mvKeys.size(); ++i) o.angle[i] = F.mvKeys[i].angle;
    o.off.push_back(0);
    for (const auto& node : F.mFeatVec) {  // std::map: ascending NodeId
      o.ids.push_back(node.first);
      o.feat.insert(o.feat.end(), node.second.begin(), node.second.end());
      o.off.push_back((uint32_t)o.feat.size());
    }
    o.f.n = F.N;
    o.f.desc = F.mDescriptors.data;
    o.f.angle = o.angle.data();
    o.f.valid = nullptr;
    o.f.nnodes = (int)o.ids.size();
    o.f.node_id = o.ids.data();
    o.f.node_off = o.off.data();
    o.f.feat = o.feat.data();
  }

  float mfNNratio;
  bool mbCheckOrientation;
  BowKFFrame mBowKFFrame = BowKFFrame::Stub;
};

}  // namespace ORB_SLAM2

// ---------------------------------------------------------------------------
// SURVEY.md §8(f), the callers either side of the path, with the reference's
// own shapes:
//   * DBoW2::BowVector / FeatureVector (Thirdparty/DBoW2/DBoW2/BowVector.h,
//     FeatureVector.h: std::maps keyed by word / node id) and
//     ORB_SLAM2::ORBVocabulary (DBoW2::TemplatedVocabulary<FORB::TDescriptor,
//     FORB>, include/ORBVocabulary.h) with loadFromTextFile / empty /
//     transform(features, BowVector&, FeatureVector&, levelsup), as
//     Frame::ComputeBoW (src/Frame.cc:373-382) and System's loader call them;
//   * Frame::ComputeStereoMatches (src/Frame.cc:446-620) as a template over
//     the caller's Frame, reading and writing exactly the members the
//     reference's member function does.
// ---------------------------------------------------------------------------
#ifndef ORBX_COMPAT_NO_DBOW2
namespace DBoW2 {
typedef unsigned int WordId;
typedef double WordValue;
typedef unsigned int NodeId;
class BowVector : public std::map<WordId, WordValue> {};
class FeatureVector : public std::map<NodeId, std::vector<unsigned int> > {};
}  // namespace DBoW2
#endif

namespace ORB_SLAM2 {

class ORBVocabulary {
 public:
  ORBVocabulary() {}
  ~ORBVocabulary() { orbv_vocab_destroy(v_); }
  ORBVocabulary(const ORBVocabulary&) = delete;
  ORBVocabulary& operator=(const ORBVocabulary&) = delete;

  // TemplatedVocabulary::loadFromTextFile (TemplatedVocabulary.h:1126-1259)
  bool loadFromTextFile(const std::string& filename) {
    orbv_vocab* v = nullptr;
    if (orbv_vocab_load_text(filename.c_str(), 0, &v) != ORBX_OK) return false;
    orbv_vocab_destroy(v_);
    v_ = v;
    return true;
  }
  bool empty() const {
    int nwords = 0;
    return !v_ || orbv_vocab_info(v_, nullptr, nullptr, nullptr, nullptr, nullptr, &nwords) || nwords == 0;
  }
  // transform(features, v, fv, levelsup) (TemplatedVocabulary.h:1338-1424):
  // features = Converter::toDescriptorVector(mDescriptors), one 1 x 32 row each
  void transform(const std::vector<cv::Mat>& features, DBoW2::BowVector& v, DBoW2::FeatureVector& fv,
                 int levelsup) const {
    v.clear();
    fv.clear();
    const int n = (int)features.size();
    if (n == 0) return;
    std::vector<uint8_t> desc((size_t)n * 32);
    for (int i = 0; i < n; ++i) memcpy(desc.data() + (size_t)i * 32, features[i].ptr(0), 32);
    std::vector<uint32_t> word(n), node(n), off(n + 1), feat(n);
    std::vector<double> value(n);
    int nb = 0, nf = 0;
    orbx_throw(orbv_transform(v_, desc.data(), n, levelsup, word.data(), value.data(), &nb, node.data(),
                              off.data(), feat.data(), &nf),
               "ORBVocabulary::transform");
    for (int i = 0; i < nb; ++i) v.insert(v.end(), std::make_pair(word[i], value[i]));
    for (int j = 0; j < nf; ++j)
      fv.insert(fv.end(), std::make_pair(node[j], std::vector<unsigned int>(feat.begin() + off[j],
                                                                              feat.begin() + off[j + 1])));
  }

 private:
  orbv_vocab* v_ = nullptr;
};

// Frame::ComputeStereoMatches (src/Frame.cc:446-620) for a stereo Frame whose
// two extractors just ran on its images (their pyramids stay on the device
// for the search).  FR: the reference's Frame -- reads N, mvKeys, mvKeysRight,
// mDescriptors, mDescriptorsRight, mb, mbf, mpORBextractorLeft / Right;
// writes mvuRight / mvDepth (-1 where no match survives, :448-449).
template <class FR>
void ComputeStereoMatches(FR& F) {
  F.mvuRight = std::vector<float>(F.N, -1.0f);
  F.mvDepth = std::vector<float>(F.N, -1.0f);
  int kept = 0;
  orbx_throw(orbx_stereo_match(F.mpORBextractorLeft->Orbx(), F.mpORBextractorRight->Orbx(),
                               reinterpret_cast<const orbx_keypoint*>(F.mvKeys.data()), F.mDescriptors.data,
                               (int)F.mvKeys.size(), reinterpret_cast<const orbx_keypoint*>(F.mvKeysRight.data()),
                               F.mDescriptorsRight.data, (int)F.mvKeysRight.size(), F.mb, F.mbf,
                               F.mvuRight.data(), F.mvDepth.data(), &kept),
             "ComputeStereoMatches");
}

}  // namespace ORB_SLAM2

#endif
