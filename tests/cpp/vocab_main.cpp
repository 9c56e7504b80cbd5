// ORBVocabulary as System / Frame::ComputeBoW / LoopClosing use it
// (src/System.cc:59-62, src/Frame.cc:373-382, src/LoopClosing.cc:149):
// load ORBvoc-format text, transform two frames' descriptor rows (levelsup
// 4), SearchByBoW(KF, KF) on the resulting FeatureVectors -- compiled
// against orb-slam-system_amd/cpp/orbslam2_compat.hpp.  Used by
// tests/test_cpp_adapter.py.
//   vocab_main voc.txt a.raw b.raw W H out.bin
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "orbslam2_compat.hpp"

using namespace ORB_SLAM2;

// the KeyFrame / MapPoint members SearchByBoW reads (KeyFrame.h, MapPoint.h)
struct TMapPoint {
  bool isBad() { return false; }
};
struct TKeyFrame {
  std::vector<TMapPoint*> mvpMapPoints;
  std::vector<cv::KeyPoint> mvKeysUn;
  DBoW2::BowVector mBowVec;
  DBoW2::FeatureVector mFeatVec;
  cv::Mat mDescriptors;
  std::vector<TMapPoint*> GetMapPointMatches() { return mvpMapPoints; }
};

static std::vector<uint8_t> load(const char* p, size_t n) {
  std::vector<uint8_t> v(n);
  FILE* f = fopen(p, "rb");
  if (!f || fread(v.data(), 1, n, f) != n) { fprintf(stderr, "read %s\n", p); exit(2); }
  fclose(f);
  return v;
}

// Converter::toDescriptorVector (src/Converter.cc:27-35): one row per keypoint
static std::vector<cv::Mat> toDescriptorVector(const cv::Mat& d) {
  std::vector<cv::Mat> v;
  for (int j = 0; j < d.rows; ++j) v.push_back(d.row(j));
  return v;
}

int main(int argc, char** argv) {
  if (argc != 7) return 2;
  const int W = atoi(argv[4]), H = atoi(argv[5]);
  auto a = load(argv[2], (size_t)W * H), b = load(argv[3], (size_t)W * H);
  ORBVocabulary voc;
  if (!voc.loadFromTextFile(argv[1]) || voc.empty()) { fprintf(stderr, "vocab\n"); return 3; }
  ORBextractor ex(2000, 1.2f, 8, 20, 7);
  TKeyFrame kf1, kf2;
  ex(cv::Mat(H, W, CV_8UC1, a.data()), cv::Mat(), kf1.mvKeysUn, kf1.mDescriptors);
  ex(cv::Mat(H, W, CV_8UC1, b.data()), cv::Mat(), kf2.mvKeysUn, kf2.mDescriptors);
  voc.transform(toDescriptorVector(kf1.mDescriptors), kf1.mBowVec, kf1.mFeatVec, 4);  // Frame.cc:378
  voc.transform(toDescriptorVector(kf2.mDescriptors), kf2.mBowVec, kf2.mFeatVec, 4);
  std::vector<TMapPoint> mp2(kf2.mvKeysUn.size());
  TMapPoint mp;
  kf1.mvpMapPoints.assign(kf1.mvKeysUn.size(), &mp);
  kf2.mvpMapPoints.resize(mp2.size());
  for (size_t i = 0; i < mp2.size(); ++i) kf2.mvpMapPoints[i] = &mp2[i];
  ORBmatcher m(0.75f, true);  // LoopClosing.cc:129
  std::vector<TMapPoint*> vpMatches12;
  const int nm = m.SearchByBoW(&kf1, &kf2, vpMatches12);
  std::vector<int32_t> m12(kf1.mvKeysUn.size(), -1);
  for (size_t i = 0; i < vpMatches12.size(); ++i)
    if (vpMatches12[i]) m12[i] = (int32_t)(vpMatches12[i] - mp2.data());
  std::vector<uint32_t> words, nodes, off{0}, feat;
  std::vector<double> values;
  for (const auto& w : kf1.mBowVec) {
    words.push_back(w.first);
    values.push_back(w.second);
  }
  for (const auto& n : kf1.mFeatVec) {
    nodes.push_back(n.first);
    feat.insert(feat.end(), n.second.begin(), n.second.end());
    off.push_back((uint32_t)feat.size());
  }
  FILE* o = fopen(argv[6], "wb");
  int hdr[4] = {(int)kf1.mvKeysUn.size(), (int)words.size(), (int)nodes.size(), nm};
  fwrite(hdr, sizeof(int), 4, o);
  fwrite(words.data(), 4, words.size(), o);
  fwrite(values.data(), 8, values.size(), o);
  fwrite(nodes.data(), 4, nodes.size(), o);
  fwrite(off.data(), 4, off.size(), o);
  fwrite(feat.data(), 4, feat.size(), o);
  fwrite(m12.data(), 4, m12.size(), o);
  fclose(o);
  printf("vocab ok: K1=%zu words=%zu nodes=%zu matches=%d\n", kf1.mvKeysUn.size(), words.size(), nodes.size(), nm);
  return 0;
}
