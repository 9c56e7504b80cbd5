// compat_latency -- per-call latency of the reference-shaped call site:
// ORB_SLAM2::ORBextractor::operator() from cpp/orbslam2_compat.hpp, called one
// frame at a time as Frame::ExtractORB does (src/Frame.cc:227-233), with
// mvImagePyramid refilled on every call (src/ORBextractor.cc:497-515) and
// read afterwards the way Frame::ComputeStereoMatches reads it
// (src/Frame.cc:543-560: one pixel per level touched here).
//   compat_latency W H nfeatures warm calls frames.raw nframes
// Frames: nframes W x H images back to back.  Prints one JSON object.
// ORBX_CELL_GUARD=1 in the environment selects the upstream cell guard.
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>
#include <vector>

#include "../orb-slam-system_amd/cpp/orbslam2_compat.hpp"

using namespace ORB_SLAM2;

static double pct(std::vector<double> v, double q) {
  std::sort(v.begin(), v.end());
  size_t i = (size_t)(q / 100.0 * (double)(v.size() - 1) + 0.5);
  return v[std::min(i, v.size() - 1)];
}

int main(int argc, char** argv) {
  if (argc != 8) {
    fprintf(stderr, "usage: compat_latency W H nfeatures warm calls frames.raw nframes\n");
    return 2;
  }
  const int W = atoi(argv[1]), H = atoi(argv[2]), nf = atoi(argv[3]);
  const int warm = atoi(argv[4]), calls = atoi(argv[5]), nfr = atoi(argv[7]);
  std::vector<uint8_t> raw((size_t)W * H * nfr);
  FILE* f = fopen(argv[6], "rb");
  if (!f || fread(raw.data(), 1, raw.size(), f) != raw.size()) {
    fprintf(stderr, "compat_latency: cannot read %s\n", argv[6]);
    return 2;
  }
  fclose(f);
  std::vector<cv::Mat> frames;
  for (int i = 0; i < nfr; ++i) frames.emplace_back(H, W, CV_8UC1, raw.data() + (size_t)i * W * H);
  printf("{");
  const char* sep = "";
  for (int pyr = 1; pyr >= 0; --pyr) {
    ORBextractor ex(nf, 1.2f, 8, 20, 7);
    ex.SetPyramidToHost(pyr != 0);
    std::vector<cv::KeyPoint> kps;
    cv::Mat desc;
    std::vector<double> ts;
    long long touch = 0;
    for (int i = 0; i < warm + calls; ++i) {
      const auto t0 = std::chrono::steady_clock::now();
      ex(frames[i % nfr], cv::Mat(), kps, desc);
      if (pyr)
        for (int l = 0; l < 8; ++l) {  // the stereo search reads the levels next
          const cv::Mat& m = ex.mvImagePyramid[l];
          touch += m.ptr(m.rows / 2)[m.cols / 2];
        }
      const auto t1 = std::chrono::steady_clock::now();
      if (i >= warm) ts.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    long long nc = 0, nre = 0;
    orbx_extractor_stats(ex.Orbx(), &nc, &nre);
    printf("%s\"%s\": {\"p50_us\": %.1f, \"p99_us\": %.1f, \"max_us\": %.1f, \"calls\": %d, "
           "\"keypoints\": %zu, \"refetches\": %lld, \"extract_calls\": %lld, \"checksum\": %lld}",
           sep, pyr ? "operator_with_mvImagePyramid" : "operator_no_pyramid", pct(ts, 50), pct(ts, 99),
           *std::max_element(ts.begin(), ts.end()), calls, kps.size(), nre, nc, touch);
    sep = ", ";
  }
  printf("}\n");
  return 0;
}
