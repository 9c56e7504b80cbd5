// api_misc.hip -- C ABI of SURVEY.md §8f rank 4: distinctive descriptors and
// keypoint undistortion.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>

#include "../../include/orbx.h"
#include "api_common.h"

namespace orbx {
struct UndistortArgs {
  double fx, fy, cx, cy, ifx, ify;
  double k[14];
};
__global__ void k_distinctive(const uint8_t*, const int32_t*, int, int32_t*);
__global__ void k_undistort(const orbx_keypoint*, int, const UndistortArgs, orbx_keypoint*);
}  // namespace orbx

using namespace orbx;

static int check_device(int device) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return ORBX_ERR_NO_DEVICE;
  return hipSetDevice(device) == hipSuccess ? ORBX_OK : ORBX_ERR_HIP;
}

extern "C" int orbm_compute_distinctive_descriptors(const uint8_t* desc, const int32_t* off,
                                                    int nmp, int device, int32_t* best) {
  if (nmp < 0 || (nmp > 0 && (!off || !best))) return ORBX_ERR_ARG;
  if (nmp == 0) return ORBX_OK;
  const int total = off[nmp];
  if (off[0] != 0 || total < 0 || (total > 0 && !desc)) return ORBX_ERR_ARG;
  for (int m = 0; m < nmp; ++m)
    if (off[m + 1] < off[m] || off[m + 1] - off[m] > (1 << 20)) return ORBX_ERR_ARG;
  int rc = check_device(device);
  if (rc) return rc;
  uint8_t* d_desc = nullptr;
  int32_t *d_off = nullptr, *d_best = nullptr;
  rc = ORBX_ERR_HIP;
  if (hipMalloc((void**)&d_desc, std::max(total, 1) * (size_t)32) == hipSuccess &&
      hipMalloc((void**)&d_off, (nmp + 1) * sizeof(int32_t)) == hipSuccess &&
      hipMalloc((void**)&d_best, nmp * sizeof(int32_t)) == hipSuccess &&
      (total == 0 || hipMemcpy(d_desc, desc, (size_t)total * 32, hipMemcpyHostToDevice) == hipSuccess) &&
      hipMemcpy(d_off, off, (nmp + 1) * sizeof(int32_t), hipMemcpyHostToDevice) == hipSuccess) {
    hipLaunchKernelGGL(k_distinctive, dim3((nmp + 3) / 4), dim3(256), 0, 0, d_desc, d_off, nmp,
                       d_best);
    if (hipGetLastError() == hipSuccess &&
        hipMemcpy(best, d_best, nmp * sizeof(int32_t), hipMemcpyDeviceToHost) == hipSuccess)
      rc = ORBX_OK;
  }
  if (d_desc) hipFree(d_desc);
  if (d_off) hipFree(d_off);
  if (d_best) hipFree(d_best);
  return rc;
}

extern "C" int orbx_undistort_keypoints(const orbx_keypoint* kps, int n, const float* K,
                                        const float* dist, int ndist, int device,
                                        orbx_keypoint* out) {
  if (n < 0 || !K || (ndist > 0 && !dist) || ndist < 0 || ndist > 14 || (n > 0 && (!kps || !out)))
    return ORBX_ERR_ARG;
  if (n == 0) return ORBX_OK;
  if (ndist == 0 || dist[0] == 0.0f) { /* mvKeysUn = mvKeys (:386-390) */
    memmove(out, kps, n * sizeof(orbx_keypoint));
    return ORBX_OK;
  }
  int rc = check_device(device);
  if (rc) return rc;
  UndistortArgs A;
  memset(&A, 0, sizeof(A));
  A.fx = K[0];
  A.fy = K[4];
  A.cx = K[2];
  A.cy = K[5];
  A.ifx = 1. / A.fx;
  A.ify = 1. / A.fy;
  for (int j = 0; j < ndist; ++j) A.k[j] = dist[j];
  orbx_keypoint *d_in = nullptr, *d_out = nullptr;
  rc = ORBX_ERR_HIP;
  if (hipMalloc((void**)&d_in, n * sizeof(orbx_keypoint)) == hipSuccess &&
      hipMalloc((void**)&d_out, n * sizeof(orbx_keypoint)) == hipSuccess &&
      hipMemcpy(d_in, kps, n * sizeof(orbx_keypoint), hipMemcpyHostToDevice) == hipSuccess) {
    hipLaunchKernelGGL(k_undistort, dim3((n + 255) / 256), dim3(256), 0, 0, d_in, n, A, d_out);
    if (hipGetLastError() == hipSuccess &&
        hipMemcpy(out, d_out, n * sizeof(orbx_keypoint), hipMemcpyDeviceToHost) == hipSuccess)
      rc = ORBX_OK;
  }
  if (d_in) hipFree(d_in);
  if (d_out) hipFree(d_out);
  return rc;
}
