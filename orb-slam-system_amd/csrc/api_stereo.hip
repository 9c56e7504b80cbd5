// api_stereo.hip -- C ABI of the stereo matcher: Frame::ComputeStereoMatches
// (/root/reference/src/Frame.cc:446-620) on the device-resident pyramids of
// the left and right extractors.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <cmath>

#include "../../include/orbx.h"
#include "api_common.h"
#include "geometry.h"
#include "plan_internal.h"

namespace orbx {
__global__ void k_stereo_rows(const orbx_keypoint*, const int*, const StereoArgs, int*, uint2*,
                              int*);
__global__ void k_stereo_match(const orbx_keypoint*, const uint8_t*, const int*,
                               const orbx_keypoint*, const uint8_t*, const uint8_t*,
                               const uint8_t*, size_t, size_t, const uint8_t*, const uint8_t*,
                               size_t, const StereoArgs, const int*, const uint2*, float*,
                               float*, int*, int*);
__global__ void k_stereo_filter(const int*, const StereoArgs, float*, float*, const int*, int*);
}  // namespace orbx

using namespace orbx;

struct orbs_plan {
  int device = 0, max_batch = 0, waves = 4;
  int sm_div = 0; /* ORBX_DEBUG_SMDIV: k_stereo_match keypoints per wave, profiling only */
  orbx_params params;
  int W = 0, H = 0;
  StereoArgs args;
  int* d_rowoff = nullptr;
  uint2* d_rows = nullptr; /* CSR entries {iR | octave << 16, x} (kernels_stereo.hip) */
  int* d_sad = nullptr;
  int* d_err = nullptr;
  /* host drop-in (orbx_stereo_match) staging, batch 1 */
  orbx_keypoint *d_kl = nullptr, *d_kr = nullptr;
  uint8_t *d_dl = nullptr, *d_dr = nullptr;
  int* d_cnt = nullptr; /* [2]: left, right */
  float *d_ur = nullptr, *d_dep = nullptr;
  int* d_nm = nullptr;
  hipStream_t stream = nullptr;
  StageTimer timer;
};

static void splan_free(orbs_plan* sp) {
  if (!sp) return;
  hipSetDevice(sp->device);
  void* bufs[] = {sp->d_rowoff, sp->d_rows, sp->d_sad, sp->d_err, sp->d_kl, sp->d_kr,
                  sp->d_dl,     sp->d_dr,   sp->d_cnt, sp->d_ur,  sp->d_dep, sp->d_nm};
  for (void* b : bufs)
    if (b) hipFree(b);
  sp->timer.release();
  if (sp->stream) hipStreamDestroy(sp->stream);
  delete sp;
}

static int splan_create(const orbx_plan* g, int max_batch, orbs_plan** out) {
  *out = nullptr;
  const Plan& P = g->P;
  const int L = P.params.nlevels;
  if (P.H > ORBX_STEREO_MAXROWS || P.kcap > 65535 || L > ORBX_MAX_LEVELS) return ORBX_ERR_UNSUPPORTED;
  orbs_plan* sp = new orbs_plan();
  sp->device = g->device;
  sp->max_batch = max_batch;
  sp->params = P.params;
  sp->W = P.W;
  sp->H = P.H;
  StereoArgs& A = sp->args;
  memset(&A, 0, sizeof(A));
  A.nlevels = L;
  A.nrows = P.H; /* mvImagePyramid[0].rows (:453) */
  A.kcap = P.kcap;
  float smax = 0.f;
  for (int l = 0; l < L; ++l) {
    const LevelInfo& lv = P.levels[l];
    const LevelInfo& u = P.levels[lv.unique];
    A.off[l] = lv.unique == 0 ? -1 : u.pyr_off;
    A.pitch[l] = u.pitch;
    A.w[l] = lv.w;
    A.h[l] = lv.h;
    A.scale[l] = P.tables.scale[l];
    A.inv_scale[l] = P.tables.inv_scale[l];
    smax = std::max(smax, A.scale[l]);
  }
  /* a keypoint spans ceil(y + 2s) - floor(y - 2s) + 1 <= 4s + 3 rows */
  const int span = (int)std::ceil(4.0 * smax) + 3;
  A.rcap = P.kcap * span;
  sp->waves = std::max(4, std::min(P.kcap, P.params.nfeatures + 256));
#ifdef ORBX_PROFILING
  if (const char* e = getenv("ORBX_DEBUG_SMDIV")) sp->sm_div = atoi(e); /* profiling builds only */
#endif
  hipSetDevice(sp->device);
  const size_t B = (size_t)max_batch;
  const size_t K = (size_t)std::max(P.kcap, 1);
  if (hipMalloc((void**)&sp->d_rowoff, B * (A.nrows + 1) * sizeof(int)) != hipSuccess ||
      hipMalloc((void**)&sp->d_rows, B * (size_t)std::max(A.rcap, 1) * sizeof(uint2)) != hipSuccess ||
      hipMalloc((void**)&sp->d_sad, B * K * sizeof(int)) != hipSuccess ||
      hipMalloc((void**)&sp->d_err, 16) != hipSuccess ||
      hipMemset(sp->d_err, 0, 16) != hipSuccess ||
      hipStreamCreateWithFlags(&sp->stream, hipStreamNonBlocking) != hipSuccess) {
    splan_free(sp);
    return ORBX_ERR_HIP;
  }
  if (A.nrows * sizeof(int) > 64 * 1024 &&
      hipFuncSetAttribute((const void*)k_stereo_rows, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)(A.nrows * sizeof(int))) != hipSuccess) {
    splan_free(sp);
    return ORBX_ERR_HIP;
  }
  *out = sp;
  return ORBX_OK;
}

extern "C" int orbs_plan_create(const orbx_plan* geometry, int max_batch, orbs_plan** out) {
  if (!geometry || !out || max_batch < 1) return ORBX_ERR_ARG;
  return splan_create(geometry, max_batch, out);
}

extern "C" int orbs_plan_destroy(orbs_plan* sp) {
  splan_free(sp);
  return ORBX_OK;
}

static bool same_geometry(const orbs_plan* sp, const orbx_plan* p) {
  return p && p->P.W == sp->W && p->P.H == sp->H && p->device == sp->device &&
         p->P.params.nfeatures == sp->params.nfeatures &&
         p->P.params.nlevels == sp->params.nlevels &&
         p->P.params.scale_factor == sp->params.scale_factor;
}

/* the reference's left and right extractors share their parameters
 * (Tracking.cc:76-82); the pyramids must have identical level sizes */
static bool same_geometry_pair(const orbx_plan* a, const orbx_plan* b) {
  return a->P.W == b->P.W && a->P.H == b->P.H && a->device == b->device &&
         a->P.params.nlevels == b->P.params.nlevels &&
         a->P.params.scale_factor == b->P.params.scale_factor;
}

static int splan_launch(orbs_plan* sp, int n, const uint8_t* fl, const uint8_t* fr, size_t fstride,
                        size_t rstride, const uint8_t* pyr_l, const uint8_t* pyr_r,
                        size_t pstride, const orbx_keypoint* kl, const uint8_t* dl,
                        const int* cl, const orbx_keypoint* kr, const uint8_t* dr,
                        const int* cr, float mb, float mbf, float* ur, float* dep, int* nm,
                        hipStream_t s) {
  StereoArgs A = sp->args;
  A.mb = mb;
  A.mbf = mbf;
  sp->timer.begin(ORBX_STAGE_SROWS, s);
  hipLaunchKernelGGL(k_stereo_rows, dim3(n), dim3(1024), A.nrows * sizeof(int), s, kr, cr, A,
                     sp->d_rowoff, sp->d_rows, sp->d_err);
  sp->timer.end(ORBX_STAGE_SROWS, s);
  sp->timer.begin(ORBX_STAGE_SMATCH, s);
  // waves stride over the left keypoints: about 4 per wave once the batch
  // fills the chip (1 / 2 / 4 / 8 / 12 per wave: 0.399 / 0.391 / 0.386 /
  // 0.392 / 0.403 ms at c5), one per wave for small batches
  int sw = std::min(sp->waves, std::max((sp->waves + 3) / 4, (16384 + n - 1) / n));
  if (sp->sm_div > 0) sw = std::max(4, sp->waves / sp->sm_div);
  hipLaunchKernelGGL(k_stereo_match, dim3((sw + 3) / 4, n), dim3(256), 0, s, kl, dl, cl,
                     kr, dr, fl, fr, fstride, rstride, pyr_l, pyr_r, pstride, A, sp->d_rowoff,
                     sp->d_rows, ur, dep, sp->d_sad, sp->d_err);
  sp->timer.end(ORBX_STAGE_SMATCH, s);
  sp->timer.begin(ORBX_STAGE_SFILTER, s);
  hipLaunchKernelGGL(k_stereo_filter, dim3(n), dim3(256), 0, s, cl, A, ur, dep, sp->d_sad, nm);
  sp->timer.end(ORBX_STAGE_SFILTER, s);
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_ERR_HIP;
}

extern "C" int orbs_plan_match(orbs_plan* sp, int nframes, const orbx_plan* left,
                               const orbx_plan* right, const uint8_t* d_frames_l,
                               const uint8_t* d_frames_r, size_t frame_stride, size_t row_stride,
                               const orbx_keypoint* d_kps_l, const uint8_t* d_desc_l,
                               const int* d_count_l, const orbx_keypoint* d_kps_r,
                               const uint8_t* d_desc_r, const int* d_count_r, float mb, float mbf,
                               float* d_uright, float* d_depth, int* d_nmatches, void* stream) {
  if (!sp || nframes < 1 || nframes > sp->max_batch || !same_geometry(sp, left) ||
      !same_geometry(sp, right) || nframes > left->max_batch || nframes > right->max_batch ||
      !d_frames_l || !d_frames_r || !d_kps_l || !d_desc_l || !d_count_l || !d_kps_r ||
      !d_desc_r || !d_count_r || !d_uright || !d_depth || !d_nmatches)
    return ORBX_ERR_ARG;
  if (row_stride < (size_t)sp->W || frame_stride < row_stride * (size_t)sp->H) return ORBX_ERR_ARG;
  /* 24-bit row offsets, 32-bit offsets within a frame */
  if (row_stride >= ((size_t)1 << 24) || row_stride * (size_t)sp->H >= ((size_t)1 << 32))
    return ORBX_ERR_UNSUPPORTED;
  ORBX_TRY(hipSetDevice(sp->device));
  return splan_launch(sp, nframes, d_frames_l, d_frames_r, frame_stride, row_stride, left->d_pyr,
                      right->d_pyr, left->pyr_stride, d_kps_l, d_desc_l, d_count_l, d_kps_r,
                      d_desc_r, d_count_r, mb, mbf, d_uright, d_depth, d_nmatches,
                      (hipStream_t)stream);
}

extern "C" int orbs_plan_check(orbs_plan* sp, void* stream) {
  if (!sp) return ORBX_ERR_ARG;
  ORBX_TRY(hipSetDevice(sp->device));
  ORBX_TRY(hipStreamSynchronize((hipStream_t)stream));
  int err = 0;
  ORBX_TRY(hipMemcpy(&err, sp->d_err, sizeof(int), hipMemcpyDeviceToHost));
  if (err) {
    ORBX_TRY(hipMemset(sp->d_err, 0, sizeof(int)));
    return ORBX_ERR_ARG;
  }
  return ORBX_OK;
}

extern "C" int orbs_plan_set_timing(orbs_plan* sp, int enable) {
  if (!sp) return ORBX_ERR_ARG;
  hipSetDevice(sp->device);
  sp->timer.reset(enable != 0);
  return ORBX_OK;
}

extern "C" int orbs_plan_stage_times(orbs_plan* sp, double* ms, int* launches, int n) {
  if (!sp) return ORBX_ERR_ARG;
  hipSetDevice(sp->device);
  return sp->timer.collect(ms, launches, n);
}

// ---------------------------------------------------------------------------
// Frame::ComputeStereoMatches drop-in on the last orbx_extract of the left and
// right extractors (their mvImagePyramid stays on the device).
// ---------------------------------------------------------------------------
extern "C" int orbx_stereo_match(orbx_extractor* left, orbx_extractor* right,
                                 const orbx_keypoint* kps_l, const uint8_t* desc_l, int nl,
                                 const orbx_keypoint* kps_r, const uint8_t* desc_r, int nr,
                                 float mb, float mbf, float* uright, float* depth,
                                 int* nmatches) {
  if (!left || !right || !left->plan || !right->plan || !left->have_frame ||
      !right->have_frame || nl < 0 || nr < 0 || (nl > 0 && (!kps_l || !desc_l || !uright || !depth)) ||
      (nr > 0 && (!kps_r || !desc_r)))
    return ORBX_ERR_ARG;
  if (nmatches) *nmatches = 0;
  if (nl == 0) return ORBX_OK;
  orbs_plan* sp = reinterpret_cast<orbs_plan*>(left->stereo);
  if (sp && !same_geometry(sp, left->plan)) {
    splan_free(sp);
    left->stereo = sp = nullptr;
  }
  if (!same_geometry_pair(left->plan, right->plan)) return ORBX_ERR_ARG;
  if (!sp) {
    int rc = splan_create(left->plan, 1, &sp);
    if (rc) return rc;
    const size_t K = (size_t)std::max(left->plan->P.kcap, 1);
    if (hipMalloc((void**)&sp->d_kl, K * sizeof(orbx_keypoint)) != hipSuccess ||
        hipMalloc((void**)&sp->d_kr, K * sizeof(orbx_keypoint)) != hipSuccess ||
        hipMalloc((void**)&sp->d_dl, K * 32) != hipSuccess ||
        hipMalloc((void**)&sp->d_dr, K * 32) != hipSuccess ||
        hipMalloc((void**)&sp->d_cnt, 2 * sizeof(int)) != hipSuccess ||
        hipMalloc((void**)&sp->d_ur, K * sizeof(float)) != hipSuccess ||
        hipMalloc((void**)&sp->d_dep, K * sizeof(float)) != hipSuccess ||
        hipMalloc((void**)&sp->d_nm, sizeof(int)) != hipSuccess) {
      splan_free(sp);
      return ORBX_ERR_HIP;
    }
    left->stereo = sp;
  }
  if (nl > sp->args.kcap || nr > sp->args.kcap) return ORBX_ERR_CAPACITY;
  ORBX_TRY(hipSetDevice(sp->device));
  hipStream_t s = sp->stream;
  /* the extractors' kernels ran on their own streams and finished (orbx_extract is synchronous) */
  const int cnt[2] = {nl, nr};
  ORBX_TRY(hipMemcpyAsync(sp->d_kl, kps_l, nl * sizeof(orbx_keypoint), hipMemcpyHostToDevice, s));
  ORBX_TRY(hipMemcpyAsync(sp->d_dl, desc_l, (size_t)nl * 32, hipMemcpyHostToDevice, s));
  if (nr > 0) {
    ORBX_TRY(hipMemcpyAsync(sp->d_kr, kps_r, nr * sizeof(orbx_keypoint), hipMemcpyHostToDevice, s));
    ORBX_TRY(hipMemcpyAsync(sp->d_dr, desc_r, (size_t)nr * 32, hipMemcpyHostToDevice, s));
  }
  ORBX_TRY(hipMemcpyAsync(sp->d_cnt, cnt, sizeof(cnt), hipMemcpyHostToDevice, s));
  const size_t fs = (size_t)left->W * left->H;
  int rc = splan_launch(sp, 1, left->d_img, right->d_img, fs, (size_t)left->W, left->plan->d_pyr,
                        right->plan->d_pyr, left->plan->pyr_stride, sp->d_kl, sp->d_dl, sp->d_cnt,
                        sp->d_kr, sp->d_dr, sp->d_cnt + 1, mb, mbf, sp->d_ur, sp->d_dep, sp->d_nm,
                        s);
  if (rc) return rc;
  int nm = 0;
  ORBX_TRY(hipMemcpyAsync(uright, sp->d_ur, nl * sizeof(float), hipMemcpyDeviceToHost, s));
  ORBX_TRY(hipMemcpyAsync(depth, sp->d_dep, nl * sizeof(float), hipMemcpyDeviceToHost, s));
  ORBX_TRY(hipMemcpyAsync(&nm, sp->d_nm, sizeof(int), hipMemcpyDeviceToHost, s));
  rc = orbs_plan_check(sp, s);
  if (rc) return rc;
  if (nmatches) *nmatches = nm;
  return ORBX_OK;
}

void orbx_stereo_release(orbx_extractor* e) {
  if (e && e->stereo) {
    splan_free(reinterpret_cast<orbs_plan*>(e->stereo));
    e->stereo = nullptr;
  }
}
