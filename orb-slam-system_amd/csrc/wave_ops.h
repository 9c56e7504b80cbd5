// wave_ops.h -- wave64 reductions and scans on DPP / v_readlane (CDNA4).
// __shfl / __shfl_up compile to ds_bpermute: an LDS round trip per step.
// These use DPP row shifts and row broadcasts (gfx9 DPP: row_shr:n =
// 0x110 + n, row_bcast:15 = 0x142, row_bcast:31 = 0x143) and readlane, so a
// 64-lane scan is 6 VALU ops.  Callers keep all 64 lanes active (DPP reads
// inactive lanes' stale registers).
#ifndef ORBX_WAVE_OPS_H
#define ORBX_WAVE_OPS_H

#include <hip/hip_runtime.h>

namespace orbx {

// inclusive prefix sum over the 64 lanes
__device__ __forceinline__ int wave_incl_scan(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return x;
}

// sum over the 64 lanes, wave-uniform
__device__ __forceinline__ int wave_sum(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);
  return __builtin_amdgcn_readlane(x, 15) + __builtin_amdgcn_readlane(x, 31) +
         __builtin_amdgcn_readlane(x, 47) + __builtin_amdgcn_readlane(x, 63);
}

// minimum over the 64 lanes (unsigned), wave-uniform
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)x, 0x111, 0xf, 0xf, false));
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)x, 0x112, 0xf, 0xf, false));
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)x, 0x114, 0xf, 0xf, false));
  x = min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)0xFFFFFFFF, (int)x, 0x118, 0xf, 0xf, false));
  return min(min((uint32_t)__builtin_amdgcn_readlane((int)x, 15), (uint32_t)__builtin_amdgcn_readlane((int)x, 31)),
             min((uint32_t)__builtin_amdgcn_readlane((int)x, 47), (uint32_t)__builtin_amdgcn_readlane((int)x, 63)));
}

// set bits of a wave-wide mask below this lane (v_mbcnt_lo/hi, no and/bcnt)
__device__ __forceinline__ int lanes_below(unsigned long long m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// value of lane l (l wave-uniform)
__device__ __forceinline__ int lane_value(int x, int l) { return __builtin_amdgcn_readlane(x, l); }
__device__ __forceinline__ uint32_t lane_value(uint32_t x, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)x, l);
}

#ifndef ORBX_XCD_FRAMES
#define ORBX_XCD_FRAMES 1
#endif
// (unit, frame) of a workgroup of a grid (units, frames).  Workgroups are
// dispatched round-robin over the 8 XCDs in linear-id order, so with
// ORBX_XCD_FRAMES every unit of frame f runs on XCD f % 8, in unit order:
// strips / tiles / keypoint groups / row chunks that share 128-B lines, ring
// rows or a whole descriptor set of one frame meet in one L2 instead of being
// fetched from HBM by several XCDs (falls back to the plain grid when the
// frame count is not a multiple of 8).
__device__ __forceinline__ void frame_unit(int& unit, int& f) {
  if (ORBX_XCD_FRAMES && (gridDim.y & 7) == 0) {
    const int L = (int)(blockIdx.x + blockIdx.y * gridDim.x), k = L >> 3;
    const int q = k / (int)gridDim.x;
    unit = k - q * (int)gridDim.x;
    f = (L & 7) + 8 * q;
  } else {
    unit = (int)blockIdx.x;
    f = (int)blockIdx.y;
  }
}

}  // namespace orbx

#endif
