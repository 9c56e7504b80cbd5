// kernels_bow.hip -- gfx950 kernels of the DBoW2 vocabulary transform
// (/root/reference/Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1126-1259),
// the producer of the FeatureVectors SearchByBoW consumes
// (Frame::ComputeBoW, /root/reference/src/Frame.cc:375-382).
//
//   transform(feature, word, weight, nid, levelsup) (:1222-1259) -> k_bow_descend
//     16 lanes per descriptor: lane j scores child j (j, j+16, ...) of the
//     current node (children stored contiguously per parent), a 16-lane
//     min over (distance, child index) is the reference's first strict '<'
//     minimum, and the group steps down one level per iteration.
//   BowVector / FeatureVector assembly (:1126-1191, BowVector.cpp,
//   FeatureVector.cpp) -> k_bow_assemble: one workgroup per frame, LDS bitonic
//   sort of (node, feature) and (word, feature) keys (std::map order,
//   push order inside a key), in-order double sums per word and the
//   sequential L1/L2 norm of BowVector::normalize.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "wave_ops.h"

namespace orbx {

struct BowRes {
  uint32_t word, nid;
  double w;
};

#define BOW_NID_UNSET 0xFFFFFFFFu
#define BOW_DEVERR_NID 8

__global__ __launch_bounds__(256) void k_bow_descend(
    const uint8_t* __restrict__ desc, const int* __restrict__ counts, int kcap,
    const int* __restrict__ cbeg, const int* __restrict__ cid, const uint8_t* __restrict__ cdesc,
    const uint32_t* __restrict__ word, const double* __restrict__ weight, int nid_level,
    BowRes* __restrict__ out) {
  const int g = threadIdx.x & 15;                   // lane in the 16-lane group
  const int f = blockIdx.y;
  const int i = blockIdx.x * 16 + (threadIdx.x >> 4);  // descriptor
  const int n = counts[f];
  if (i >= n) return;  // whole groups leave together
  const uint4* fp = reinterpret_cast<const uint4*>(desc + ((size_t)f * kcap + i) * 32);
  const uint4 a0 = fp[0], a1 = fp[1];
  uint32_t node = 0, nid = nid_level <= 0 ? 0u : BOW_NID_UNSET;
  int level = 0;
  while (true) {
    const int b = cbeg[node], e = cbeg[node + 1];
    if (b == e) break;  // isLeaf(): children.empty()
    ++level;
    uint32_t key = 0xFFFFFFFFu;
    for (int j = b + g; j < e; j += 16) {
      const uint4* cp = reinterpret_cast<const uint4*>(cdesc + (size_t)j * 32);
      const uint4 b0 = cp[0], b1 = cp[1];
      const uint32_t d = __popc(a0.x ^ b0.x) + __popc(a0.y ^ b0.y) + __popc(a0.z ^ b0.z) +
                         __popc(a0.w ^ b0.w) + __popc(a1.x ^ b1.x) + __popc(a1.y ^ b1.y) +
                         __popc(a1.z ^ b1.z) + __popc(a1.w ^ b1.w);
      key = min(key, (d << 16) | (uint32_t)(j - b));
    }
#pragma unroll
    for (int s = 8; s >= 1; s >>= 1) key = min(key, (uint32_t)__shfl_xor((int)key, s, 16));
    node = (uint32_t)cid[b + (int)(key & 0xFFFFu)];
    if (level == nid_level) nid = node;
  }
  if (g == 0) {
    BowRes r;
    r.word = word[node];
    r.nid = nid;
    r.w = weight[node];
    out[(size_t)f * kcap + i] = r;
  }
}

#define BA_THREADS 1024

__device__ void bitonic_sort_u64(unsigned long long* k, int P) {
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < (P >> 1); t += BA_THREADS) {
        const int lo = 2 * t - (t & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const unsigned long long x = k[lo], y = k[hi];
        if ((x > y) == up) {
          k[lo] = y;
          k[hi] = x;
        }
      }
      __syncthreads();
    }
  }
}

// one workgroup per frame; n <= P <= 8192 (host-checked)
__global__ __launch_bounds__(BA_THREADS) void k_bow_assemble(
    const BowRes* __restrict__ res, const int* __restrict__ counts, int kcap, int P, int tf,
    int must, int l2, uint32_t* __restrict__ bow_word, double* __restrict__ bow_value,
    int* __restrict__ nbow, uint32_t* __restrict__ fv_node, uint32_t* __restrict__ fv_off,
    uint32_t* __restrict__ fv_feat, int* __restrict__ nfv, int* __restrict__ err) {
  extern __shared__ unsigned long long keys[];  // P
  __shared__ int s_cnt[2];
  __shared__ double s_norm;
  const int f = blockIdx.x, tid = threadIdx.x;
  const int n = counts[f];
  const BowRes* R = res + (size_t)f * kcap;
  uint32_t* BW = bow_word + (size_t)f * kcap;
  double* BV = bow_value + (size_t)f * kcap;
  uint32_t* FN = fv_node + (size_t)f * kcap;
  uint32_t* FO = fv_off + (size_t)f * (kcap + 1);
  uint32_t* FF = fv_feat + (size_t)f * kcap;
  const unsigned long long NONE = ~0ull;
  // ---- FeatureVector: sort (nid, i) of the non-stopped features ----
  bool bad = false;
  for (int i = tid; i < P; i += BA_THREADS) {
    unsigned long long key = NONE;
    if (i < n) {
      const BowRes r = R[i];
      if (r.w > 0) {
        if (r.nid == BOW_NID_UNSET) bad = true;  // the reference reads an unset NodeId
        key = ((unsigned long long)r.nid << 32) | (unsigned)i;
      }
    }
    keys[i] = key;
  }
  if (bad) atomicOr(err, BOW_DEVERR_NID);
  if (tid < 2) s_cnt[tid] = 0;
  __syncthreads();
  bitonic_sort_u64(keys, P);
  // heads of runs -> node index by a block-wide count (ordered: ranks by scan)
  // simple two-pass: count valid entries and heads, then each head finds its
  // rank by counting heads before it with a per-thread chunk scan
  const int chunk = (P + BA_THREADS - 1) / BA_THREADS;
  const int c0 = min(P, tid * chunk), c1 = min(P, c0 + chunk);
  int heads = 0, valid = 0;
  for (int i = c0; i < c1; ++i) {
    const unsigned long long k = keys[i];
    if (k == NONE) continue;
    ++valid;
    if (i == 0 || (keys[i - 1] >> 32) != (k >> 32)) ++heads;
  }
  // block exclusive scan of heads (and total valid)
  __shared__ int s_scan[BA_THREADS / 64 + 1];
  {
    const int lane = tid & 63, wave = tid >> 6;
    const int incl = orbx::wave_incl_scan(heads);
    if (lane == 63) s_scan[wave] = incl;
    atomicAdd(&s_cnt[0], valid);
    __syncthreads();
    if (tid == 0) {
      int run = 0;
      for (int w = 0; w < BA_THREADS / 64; ++w) {
        const int t = s_scan[w];
        s_scan[w] = run;
        run += t;
      }
      s_scan[BA_THREADS / 64] = run;
    }
    __syncthreads();
    int q = s_scan[wave] + incl - heads;
    for (int i = c0; i < c1; ++i) {
      const unsigned long long k = keys[i];
      if (k == NONE) continue;
      if (i == 0 || (keys[i - 1] >> 32) != (k >> 32)) {
        FN[q] = (uint32_t)(k >> 32);
        FO[q] = (uint32_t)i;
        ++q;
      }
      FF[i] = (uint32_t)(k & 0xFFFFFFFFu);
    }
  }
  const int nf = s_cnt[0], nq = s_scan[BA_THREADS / 64];
  if (tid == 0) {
    FO[nq] = (uint32_t)nf;
    nfv[f] = nq;
  }
  __syncthreads();
  // ---- BowVector: sort (word, i) ----
  for (int i = tid; i < P; i += BA_THREADS) {
    unsigned long long key = NONE;
    if (i < n) {
      const BowRes r = R[i];
      if (r.w > 0) key = ((unsigned long long)r.word << 32) | (unsigned)i;
    }
    keys[i] = key;
  }
  __syncthreads();
  bitonic_sort_u64(keys, P);
  heads = 0;
  for (int i = c0; i < c1; ++i) {
    const unsigned long long k = keys[i];
    if (k != NONE && (i == 0 || (keys[i - 1] >> 32) != (k >> 32))) ++heads;
  }
  int q0;
  {
    const int lane = tid & 63, wave = tid >> 6;
    const int incl = orbx::wave_incl_scan(heads);
    __syncthreads();
    if (lane == 63) s_scan[wave] = incl;
    __syncthreads();
    if (tid == 0) {
      int run = 0;
      for (int w = 0; w < BA_THREADS / 64; ++w) {
        const int t = s_scan[w];
        s_scan[w] = run;
        run += t;
      }
      s_scan[BA_THREADS / 64] = run;
    }
    __syncthreads();
    q0 = s_scan[wave] + incl - heads;
  }
  const int m = s_scan[BA_THREADS / 64];
  // per word: addWeight's in-order += (TF, TF_IDF) or the first value
  // (addIfNotExist: IDF, BINARY)
  {
    int q = q0;
    for (int i = c0; i < c1; ++i) {
      const unsigned long long k = keys[i];
      if (k == NONE || !(i == 0 || (keys[i - 1] >> 32) != (k >> 32))) continue;
      double s = R[(uint32_t)(k & 0xFFFFFFFFu)].w;
      if (tf)
        for (int e = i + 1; e < nf && (keys[e] >> 32) == (k >> 32); ++e)
          s += R[(uint32_t)(keys[e] & 0xFFFFFFFFu)].w;
      BW[q] = (uint32_t)(k >> 32);
      BV[q] = s;
      ++q;
    }
  }
  __syncthreads();
  if (tf && m > 0 && !must) {  // :1164-1170
    const double nd = (double)m;
    for (int q = tid; q < m; q += BA_THREADS) BV[q] /= nd;
  }
  if (must) {  // BowVector::normalize: sequential sum in ascending word order
    double* vals = reinterpret_cast<double*>(keys);
    for (int q = tid; q < m; q += BA_THREADS) vals[q] = BV[q];
    __syncthreads();
    if (tid == 0) {
      double norm = 0.0;
      if (!l2) {
        for (int q = 0; q < m; ++q) norm += fabs(vals[q]);
      } else {
        for (int q = 0; q < m; ++q) norm = fma(vals[q], vals[q], norm);  // -march=native FMA
        norm = sqrt(norm);
      }
      s_norm = norm;
    }
    __syncthreads();
    const double norm = s_norm;
    if (norm > 0.0)
      for (int q = tid; q < m; q += BA_THREADS) BV[q] = vals[q] / norm;
  }
  if (tid == 0) nbow[f] = m;
}

}  // namespace orbx
