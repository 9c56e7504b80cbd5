// api_bow.hip -- C ABI of the DBoW2 vocabulary transform on the device:
// TemplatedVocabulary::loadFromTextFile / transform
// (/root/reference/Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:1126-1259,1338-1424).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/orbx.h"
#include "api_common.h"

namespace orbx {
struct BowRes {
  uint32_t word, nid;
  double w;
};
__global__ void k_bow_descend(const uint8_t*, const int*, int, const int*, const int*,
                              const uint8_t*, const uint32_t*, const double*, int, BowRes*);
__global__ void k_bow_assemble(const BowRes*, const int*, int, int, int, int, int, uint32_t*,
                               double*, int*, uint32_t*, uint32_t*, uint32_t*, int*, int*);
}  // namespace orbx

using namespace orbx;

#define ORBV_MAX_SORT 8192

struct orbv_vocab {
  int device = 0;
  int k = 0, L = 0, scoring = 0, weighting = 0, nnodes = 0, nwords = 0;
  int* d_cbeg = nullptr;
  int* d_cid = nullptr;
  uint8_t* d_cdesc = nullptr;
  uint32_t* d_word = nullptr;
  double* d_weight = nullptr;
  int* d_err = nullptr;
  BowRes* d_res = nullptr;
  size_t res_cap = 0;
  /* outgrown d_res buffers: launches on callers' streams may still read
   * them, so they are freed with the vocabulary, not on growth (no device
   * synchronisation on the transform path) */
  std::vector<void*> retired;
  /* host drop-in staging (one frame) */
  uint8_t* d_desc1 = nullptr;
  int* d_cnt1 = nullptr;
  uint32_t *d_bw = nullptr, *d_fn = nullptr, *d_fo = nullptr, *d_ff = nullptr;
  double* d_bv = nullptr;
  int* d_n2 = nullptr;
  int cap1 = 0;
  hipStream_t stream = nullptr;
};

static void vocab_free(orbv_vocab* v) {
  if (!v) return;
  hipSetDevice(v->device);
  void* bufs[] = {v->d_cbeg, v->d_cid, v->d_cdesc, v->d_word, v->d_weight, v->d_err, v->d_res,
                  v->d_desc1, v->d_cnt1, v->d_bw, v->d_fn, v->d_fo, v->d_ff, v->d_bv, v->d_n2};
  for (void* b : bufs)
    if (b) hipFree(b);
  for (void* b : v->retired) hipFree(b);
  if (v->stream) hipStreamDestroy(v->stream);
  delete v;
}

template <typename T>
static int upload_vec(T** dst, const std::vector<T>& h) {
  const size_t n = std::max<size_t>(h.size(), 1);
  if (hipMalloc((void**)dst, n * sizeof(T)) != hipSuccess) return ORBX_ERR_HIP;
  if (!h.empty() && hipMemcpy(*dst, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice) != hipSuccess)
    return ORBX_ERR_HIP;
  return ORBX_OK;
}

extern "C" int orbv_vocab_create(int k, int L, int scoring, int weighting, int nrec,
                                 const int32_t* parent, const int32_t* is_leaf,
                                 const uint8_t* desc, const double* weight, int device,
                                 orbv_vocab** out) {
  if (!out) return ORBX_ERR_ARG;
  *out = nullptr;
  /* header check of loadFromTextFile (:1356-1360) */
  if (k < 0 || k > 20 || L < 1 || L > 10 || scoring < 0 || scoring > 5 || weighting < 0 ||
      weighting > 3 || nrec < 0 || (nrec > 0 && (!parent || !is_leaf || !desc || !weight)))
    return ORBX_ERR_ARG;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return ORBX_ERR_NO_DEVICE;
  const int n = nrec + 1;
  /* m_nodes[pid].children.push_back(nid) in record order; children of a
   * node stored contiguously (CSR) with their descriptors next to each other */
  std::vector<int> cnt(n + 1, 0), cbeg(n + 1, 0), cid(std::max(nrec, 0)), fill(n, 0);
  std::vector<uint32_t> word(n, 0);
  std::vector<double> w(n, 0.0);
  int nwords = 0;
  for (int i = 1; i < n; ++i) {
    const int pid = parent[i - 1];
    if (pid < 0 || pid >= i) return ORBX_ERR_ARG; /* m_nodes[pid] must already exist */
    cnt[pid]++;
    w[i] = weight[i - 1];
    if (is_leaf[i - 1] > 0) word[i] = (uint32_t)nwords++;
  }
  for (int i = 0; i < n; ++i) cbeg[i + 1] = cbeg[i] + cnt[i];
  std::vector<uint8_t> cdesc((size_t)std::max(nrec, 1) * 32, 0);
  for (int i = 1; i < n; ++i) {
    const int pid = parent[i - 1];
    const int slot = cbeg[pid] + fill[pid]++;
    cid[slot] = i;
    memcpy(&cdesc[(size_t)slot * 32], desc + (size_t)(i - 1) * 32, 32);
  }
  for (int i = 0; i < n; ++i)
    if (cnt[i] > 65535) return ORBX_ERR_UNSUPPORTED;
  orbv_vocab* v = new orbv_vocab();
  v->device = device;
  v->k = k; v->L = L; v->scoring = scoring; v->weighting = weighting;
  v->nnodes = n;
  v->nwords = nwords;
  if (hipSetDevice(device) != hipSuccess || upload_vec(&v->d_cbeg, cbeg) ||
      upload_vec(&v->d_cid, cid) || upload_vec(&v->d_cdesc, cdesc) ||
      upload_vec(&v->d_word, word) || upload_vec(&v->d_weight, w) ||
      hipMalloc((void**)&v->d_err, 16) != hipSuccess || hipMemset(v->d_err, 0, 16) != hipSuccess ||
      hipStreamCreateWithFlags(&v->stream, hipStreamNonBlocking) != hipSuccess) {
    vocab_free(v);
    return ORBX_ERR_HIP;
  }
  if (hipFuncSetAttribute((const void*)k_bow_assemble, hipFuncAttributeMaxDynamicSharedMemorySize,
                          ORBV_MAX_SORT * 8) != hipSuccess) {
    vocab_free(v);
    return ORBX_ERR_HIP;
  }
  *out = v;
  return ORBX_OK;
}

/* loadFromTextFile (:1338-1424): header "k L scoring weighting", then one
 * node per line: "parent isLeaf d0 .. d31 weight".  A failed extraction
 * yields 0 as operator>> does since C++11.  The reference also turns the
 * empty line after a final newline into a phantom child of the root with an
 * uninitialised descriptor; that line is skipped here. */
extern "C" int orbv_vocab_load_text(const char* path, int device, orbv_vocab** out) {
  if (!path || !out) return ORBX_ERR_ARG;
  *out = nullptr;
  FILE* f = fopen(path, "rb");
  if (!f) return ORBX_ERR_ARG;
  std::string data;
  char buf[1 << 16];
  size_t r;
  while ((r = fread(buf, 1, sizeof(buf), f)) > 0) data.append(buf, r);
  fclose(f);
  size_t pos = 0;
  auto next_line = [&](std::string& line) -> bool {
    if (pos >= data.size()) return false;
    size_t e = data.find('\n', pos);
    if (e == std::string::npos) e = data.size();
    line.assign(data, pos, e - pos);
    pos = e + 1;
    return true;
  };
  std::string line;
  if (!next_line(line)) return ORBX_ERR_ARG;
  int hdr[4] = {0, 0, 0, 0};
  {
    const char* p = line.c_str();
    for (int i = 0; i < 4; ++i) {
      char* end;
      long x = strtol(p, &end, 10);
      if (end == p) break;
      hdr[i] = (int)x;
      p = end;
    }
  }
  std::vector<int32_t> parent, leaf;
  std::vector<uint8_t> desc;
  std::vector<double> weight;
  while (next_line(line)) {
    const char* p = line.c_str();
    while (*p == ' ' || *p == '\t' || *p == '\r') ++p;
    if (!*p) continue; /* blank line */
    bool ok = true;
    auto get_long = [&](long* x) {
      *x = 0;
      if (!ok) return;
      char* end;
      long t = strtol(p, &end, 10);
      if (end == p) { ok = false; return; }
      *x = t;
      p = end;
    };
    long pid, isl;
    get_long(&pid);
    get_long(&isl);
    uint8_t d[32];
    for (int i = 0; i < 32; ++i) {
      long t;
      get_long(&t);
      d[i] = (uint8_t)t; /* FORB::fromString: (unsigned char)n */
    }
    double wt = 0.0;
    if (ok) {
      char* end;
      double t = strtod(p, &end);
      if (end != p) wt = t;
    }
    parent.push_back((int32_t)pid);
    leaf.push_back((int32_t)isl);
    desc.insert(desc.end(), d, d + 32);
    weight.push_back(wt);
  }
  return orbv_vocab_create(hdr[0], hdr[1], hdr[2], hdr[3], (int)parent.size(), parent.data(),
                           leaf.data(), desc.data(), weight.data(), device, out);
}

extern "C" int orbv_vocab_destroy(orbv_vocab* v) {
  vocab_free(v);
  return ORBX_OK;
}

extern "C" int orbv_vocab_info(const orbv_vocab* v, int* k, int* L, int* scoring,
                               int* weighting, int* nnodes, int* nwords) {
  if (!v) return ORBX_ERR_ARG;
  if (k) *k = v->k;
  if (L) *L = v->L;
  if (scoring) *scoring = v->scoring;
  if (weighting) *weighting = v->weighting;
  if (nnodes) *nnodes = v->nnodes;
  if (nwords) *nwords = v->nwords;
  return ORBX_OK;
}

static int next_pow2(int x) {
  int p = 1;
  while (p < x) p <<= 1;
  return p;
}

extern "C" int orbv_transform_batch(orbv_vocab* v, int nframes, const uint8_t* d_desc,
                                    const int* d_counts, int kcap, int levelsup,
                                    uint32_t* d_bow_word, double* d_bow_value, int* d_nbow,
                                    uint32_t* d_fv_node, uint32_t* d_fv_off, uint32_t* d_fv_feat,
                                    int* d_nfv, void* stream) {
  if (!v || nframes < 1 || kcap < 1 || !d_desc || !d_counts || !d_bow_word || !d_bow_value ||
      !d_nbow || !d_fv_node || !d_fv_off || !d_fv_feat || !d_nfv)
    return ORBX_ERR_ARG;
  const int P = next_pow2(kcap);
  if (P > ORBV_MAX_SORT) return ORBX_ERR_UNSUPPORTED;
  ORBX_TRY(hipSetDevice(v->device));
  hipStream_t s = (hipStream_t)stream;
  const size_t need = (size_t)nframes * kcap;
  if (need > v->res_cap) {
    /* geometric growth: the retired buffers (which launches on other
     * streams may still read) stay below twice the current one */
    const size_t cap = std::max(need, v->res_cap + v->res_cap / 2);
    if (v->d_res) v->retired.push_back(v->d_res);
    v->d_res = nullptr;
    v->res_cap = 0;
    ORBX_TRY(hipMalloc((void**)&v->d_res, cap * sizeof(BowRes)));
    v->res_cap = cap;
  }
  if (v->nwords == 0) { /* if(empty()) return;  (:1133): empty vectors */
    ORBX_TRY(hipMemsetAsync(d_nbow, 0, nframes * sizeof(int), s));
    ORBX_TRY(hipMemsetAsync(d_nfv, 0, nframes * sizeof(int), s));
    ORBX_TRY(hipMemsetAsync(d_fv_off, 0, (size_t)nframes * (kcap + 1) * sizeof(uint32_t), s));
    return ORBX_OK;
  }
  const int nid_level = v->L - levelsup;
  const int tf = v->weighting == 0 || v->weighting == 1; /* TF_IDF || TF */
  const int must = v->scoring != 5;                      /* all but DotProductScoring */
  const int l2 = v->scoring == 1;                        /* L2Scoring */
  hipLaunchKernelGGL(k_bow_descend, dim3((kcap + 15) / 16, nframes), dim3(256), 0, s, d_desc,
                     d_counts, kcap, v->d_cbeg, v->d_cid, v->d_cdesc, v->d_word, v->d_weight,
                     nid_level, v->d_res);
  hipLaunchKernelGGL(k_bow_assemble, dim3(nframes), dim3(1024), (size_t)P * 8, s, v->d_res,
                     d_counts, kcap, P, tf, must, l2, d_bow_word, d_bow_value, d_nbow, d_fv_node,
                     d_fv_off, d_fv_feat, d_nfv, v->d_err);
  return hipGetLastError() == hipSuccess ? ORBX_OK : ORBX_ERR_HIP;
}

extern "C" int orbv_check(orbv_vocab* v, void* stream) {
  if (!v) return ORBX_ERR_ARG;
  ORBX_TRY(hipSetDevice(v->device));
  ORBX_TRY(hipStreamSynchronize((hipStream_t)stream));
  int err = 0;
  ORBX_TRY(hipMemcpy(&err, v->d_err, sizeof(int), hipMemcpyDeviceToHost));
  if (err) {
    ORBX_TRY(hipMemset(v->d_err, 0, sizeof(int)));
    return ORBX_ERR_ARG; /* the reference would read an unset NodeId */
  }
  return ORBX_OK;
}

extern "C" int orbv_transform(orbv_vocab* v, const uint8_t* desc, int n, int levelsup,
                              uint32_t* bow_word, double* bow_value, int* nbow,
                              uint32_t* fv_node, uint32_t* fv_off, uint32_t* fv_feat, int* nfv) {
  if (!v || n < 0 || (n > 0 && !desc) || !nbow || !nfv || !fv_off) return ORBX_ERR_ARG;
  *nbow = 0;
  *nfv = 0;
  fv_off[0] = 0;
  if (n == 0) return ORBX_OK;
  if (!bow_word || !bow_value || !fv_node || !fv_feat) return ORBX_ERR_ARG;
  if (next_pow2(n) > ORBV_MAX_SORT) return ORBX_ERR_UNSUPPORTED;
  ORBX_TRY(hipSetDevice(v->device));
  if (n > v->cap1) {
    void* bufs[] = {v->d_desc1, v->d_cnt1, v->d_bw, v->d_fn, v->d_fo, v->d_ff, v->d_bv, v->d_n2};
    for (void* b : bufs)
      if (b) hipFree(b);
    v->d_desc1 = nullptr; v->d_cnt1 = nullptr; v->d_bw = nullptr; v->d_fn = nullptr;
    v->d_fo = nullptr; v->d_ff = nullptr; v->d_bv = nullptr; v->d_n2 = nullptr;
    v->cap1 = 0;
    const size_t c = (size_t)next_pow2(n);
    if (hipMalloc((void**)&v->d_desc1, c * 32) != hipSuccess ||
        hipMalloc((void**)&v->d_cnt1, sizeof(int)) != hipSuccess ||
        hipMalloc((void**)&v->d_bw, c * 4) != hipSuccess ||
        hipMalloc((void**)&v->d_fn, c * 4) != hipSuccess ||
        hipMalloc((void**)&v->d_fo, (c + 1) * 4) != hipSuccess ||
        hipMalloc((void**)&v->d_ff, c * 4) != hipSuccess ||
        hipMalloc((void**)&v->d_bv, c * 8) != hipSuccess ||
        hipMalloc((void**)&v->d_n2, 2 * sizeof(int)) != hipSuccess)
      return ORBX_ERR_HIP;
    v->cap1 = (int)c;
  }
  hipStream_t s = v->stream;
  ORBX_TRY(hipMemcpyAsync(v->d_desc1, desc, (size_t)n * 32, hipMemcpyHostToDevice, s));
  ORBX_TRY(hipMemcpyAsync(v->d_cnt1, &n, sizeof(int), hipMemcpyHostToDevice, s));
  int rc = orbv_transform_batch(v, 1, v->d_desc1, v->d_cnt1, n, levelsup, v->d_bw, v->d_bv,
                                v->d_n2, v->d_fn, v->d_fo, v->d_ff, v->d_n2 + 1, s);
  if (rc) return rc;
  int cnts[2] = {0, 0};
  ORBX_TRY(hipMemcpyAsync(cnts, v->d_n2, sizeof(cnts), hipMemcpyDeviceToHost, s));
  ORBX_TRY(hipStreamSynchronize(s));
  rc = orbv_check(v, s);
  if (rc) return rc;
  *nbow = cnts[0];
  *nfv = cnts[1];
  ORBX_TRY(hipMemcpyAsync(bow_word, v->d_bw, (size_t)cnts[0] * 4, hipMemcpyDeviceToHost, s));
  ORBX_TRY(hipMemcpyAsync(bow_value, v->d_bv, (size_t)cnts[0] * 8, hipMemcpyDeviceToHost, s));
  ORBX_TRY(hipMemcpyAsync(fv_node, v->d_fn, (size_t)cnts[1] * 4, hipMemcpyDeviceToHost, s));
  ORBX_TRY(hipMemcpyAsync(fv_off, v->d_fo, (size_t)(cnts[1] + 1) * 4, hipMemcpyDeviceToHost, s));
  int nfeat = 0;
  ORBX_TRY(hipMemcpyAsync(&nfeat, v->d_fo + cnts[1], 4, hipMemcpyDeviceToHost, s));
  ORBX_TRY(hipStreamSynchronize(s));
  ORBX_TRY(hipMemcpyAsync(fv_feat, v->d_ff, (size_t)nfeat * 4, hipMemcpyDeviceToHost, s));
  ORBX_TRY(hipStreamSynchronize(s));
  return ORBX_OK;
}
