"""orbx -- Python host binding of liborbx.so (the MI355X ORB front end).

Thin ctypes layer over the C ABI in include/orbx.h.  It mirrors the
reference interfaces for tests and the benchmark:

  Extractor      ORB_SLAM2::ORBextractor  (/root/reference/include/ORBextractor.h:25-91)
  search_by_bow  ORBmatcher::SearchByBoW(KF, KF) (/root/reference/src/ORBmatcher.cc:278-366)
  compute_stereo_matches  Frame::ComputeStereoMatches (/root/reference/src/Frame.cc:446-620)
  descriptor_distance_batch  ORBmatcher::DescriptorDistance (ORBmatcher.cc:896-908)
  Plan / MatchPlan  batched device-resident throughput path (bench.py)

The library is mandatory: importing this package raises if liborbx.so is
missing, and every compute call runs the HIP kernels (there is no CPU path).
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(HERE), "liborbx.so")
if os.environ.get("ORBX_VARIANT"):  # profiling only: tools/variant.sh builds liborbx_<name>.so
    LIB_PATH = os.path.join(os.path.dirname(HERE), "liborbx_%s.so" % os.environ["ORBX_VARIANT"])

if not os.path.exists(LIB_PATH):
    raise ImportError("liborbx.so not built (%s): run __graft_entry__.build() or "
                      "make -C orb-slam-system_amd" % LIB_PATH)

try:
    # Load torch (and its bundled libamdhip64.so.7) first: liborbx.so then binds to the
    # same HIP runtime by SONAME, so one process never holds two HIP runtimes.
    import torch as _torch  # noqa: F401
except ImportError:  # pragma: no cover - torch is plumbing only
    _torch = None

_lib = ctypes.CDLL(LIB_PATH)

KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
assert KEYPOINT_DTYPE.itemsize == 28

OK, ERR_ARG, ERR_CELL_ROI, ERR_LEVEL_SIZE, ERR_QUADTREE, ERR_CAPACITY, ERR_UNSUPPORTED, \
    ERR_HIP, ERR_NO_DEVICE = 0, -1, -2, -3, -4, -5, -6, -7, -8
ORBM_PLAN_ZERO_TAIL, ORBM_PLAN_VALU = 1, 2  # orbm_plan_set_options flags (include/orbx.h)
ORBX_PLAN_PYR_TILES, ORBX_PLAN_BRIEF_PATCH, ORBX_PLAN_BRIEF_LEVEL = 1, 8, 16  # orbx_plan_set_options flags

EXPORTED = [
    "orbx_abi_version", "orbx_status_string", "orbx_device_count", "orbx_tables",
    "orbx_geometry_compute", "orbx_resize_tables", "orbx_extractor_create",
    "orbx_extractor_destroy", "orbx_extractor_capacity", "orbx_extract", "orbx_extractor_level",
    "orbx_extractor_set_options", "orbx_extractor_level_host", "orbx_extractor_stats",
    "orbx_boundary_record_bytes", "orbx_boundary_pack", "orbx_boundary_unpack",
    "orbx_plan_create", "orbx_plan_destroy", "orbx_plan_geometry", "orbx_plan_extract",
    "orbx_plan_check", "orbx_plan_debug_counters", "orbx_debug_set_fast_ccap", "orbx_plan_set_options", "orbx_plan_level", "orbx_stage_count", "orbx_stage_name", "orbx_plan_set_timing",
    "orbx_plan_stage_times", "orbx_synth_frames", "orbm_search_by_bow", "orbm_search_by_bow_kf_frame",
    "orbm_descriptor_distance_batch", "orbm_plan_create", "orbm_plan_destroy",
    "orbm_plan_match_frames", "orbm_plan_set_timing", "orbm_plan_stage_times", "orbm_plan_set_options",
    "orbx_stereo_match", "orbs_plan_create", "orbs_plan_destroy", "orbs_plan_match",
    "orbs_plan_check", "orbs_plan_set_timing", "orbs_plan_stage_times",
    "orbv_vocab_load_text", "orbv_vocab_create", "orbv_vocab_destroy", "orbv_vocab_info",
    "orbv_transform", "orbv_transform_batch", "orbv_check", "orbm_search_by_projection",
    "orbm_proj_plan_create", "orbm_proj_plan_destroy", "orbm_proj_plan_search",
    "orbm_compute_distinctive_descriptors", "orbx_undistort_keypoints", "orbx_selftest_sincos",
    "orbx_selftest_sincos_range",
]


class Params(ctypes.Structure):
    _fields_ = [("nfeatures", ctypes.c_int), ("scale_factor", ctypes.c_float),
                ("nlevels", ctypes.c_int), ("ini_th_fast", ctypes.c_int),
                ("min_th_fast", ctypes.c_int), ("cell_guard", ctypes.c_int)]


def params(nfeatures, scale_factor, nlevels, ini_th, min_th, cell_guard="strict"):
    return Params(nfeatures, scale_factor, nlevels, ini_th, min_th,
                  1 if cell_guard in ("empty", 1, True) else 0)


class Geometry(ctypes.Structure):
    _fields_ = [("nlevels", ctypes.c_int)] + [
        (n, ctypes.c_int * 32) for n in ("width", "height", "alias", "ncols", "nrows", "wcell",
                                         "hcell", "ncells_bad", "features", "nini", "kcap_level")
    ] + [("kcap", ctypes.c_int), ("pixels", ctypes.c_longlong), ("bytes_pyr_fast", ctypes.c_longlong)]

    def level(self, name):
        return list(getattr(self, name))[:self.nlevels]


class ProjQuery(ctypes.Structure):
    _fields_ = [("x", ctypes.c_float), ("y", ctypes.c_float), ("radius", ctypes.c_float),
                ("min_level", ctypes.c_int32), ("max_level", ctypes.c_int32),
                ("xr", ctypes.c_float), ("angle", ctypes.c_float)]


PROJ_QUERY_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("radius", "<f4"), ("min_level", "<i4"),
                             ("max_level", "<i4"), ("xr", "<f4"), ("angle", "<f4")])


class ProjFrame(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("keys", ctypes.c_void_p), ("desc", ctypes.c_void_p),
                ("uright", ctypes.c_void_p), ("occupied", ctypes.c_void_p),
                ("min_x", ctypes.c_float), ("min_y", ctypes.c_float),
                ("grid_w_inv", ctypes.c_float), ("grid_h_inv", ctypes.c_float)]


class ProjProblem(ctypes.Structure):
    _fields_ = [("frame", ProjFrame), ("q", ctypes.c_void_p), ("qdesc", ctypes.c_void_p),
                ("nq", ctypes.c_int), ("match", ctypes.c_void_p), ("nmatches", ctypes.c_void_p)]


class BowFrame(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int), ("desc", ctypes.c_void_p), ("angle", ctypes.c_void_p),
                ("valid", ctypes.c_void_p), ("nnodes", ctypes.c_int), ("node_id", ctypes.c_void_p),
                ("node_off", ctypes.c_void_p), ("feat", ctypes.c_void_p)]


P, I, F, SZ = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
_sig = {
    "orbx_abi_version": (I, []),
    "orbx_status_string": (ctypes.c_char_p, [I]),
    "orbx_device_count": (I, []),
    "orbx_tables": (I, [P, P, P, P, P, P, P]),
    "orbx_geometry_compute": (I, [P, I, I, P]),
    "orbx_resize_tables": (I, [P, I, I, I, P, P, P, P]),
    "orbx_extractor_create": (I, [P, I, P]),
    "orbx_extractor_destroy": (I, [P]),
    "orbx_extractor_capacity": (I, [P, I, I, P]),
    "orbx_extract": (I, [P, P, I, I, SZ, P, I, P, P]),
    "orbx_extractor_level": (I, [P, I, P, SZ, P, P]),
    "orbx_extractor_set_options": (I, [P, I]),
    "orbx_extractor_level_host": (I, [P, I, P, P, P, P]),
    "orbx_extractor_stats": (I, [P, P, P]),
    "orbx_boundary_record_bytes": (SZ, [I]),
    "orbx_boundary_pack": (I, [P, P, P, I, P, P]),
    "orbx_boundary_unpack": (I, [P, I, P, P, P, P]),
    "orbx_plan_create": (I, [P, I, I, I, I, P]),
    "orbx_plan_destroy": (I, [P]),
    "orbx_plan_geometry": (I, [P, P]),
    "orbx_plan_extract": (I, [P, P, I, SZ, SZ, P, P, P, P]),
    "orbx_plan_check": (I, [P, P]),
    "orbx_plan_debug_counters": (I, [P, P]),
    "orbx_debug_set_fast_ccap": (I, [I]),
    "orbx_plan_set_options": (I, [P, I]),
    "orbx_plan_level": (I, [P, I, I, P, SZ, P, P, P]),
    "orbx_stage_count": (I, []),
    "orbx_stage_name": (ctypes.c_char_p, [I]),
    "orbx_plan_set_timing": (I, [P, I]),
    "orbx_plan_stage_times": (I, [P, P, P, I]),
    "orbx_synth_frames": (I, [P, I, I, SZ, I, I, I, P]),
    "orbm_search_by_bow": (I, [P, P, F, I, I, P, P]),
    "orbm_search_by_bow_kf_frame": (I, [P, P, F, I, I, P, P]),
    "orbm_descriptor_distance_batch": (I, [P, I, P, I, P, P, I, I, P]),
    "orbm_plan_create": (I, [I, I, I, I, P]),
    "orbm_plan_destroy": (I, [P]),
    "orbm_plan_match_frames": (I, [P, I, P, P, P, P, P, P, F, I, P, P, P]),
    "orbm_plan_set_timing": (I, [P, I]),
    "orbm_plan_set_options": (I, [P, I]),
    "orbm_plan_stage_times": (I, [P, P, P, I]),
    "orbx_stereo_match": (I, [P, P, P, P, I, P, P, I, F, F, P, P, P]),
    "orbs_plan_create": (I, [P, I, P]),
    "orbs_plan_destroy": (I, [P]),
    "orbs_plan_match": (I, [P, I, P, P, P, P, SZ, SZ, P, P, P, P, P, P, F, F, P, P, P, P]),
    "orbs_plan_check": (I, [P, P]),
    "orbs_plan_set_timing": (I, [P, I]),
    "orbs_plan_stage_times": (I, [P, P, P, I]),
    "orbv_vocab_load_text": (I, [ctypes.c_char_p, I, P]),
    "orbv_vocab_create": (I, [I, I, I, I, I, P, P, P, P, I, P]),
    "orbv_vocab_destroy": (I, [P]),
    "orbv_vocab_info": (I, [P, P, P, P, P, P, P]),
    "orbv_transform": (I, [P, P, I, I, P, P, P, P, P, P, P]),
    "orbv_transform_batch": (I, [P, I, P, P, I, I, P, P, P, P, P, P, P, P]),
    "orbv_check": (I, [P, P]),
    "orbm_search_by_projection": (I, [I, P, P, P, I, F, I, I, I, P, P]),
    "orbm_proj_plan_create": (I, [I, I, I, I, P]),
    "orbm_proj_plan_destroy": (I, [P]),
    "orbm_proj_plan_search": (I, [P, I, I, P, F, I, I, P]),
    "orbm_compute_distinctive_descriptors": (I, [P, P, I, I, P]),
    "orbx_undistort_keypoints": (I, [P, I, P, P, I, I, P]),
    "orbx_selftest_sincos": (I, [P, I, P, P]),
    "orbx_selftest_sincos_range": (I, [ctypes.c_uint32, I, P, I]),
}
for _n, (_r, _a) in _sig.items():
    _f = getattr(_lib, _n)
    _f.restype = _r
    _f.argtypes = _a


def lib():
    return _lib


class OrbxError(RuntimeError):
    def __init__(self, code, what=""):
        msg = _lib.orbx_status_string(code).decode()
        super().__init__("%s: %s (%d)" % (what, msg, code) if what else "%s (%d)" % (msg, code))
        self.code = code


def _check(rc, what=""):
    if rc != OK:
        raise OrbxError(rc, what)
    return rc


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def device_count():
    return _lib.orbx_device_count()


def stage_names():
    return [_lib.orbx_stage_name(i).decode() for i in range(_lib.orbx_stage_count())]


# --------------------------------------------------------------------------- host-only tables
def tables(prm):
    L = prm.nlevels
    s, inv, s2, inv2 = (np.zeros(L, np.float32) for _ in range(4))
    fpl = np.zeros(L, np.int32)
    umax = np.zeros(16, np.int32)
    _check(_lib.orbx_tables(ctypes.byref(prm), _p(s), _p(inv), _p(s2), _p(inv2), _p(fpl), _p(umax)))
    return dict(scale=s, inv_scale=inv, sigma2=s2, inv_sigma2=inv2, features_per_level=fpl,
                umax=umax)


def geometry(prm, width, height):
    g = Geometry()
    _check(_lib.orbx_geometry_compute(ctypes.byref(prm), width, height, ctypes.byref(g)), "geometry")
    return g


def resize_tables(prm, width, height, level):
    g = geometry(prm, width, height)
    w, h = g.width[level], g.height[level]
    xofs = np.zeros(w, np.int32)
    alpha = np.zeros(2 * w, np.int16)
    yofs = np.zeros(h, np.int32)
    beta = np.zeros(2 * h, np.int16)
    _check(_lib.orbx_resize_tables(ctypes.byref(prm), width, height, level, _p(xofs), _p(alpha),
                                   _p(yofs), _p(beta)))
    return xofs, alpha.reshape(w, 2), yofs, beta.reshape(h, 2)


# --------------------------------------------------------------------------- ORBextractor
class Extractor:
    """ORB_SLAM2::ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)."""

    def __init__(self, nfeatures, scale_factor, nlevels, ini_th, min_th, cell_guard="strict",
                 device=0):
        self.params = params(nfeatures, scale_factor, nlevels, ini_th, min_th, cell_guard)
        self._t = tables(self.params)
        h = ctypes.c_void_p()
        _check(_lib.orbx_extractor_create(ctypes.byref(self.params), device, ctypes.byref(h)),
               "orbx_extractor_create")
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            _lib.orbx_extractor_destroy(self._h)
            self._h = None

    # getters (ORBextractor.h:43-63)
    def GetLevels(self):
        return self.params.nlevels

    def GetScaleFactor(self):
        return self.params.scale_factor

    def GetScaleFactors(self):
        return self._t["scale"].tolist()

    def GetInverseScaleFactors(self):
        return self._t["inv_scale"].tolist()

    def GetScaleSigmaSquares(self):
        return self._t["sigma2"].tolist()

    def GetInverseScaleSigmaSquares(self):
        return self._t["inv_sigma2"].tolist()

    def __call__(self, image, mask=None):
        """operator()(image, mask, keypoints, descriptors) -> (keypoints, descriptors)."""
        return self.extract(image)

    def extract(self, image):
        img = np.ascontiguousarray(image, dtype=np.uint8)
        if img.ndim != 2:
            raise OrbxError(ERR_ARG, "CV_8UC1 image expected")
        h, w = img.shape
        cap = ctypes.c_int(0)
        _check(_lib.orbx_extractor_capacity(self._h, w, h, ctypes.byref(cap)), "capacity")
        kps = np.zeros(max(cap.value, 1), KEYPOINT_DTYPE)
        desc = np.zeros((max(cap.value, 1), 32), np.uint8)
        n = ctypes.c_int(0)
        _check(_lib.orbx_extract(self._h, _p(img), w, h, w, _p(kps), cap.value, _p(desc),
                                 ctypes.byref(n)), "orbx_extract")
        return kps[:n.value].copy(), desc[:n.value].copy()

    def level(self, l):
        w, h = ctypes.c_int(), ctypes.c_int()
        _check(_lib.orbx_extractor_level(self._h, l, None, 0, ctypes.byref(w), ctypes.byref(h)))
        out = np.zeros((h.value, w.value), np.uint8)
        _check(_lib.orbx_extractor_level(self._h, l, _p(out), w.value, None, None))
        return out

    def set_options(self, pyramid_to_host=False, pinned_h2d=False):
        """ORBX_EXTRACTOR_* options (include/orbx.h)"""
        _check(_lib.orbx_extractor_set_options(self._h, (1 if pyramid_to_host else 0)
                                               | (2 if pinned_h2d else 0)), "orbx_extractor_set_options")

    def level_host(self, l):
        """copy of the host pyramid level the last extract() brought back
        (pyramid_to_host option)"""
        d, st = ctypes.c_void_p(), ctypes.c_size_t()
        w, h = ctypes.c_int(), ctypes.c_int()
        _check(_lib.orbx_extractor_level_host(self._h, l, ctypes.byref(d), ctypes.byref(st),
                                              ctypes.byref(w), ctypes.byref(h)), "orbx_extractor_level_host")
        buf = (ctypes.c_uint8 * (st.value * (h.value - 1) + w.value)).from_address(d.value)
        a = np.frombuffer(buf, np.uint8)
        return np.lib.stride_tricks.as_strided(a, (h.value, w.value), (st.value, 1)).copy()

    def stats(self):
        c, r = ctypes.c_longlong(), ctypes.c_longlong()
        _check(_lib.orbx_extractor_stats(self._h, ctypes.byref(c), ctypes.byref(r)))
        return {"calls": c.value, "refetches": r.value}


# --------------------------------------------------------------------------- stereo
def compute_stereo_matches(left, right, kps_l, desc_l, kps_r, desc_r, mb, mbf):
    """Frame::ComputeStereoMatches (Frame.cc:446-620) for the pair whose images
    were the last extract() of Extractor `left` and `right` (their pyramids
    stay on the device).  Returns (mvuRight f32[N], mvDepth f32[N], nmatches)."""
    kl = np.ascontiguousarray(kps_l, KEYPOINT_DTYPE)
    kr = np.ascontiguousarray(kps_r, KEYPOINT_DTYPE)
    dl = np.ascontiguousarray(desc_l, np.uint8).reshape(-1, 32)
    dr = np.ascontiguousarray(desc_r, np.uint8).reshape(-1, 32)
    ur = np.full(max(len(kl), 1), -1, np.float32)
    dep = np.full(max(len(kl), 1), -1, np.float32)
    nm = ctypes.c_int(0)
    _check(_lib.orbx_stereo_match(left._h, right._h, _p(kl), _p(dl), len(kl), _p(kr), _p(dr),
                                  len(kr), float(mb), float(mbf), _p(ur), _p(dep),
                                  ctypes.byref(nm)), "orbx_stereo_match")
    return ur[:len(kl)].copy(), dep[:len(kl)].copy(), nm.value


# --------------------------------------------------------------------------- DBoW2 vocabulary
class Vocabulary:
    """DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB> (ORBVocabulary) on
    the device: loadFromTextFile + transform (TemplatedVocabulary.h:1126-1424)."""

    def __init__(self, handle):
        self._h = handle

    @classmethod
    def load_text(cls, path, device=0):
        h = ctypes.c_void_p()
        _check(_lib.orbv_vocab_load_text(os.fsencode(path), device, ctypes.byref(h)),
               "orbv_vocab_load_text")
        return cls(h)

    @classmethod
    def from_records(cls, voc, scoring=0, weighting=0, device=0):
        parent = np.ascontiguousarray(voc["parent"], np.int32)
        leaf = np.ascontiguousarray(voc["is_leaf"], np.int32)
        desc = np.ascontiguousarray(voc["desc"], np.uint8)
        w = np.ascontiguousarray(voc["weight"], np.float64)
        h = ctypes.c_void_p()
        _check(_lib.orbv_vocab_create(voc["k"], voc["L"], scoring, weighting, len(parent),
                                      _p(parent), _p(leaf), _p(desc), _p(w), device,
                                      ctypes.byref(h)), "orbv_vocab_create")
        return cls(h)

    def __del__(self):
        if getattr(self, "_h", None):
            _lib.orbv_vocab_destroy(self._h)
            self._h = None

    def info(self):
        v = [ctypes.c_int() for _ in range(6)]
        _check(_lib.orbv_vocab_info(self._h, *[ctypes.byref(x) for x in v]))
        return dict(zip(("k", "L", "scoring", "weighting", "nnodes", "nwords"),
                        [x.value for x in v]))

    def transform(self, desc, levelsup=4):
        """-> (BowVector (word ids u32, values f64), FeatureVector dict(node_id, off, feat))"""
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = len(d)
        m = max(n, 1)
        bw, bv = np.zeros(m, np.uint32), np.zeros(m, np.float64)
        fn, fo, ff = np.zeros(m, np.uint32), np.zeros(m + 1, np.uint32), np.zeros(m, np.uint32)
        nb, nf = ctypes.c_int(), ctypes.c_int()
        _check(_lib.orbv_transform(self._h, _p(d), n, levelsup, _p(bw), _p(bv), ctypes.byref(nb),
                                   _p(fn), _p(fo), _p(ff), ctypes.byref(nf)), "orbv_transform")
        nfe = int(fo[nf.value])
        return ((bw[:nb.value].copy(), bv[:nb.value].copy()),
                dict(node_id=fn[:nf.value].copy(), off=fo[:nf.value + 1].copy(),
                     feat=ff[:nfe].copy()))

    def transform_batch(self, desc, counts, levelsup=4, stream=None):
        """Device form over Plan outputs: desc cuda u8 [B, kcap, 32], counts i32 [B].
        Async; returns dict of cuda tensors (bow_word, bow_value, nbow, fv_node,
        fv_off, fv_feat, nfv), rows per frame as in orbv_transform."""
        import torch
        B, kcap = desc.shape[0], desc.shape[1]
        dev = desc.device
        o = dict(bow_word=torch.empty((B, kcap), dtype=torch.int32, device=dev),
                 bow_value=torch.empty((B, kcap), dtype=torch.float64, device=dev),
                 nbow=torch.empty(B, dtype=torch.int32, device=dev),
                 fv_node=torch.empty((B, kcap), dtype=torch.int32, device=dev),
                 fv_off=torch.empty((B, kcap + 1), dtype=torch.int32, device=dev),
                 fv_feat=torch.empty((B, kcap), dtype=torch.int32, device=dev),
                 nfv=torch.empty(B, dtype=torch.int32, device=dev))
        _check(_lib.orbv_transform_batch(self._h, B, desc.data_ptr(), counts.data_ptr(), kcap,
                                         levelsup, o["bow_word"].data_ptr(),
                                         o["bow_value"].data_ptr(), o["nbow"].data_ptr(),
                                         o["fv_node"].data_ptr(), o["fv_off"].data_ptr(),
                                         o["fv_feat"].data_ptr(), o["nfv"].data_ptr(),
                                         _stream_handle(stream)), "orbv_transform_batch")
        return o

    def check(self, stream=None):
        _check(_lib.orbv_check(self._h, _stream_handle(stream)), "orbv_check")


# --------------------------------------------------------------------------- ORBmatcher
def _bow_struct(k, keep):
    desc = np.ascontiguousarray(k["desc"], np.uint8).reshape(-1, 32)
    ang = np.ascontiguousarray(k["angle"], np.float32)
    valid = None if k.get("valid") is None else np.ascontiguousarray(k["valid"], np.uint8)
    nid = np.ascontiguousarray(k["node_id"], np.uint32)
    off = np.ascontiguousarray(k["off"], np.uint32)
    feat = np.ascontiguousarray(k["feat"], np.uint32)
    keep.extend([desc, ang, valid, nid, off, feat])
    return BowFrame(len(desc), _p(desc), _p(ang), _p(valid), len(nid), _p(nid), _p(off), _p(feat))


def search_by_bow(kf1, kf2, nnratio=0.6, check_ori=True, device=0):
    """SearchByBoW(KF1, KF2): returns (match12 int32[N1], nmatches)."""
    keep = []
    b1, b2 = _bow_struct(kf1, keep), _bow_struct(kf2, keep)
    m = np.full(max(b1.n, 1), -1, np.int32)
    nm = ctypes.c_int(0)
    _check(_lib.orbm_search_by_bow(ctypes.byref(b1), ctypes.byref(b2), float(nnratio),
                                   1 if check_ori else 0, device, _p(m), ctypes.byref(nm)),
           "orbm_search_by_bow")
    return m[:b1.n].copy(), nm.value


def search_by_bow_kf_frame(kf, fr, nnratio=0.6, check_ori=True, device=0):
    """Upstream ORB-SLAM2's SearchByBoW(KF, Frame) (bow_kf_frame=full; the
    reference ships a stub): returns (match_f int32[F.N], nmatches)."""
    keep = []
    b1, b2 = _bow_struct(kf, keep), _bow_struct(fr, keep)
    m = np.full(max(b2.n, 1), -1, np.int32)
    nm = ctypes.c_int(0)
    _check(_lib.orbm_search_by_bow_kf_frame(ctypes.byref(b1), ctypes.byref(b2), float(nnratio),
                                            1 if check_ori else 0, device, _p(m), ctypes.byref(nm)),
           "orbm_search_by_bow_kf_frame")
    return m[:b2.n].copy(), nm.value


def descriptor_distance_batch(a, b, ia, ib, device=0):
    a = np.ascontiguousarray(a, np.uint8).reshape(-1, 32)
    b = np.ascontiguousarray(b, np.uint8).reshape(-1, 32)
    ia = np.ascontiguousarray(ia, np.int32)
    ib = np.ascontiguousarray(ib, np.int32)
    out = np.zeros(len(ia), np.int32)
    _check(_lib.orbm_descriptor_distance_batch(_p(a), len(a), _p(b), len(b), _p(ia), _p(ib),
                                               len(ia), device, _p(out)))
    return out


def search_by_projection(mode, frame, queries, qdesc, nnratio=0.6, th_dist=100, check_ori=True,
                         device=0):
    """ORBmatcher::SearchByProjection in query form (orbm_search_by_projection).
    frame = dict(keys, desc, uright|None, occupied|None, min_x, min_y, grid_w_inv,
    grid_h_inv); queries = PROJ_QUERY_DTYPE array.  Returns (match int32[n], nmatches)."""
    keys = np.ascontiguousarray(frame["keys"], KEYPOINT_DTYPE)
    desc = np.ascontiguousarray(frame["desc"], np.uint8).reshape(-1, 32)
    ur = None if frame.get("uright") is None else np.ascontiguousarray(frame["uright"], np.float32)
    occ = None if frame.get("occupied") is None else np.ascontiguousarray(frame["occupied"], np.uint8)
    q = np.ascontiguousarray(queries, PROJ_QUERY_DTYPE)
    qd = np.ascontiguousarray(qdesc, np.uint8).reshape(-1, 32)
    F = ProjFrame(len(keys), _p(keys), _p(desc), _p(ur), _p(occ), frame["min_x"], frame["min_y"],
                  frame["grid_w_inv"], frame["grid_h_inv"])
    m = np.full(max(len(keys), 1), -1, np.int32)
    nm = ctypes.c_int(0)
    _check(_lib.orbm_search_by_projection(mode, ctypes.byref(F), _p(q), _p(qd), len(q),
                                          float(nnratio), int(th_dist), 1 if check_ori else 0,
                                          device, _p(m), ctypes.byref(nm)),
           "orbm_search_by_projection")
    return m[:len(keys)].copy(), nm.value


class ProjPlan:
    """Batched SearchByProjection (orbm_proj_plan_*): many (frame, queries)
    problems on device-resident data in one set of launches."""

    def __init__(self, max_problems, max_n, max_nq, device=0):
        h = ctypes.c_void_p()
        _check(_lib.orbm_proj_plan_create(max_problems, max_n, max_nq, device, ctypes.byref(h)),
               "orbm_proj_plan_create")
        self._h, self.device = h, device

    def __del__(self):
        if getattr(self, "_h", None):
            _lib.orbm_proj_plan_destroy(self._h)
            self._h = None

    def search(self, mode, problems, nnratio=0.6, th_dist=100, check_ori=True, stream=None):
        """problems: list of dicts of cuda tensors -- keys [n, 28] u8 (orbx_keypoint
        rows), desc [n, 32] u8, uright [n] f32 or None, occupied [n] u8 or None,
        q [nq] rows of PROJ_QUERY_DTYPE as u8 [nq, 28], qdesc [nq, 32] u8,
        match [n] i32 and nmatches [1] i32 (outputs) -- plus the grid floats
        min_x, min_y, grid_w_inv, grid_h_inv.  Asynchronous."""
        def ptr(t):
            return None if t is None else t.data_ptr()
        arr = (ProjProblem * max(len(problems), 1))()
        for i, pb in enumerate(problems):
            n = pb["keys"].shape[0]
            arr[i].frame = ProjFrame(n, ptr(pb["keys"]), ptr(pb["desc"]), ptr(pb.get("uright")),
                                     ptr(pb.get("occupied")), pb["min_x"], pb["min_y"],
                                     pb["grid_w_inv"], pb["grid_h_inv"])
            arr[i].q, arr[i].qdesc, arr[i].nq = ptr(pb["q"]), ptr(pb["qdesc"]), pb["q"].shape[0]
            arr[i].match, arr[i].nmatches = ptr(pb["match"]), ptr(pb["nmatches"])
        _check(_lib.orbm_proj_plan_search(self._h, mode, len(problems), ctypes.cast(arr, ctypes.c_void_p),
                                          float(nnratio), int(th_dist), 1 if check_ori else 0,
                                          _stream_handle(stream)), "orbm_proj_plan_search")


def compute_distinctive_descriptors(groups, device=0):
    """MapPoint::ComputeDistinctiveDescriptors for a list of (N_m, 32) descriptor
    arrays; returns int32[len(groups)] chosen rows (-1 for empty)."""
    off = np.zeros(len(groups) + 1, np.int32)
    off[1:] = np.cumsum([len(g) for g in groups])
    desc = np.ascontiguousarray(np.concatenate([np.asarray(g, np.uint8).reshape(-1, 32)
                                                for g in groups]) if groups else
                                np.zeros((0, 32), np.uint8))
    best = np.zeros(max(len(groups), 1), np.int32)
    _check(_lib.orbm_compute_distinctive_descriptors(_p(desc), _p(off), len(groups), device,
                                                     _p(best)), "distinctive descriptors")
    return best[:len(groups)].copy()


def undistort_keypoints(kps, K, dist, device=0):
    """Frame::UndistortKeyPoints (cv::undistortPoints, OpenCV 3.4 algorithm)."""
    k = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
    K9 = np.ascontiguousarray(K, np.float32).reshape(9)
    D = np.ascontiguousarray(dist, np.float32).reshape(-1)
    out = np.zeros_like(k)
    _check(_lib.orbx_undistort_keypoints(_p(k), len(k), _p(K9), _p(D), len(D), device, _p(out)),
           "orbx_undistort_keypoints")
    return out


# --------------------------------------------------------------------------- batched device path
def _check_dev(t, itemsize, rows, name, tail=None):
    """Validate a caller-supplied cuda tensor before its pointer crosses the C
    ABI: cuda device, contiguous, element size, >= rows leading entries and
    the expected trailing shape (the kernels trust these)."""
    if not getattr(t, "is_cuda", False):
        raise OrbxError(ERR_ARG, "%s: cuda tensor expected" % name)
    if not t.is_contiguous():
        raise OrbxError(ERR_ARG, "%s: contiguous tensor expected" % name)
    if itemsize is not None and t.element_size() != itemsize:
        raise OrbxError(ERR_ARG, "%s: element size %d expected" % (name, itemsize))
    if t.dim() < 1 or t.shape[0] < rows:
        raise OrbxError(ERR_ARG, "%s: at least %d rows expected" % (name, rows))
    if tail is not None and tuple(t.shape[1:]) != tuple(tail):
        raise OrbxError(ERR_ARG, "%s: shape [*, %s] expected, got %s"
                        % (name, ", ".join(map(str, tail)), tuple(t.shape)))


def _stream_handle(stream):
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    return getattr(stream, "cuda_stream", stream)


class Plan:
    """Batched device-resident extraction of `max_batch` frames of W x H."""

    def __init__(self, prm, width, height, max_batch, device=0):
        import torch
        self.params, self.W, self.H, self.max_batch, self.device = prm, width, height, max_batch, device
        h = ctypes.c_void_p()
        _check(_lib.orbx_plan_create(ctypes.byref(prm), width, height, max_batch, device,
                                     ctypes.byref(h)), "orbx_plan_create")
        self._h = h
        self.geo = Geometry()
        _check(_lib.orbx_plan_geometry(self._h, ctypes.byref(self.geo)))
        self.kcap = self.geo.kcap
        dev = torch.device("cuda", device)
        self.kps = torch.empty((max_batch, max(self.kcap, 1), 28), dtype=torch.uint8, device=dev)
        self.desc = torch.empty((max_batch, max(self.kcap, 1), 32), dtype=torch.uint8, device=dev)
        self.counts = torch.zeros(max_batch, dtype=torch.int32, device=dev)

    def __del__(self):
        if getattr(self, "_h", None):
            _lib.orbx_plan_destroy(self._h)
            self._h = None

    def extract(self, frames, stream=None, out=None):
        """frames: cuda uint8 tensor [B, H, W] (row stride W).  Async.
        out: optional (kps [>=B, kcap, 28] u8, desc [>=B, kcap, 32] u8, counts [>=B] i32)."""
        B = frames.shape[0]
        assert frames.dtype.itemsize == 1 and frames.is_contiguous()
        assert frames.shape[1] == self.H and frames.shape[2] == self.W and B <= self.max_batch
        kps, desc, counts = out if out is not None else (self.kps, self.desc, self.counts)
        _check_dev(frames, None, B, "frames")
        _check_dev(kps, 1, B, "kps", (self.kcap, 28))
        _check_dev(desc, 1, B, "desc", (self.kcap, 32))
        _check_dev(counts, 4, B, "counts")
        _check(_lib.orbx_plan_extract(self._h, frames.data_ptr(), B, self.W * self.H, self.W,
                                      kps.data_ptr(), desc.data_ptr(), counts.data_ptr(),
                                      _stream_handle(stream)), "orbx_plan_extract")

    def check(self, stream=None):
        _check(_lib.orbx_plan_check(self._h, _stream_handle(stream)), "orbx_plan_check")

    def debug_counters(self):
        """{'fast_overflow_strips': n} since the last call (synchronises the plan's stream)"""
        v = ctypes.c_int(0)
        _check(_lib.orbx_plan_debug_counters(self._h, ctypes.byref(v)), "orbx_plan_debug_counters")
        return {"fast_overflow_strips": v.value}

    def set_options(self, pyramid="auto", brief="auto"):
        """pyramid: 'auto' or 'tiles' (k_pyramid, the one pyramid path since
        the round-4 streaming kernels were retired); brief: 'auto' (the
        planner's choice), 'patch' (per-keypoint blur, k_orient_brief) or
        'level' (every level blurred once, k_blur + k_orient_brief_lb).
        Every combination gives the same results."""
        flags = {"auto": 0, "tiles": ORBX_PLAN_PYR_TILES}[pyramid]
        flags |= {"auto": 0, "patch": ORBX_PLAN_BRIEF_PATCH, "level": ORBX_PLAN_BRIEF_LEVEL}[brief]
        _check(_lib.orbx_plan_set_options(self._h, flags), "orbx_plan_set_options")

    def level(self, frame, lvl, stream=None):
        """pyramid level `lvl` (>= 1, not aliasing level 0) of frame `frame` of
        the last extract, as a host array (synchronises the stream)"""
        w, h = ctypes.c_int(0), ctypes.c_int(0)
        _check(_lib.orbx_plan_level(self._h, frame, lvl, None, 0, ctypes.byref(w), ctypes.byref(h),
                                    _stream_handle(stream)), "orbx_plan_level")
        out = np.empty((h.value, w.value), np.uint8)
        _check(_lib.orbx_plan_level(self._h, frame, lvl, _p(out), w.value, None, None,
                                    _stream_handle(stream)), "orbx_plan_level")
        return out

    def set_timing(self, enable):
        _check(_lib.orbx_plan_set_timing(self._h, 1 if enable else 0))

    def stage_times(self):
        n = _lib.orbx_stage_count()
        ms = np.zeros(n, np.float64)
        cnt = np.zeros(n, np.int32)
        _check(_lib.orbx_plan_stage_times(self._h, _p(ms), _p(cnt), n))
        return {name: (ms[i], int(cnt[i])) for i, name in enumerate(stage_names())}

    def results(self, B):
        """host copies: list of (keypoints structured array, descriptors) for frames 0..B-1"""
        counts = self.counts[:B].cpu().numpy()
        kraw = self.kps[:B].cpu().numpy()
        draw = self.desc[:B].cpu().numpy()
        out = []
        for f in range(B):
            n = int(counts[f])
            k = kraw[f, :n].copy().view(KEYPOINT_DTYPE).reshape(n)
            out.append((k, draw[f, :n].copy()))
        return out


class MatchPlan:
    """Batched brute-force SearchByBoW between extractor frames (single node, top-N).

    zero_tail=True asserts that bytes 24..31 of every descriptor are zero (true
    of Plan.extract outputs) and lets the distance kernels skip them; valu=True
    takes the xor/popcount distance kernel instead of the MFMA one."""

    def __init__(self, max_pairs, kcap, topn=2000, device=0, zero_tail=False, valu=False):
        import torch
        h = ctypes.c_void_p()
        _check(_lib.orbm_plan_create(max_pairs, kcap, topn, device, ctypes.byref(h)),
               "orbm_plan_create")
        self._h, self.kcap, self.topn, self.max_pairs = h, kcap, topn, max_pairs
        _check(_lib.orbm_plan_set_options(h, (ORBM_PLAN_ZERO_TAIL if zero_tail else 0)
                                          | (ORBM_PLAN_VALU if valu else 0)), "orbm_plan_set_options")
        dev = torch.device("cuda", device)
        self.match12 = torch.empty((max_pairs, kcap), dtype=torch.int32, device=dev)
        self.nmatches = torch.zeros(max_pairs, dtype=torch.int32, device=dev)

    def __del__(self):
        if getattr(self, "_h", None):
            _lib.orbm_plan_destroy(self._h)
            self._h = None

    def match(self, npairs, kps_a, desc_a, cnt_a, kps_b, desc_b, cnt_b, nnratio=0.6,
              check_ori=True, stream=None, out_offset=0):
        if npairs < 1 or out_offset < 0 or npairs + out_offset > self.max_pairs:
            raise OrbxError(ERR_ARG, "MatchPlan.match: npairs %d + out_offset %d > max_pairs %d"
                            % (npairs, out_offset, self.max_pairs))
        for t, name, shape in ((kps_a, "kps_a", (self.kcap, 28)), (desc_a, "desc_a", (self.kcap, 32)),
                               (kps_b, "kps_b", (self.kcap, 28)), (desc_b, "desc_b", (self.kcap, 32))):
            _check_dev(t, 1, npairs, name, shape)
        _check_dev(cnt_a, 4, npairs, "cnt_a")
        _check_dev(cnt_b, 4, npairs, "cnt_b")
        m = self.match12[out_offset:]
        nm = self.nmatches[out_offset:]
        _check(_lib.orbm_plan_match_frames(self._h, npairs, kps_a.data_ptr(), desc_a.data_ptr(),
                                           cnt_a.data_ptr(), kps_b.data_ptr(), desc_b.data_ptr(),
                                           cnt_b.data_ptr(), float(nnratio), 1 if check_ori else 0,
                                           m.data_ptr(), nm.data_ptr(), _stream_handle(stream)),
               "orbm_plan_match_frames")

    def set_timing(self, enable):
        _check(_lib.orbm_plan_set_timing(self._h, 1 if enable else 0))

    def stage_times(self):
        n = _lib.orbx_stage_count()
        ms = np.zeros(n, np.float64)
        cnt = np.zeros(n, np.int32)
        _check(_lib.orbm_plan_stage_times(self._h, _p(ms), _p(cnt), n))
        return {name: (ms[i], int(cnt[i])) for i, name in enumerate(stage_names())}


class StereoPlan:
    """Batched device stereo matcher (Frame::ComputeStereoMatches) over the
    outputs and pyramids of a left and a right Plan of the same geometry."""

    def __init__(self, plan, max_batch=None, device=0):
        import torch
        max_batch = max_batch or plan.max_batch
        h = ctypes.c_void_p()
        _check(_lib.orbs_plan_create(plan._h, max_batch, ctypes.byref(h)), "orbs_plan_create")
        self._h, self.kcap, self.max_batch = h, plan.kcap, max_batch
        dev = torch.device("cuda", device)
        self.uright = torch.empty((max_batch, max(self.kcap, 1)), dtype=torch.float32, device=dev)
        self.depth = torch.empty((max_batch, max(self.kcap, 1)), dtype=torch.float32, device=dev)
        self.nmatches = torch.zeros(max_batch, dtype=torch.int32, device=dev)

    def __del__(self):
        if getattr(self, "_h", None):
            _lib.orbs_plan_destroy(self._h)
            self._h = None

    def match(self, left, right, frames_l, frames_r, mb, mbf, left_out=None, right_out=None,
              stream=None):
        """frames_*: the cuda [B, H, W] tensors the plans last extracted.  Async."""
        B = frames_l.shape[0]
        if B > self.max_batch or frames_r.shape[0] < B:
            raise OrbxError(ERR_ARG, "StereoPlan.match: batch %d > max_batch %d" % (B, self.max_batch))
        _check_dev(frames_l, 1, B, "frames_l", (left.H, left.W))
        _check_dev(frames_r, 1, B, "frames_r", (left.H, left.W))
        kl, dl, cl = left_out if left_out is not None else (left.kps, left.desc, left.counts)
        kr, dr, cr = right_out if right_out is not None else (right.kps, right.desc, right.counts)
        for t, name, shape in ((kl, "kps_l", (self.kcap, 28)), (dl, "desc_l", (self.kcap, 32)),
                               (kr, "kps_r", (self.kcap, 28)), (dr, "desc_r", (self.kcap, 32))):
            _check_dev(t, 1, B, name, shape)
        _check_dev(cl, 4, B, "counts_l")
        _check_dev(cr, 4, B, "counts_r")
        _check(_lib.orbs_plan_match(self._h, B, left._h, right._h, frames_l.data_ptr(),
                                    frames_r.data_ptr(), left.W * left.H, left.W, kl.data_ptr(),
                                    dl.data_ptr(), cl.data_ptr(), kr.data_ptr(), dr.data_ptr(),
                                    cr.data_ptr(), float(mb), float(mbf), self.uright.data_ptr(),
                                    self.depth.data_ptr(), self.nmatches.data_ptr(),
                                    _stream_handle(stream)), "orbs_plan_match")

    def check(self, stream=None):
        _check(_lib.orbs_plan_check(self._h, _stream_handle(stream)), "orbs_plan_check")

    def set_timing(self, enable):
        _check(_lib.orbs_plan_set_timing(self._h, 1 if enable else 0))

    def stage_times(self):
        n = _lib.orbx_stage_count()
        ms = np.zeros(n, np.float64)
        cnt = np.zeros(n, np.int32)
        _check(_lib.orbs_plan_stage_times(self._h, _p(ms), _p(cnt), n))
        return {name: (ms[i], int(cnt[i])) for i, name in enumerate(stage_names())}


def selftest_sincos(x):
    """(sin, cos) the BRIEF kernel uses for each float angle of the cuda float32
    tensor x (radians); returns a cuda float32 tensor [n, 2]."""
    import torch
    out = torch.empty((x.numel(), 2), dtype=torch.float32, device=x.device)
    _check(_lib.orbx_selftest_sincos(x.data_ptr(), x.numel(), out.data_ptr(), None),
           "orbx_selftest_sincos")
    torch.cuda.synchronize(x.device)
    return out


def synth_frames(out, first_idx, kind="rects", stream=None):
    """Fill a cuda uint8 tensor [B, H, W] with synthetic frames (orbx/synth.py spec)."""
    from . import synth
    B, H, W = out.shape
    _check(_lib.orbx_synth_frames(out.data_ptr(), W, H, W * H, B, first_idx, synth.KINDS[kind],
                                  _stream_handle(stream)), "orbx_synth_frames")
