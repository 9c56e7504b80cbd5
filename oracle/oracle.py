"""TEST INFRASTRUCTURE ONLY -- ctypes binding of the CPU restatement (the oracle).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module.  The product (orb-slam-system_amd/liborbx.so) never
touches it.  Parity status: "parity unpinned" vs the reference binary (see
oracle/orb_oracle.h and DESIGN.md §Oracle).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liborb_oracle.so")

KEYPOINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                           ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
assert KEYPOINT_DTYPE.itemsize == 28

OO_OK, OO_ERR_ARG, OO_ERR_CELL_ROI, OO_ERR_LEVEL_SIZE, OO_ERR_QUADTREE, OO_ERR_CAPACITY, \
    OO_ERR_UNSUPPORTED = 0, -1, -2, -3, -4, -5, -6

_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        i, f = ctypes.c_int, ctypes.c_float
        L.oo_create.restype = P
        L.oo_create.argtypes = [i, f, i, i, i, i]
        L.oo_destroy.argtypes = [P]
        L.oo_get_tables.argtypes = [P, P, P, P, P, P, P]
        L.oo_extract.argtypes = [P, P, i, i, i, P, i, P, P]
        L.oo_level_size.argtypes = [P, i, P, P]
        L.oo_level_pixels.restype = P
        L.oo_level_pixels.argtypes = [P, i]
        L.oo_level_candidates.argtypes = [P, i, P, i]
        L.oo_level_keys.argtypes = [P, i, P, i]
        L.oo_fast_atan2.restype = f
        L.oo_fast_atan2.argtypes = [f, f]
        L.oo_fast_detect.argtypes = [P, i, i, i, i, i, P, i]
        L.oo_resize_linear.argtypes = [P, i, i, i, P, i, i, i]
        L.oo_resize_area2.argtypes = [P, i, i, i, P, i, i, i]
        L.oo_gaussian_blur7.argtypes = [P, i, i, i, P, i]
        L.oo_gaussian_kernel7.argtypes = [P]
        L.oo_brief_descriptor.argtypes = [P, i, i, i, f, P]
        L.oo_descriptor_distance.argtypes = [P, P]
        L.oo_search_by_bow.argtypes = [i, P, P, P, i, P, P, P, i, P, P, P, i, P, P, P, f, i, P]
        L.oo_search_by_bow_kf_frame.argtypes = [i, P, P, P, i, P, P, P, i, P, P, i, P, P, P, f, i, P]
        L.oo_vocab_from_records.restype = P
        L.oo_vocab_from_records.argtypes = [i, i, i, i, i, P, P, P, P]
        L.oo_vocab_destroy.argtypes = [P]
        L.oo_vocab_info.argtypes = [P, P, P, P, P, P, P]
        L.oo_vocab_transform.argtypes = [P, P, i, i, P, P, P, P, P, P, P]
        L.oo_features_in_area.argtypes = [i, P, f, f, f, f, f, f, f, i, i, P]
        L.oo_search_by_projection.argtypes = [i, i, P, P, P, P, f, f, f, f, i, P, P, f, i, i, P]
        L.oo_distinctive_descriptor.argtypes = [P, i]
        L.oo_undistort_keypoints.argtypes = [P, i, P, P, i, P]
        L.oo_compute_stereo_matches.argtypes = [i, P, P, i, P, P, i, P, P, P, P, P, P, P, f, f,
                                                P, P]
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class OracleError(RuntimeError):
    def __init__(self, code):
        super().__init__("oracle error %d" % code)
        self.code = code


class Extractor:
    """CPU restatement of ORB_SLAM2::ORBextractor (ORBextractor.cc:116-515)."""

    def __init__(self, nfeatures, scale_factor, nlevels, ini_th, min_th, cell_guard="strict"):
        self.nfeatures, self.nlevels = nfeatures, nlevels
        self._h = lib().oo_create(nfeatures, scale_factor, nlevels, ini_th, min_th,
                                  1 if cell_guard == "empty" else 0)
        if not self._h:
            raise ValueError("bad extractor parameters")

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            try:
                lib().oo_destroy(self._h)
            except TypeError:  # interpreter teardown
                pass
            self._h = None

    def tables(self):
        L = self.nlevels
        s, inv, s2, inv2 = (np.zeros(L, np.float32) for _ in range(4))
        fpl = np.zeros(L, np.int32)
        umax = np.zeros(16, np.int32)
        lib().oo_get_tables(self._h, _p(s), _p(inv), _p(s2), _p(inv2), _p(fpl), _p(umax))
        return dict(scale=s, inv_scale=inv, sigma2=s2, inv_sigma2=inv2, features_per_level=fpl,
                    umax=umax)

    def extract(self, img):
        img = np.ascontiguousarray(img, dtype=np.uint8)
        h, w = img.shape
        cap = 4 * self.nfeatures + 64 * self.nlevels + 64
        kps = np.zeros(cap, KEYPOINT_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = ctypes.c_int(0)
        rc = lib().oo_extract(self._h, _p(img), w, h, w, _p(kps), cap, _p(desc), ctypes.byref(n))
        if rc != OO_OK:
            raise OracleError(rc)
        return kps[:n.value].copy(), desc[:n.value].copy()

    def level(self, l):
        w, h = ctypes.c_int(), ctypes.c_int()
        lib().oo_level_size(self._h, l, ctypes.byref(w), ctypes.byref(h))
        ptr = lib().oo_level_pixels(self._h, l)
        buf = (ctypes.c_uint8 * (w.value * h.value)).from_address(ptr)
        return np.frombuffer(buf, np.uint8).reshape(h.value, w.value).copy()

    def candidates(self, l):
        n = lib().oo_level_candidates(self._h, l, None, 0)
        out = np.zeros(n, KEYPOINT_DTYPE)
        lib().oo_level_candidates(self._h, l, _p(out), n)
        return out

    def level_keys(self, l):
        n = lib().oo_level_keys(self._h, l, None, 0)
        out = np.zeros(n, KEYPOINT_DTYPE)
        lib().oo_level_keys(self._h, l, _p(out), n)
        return out


def fast_atan2(y, x):
    return lib().oo_fast_atan2(float(y), float(x))


def fast_detect(img, threshold, nonmax=True):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    cap = w * h + 1
    out = np.zeros(cap, KEYPOINT_DTYPE)
    n = lib().oo_fast_detect(_p(img), w, h, w, threshold, 1 if nonmax else 0, _p(out), cap)
    return out[:n].copy()


def resize_linear(src, dw, dh):
    src = np.ascontiguousarray(src, dtype=np.uint8)
    sh, sw = src.shape
    dst = np.zeros((dh, dw), np.uint8)
    lib().oo_resize_linear(_p(src), sw, sh, sw, _p(dst), dw, dh, dw)
    return dst


def resize_area2(src):
    """cv::resize to exactly half size (the INTER_AREA fast path)"""
    src = np.ascontiguousarray(src, dtype=np.uint8)
    sh, sw = src.shape
    dh, dw = sh // 2, sw // 2
    dst = np.zeros((dh, dw), np.uint8)
    lib().oo_resize_area2(_p(src), sw, sh, sw, _p(dst), dw, dh, dw)
    return dst


def gaussian_blur7(src):
    src = np.ascontiguousarray(src, dtype=np.uint8)
    h, w = src.shape
    dst = np.zeros_like(src)
    lib().oo_gaussian_blur7(_p(src), w, h, w, _p(dst), w)
    return dst


def gaussian_kernel7():
    k = np.zeros(7, np.int32)
    lib().oo_gaussian_kernel7(_p(k))
    return k


def brief_descriptor(blurred, cx, cy, angle_deg):
    blurred = np.ascontiguousarray(blurred, dtype=np.uint8)
    d = np.zeros(32, np.uint8)
    lib().oo_brief_descriptor(_p(blurred), blurred.shape[1], cx, cy, float(angle_deg), _p(d))
    return d


def descriptor_distance(a, b):
    a = np.ascontiguousarray(a, np.uint8)
    b = np.ascontiguousarray(b, np.uint8)
    return lib().oo_descriptor_distance(_p(a), _p(b))


def search_by_bow(kf1, kf2, nnratio=0.6, check_ori=True):
    """kf = dict(desc (N,32) u8, angle (N,) f32, valid (N,) u8 or None,
    node_id (M,) u32 ascending, off (M+1,) u32, feat u32)."""
    def unpack(k):
        d = np.ascontiguousarray(k["desc"], np.uint8)
        a = np.ascontiguousarray(k["angle"], np.float32)
        v = None if k.get("valid") is None else np.ascontiguousarray(k["valid"], np.uint8)
        nid = np.ascontiguousarray(k["node_id"], np.uint32)
        off = np.ascontiguousarray(k["off"], np.uint32)
        feat = np.ascontiguousarray(k["feat"], np.uint32)
        return d, a, v, nid, off, feat
    d1, a1, v1, n1, o1, f1 = unpack(kf1)
    d2, a2, v2, n2, o2, f2 = unpack(kf2)
    m = np.full(len(d1), -1, np.int32)
    nm = lib().oo_search_by_bow(len(d1), _p(d1), _p(a1), _p(v1), len(n1), _p(n1), _p(o1), _p(f1),
                                len(d2), _p(d2), _p(a2), _p(v2), len(n2), _p(n2), _p(o2), _p(f2),
                                float(nnratio), 1 if check_ori else 0, _p(m))
    return m, nm


def search_by_bow_kf_frame(kf, fr, nnratio=0.6, check_ori=True):
    """Upstream ORB-SLAM2's SearchByBoW(KeyFrame*, Frame&) (the reference
    ships a stub, src/ORBmatcher.cc:88-119): kf / fr as search_by_bow's
    dicts (fr's valid is not used).  Returns (match_f int32[F.N]: KF index
    whose MapPoint Frame feature j received, -1 = none; nmatches)."""
    d1 = np.ascontiguousarray(kf["desc"], np.uint8)
    a1 = np.ascontiguousarray(kf["angle"], np.float32)
    v1 = None if kf.get("valid") is None else np.ascontiguousarray(kf["valid"], np.uint8)
    n1, o1, f1 = (np.ascontiguousarray(kf[k], np.uint32) for k in ("node_id", "off", "feat"))
    d2 = np.ascontiguousarray(fr["desc"], np.uint8)
    a2 = np.ascontiguousarray(fr["angle"], np.float32)
    n2, o2, f2 = (np.ascontiguousarray(fr[k], np.uint32) for k in ("node_id", "off", "feat"))
    m = np.full(max(len(d2), 1), -1, np.int32)
    nm = lib().oo_search_by_bow_kf_frame(len(d1), _p(d1), _p(a1), _p(v1), len(n1), _p(n1), _p(o1), _p(f1),
                                         len(d2), _p(d2), _p(a2), len(n2), _p(n2), _p(o2), _p(f2),
                                         float(nnratio), 1 if check_ori else 0, _p(m))
    return m[:len(d2)].copy(), nm


def compute_stereo_matches(kl, dl, kr, dr, scale, inv_scale, lpyr, rpyr, mb, mbf):
    """Frame::ComputeStereoMatches (src/Frame.cc:446-620) on one rectified pair.
    lpyr / rpyr: lists of uint8 level images (mvImagePyramid of the left /
    right extractor).  Returns (uRight, depth, nkept); raises OracleError
    where the reference would index out of range or throw."""
    kl = np.ascontiguousarray(kl, KEYPOINT_DTYPE)
    kr = np.ascontiguousarray(kr, KEYPOINT_DTYPE)
    dl = np.ascontiguousarray(dl, np.uint8).reshape(-1, 32)
    dr = np.ascontiguousarray(dr, np.uint8).reshape(-1, 32)
    scale = np.ascontiguousarray(scale, np.float32)
    inv_scale = np.ascontiguousarray(inv_scale, np.float32)
    L = len(lpyr)
    lp = [np.ascontiguousarray(a, np.uint8) for a in lpyr]
    rp = [np.ascontiguousarray(a, np.uint8) for a in rpyr]
    for a, b in zip(lp, rp):
        assert a.shape == b.shape
    lptr = (ctypes.c_void_p * L)(*[a.ctypes.data for a in lp])
    rptr = (ctypes.c_void_p * L)(*[a.ctypes.data for a in rp])
    lw = np.array([a.shape[1] for a in lp], np.int32)
    lh = np.array([a.shape[0] for a in lp], np.int32)
    ur = np.zeros(len(kl), np.float32)
    dep = np.zeros(len(kl), np.float32)
    rc = lib().oo_compute_stereo_matches(len(kl), _p(kl), _p(dl), len(kr), _p(kr), _p(dr), L,
                                         _p(scale), _p(inv_scale), ctypes.cast(lptr, ctypes.c_void_p),
                                         ctypes.cast(rptr, ctypes.c_void_p), _p(lw), _p(lh), _p(lw),
                                         float(mb), float(mbf), _p(ur), _p(dep))
    if rc < 0:
        raise OracleError(rc)
    return ur, dep, rc


def parse_vocabulary_text(path):
    """TemplatedVocabulary::loadFromTextFile (TemplatedVocabulary.h:1338-1424)
    on the text: header "k L scoring weighting", node records "parent isLeaf
    d0..d31 weight".  Failed extractions give 0 (C++11 operator>>); blank
    lines are skipped (the reference turns a trailing one into a phantom root
    child with an uninitialised descriptor -- see DESIGN.md)."""
    with open(path) as f:
        lines = f.read().split("\n")

    def num(tok, cast):
        try:
            return cast(tok), True
        except (ValueError, IndexError):
            return cast(0), False

    hdr = lines[0].split()
    head = []
    for j in range(4):
        v, ok = num(hdr[j] if j < len(hdr) else "", int)
        head.append(v)
    parent, leaf, desc, weight = [], [], [], []
    for ln in lines[1:]:
        t = ln.split()
        if not t:
            continue
        vals, ok = [], True
        for j in range(34):
            if ok:
                v, ok = num(t[j] if j < len(t) else "", int)
            else:
                v = 0
            vals.append(v)
        w = 0.0
        if ok and len(t) > 34:
            w, _ = num(t[34], float)
        parent.append(vals[0])
        leaf.append(vals[1])
        desc.append([x & 0xFF for x in vals[2:34]])
        weight.append(w)
    return dict(k=head[0], L=head[1], scoring=head[2], weighting=head[3],
                parent=np.array(parent, np.int32), is_leaf=np.array(leaf, np.int32),
                desc=np.array(desc, np.uint8).reshape(-1, 32), weight=np.array(weight, np.float64))


class Vocabulary:
    """CPU restatement of DBoW2::TemplatedVocabulary<FORB> (load + transform)."""

    def __init__(self, voc, scoring=0, weighting=0):
        self.voc = voc
        parent = np.ascontiguousarray(voc["parent"], np.int32)
        leaf = np.ascontiguousarray(voc["is_leaf"], np.int32)
        desc = np.ascontiguousarray(voc["desc"], np.uint8)
        w = np.ascontiguousarray(voc["weight"], np.float64)
        self._keep = (parent, leaf, desc, w)
        self._h = lib().oo_vocab_from_records(voc["k"], voc["L"], scoring, weighting, len(parent),
                                              _p(parent), _p(leaf), _p(desc), _p(w))
        if not self._h:
            raise OracleError(OO_ERR_ARG)

    @classmethod
    def load_text(cls, path):
        v = parse_vocabulary_text(path)
        return cls(v, v["scoring"], v["weighting"])

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            try:
                lib().oo_vocab_destroy(self._h)
            except TypeError:  # interpreter teardown
                pass
            self._h = None

    def transform(self, desc, levelsup=4):
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = len(d)
        m = max(n, 1)
        bw, bv = np.zeros(m, np.uint32), np.zeros(m, np.float64)
        fn, fo, ff = np.zeros(m, np.uint32), np.zeros(m + 1, np.uint32), np.zeros(m, np.uint32)
        nb, nf = ctypes.c_int(), ctypes.c_int()
        rc = lib().oo_vocab_transform(self._h, _p(d), n, levelsup, _p(bw), _p(bv), ctypes.byref(nb),
                                      _p(fn), _p(fo), _p(ff), ctypes.byref(nf))
        if rc != OO_OK:
            raise OracleError(rc)
        nfe = int(fo[nf.value])
        return ((bw[:nb.value].copy(), bv[:nb.value].copy()),
                dict(node_id=fn[:nf.value].copy(), off=fo[:nf.value + 1].copy(),
                     feat=ff[:nfe].copy()))


PROJ_QUERY_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("radius", "<f4"), ("min_level", "<i4"),
                             ("max_level", "<i4"), ("xr", "<f4"), ("angle", "<f4")])


def features_in_area(frame, x, y, r, min_level=-1, max_level=-1):
    """Frame::GetFeaturesInArea (src/Frame.cc:307-358), in visiting order."""
    keys = np.ascontiguousarray(frame["keys"], KEYPOINT_DTYPE)
    out = np.zeros(max(len(keys), 1), np.int32)
    n = lib().oo_features_in_area(len(keys), _p(keys), frame["min_x"], frame["min_y"],
                                  frame["grid_w_inv"], frame["grid_h_inv"], float(x), float(y),
                                  float(r), int(min_level), int(max_level), _p(out))
    return out[:n].copy()


def search_by_projection(mode, frame, queries, qdesc, nnratio=0.6, th_dist=100, check_ori=True):
    """ORBmatcher::SearchByProjection, query form (modes 1-3, see orb_oracle.h)."""
    keys = np.ascontiguousarray(frame["keys"], KEYPOINT_DTYPE)
    desc = np.ascontiguousarray(frame["desc"], np.uint8).reshape(-1, 32)
    ur = None if frame.get("uright") is None else np.ascontiguousarray(frame["uright"], np.float32)
    occ = None if frame.get("occupied") is None else np.ascontiguousarray(frame["occupied"], np.uint8)
    q = np.ascontiguousarray(queries, PROJ_QUERY_DTYPE)
    qd = np.ascontiguousarray(qdesc, np.uint8).reshape(-1, 32)
    m = np.full(max(len(keys), 1), -1, np.int32)
    nm = lib().oo_search_by_projection(mode, len(keys), _p(keys), _p(desc), _p(ur), _p(occ),
                                       frame["min_x"], frame["min_y"], frame["grid_w_inv"],
                                       frame["grid_h_inv"], len(q), _p(q), _p(qd), float(nnratio),
                                       int(th_dist), 1 if check_ori else 0, _p(m))
    return m[:len(keys)].copy(), nm


def distinctive_descriptor(desc):
    """MapPoint::ComputeDistinctiveDescriptors: index of the chosen row (-1 if none)."""
    d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    return lib().oo_distinctive_descriptor(_p(d), len(d))


def undistort_keypoints(kps, K, dist):
    """Frame::UndistortKeyPoints (cv::undistortPoints restatement)."""
    k = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
    K9 = np.ascontiguousarray(K, np.float32).reshape(9)
    D = np.ascontiguousarray(dist, np.float32).reshape(-1)
    out = np.zeros_like(k)
    lib().oo_undistort_keypoints(_p(k), len(k), _p(K9), _p(D), len(D), _p(out))
    return out
