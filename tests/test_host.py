"""Host-side checks of liborbx.so that need no GPU: exported C ABI, constant
tables, level geometry, resize coefficient tables, the BRIEF sin/cos
exception table, and loud failure without a device."""
import os
import re
import subprocess

import numpy as np
import pytest

from orbx import synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "orb-slam-system_amd")
HEADER = os.path.join(ROOT, "include", "orbx.h")


def test_library_exports_every_header_function(orbx_mod):
    txt = open(HEADER).read()
    decl = set(re.findall(r"^\w[\w\s\*]*?\b(orb[xmsv]_\w+)\s*\(", txt, re.M))
    assert len(decl) >= 25
    missing = [n for n in decl if not hasattr(orbx_mod.lib(), n)]
    assert not missing, missing
    assert set(orbx_mod.EXPORTED) == decl
    assert orbx_mod.lib().orbx_abi_version() == 2  # include/orbx.h ORBX_ABI_VERSION (flags 2 / 4 retired)


@pytest.mark.parametrize("nf,L", [(1000, 8), (2000, 8), (1200, 8), (1000, 1), (1500, 6)])
def test_tables_match_oracle(orbx_mod, oracle, nf, L):
    sf = 1.3 if L == 6 else 1.2
    t = orbx_mod.tables(orbx_mod.params(nf, sf, L, 20, 7))
    r = oracle.Extractor(nf, sf, L, 20, 7).tables()
    for k in ("scale", "inv_scale", "sigma2", "inv_sigma2", "features_per_level", "umax"):
        assert np.array_equal(t[k], r[k]), k


@pytest.mark.parametrize("w,h,nf,guard", [(640, 480, 1000, "strict"), (1241, 376, 2000, "strict"),
                                          (1920, 1080, 2000, "empty"), (752, 480, 1200, "strict")])
def test_geometry_matches_oracle_levels(orbx_mod, oracle, w, h, nf, guard):
    prm = orbx_mod.params(nf, 1.2, 8, 20, 7, guard)
    g = orbx_mod.geometry(prm, w, h)
    e = oracle.Extractor(nf, 1.2, 8, 20, 7, cell_guard=guard)
    k, _ = e.extract(synth.frame(w, h, 9, "noise"))
    for l in range(8):
        assert e.level(l).shape == (g.height[l], g.width[l])
        assert len(e.level_keys(l)) <= g.kcap_level[l]
    assert g.alias[1] == 0  # mvScaleFactor[1] == 1: level 1 is a copy of level 0
    assert len(k) <= g.kcap


def test_strict_guard_geometry(orbx_mod):
    with pytest.raises(orbx_mod.OrbxError) as e:
        orbx_mod.geometry(orbx_mod.params(2000, 1.2, 8, 20, 7, "strict"), 1920, 1080)
    assert e.value.code == orbx_mod.ERR_CELL_ROI
    g = orbx_mod.geometry(orbx_mod.params(2000, 1.2, 8, 20, 7, "empty"), 1920, 1080)
    # 1080p: last FAST cell column has negative width at levels 0/1 (1920), 2 (1600), 3 (1333)
    assert [g.ncells_bad[l] > 0 for l in range(8)] == [True, True, True, True] + [False] * 4


@pytest.mark.parametrize("w,h,ok", [(4127, 4127, True), (4128, 1000, True), (8223, 2079, True),
                                    (2079, 8223, True), (8224, 600, False), (4200, 4200, False),
                                    (4200, 2100, False), (2100, 4200, False), (4127, 2079, True)])
def test_large_frame_geometry(orbx_mod, w, h, ok):
    """Frames past 4127 px: the FAST key packing trades coordinate bits
    (13-bit x / 11-bit y or the reverse); beyond both it is unsupported."""
    prm = orbx_mod.params(2000, 1.2, 8, 20, 7, "empty")
    if ok:
        g = orbx_mod.geometry(prm, w, h)
        assert (g.width[0], g.height[0]) == (w, h)
    else:
        with pytest.raises(orbx_mod.OrbxError) as e:
            orbx_mod.geometry(prm, w, h)
        assert e.value.code == orbx_mod.ERR_UNSUPPORTED


def test_level_too_small(orbx_mod):
    with pytest.raises(orbx_mod.OrbxError) as e:
        orbx_mod.geometry(orbx_mod.params(1000, 1.2, 14, 20, 7), 320, 240)
    assert e.value.code == orbx_mod.ERR_LEVEL_SIZE


def _apply_lut(src, xofs, alpha, yofs, beta):
    sh, sw = src.shape
    s = src.astype(np.int64)
    a0, a1 = alpha[:, 0].astype(np.int64), alpha[:, 1].astype(np.int64)
    x1 = np.where(alpha[:, 1] == 0, xofs, np.minimum(xofs + 1, sw - 1))
    r0 = np.clip(yofs, 0, sh - 1)
    r1 = np.clip(yofs + 1, 0, sh - 1)
    D0 = s[r0][:, xofs] * a0 + s[r0][:, x1] * a1
    D1 = s[r1][:, xofs] * a0 + s[r1][:, x1] * a1
    b0, b1 = beta[:, 0:1].astype(np.int64), beta[:, 1:2].astype(np.int64)
    return ((((b0 * (D0 >> 4)) >> 16) + ((b1 * (D1 >> 4)) >> 16) + 2) >> 2).astype(np.uint8)


@pytest.mark.parametrize("w,h", [(640, 480), (1241, 376), (1920, 1080)])
def test_resize_tables_reproduce_oracle_resize(orbx_mod, oracle, w, h):
    prm = orbx_mod.params(2000, 1.2, 8, 20, 7, "empty")
    g = orbx_mod.geometry(prm, w, h)
    img = synth.frame(w, h, 3, "noise")
    prev = img
    for l in range(1, 8):
        ref = oracle.resize_linear(prev, g.width[l], g.height[l])
        if g.alias[l] == l:
            got = _apply_lut(prev, *orbx_mod.resize_tables(prm, w, h, l))
            assert np.array_equal(got, ref), l
        else:
            assert np.array_equal(ref, prev)
        prev = ref


def test_release_library_reads_no_profiling_knobs():
    """The ORBX_DEBUG_* / ORBX_CHUNK environment knobs (phase early exits, grid
    divisors, chunked passes) exist only in profiling builds (-DORBX_PROFILING,
    tools/variant.sh): the release liborbx.so does not contain their names, so
    an inherited environment cannot change its results.  The FAST corner-list
    test hook is a C entry point (orbx_debug_set_fast_ccap), not a variable
    (ADVICE r5)."""
    blob = open(os.path.join(PKG, "liborbx.so"), "rb").read()
    for knob in (b"ORBX_DEBUG_STOP", b"ORBX_DEBUG_OBDIV", b"ORBX_CHUNK", b"ORBX_DEBUG_OVERLAP",
                 b"ORBX_DEBUG_SMDIV", b"ORBX_DEBUG_PYR_TILE", b"ORBX_DEBUG_PYR_MAXSEG", b"ORBX_DEBUG_CCAP", b"ORBX_DEBUG_QT_WIDE"):
        assert knob not in blob, knob
    assert b"orbx_debug_set_fast_ccap" in blob


def test_no_device_fails_loudly(orbx_mod):
    if orbx_mod.device_count() > 0:
        pytest.skip("GPU visible")
    with pytest.raises(orbx_mod.OrbxError) as e:
        orbx_mod.Extractor(1000, 1.2, 8, 20, 7)
    assert e.value.code == orbx_mod.ERR_NO_DEVICE
    with pytest.raises(orbx_mod.OrbxError):
        orbx_mod.search_by_bow(dict(desc=np.zeros((1, 32), np.uint8), angle=np.zeros(1, np.float32),
                                    node_id=np.zeros(1, np.uint32), off=np.array([0, 1], np.uint32),
                                    feat=np.zeros(1, np.uint32)),
                               dict(desc=np.zeros((1, 32), np.uint8), angle=np.zeros(1, np.float32),
                                    node_id=np.zeros(1, np.uint32), off=np.array([0, 1], np.uint32),
                                    feat=np.zeros(1, np.uint32)))


@pytest.mark.slow
def test_sincos_exception_table_is_current(tmp_path):
    """Exhaustive: every reachable BRIEF angle, host glibc sincosf vs the device routine."""
    exe = tmp_path / "gen_sincos"
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe),
                           os.path.join(ROOT, "tools", "gen_sincos_table.c"), "-lm", "-lpthread"])
    out = tmp_path / "t.inc"
    subprocess.check_call([str(exe), str(out)], stdout=subprocess.DEVNULL)
    committed = open(os.path.join(ROOT, "orb-slam-system_amd", "csrc", "sincos_exceptions.inc")).read()
    assert out.read_text() == committed


# every geometry the GPU parity suite runs (test_gpu_parity.py), so the
# tile kernel's duplicate-store invariant (non-owned edge-dword bytes equal
# their owner's) is checked wherever the kernel runs
PYR_CASES = [(640, 480, 1000, 8, 1.2), (1241, 376, 2000, 8, 1.2), (1920, 1080, 2000, 8, 1.2),
             (752, 480, 1200, 4, 1.5), (640, 480, 500, 14, 1.1), (1000, 700, 500, 3, 1.9),
             (320, 240, 500, 2, 1.2), (4096, 400, 2000, 8, 1.2), (5000, 720, 2000, 8, 1.2),
             (600, 4400, 2000, 8, 1.2), (642, 361, 1000, 8, 1.2), (644, 362, 1000, 8, 1.2),
             (640, 480, 1000, 12, 1.1), (640, 480, 1000, 8, 1.3), (752, 480, 1200, 6, 1.5),
             (1241, 376, 2000, 4, 1.7), (640, 480, 800, 3, 1.95), (1280, 600, 1000, 6, 2.0),
             (1920, 1080, 2000, 6, 2.0)]


@pytest.mark.parametrize("W,H,nf,L,sf", PYR_CASES)
def test_fused_pyramid_tiling_matches_oracle(oracle, tmp_path, W, H, nf, L, sf):
    """Host emulation of k_pyramid's tiles (LDS regions, owned partitions)
    on the planner's tables: every unique level written exactly once, no read
    outside a staged region, and the levels equal the oracle's pyramid."""
    exe = tmp_path / "pyr"
    csrc = os.path.join(PKG, "csrc")
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", csrc,
                           os.path.join(ROOT, "tests", "cpp", "pyramid_emu.cpp"),
                           os.path.join(csrc, "geometry.cpp"), "-o", str(exe)])
    img = synth.frame(W, H, 3, "noise")
    (tmp_path / "in.raw").write_bytes(img.tobytes())
    out = tmp_path / "out.bin"
    subprocess.check_call([str(exe), str(tmp_path / "in.raw"), str(W), str(H), str(nf), str(L),
                           repr(sf), str(out)])
    raw = np.frombuffer(out.read_bytes(), np.uint8)
    ref = oracle.Extractor(nf, sf, L, 20, 7, cell_guard="empty")
    ref.extract(img)
    off = 0
    for l in range(1, L):
        lv = ref.level(l)
        if lv.shape == ref.level(l - 1).shape:
            continue  # alias of the previous level (cv::resize copy)
        assert np.array_equal(raw[off:off + lv.size].reshape(lv.shape), lv), "level %d" % l
        off += lv.size
    assert off == raw.size


