"""DBoW2 vocabulary transform (Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h:
1126-1259, loader :1338-1424): the producer of the FeatureVectors that
SearchByBoW consumes (Frame::ComputeBoW, src/Frame.cc:375-382, levelsup 4).

The reference vocabulary (ORBvoc.txt) is not in the tree
(.MISSING_LARGE_BLOBS), so vocabularies are synthetic trees
(orbx/synth.py vocabulary) written in the reference's text format.
CPU: oracle known answers (hand-built tree), text loader round trip, the
BowVector/FeatureVector invariants.  GPU: orbv_transform / orbv_transform_batch
vs the oracle -- word ids, node ids and feature lists exact, BowVector values
bit-exact (IEEE double) -- and SearchByBoW on the resulting FeatureVectors.
"""
import numpy as np
import pytest

from orbx import synth


def _tiny_vocab():
    # root -> A(1), B(2); A -> a1(3), a2(4); B -> b1(5) (leaf), b2(6) (stopped leaf)
    z = np.zeros(32, np.uint8)
    A = z.copy(); B = np.full(32, 0xFF, np.uint8)
    a1 = z.copy(); a2 = z.copy(); a2[:4] = 0xFF
    b1 = B.copy(); b2 = B.copy(); b2[:4] = 0
    return dict(k=2, L=2, parent=np.array([0, 0, 1, 1, 2, 2], np.int32),
                is_leaf=np.array([0, 0, 1, 1, 1, 1], np.int32),
                desc=np.stack([A, B, a1, a2, b1, b2]),
                weight=np.array([0, 0, 1.5, 2.5, 4.0, 0.0], np.float64))


def test_oracle_tiny_tree_known_answer(oracle):
    v = oracle.Vocabulary(_tiny_vocab())
    f = np.zeros((5, 32), np.uint8)
    f[1, :4] = 0xFF          # -> A, then a2 (distance 0)
    f[2, :] = 0xFF           # -> B, b1
    f[3, :] = 0xFF
    f[3, :4] = 0             # -> B, b2: stopped (weight 0)
    f[4, 0] = 0x01           # -> A, a1 (tie-free)
    (bw, bv), fv = v.transform(f, levelsup=1)  # nid level 1: A = 1, B = 2
    # words: a1 = 0, a2 = 1, b1 = 2, b2 = 3 (leaf order)
    assert bw.tolist() == [0, 1, 2]
    raw = np.array([1.5 + 1.5, 2.5, 4.0])  # a1 twice (features 0, 4)
    np.testing.assert_array_equal(bv, raw / np.abs(raw).sum())  # L1 normalised
    assert fv["node_id"].tolist() == [1, 2]
    assert fv["off"].tolist() == [0, 3, 4]
    assert fv["feat"].tolist() == [0, 1, 4, 2]


def test_oracle_ties_take_first_child(oracle):
    voc = _tiny_vocab()
    voc["desc"][1] = voc["desc"][0]  # A == B: every feature ties at level 1 -> A (first)
    v = oracle.Vocabulary(voc)
    f = np.full((3, 32), 0xFF, np.uint8)
    (bw, bv), fv = v.transform(f, levelsup=1)
    assert fv["node_id"].tolist() == [1]


def test_oracle_text_roundtrip(oracle, tmp_path):
    voc = synth.vocabulary(6, 3, seed=5)
    p = tmp_path / "voc.txt"
    synth.write_vocabulary_text(p, voc, scoring=1, weighting=0)
    back = oracle.parse_vocabulary_text(p)
    assert (back["k"], back["L"], back["scoring"], back["weighting"]) == (6, 3, 1, 0)
    for key in ("parent", "is_leaf", "desc", "weight"):
        assert np.array_equal(back[key], voc[key]), key


def test_oracle_featurevector_invariants(oracle):
    voc = synth.vocabulary(10, 4, seed=7)
    v = oracle.Vocabulary(voc)
    ex = oracle.Extractor(1000, 1.2, 8, 20, 7)
    k, d = ex.extract(synth.frame(640, 480, 9))
    (bw, bv), fv = v.transform(d, levelsup=2)
    assert np.all(np.diff(bw.astype(np.int64)) > 0) and abs(bv.sum() - 1.0) < 1e-12
    assert np.all(np.diff(fv["node_id"].astype(np.int64)) > 0)
    for j in range(len(fv["node_id"])):
        seg = fv["feat"][fv["off"][j]:fv["off"][j + 1]]
        assert np.all(np.diff(seg.astype(np.int64)) > 0)
    assert len(fv["feat"]) <= len(d)


def test_oracle_rejects_bad_header(oracle):
    voc = _tiny_vocab()
    voc["k"] = 21  # :1356: m_k > 20
    with pytest.raises(oracle.OracleError):
        oracle.Vocabulary(voc)


VOCABS = [
    # (k, L, seed, prune, scoring, weighting, levelsup)
    (10, 6, 1, 0.0, 0, 0, 4),   # ORBvoc.txt shape: k 10, L 6, L1 / TF-IDF, levelsup 4
    (10, 3, 2, 0.0, 1, 0, 1),   # L2 scoring (FMA square-accumulate)
    (5, 4, 3, 0.0, 5, 1, 2),    # dot product (no normalise: divide by #words), TF
    (8, 4, 4, 0.0, 0, 2, 4),    # IDF: addIfNotExist; nid_level 0 -> root
    (6, 5, 5, 0.2, 0, 3, 3),    # BINARY, shallow leaves (level >= 2; nid level 2)
]


def _same(g, r):
    (gbw, gbv), gfv = g
    (rbw, rbv), rfv = r
    assert np.array_equal(gbw, rbw)
    assert np.array_equal(gbv.view(np.uint64), rbv.view(np.uint64))
    for key in ("node_id", "off", "feat"):
        assert np.array_equal(gfv[key], rfv[key]), key


@pytest.mark.gpu
@pytest.mark.parametrize("k,L,seed,prune,scoring,weighting,levelsup", VOCABS)
def test_transform_matches_oracle(gpu, oracle, k, L, seed, prune, scoring, weighting, levelsup):
    voc = synth.vocabulary(k, L, seed=seed, prune=prune)
    gv = gpu.Vocabulary.from_records(voc, scoring, weighting)
    ov = oracle.Vocabulary(voc, scoring, weighting)
    ex = oracle.Extractor(2000, 1.2, 8, 20, 7)
    for idx in range(3):
        k_, d = ex.extract(synth.frame(1241, 376, 70 + idx))
        _same(gv.transform(d, levelsup), ov.transform(d, levelsup))
    rnd = np.random.default_rng(seed).integers(0, 256, (3000, 32), dtype=np.uint8)
    _same(gv.transform(rnd, levelsup), ov.transform(rnd, levelsup))
    _same(gv.transform(rnd[:0], levelsup), ov.transform(rnd[:0], levelsup))


@pytest.mark.gpu
def test_transform_text_loader_matches_oracle(gpu, oracle, tmp_path):
    voc = synth.vocabulary(10, 4, seed=11)
    p = tmp_path / "voc.txt"
    synth.write_vocabulary_text(p, voc, scoring=0, weighting=0)
    gv = gpu.Vocabulary.load_text(p)
    info = gv.info()
    assert (info["k"], info["L"], info["nnodes"]) == (10, 4, len(voc["parent"]) + 1)
    ov = oracle.Vocabulary.load_text(p)
    d = np.random.default_rng(3).integers(0, 256, (1500, 32), dtype=np.uint8)
    _same(gv.transform(d, 2), ov.transform(d, 2))


@pytest.mark.gpu
def test_transform_unset_nodeid_errors(gpu, oracle):
    # header L = 2 but every leaf at level 1; levelsup 0 -> nid level 2 is never reached
    voc = synth.vocabulary(4, 1, seed=12, stop_frac=0.0)
    voc["L"] = 2
    gv = gpu.Vocabulary.from_records(voc)
    d = np.random.default_rng(4).integers(0, 256, (10, 32), dtype=np.uint8)
    with pytest.raises(oracle.OracleError):
        oracle.Vocabulary(voc).transform(d, 0)
    with pytest.raises(gpu.OrbxError) as e:
        gv.transform(d, 0)
    assert e.value.code == gpu.ERR_ARG


@pytest.mark.gpu
def test_search_by_bow_on_vocabulary_featurevectors(gpu, oracle):
    """Frame::ComputeBoW -> SearchByBoW(KF, KF) with real multi-node FeatureVectors."""
    voc = synth.vocabulary(10, 6, seed=1)
    gv = gpu.Vocabulary.from_records(voc)
    ex = oracle.Extractor(2000, 1.2, 8, 20, 7)
    k1, d1 = ex.extract(synth.frame(1241, 376, 80))
    k2, d2 = ex.extract(synth.frame(1241, 376, 81))
    _, fv1 = gv.transform(d1, 4)
    _, fv2 = gv.transform(d2, 4)
    kf1 = dict(desc=d1, angle=k1["angle"], valid=None, **fv1)
    kf2 = dict(desc=d2, angle=k2["angle"], valid=None, **fv2)
    m, nm = gpu.search_by_bow(kf1, kf2, 0.75, True)
    rm, rnm = oracle.search_by_bow(kf1, kf2, 0.75, True)
    assert nm == rnm and np.array_equal(m, rm) and nm > 0


@pytest.mark.gpu
def test_transform_batch_on_plan_outputs(gpu, oracle):
    """orbv_transform_batch over orbx_plan_extract outputs == per-frame oracle."""
    import torch
    W, H, B = 640, 480, 4
    plan = gpu.Plan(gpu.params(1000, 1.2, 8, 20, 7), W, H, B)
    frames = torch.from_numpy(synth.frames(W, H, 90, B)).cuda()
    plan.extract(frames)
    voc = synth.vocabulary(10, 6, seed=1)
    gv = gpu.Vocabulary.from_records(voc)
    o = gv.transform_batch(plan.desc, plan.counts, 4)
    gv.check()
    plan.check()
    ov = oracle.Vocabulary(voc)
    res = plan.results(B)
    h = {k: v.cpu().numpy() for k, v in o.items()}
    for f in range(B):
        (rbw, rbv), rfv = ov.transform(res[f][1], 4)
        nb, nf = h["nbow"][f], h["nfv"][f]
        assert np.array_equal(h["bow_word"][f, :nb].astype(np.uint32), rbw)
        assert np.array_equal(h["bow_value"][f, :nb].view(np.uint64), rbv.view(np.uint64))
        assert np.array_equal(h["fv_node"][f, :nf].astype(np.uint32), rfv["node_id"])
        assert np.array_equal(h["fv_off"][f, :nf + 1].astype(np.uint32), rfv["off"])
        nfe = int(rfv["off"][-1])
        assert np.array_equal(h["fv_feat"][f, :nfe].astype(np.uint32), rfv["feat"])
