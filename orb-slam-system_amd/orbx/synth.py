"""Deterministic synthetic grayscale frames.

splitmix64 stream, element i of the stream seeded with s is
``mix(s + (i+1) * 0x9E3779B97F4A7C15)`` (counter form of the sequential
generator), with ``seed = 0x5EED0000 + frame_idx``.

kinds:
  rects  horizontal gradient 64->192, then 96 axis-aligned rectangles
         (stream elements 5r..5r+4: x0, x1, y0, y1 mod W/H, value mod 256; later
         rectangles overwrite earlier ones; corners inclusive), then additive
         noise U{-6..6} (element 480 + y*W + x, mod 13, minus 6), clamped.
  pan    temporally correlated stream: frame t shows the rectangles of
         rects frame t - t % 16 (the clip's first frame) shifted right by
         2 * (t % 16) px (clipped at the right edge), over the same
         gradient, with frame t's own noise -- consecutive frames share most
         corners, so SearchByBoW commits hundreds of matches per pair.
  noise  iid U{0..255} (element y*W + x, mod 256).
  flat   constant 128.

The device generator (`orbx_synth_frames`, csrc/kernels_synth.hip) produces
the identical bytes; tests/test_gpu_parity.py checks that.
"""
import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)
SEED_BASE = 0x5EED0000
KINDS = {"rects": 0, "noise": 1, "flat": 2, "pan": 3}
PAN_CLIP, PAN_STEP = 16, 2


def _mix(z):
    z = z.astype(np.uint64, copy=False)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
    return z ^ (z >> np.uint64(31))


def stream(seed, start, count):
    i = np.arange(start + 1, start + count + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return _mix(np.uint64(seed) + i * GOLDEN)


def frame(w, h, frame_idx, kind="rects"):
    seed = SEED_BASE + frame_idx
    if kind == "flat":
        return np.full((h, w), 128, np.uint8)
    if kind == "noise":
        return (stream(seed, 0, w * h) % np.uint64(256)).astype(np.uint8).reshape(h, w)
    if kind not in ("rects", "pan"):
        raise ValueError(kind)
    phase = frame_idx % PAN_CLIP if kind == "pan" else 0
    shift = PAN_STEP * phase
    x = np.arange(w, dtype=np.int64)
    bg = 64 + (128 * x) // max(w - 1, 1)
    img = np.broadcast_to(bg, (h, w)).astype(np.int32).copy()
    r = stream(seed - phase, 0, 5 * 96).reshape(96, 5)
    for x0, x1, y0, y1, v in r:
        x0, x1 = int(x0 % np.uint64(w)), int(x1 % np.uint64(w))
        y0, y1 = int(y0 % np.uint64(h)), int(y1 % np.uint64(h))
        xa = min(x0, x1) + shift
        if xa < w:
            img[min(y0, y1):max(y0, y1) + 1, xa:max(x0, x1) + shift + 1] = int(v % np.uint64(256))
    noise = (stream(seed, 480, w * h) % np.uint64(13)).astype(np.int32).reshape(h, w) - 6
    return np.clip(img + noise, 0, 255).astype(np.uint8)


def stereo_pair(w, h, frame_idx, max_disp=64):
    """Rectified synthetic stereo pair (left, right) for the stereo matcher.

    Same scene model as ``frame(kind="rects")`` with a disparity per object:
    rectangle r (stream elements 5r..5r+4 as in rects) is seen at x - d_r in
    the right image, d_r = element 480 + r mod max_disp; the background
    gradient has disparity 2.  Noise: left element 576 + y*W + x, right
    element 576 + W*H + y*W + x (mod 13, minus 6), independent per image.
    """
    seed = SEED_BASE + frame_idx
    x = np.arange(w, dtype=np.int64)
    bgl = 64 + (128 * x) // max(w - 1, 1)
    bgr = 64 + (128 * (x + 2)) // max(w - 1, 1)
    L = np.broadcast_to(bgl, (h, w)).astype(np.int32).copy()
    R = np.broadcast_to(bgr, (h, w)).astype(np.int32).copy()
    r = stream(seed, 0, 5 * 96).reshape(96, 5)
    disp = stream(seed, 480, 96) % np.uint64(max_disp)
    for (x0, x1, y0, y1, v), d in zip(r, disp):
        x0, x1 = int(x0 % np.uint64(w)), int(x1 % np.uint64(w))
        y0, y1 = int(y0 % np.uint64(h)), int(y1 % np.uint64(h))
        xa, xb, ya, yb, d = min(x0, x1), max(x0, x1), min(y0, y1), max(y0, y1), int(d)
        val = int(v % np.uint64(256))
        L[ya:yb + 1, xa:xb + 1] = val
        ra, rb = max(xa - d, 0), xb - d
        if rb >= 0:
            R[ya:yb + 1, ra:rb + 1] = val
    nl = (stream(seed, 576, w * h) % np.uint64(13)).astype(np.int32).reshape(h, w) - 6
    nr = (stream(seed, 576 + w * h, w * h) % np.uint64(13)).astype(np.int32).reshape(h, w) - 6
    return (np.clip(L + nl, 0, 255).astype(np.uint8), np.clip(R + nr, 0, 255).astype(np.uint8))


def frames(w, h, first_idx, count, kind="rects"):
    return np.stack([frame(w, h, first_idx + i, kind) for i in range(count)])


def vocabulary(k=10, L=6, seed=1, flip=0.2, stop_frac=0.03, prune=0.0):
    """Synthetic DBoW2 vocabulary tree (the reference's ORBvoc.txt is not in
    the tree).  Nodes in breadth-first order (children of a node contiguous,
    parents before children, as loadFromTextFile requires); root children
    are random 32-B descriptors, a child is its parent with each bit flipped
    with probability round(256 * flip) / 256.  Leaves carry idf-like weights in (0.1, 8),
    `stop_frac` of them 0 (stopped words); inner nodes weight 0.  `prune`:
    probability that a node below level 1 gets no children (shallow leaves).
    Returns dict(k, L, parent, is_leaf, desc, weight) of node records."""
    rng = np.random.default_rng(seed)
    parents, descs = [], []
    f_ids = np.zeros(1, np.int64)           # frontier node ids
    f_desc = None                           # frontier descriptors (None = root)
    next_id = 1
    for level in range(1, L + 1):
        if level > 2 and prune > 0:
            keep = rng.uniform(size=len(f_ids)) >= prune
            f_ids, f_desc = f_ids[keep], f_desc[keep]
        n = len(f_ids) * k
        if n == 0:
            break
        par = np.repeat(f_ids, k)
        if f_desc is None:
            cd = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        else:
            bits = rng.integers(0, 256, (n, 256), dtype=np.uint8) < int(round(flip * 256))
            cd = np.repeat(f_desc, k, axis=0) ^ np.packbits(bits, axis=1)
        parents.append(par)
        descs.append(cd)
        f_ids = np.arange(next_id, next_id + n, dtype=np.int64)
        f_desc = cd
        next_id += n
    parent = np.concatenate(parents).astype(np.int32)
    desc = np.concatenate(descs)
    nrec = len(parent)
    has_child = np.zeros(nrec + 1, bool)
    has_child[parent] = True
    is_leaf = (~has_child[1:]).astype(np.int32)
    w = rng.uniform(0.1, 8.0, nrec)
    w[rng.uniform(size=nrec) < stop_frac] = 0.0
    weight = np.where(is_leaf == 1, w, 0.0)
    return dict(k=k, L=L, parent=parent, is_leaf=is_leaf, desc=desc.reshape(nrec, 32),
                weight=weight.astype(np.float64))


def write_vocabulary_text(path, voc, scoring=0, weighting=0):
    """TemplatedVocabulary::saveToTextFile format (TemplatedVocabulary.h:1430-1455)."""
    with open(path, "w") as f:
        f.write("%d %d %d %d\n" % (voc["k"], voc["L"], scoring, weighting))
        for p, l, d, w in zip(voc["parent"], voc["is_leaf"], voc["desc"], voc["weight"]):
            f.write("%d %d %s %s\n" % (p, l, " ".join(str(int(x)) for x in d), repr(float(w))))
