"""numpy emulations of the GPU *reformulations* (not of the reference).

The HIP kernels do not run the reference's algorithms literally:
  * k_fast_cells computes one FAST "strength" A(p) per pixel and derives both
    thresholds' corner sets, scores and NMS from it;
  * k_quadtree replaces DistributeOctTree's std::list with per-pass arrays,
    two scans and per-node arg-max.
These emulations restate exactly what the kernels compute so the CPU test
suite can check the reformulations against the oracle (the literal
restatement) on many inputs without a GPU.  Used only by tests/.
"""
import numpy as np

CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3),
          (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def fast_strength(img):
    """A(p) for every pixel with a full 3-px ring (0 elsewhere)."""
    img = img.astype(np.int32)
    h, w = img.shape
    A = np.zeros((h, w), np.int32)
    if h < 7 or w < 7:
        return A
    core = img[3:h - 3, 3:w - 3]
    ring = np.stack([img[3 + dy:h - 3 + dy, 3 + dx:w - 3 + dx] for dx, dy in CIRCLE])
    ext = np.concatenate([ring, ring[:8]])
    mn = np.stack([ext[k:k + 9].min(0) for k in range(16)]).max(0)  # max_arc min
    mx = np.stack([ext[k:k + 9].max(0) for k in range(16)]).min(0)  # min_arc max
    A[3:h - 3, 3:w - 3] = np.maximum(0, np.maximum(mn - core, core - mx))
    return A


def nms_band(Ab, th):
    """cv::FAST NMS on a cell's scan band given A values of the band."""
    bh, bw = Ab.shape
    corner = Ab > th
    buf = np.where(corner, Ab - 1, 0)
    pad = np.zeros((bh + 2, bw + 2), np.int32)
    pad[1:-1, 1:-1] = buf
    keep = corner.copy()
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            if dx == 0 and dy == 0:
                continue
            keep &= buf > pad[1 + dy:1 + dy + bh, 1 + dx:1 + dx + bw]
    return keep, buf


def cell_rects(w, h):
    """ComputeKeyPointsOctTree cell grid (ORBextractor.cc:300-328)."""
    f32 = np.float32
    minB, maxBX, maxBY = 16, w - 16, h - 16
    width, height = f32(maxBX - minB), f32(maxBY - minB)
    nCols, nRows = int(width / f32(30)), int(height / f32(30))
    wCell = int(np.ceil(width / f32(nCols))) if nCols else 0
    hCell = int(np.ceil(height / f32(nRows))) if nRows else 0
    rects = []
    for i in range(nRows):
        iniY = f32(minB + i * hCell)
        maxY = min(f32(iniY + hCell + 6), f32(maxBY))
        for j in range(nCols):
            iniX = f32(minB + j * wCell)
            maxX = min(f32(iniX + wCell + 6), f32(maxBX))
            rects.append((int(iniX), int(iniY), int(maxX - iniX), int(maxY - iniY), i, j, wCell, hCell))
    return rects


def fast_cells(level, ini_th, min_th, cell_guard="empty"):
    """vToDistributeKeys of one level as the kernel computes it: (x_rel, y_rel, score)."""
    h, w = level.shape
    A = fast_strength(level)
    out = []
    for (x, y, cw, ch, i, j, wCell, hCell) in cell_rects(w, h):
        if cw < 0 or ch < 0:
            if cell_guard != "empty":
                raise RuntimeError("negative cell")
            continue
        if cw < 7 or ch < 7:
            continue
        # the cell's A values: FAST reads only the cell, A needs the ring inside the cell
        Ab = A[y + 3:y + ch - 3, x + 3:x + cw - 3]
        keep, buf = nms_band(Ab, ini_th)
        if not keep.any():
            keep, buf = nms_band(Ab, min_th)
        ys, xs = np.nonzero(keep)
        for by, bx in zip(ys, xs):
            out.append((x + 3 + bx - 16, y + 3 + by - 16, int(Ab[by, bx]) - 1))
    return np.array(out, np.int64).reshape(-1, 3)


def quadtree(keys, N, Wr, Hr, max_passes=64):
    """k_quadtree's pass/scan formulation.  keys: (x_rel, y_rel, score) rows in
    vToDistributeKeys order.  Returns the selected rows in output order."""
    C = len(keys)
    nIni = Wr // Hr
    hX = np.float32(np.float32(Wr) / np.float32(nIni if nIni > 0 else 1))
    rect = [(int(np.float32(hX * np.float32(i))), int(np.float32(hX * np.float32(i + 1))), 0, Hr)
            for i in range(nIni)]
    node = np.full(C, -1, np.int64)
    for k in range(C):
        if nIni > 0:
            idx = int(np.float32(np.float32(keys[k, 0]) / hX))
            if 0 <= idx < nIni:
                node[k] = idx
    cnt = np.bincount(node[node >= 0], minlength=len(rect)).tolist() if C else [0] * len(rect)

    def quad(k, r):
        x0, x1, y0, y1 = r
        hx, hy = (x1 - x0) // 2, (y1 - y0) // 2
        return int(keys[k, 0] >= x0 + hx) + 2 * int(keys[k, 1] >= y0 + hy)

    def child(r, q):
        x0, x1, y0, y1 = r
        hx, hy = (x1 - x0) // 2, (y1 - y0) // 2
        nx0, nx1 = (x0 + hx, x1) if q & 1 else (x0, x0 + hx)
        ny0, ny1 = (y0 + hy, y1) if q & 2 else (y0, y0 + hy)
        return (nx0, nx1, ny0, ny1)

    for _ in range(max_passes):
        S = len(rect)
        ch = np.zeros((S, 4), np.int64)
        for k in range(C):
            n = node[k]
            if n >= 0 and cnt[n] >= 2:
                ch[n, quad(k, rect[n])] += 1
        nch = [(int((ch[i] > 0).sum()) if cnt[i] >= 2 else 0) for i in range(S)]
        base = np.zeros(S, np.int64)
        acc = 0
        for i in range(S - 1, -1, -1):  # children of later parents first
            base[i] = acc
            acc += nch[i]
        totC = acc
        kept = np.cumsum([0] + [int(c == 1) for c in cnt])[:-1]
        newS = totC + int(sum(1 for c in cnt if c == 1))
        pos = np.full((S, 4), -1, np.int64)
        nrect = [None] * newS
        ncnt = [0] * newS
        split = False
        for i in range(S):
            if cnt[i] >= 2:
                p = base[i]
                for q in (3, 2, 1, 0):
                    if ch[i, q] > 0:
                        nrect[p] = child(rect[i], q)
                        ncnt[p] = int(ch[i, q])
                        split |= ch[i, q] >= 2
                        pos[i, q] = p
                        p += 1
            elif cnt[i] == 1:
                p = totC + kept[i]
                nrect[p], ncnt[p] = rect[i], 1
                pos[i, 0] = p
        for k in range(C):
            n = node[k]
            if n < 0:
                continue
            node[k] = pos[n, quad(k, rect[n])] if cnt[n] >= 2 else pos[n, 0]
        rect, cnt = nrect, ncnt
        if newS >= N or not split:
            break
    else:
        raise RuntimeError("quadtree does not terminate")
    best = {}
    for k in range(C):
        n = node[k]
        if n < 0:
            continue
        b = best.get(n)
        if b is None or keys[k, 2] > keys[b, 2]:
            best[n] = k
    return np.array([keys[best[i]] for i in range(len(rect))], np.int64).reshape(-1, 3)


def prefilters(img, t):
    """The GPU FAST kernel's two pre-tests (kernels_extract.hip k_fast_strips):
    cardinal (points 0/8 and 4/12) and 4-of-8 even points cyclically
    consecutive; both must hold wherever A > t."""
    img = img.astype(np.int32)
    h, w = img.shape
    core = img[3:h - 3, 3:w - 3]
    ring = [img[3 + dy:h - 3 + dy, 3 + dx:w - 3 + dx] for dx, dy in CIRCLE]
    hi, lo = core + t, core - t
    card = (((ring[0] > hi) | (ring[8] > hi)) & ((ring[4] > hi) | (ring[12] > hi))) | \
           (((ring[0] < lo) | (ring[8] < lo)) & ((ring[4] < lo) | (ring[12] < lo)))
    ev = np.zeros(core.shape, bool)
    for bright in (True, False):
        bits = [(ring[2 * k] > hi) if bright else (ring[2 * k] < lo) for k in range(8)]
        for k in range(8):
            ev |= bits[k] & bits[(k + 1) % 8] & bits[(k + 2) % 8] & bits[(k + 3) % 8]
    return card, ev
