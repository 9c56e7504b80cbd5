"""Host emulation of k_match_cand_mfma's wave-level list maintenance
(kernels_match.hip mfma_tile_pk, MC_TOP3): per lane a sorted top-T list
(T = ORBM_T = 8) of (distance, position) keys below the distance cap; per
tile each lane brings 16 new keys, its three smallest come from two med3
chains and a bitonic half-cleaner, m1 and m2 are inserted in every lane once
any lane needs them, and only when some lane's m3 still beats its last entry
do the remaining keys (the lane's already-inserted ones masked) take the
per-key path.  The result must be the T smallest keys under the cap, as the
plain per-key insertion gives (ORBmatcher.cc:278-366 needs the best and
second-best unmatched candidates in list order)."""
import numpy as np
import pytest

T = 8
BIG = 1 << 40


def med3(a, b, c):
    return max(min(a, b), min(max(a, b), c))


def insert(L, k):
    # kernels_match.hip topk_insert: last slot first, in place
    for t in range(T - 1, 0, -1):
        L[t] = med3(L[t - 1], k, L[t])
    L[0] = min(L[0], k)


def top3(k):
    a1, a2, a3 = min(k[0], k[1]), max(k[0], k[1]), BIG
    b1, b2, b3 = min(k[8], k[9]), max(k[8], k[9]), BIG
    for i in range(2, 8):
        a3, a2, a1 = med3(a2, k[i], a3), med3(a1, k[i], a2), min(a1, k[i])
        b3, b2, b1 = med3(b2, k[8 + i], b3), med3(b1, k[8 + i], b2), min(b1, k[8 + i])
    l1, l2, l3 = min(a1, b3), min(a2, b2), min(a3, b1)
    return min(l1, l2, l3), med3(l1, l2, l3), max(l1, l2, l3)


def wave_tile(Ls, K):
    """One tile for a wave of len(Ls) lanes: Ls[l] sorted lists, K[l] 16 keys."""
    nl = len(Ls)
    m = [top3(K[l]) for l in range(nl)]
    if not any(m[l][0] < Ls[l][T - 1] for l in range(nl)):
        return
    for l in range(nl):
        insert(Ls[l], m[l][0])
    if not any(m[l][1] < Ls[l][T - 1] for l in range(nl)):
        return
    for l in range(nl):
        insert(Ls[l], m[l][1])
    if not any(m[l][2] < Ls[l][T - 1] for l in range(nl)):
        return
    l7 = [Ls[l][T - 1] for l in range(nl)]
    kk = [[k if k > m[l][1] else BIG for k in K[l]] for l in range(nl)]
    for i in range(16):
        if any(kk[l][i] < l7[l] for l in range(nl)):
            for l in range(nl):
                insert(Ls[l], kk[l][i])


@pytest.mark.parametrize("seed", range(4))
def test_top3_wave_insertion_matches_sorted_lists(seed):
    rng = np.random.default_rng(seed)
    for trial in range(300):
        nl = int(rng.integers(1, 9))
        ntile = int(rng.integers(1, 12))
        cap = int(rng.integers(20, 300))  # distance cap: keys below cap << 16 enter
        sent = cap << 16
        Ls = [[sent] * T for _ in range(nl)]
        seen = [[] for _ in range(nl)]
        for t in range(ntile):
            K = []
            for l in range(nl):
                d = rng.integers(0, 320, 16)
                # unique keys: the position (tile, slot) in the low 16 bits
                K.append([int(d[i]) << 16 | (16 * t + i) for i in range(16)])
                seen[l] += K[l]
            wave_tile(Ls, K)
        for l in range(nl):
            want = sorted(k for k in seen[l] if k < sent)[:T]
            want += [sent] * (T - len(want))
            assert Ls[l] == want, (trial, l)
