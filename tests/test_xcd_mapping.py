"""The round-6 XCD placements, restated in Python and checked for coverage
(CPU only; the kernels themselves are exercised by the -m gpu parity tests).

* fused.h grid_work: k_grid_f's workgroup b, iteration it -> (touched
  position P, part).  Every (P, part) with P < count must be visited exactly
  once for any grid that is a multiple of 8, and a workgroup's P never
  decreases (it stops at the first P past the count).
* mpm.hip k_chunk_order_xcd: chunk c -> position j * 8 + x on XCD x.  The
  positions 0..nch-1 must all be filled exactly once, each XCD taking its
  equal share, and a chunk stays on its tile's XCD unless that XCD is over
  its share.
"""
import numpy as np
import pytest

PARTS = 7    # kGridParts
GROUP = 16   # kGridGroup
CPX = 32     # CUs an XCD (256 / 8)
KCHUNK = 256


def grid_work(b, it, S, group=GROUP):
    if group == 0:
        wt = b + it * S
        return wt // PARTS, wt % PARTS
    x, m = b & 7, (b >> 3) + it * (S >> 3)
    u = m // PARTS
    k = u // group
    return (k * 8 + x) * group + (u - k * group), m - u * PARTS


@pytest.mark.parametrize("count", [1, 5, 17, 128, 129, 896, 901, 4001])
@pytest.mark.parametrize("S", [8, 64, 7168])
@pytest.mark.parametrize("group", [0, 4, 16])
def test_grid_work_covers_every_item_once(count, S, group):
    seen = np.zeros((count, PARTS), np.int32)
    for b in range(S):
        last = -1
        it = 0
        while True:
            P, part = grid_work(b, it, S, group)
            if P >= count:
                break
            assert P >= last  # monotone: the kernel's early exit is exact
            last = P
            seen[P, part] += 1
            it += 1
    assert (seen == 1).all()


@pytest.mark.parametrize("S", [8, 7168])
def test_grid_work_parts_of_a_tile_share_an_xcd(S):
    """A tile's seven parts (and G consecutive tiles) run on one XCD."""
    xcd_of = {}
    for b in range(S):
        for it in range(4):
            P, part = grid_work(b, it, S)
            xcd_of.setdefault(P, set()).add(b & 7)
    for P, xs in xcd_of.items():
        assert xs == {(P // GROUP) % 8}


def chunk_order_xcd(tiles, sizes, tpos, ntiles):
    """The position of every chunk (k_chunk_order_xcd, one-round grids)."""
    nch = len(tiles)
    T = (nch + 7) // 8
    rem = nch - 8 * (T - 1)
    cap = [T if x < rem else T - 1 for x in range(8)]
    xs = [(tpos[t] // GROUP) % 8 if t < ntiles and tpos[t] >= 0 else c % 8 for c, t in enumerate(tiles)]
    n = [0] * 8
    rank = []
    for x in xs:  # (the kernel ranks by atomics: any order gives the same shares)
        rank.append(n[x])
        n[x] += 1
    dfc = [max(0, cap[x] - n[x]) for x in range(8)]
    pref = np.concatenate([[0], np.cumsum(dfc)])
    k = 0
    for c in range(nch):
        if rank[c] >= cap[xs[c]]:
            y = 0
            while y < 7 and pref[y + 1] <= k:
                y += 1
            xs[c] = y
            k += 1
    # size tiers within each XCD: rank by size (largest first), CPX a tier, every other full tier reversed
    pos = [None] * nch
    for x in range(8):
        members = [c for c in range(nch) if xs[c] == x]
        members.sort(key=lambda c: -sizes[c])
        full = cap[x] // CPX
        for r, c in enumerate(members):
            tier, i = divmod(r, CPX)
            j = tier * CPX + (CPX - 1 - i if (tier & 1) and tier < full else i)
            pos[c] = j * 8 + x
    return pos, xs


@pytest.mark.parametrize("nch", [1, 7, 8, 9, 100, 643, 768, 1203])
def test_chunk_order_xcd_fills_every_position_once(nch):
    rng = np.random.default_rng(nch)
    ntiles = 4864
    # skewed tiles: most chunks in a few touched groups (one XCD over its share)
    tiles = np.sort(rng.integers(0, ntiles // 4, size=nch))
    tpos = -np.ones(ntiles, np.int64)
    uniq = np.unique(tiles)
    tpos[uniq] = np.arange(len(uniq))
    sizes = rng.integers(1, KCHUNK + 1, size=nch)
    pos, xs = chunk_order_xcd(list(tiles), list(sizes), tpos, ntiles)
    assert sorted(pos) == list(range(nch))
    for c in range(nch):
        assert pos[c] % 8 == xs[c]  # position b runs on XCD b % 8
    # a chunk keeps its tile's XCD unless that XCD was over its share
    home = [(tpos[t] // GROUP) % 8 for t in tiles]
    moved = sum(1 for c in range(nch) if xs[c] != home[c])
    counts = np.bincount(home, minlength=8)
    T = (nch + 7) // 8
    assert moved <= int(np.maximum(counts - (T - 1), 0).sum())
