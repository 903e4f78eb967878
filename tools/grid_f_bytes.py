"""Per-source byte model of one k_grid_f launch (verdict item 4: "write a
per-source byte model ... check it against FETCH_SIZE / WRITE_SIZE").

Rebuilds, on the CPU, what one lego substep hands to k_grid_f -- the tiles
(8x8x7 cells) and their <= 256-particle chunks, each chunk's stencil box in
window coordinates (multi-chunk tiles publish whole windows), the touched
tiles (tiles with particles and their upper neighbours, whose low nodes the
stencils reach) -- and replays the kernel's reads in its own order: seven
one-wave workgroups per touched tile, 64 owned nodes a wave, the <= 8 window
reads of each node (zero-slot redirection outside a box), the extra chunks
of multi-chunk tiles, the cover record (64 + 32 dwords by LDS-DMA, each
wave) and the v_out store.  Lines are 128 B.  Workgroup b runs on XCD b % 8,
each XCD has its own L2, so a line is fetched from the fabric once per XCD
that reads it (with enough L2 to keep it, ~2.5 MB a substep here).

Prints the fetched bytes per source at three reuse levels:
  wave   -- every wave fetches every line it touches (no L2 reuse at all),
  xcd    -- a line once per XCD that touches it (the model for FETCH_SIZE),
  global -- a line once (one shared cache; the floor for this slot layout),
and the algorithmic figure (16 B per live cover read, 16 B per stored node).

Usage: python tools/grid_f_bytes.py [--particles 100000] [--n_grid 128]
       [--config lego.json] [--json out.json]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

T = (8, 8, 7)               # kFT0..2
W = (12, 12, 11)            # kFW0..2
FWIN = W[0] * W[1] * W[2]   # 1584 float4 a slot
CHUNK = 256
LINE = 128


def slot_loc(w0, w1, w2):
    return (w0 * W[1] + w1) * W[2] + w2


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--particles", type=int, default=100_000)
    ap.add_argument("--n_grid", type=int, default=128)
    ap.add_argument("--config", default="lego.json")
    ap.add_argument("--json", default=None)
    ap.add_argument("--map", default="cur", choices=["cur", "tile", "spatial"],
                    help="workgroup -> (tile, part) mapping: cur = b = 7 P + part (the kernel's), tile = a tile's "
                         "7 parts on one XCD, spatial = a tile's parts on one XCD and G consecutive touched "
                         "tiles (tile order) an XCD at a time")
    ap.add_argument("--group", type=int, default=4)
    a = ap.parse_args()
    from scenarios import lego_problem
    prob = lego_problem(a.particles, a.n_grid, config=a.config)
    x = prob["x"].astype(np.float32)
    ng = a.n_grid
    inv_dx = np.float32(ng / prob["cfg"]["grid_extent"])
    base = (x * inv_dx - np.float32(0.5)).astype(np.int64)  # truncation, as base_of()
    td = tuple((ng + T[d] - 1) // T[d] for d in range(3))
    tile3 = base // np.array(T)
    tid = (tile3[:, 0] * td[1] + tile3[:, 1]) * td[2] + tile3[:, 2]
    order = np.argsort(tid, kind="stable")
    tid_s, base_s = tid[order], base[order]
    tiles, first, counts = np.unique(tid_s, return_index=True, return_counts=True)
    nch = (counts + CHUNK - 1) // CHUNK
    cbase = np.concatenate([[0], np.cumsum(nch)[:-1]])
    max_chunks = int(nch.sum())
    # per tile: first chunk, chunk count, published box (window coords lo/hi per axis)
    tinfo = {}
    for t, f, c, nc, c0 in zip(tiles, first, counts, nch, cbase):
        t3 = np.array([t // (td[1] * td[2]), (t // td[2]) % td[1], t % td[2]])
        o = t3 * np.array(T) - 1
        if nc > 1:
            lo, hi = np.zeros(3, int), np.array(W) - 1
        else:
            wb = base_s[f:f + c] - o
            lo, hi = wb.min(0), wb.max(0) + 2
        tinfo[int(t)] = (int(c0), int(nc), lo, hi)
    # touched: tiles with particles and their upper neighbours t + {0,1}^3
    touched = set()
    for t in tinfo:
        t3 = (t // (td[1] * td[2]), (t // td[2]) % td[1], t % td[2])
        for d0 in (0, 1):
            for d1 in (0, 1):
                for d2 in (0, 1):
                    u = (t3[0] + d0, t3[1] + d1, t3[2] + d2)
                    if u[0] < td[0] and u[1] < td[1] and u[2] < td[2]:
                        touched.add((u[0] * td[1] + u[1]) * td[2] + u[2])
    touched = sorted(touched)
    zero_off = max_chunks * FWIN
    # touched positions: k_finish_bins scans the touched flags in tile order, so
    # the list is sorted by tile (tiles appended later by k_fused, rare, aside)
    pos = np.arange(len(touched))
    lines_wave = 0
    xcd_lines = [set() for _ in range(8)]
    glob = set()
    live_reads = 0
    stored = 0
    rec_lines_wave = 0
    rec_xcd = [set() for _ in range(8)]
    zero_line = (zero_off * 16) // LINE
    for ti_pos, T_ in zip(pos, touched):
        t3 = (T_ // (td[1] * td[2]), (T_ // td[2]) % td[1], T_ % td[2])
        for part in range(7):
            if a.map == "cur":
                xcd = (ti_pos * 7 + part) % 8
            elif a.map == "tile":
                xcd = ti_pos % 8
            else:
                xcd = (ti_pos // a.group) % 8
            wl = set()
            # cover record (64 dwords) + boxes (32 dwords): 2 + 1 lines per wave
            for r in ((ti_pos * 2 * 32 * 4) // LINE, (ti_pos * 2 * 32 * 4) // LINE + 1,
                      (10**9 + ti_pos * 32 * 4) // LINE):  # (sizes as kRecStride = 32)
                rec_xcd[xcd].add(r)
            rec_lines_wave += 3
            for q in range(64 * part, 64 * part + 64):
                l0, l1, l2 = q // 56, (q // 7) % 8, q % 7
                gi = (t3[0] * 8 + l0, t3[1] * 8 + l1, t3[2] * 7 + l2)
                if max(gi) >= ng:
                    continue
                secs = [(-1 if l < 3 else (1 if l == T[d] - 1 else 0)) for d, l in enumerate((l0, l1, l2))]
                reach = False
                for e in range(8):
                    ax, ay, az = e >> 2, (e >> 1) & 1, e & 1
                    s = (secs[0] if ax else 0, secs[1] if ay else 0, secs[2] if az else 0)
                    if (ax and secs[0] == 0) or (ay and secs[1] == 0) or (az and secs[2] == 0):
                        wl.add(zero_line)  # dead cover: the zero slot
                        continue
                    u3 = (t3[0] + s[0], t3[1] + s[1], t3[2] + s[2])
                    if min(u3) < 0 or u3[0] >= td[0] or u3[1] >= td[1] or u3[2] >= td[2]:
                        wl.add(zero_line)
                        continue
                    u = (u3[0] * td[1] + u3[1]) * td[2] + u3[2]
                    w = (l0 - s[0] * T[0] + 1, l1 - s[1] * T[1] + 1, l2 - s[2] * T[2] + 1)
                    inf = tinfo.get(u)
                    if inf is None or not all(inf[2][d] <= w[d] <= inf[3][d] for d in range(3)):
                        wl.add(zero_line)
                        continue
                    reach = True
                    c0, nc = inf[0], inf[1]
                    for c in range(c0, c0 + nc):
                        wl.add(((c * FWIN + slot_loc(*w)) * 16) // LINE)
                        live_reads += 1
                stored += reach
            lines_wave += len(wl)
            xcd_lines[xcd] |= wl
            glob |= wl
    mb = lambda n: round(n * LINE / 1e6, 3)
    out = {
        "workload": {"config": a.config, "particles": int(len(x)), "n_grid": ng},
        "map": a.map if a.map != "spatial" else f"spatial, {a.group} tiles an XCD at a time",
        "tiles_with_particles": len(tinfo), "touched_tiles": len(touched), "chunks": max_chunks,
        "multi_chunk_tiles": int((nch > 1).sum()),
        "algorithmic_MB": {"live_cover_reads_16B": round(live_reads * 16 / 1e6, 3),
                            "v_out_store_16B": round(stored * 16 / 1e6, 3)},
        "slot_fetch_MB": {"wave": mb(lines_wave), "xcd": mb(sum(len(s) for s in xcd_lines)), "global": mb(len(glob))},
        "record_fetch_MB": {"wave": mb(rec_lines_wave), "xcd": mb(sum(len(s) for s in rec_xcd))},
        "live_covers_per_stored_node": round(live_reads / max(stored, 1), 2),
    }
    print(json.dumps(out, indent=1))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
