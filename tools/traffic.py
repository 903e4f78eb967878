"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes into profiles/traffic.json.

    python tools/traffic.py <fetch_pass_dir> <write_pass_dir> [out.json]

Each pass dir holds rocprofv3's run_counter_collection.csv from a separate
`--pmc FETCH_SIZE` / `--pmc WRITE_SIZE` run (never combined with tracing).
Counters are in KiB; FETCH_SIZE is doubled (MI355X_MICROARCH.md, HBM: on gfx950
it reports half the bytes of a wide streaming read).  Averages per dispatch.
"""
import collections
import csv
import json
import os
import sys

# first match wins: k_grid_f before k_grid; k_fused counts its G2P + P2G form (<MAT, 3>) only
KERNELS = ("k_fused", "k_grid_f", "k_p2g", "k_grid", "k_g2p", "k_finish_bins", "k_permute", "k_render",
           "k_preprocess")


def kernel_key(name):
    k = next((k for k in KERNELS if k in name), None)
    if k == "k_fused" and ", 3>" not in name:
        return None
    return k


def per_dispatch(path, counter):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(os.path.join(path, "run_counter_collection.csv"))):
        if r["Counter_Name"] != counter:
            continue
        k = kernel_key(r["Kernel_Name"])
        if k:
            acc[k][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in acc.items()}


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else os.path.join(os.path.dirname(__file__), "..", "profiles", "traffic.json")
    f, w = per_dispatch(fdir, "FETCH_SIZE"), per_dispatch(wdir, "WRITE_SIZE")
    res = {}
    for k in sorted(set(f) | set(w)):
        fb, wb = 2 * 1024 * f.get(k, 0.0), 1024 * w.get(k, 0.0)
        res[k] = {"fetch_bytes": fb, "write_bytes": wb, "bytes_per_launch": fb + wb,
                  "fetch_size_kib_raw": f.get(k), "write_size_kib_raw": w.get(k)}
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    import bench  # source_sha: the kernel sources these counters were measured on
    doc = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes (tools/pmc.sh)",
           "source_sha": bench.source_sha(),
           "correction": "FETCH_SIZE x2 (gfx950), KiB -> bytes",
           # tools/pmc_probe.py's workload (bench.py only uses these numbers for the same one)
           "workload": {"config": os.environ.get("CONFIG", "lego.json"), "particles": int(os.environ.get("N", 100000)),
                        "n_grid": int(os.environ.get("NG", 128)), "material": os.environ.get("MAT") or "jelly"},
           "kernels": res}
    with open(out, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
