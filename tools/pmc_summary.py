"""Per-kernel averages of rocprofv3 --pmc passes -> one JSON.

    python tools/pmc_summary.py out.json <pass_dir> [<pass_dir> ...]

Each pass dir holds run_counter_collection.csv from its own --pmc run
(tools/pmc.sh).  Values are averaged per dispatch for each kernel family
(template arguments folded: k_fused<0, 3> and k_fused<0, 2> are reported
apart since the P2G-only / G2P-only forms differ)."""
import collections
import csv
import json
import os
import re
import sys


def family(name):
    name = re.sub(r"\(.*$", "", name)            # drop the argument list
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"gsmpm::", "", name)
    return name.strip()


def main():
    out, dirs = sys.argv[1], sys.argv[2:]
    acc = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    for d in dirs:
        for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
            acc[family(r["Kernel_Name"])][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    res = {}
    for k, cs in sorted(acc.items()):
        res[k] = {c: sum(v.values()) / len(v) for c, v in sorted(cs.items())}
        res[k]["dispatches"] = max(len(v) for v in cs.values())
        if "SQ_LDS_BANK_CONFLICT" in res[k] and res[k].get("SQ_LDS_IDX_ACTIVE"):
            res[k]["lds_conflict_frac"] = res[k]["SQ_LDS_BANK_CONFLICT"] / res[k]["SQ_LDS_IDX_ACTIVE"]
    with open(out, "w") as f:
        json.dump({"source": "rocprofv3 --pmc, separate passes per counter group (tools/pmc.sh)",
                   "per_dispatch_average": res}, f, indent=1)


if __name__ == "__main__":
    main()
