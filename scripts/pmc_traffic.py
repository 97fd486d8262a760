"""Summarise rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) into HBM bytes per kernel launch.

Usage: python scripts/pmc_traffic.py OUT.json [--qualify KERNEL@CFG:MIN_WGS ...] [CFG:]LABEL=DIR/NAME_counter_collection.csv ...
A CFG: prefix (a pass over one bench config, e.g. `bench.py --config C2 ...`) stores the kernels as "name@CFG".
--qualify KERNEL@CFG:MIN_WGS stores the dispatches of KERNEL with at least MIN_WGS workgroups as "KERNEL@CFG" (one
pass over the default bench holds both the single-subproblem C4 line and the 1024-restart batch lines); several per
kernel split it by grid size (the largest threshold met wins), e.g. k_fsep2@C5x1024:1024 and k_fsep2@C5x128:256.
FETCH_SIZE / WRITE_SIZE are in KiB.  gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE
reports half the bytes of wide reads, so it is doubled; WRITE_SIZE is taken as is.  Both counters
count Infinity-Cache hits as memory-side traffic.
"""
import csv
import json
import sys
from collections import defaultdict


def short(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").strip()
    return n.split("::")[-1].split("<")[0]


def main():
    out = sys.argv[1]
    args = sys.argv[2:]
    qual = {}
    while args and args[0] == "--qualify":
        kc, mw = args[1].rsplit(":", 1)
        kname, kcfg = kc.split("@")
        qual.setdefault(kname, []).append((int(mw), kcfg))  # several per kernel: the largest threshold met wins
        qual[kname].sort(reverse=True)
        args = args[2:]
    res = {}
    for spec in args:
        label, path = spec.split("=", 1)
        cfg = label.split(":", 1)[0] if ":" in label else None
        acc = defaultdict(lambda: defaultdict(list))
        with open(path) as f:
            for row in csv.DictReader(f):
                name = short(row["Kernel_Name"])
                if name in qual:
                    wgs = int(row["Grid_Size"]) // max(1, int(row["Workgroup_Size"]))
                    for mw, qc in qual[name]:
                        if wgs >= mw:
                            name = f"{name}@{qc}"
                            break
                acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
        for k, d in acc.items():
            e = res.setdefault(f"{k}@{cfg}" if cfg and "@" not in k else k, {})
            for cname, vals in d.items():
                scale = 1024.0 * (2.0 if cname == "FETCH_SIZE" else 1.0)
                e[cname.lower() + "_bytes_per_launch"] = scale * sum(vals) / len(vals)
                e["launches_" + cname.lower()] = len(vals)
                e.setdefault("passes", []).append(label)
    for k, e in res.items():
        if "fetch_size_bytes_per_launch" in e and "write_size_bytes_per_launch" in e:
            e["hbm_bytes_per_launch"] = e["fetch_size_bytes_per_launch"] + e["write_size_bytes_per_launch"]
    json.dump({"note": "FETCH_SIZE x2 (gfx950 wide-read correction) + WRITE_SIZE, KiB->bytes, mean per dispatch",
               "kernels": res}, open(out, "w"), indent=1, sort_keys=True)
    for k, e in sorted(res.items()):
        print(k, {kk: (round(v) if isinstance(v, float) else v) for kk, v in e.items()})


if __name__ == "__main__":
    main()
