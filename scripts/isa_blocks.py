"""Per-basic-block instruction counts of one kernel in a hipcc -S listing (static; no execution counts).

usage: python scripts/isa_blocks.py <file.s> <kernel-symbol-substring> [--from LINE --to LINE]

Prints every block with its VALU / SALU / LDS / vector-memory counts, the s_memtime stamps it holds (diagnostic
builds: MIOC_STAMPS marks the row-body phases), and its branches; used to attribute SQ_INSTS_VALU per row phase.
"""
import re
import sys


def blocks(path, sym):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and sym in l.split(":")[0] and ":" in l)
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    out, cur = [], None
    for i in range(start, end):
        l = lines[i].strip()
        m = re.match(r"^(\.LBB\d+_\d+):", l)
        if m or i == start:
            cur = {"name": m.group(1) if m else "entry", "line": i + 1, "v": 0, "s": 0, "ds": 0, "vm": 0, "mt": 0,
                   "br": []}
            out.append(cur)
            continue
        if not l or l.startswith((";", ".")):
            continue
        op = l.split()[0]
        if op.startswith("v_"):
            cur["v"] += 1
        elif op.startswith("ds_"):
            cur["ds"] += 1
        elif op.startswith(("global_", "buffer_")):
            cur["vm"] += 1
        elif op == "s_memtime":
            cur["mt"] += 1
        if op.startswith("s_cbranch") or op == "s_branch":
            cur["br"].append(l)
        if op.startswith("s_"):
            cur["s"] += 1
    return out


if __name__ == "__main__":
    path, sym = sys.argv[1], sys.argv[2]
    for b in blocks(path, sym):
        print(f"{b['name']:12s} L{b['line']:6d} v={b['v']:4d} s={b['s']:3d} ds={b['ds']:3d} vm={b['vm']:2d} "
              f"mt={b['mt']} {' | '.join(b['br'])}")
