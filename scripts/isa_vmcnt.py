"""Check hand-counted `s_waitcnt vmcnt(N)` waits in a hipcc -S listing (gfx950) by dataflow over the kernel's
instruction-level control-flow graph.

A counted wait vmcnt(N) completes every vector-memory operation except the N youngest (gfx9 family: the counter
retires loads and stores in issue order).  It is correct only if, on every path that reaches it, exactly the
intended operations are among the N youngest -- e.g. k_sdt_run's vmcnt(5) at a row's start must leave the previous
row's five output stores in flight and nothing else: so on every path, the last vector-memory LOAD before the wait is
followed by exactly 5 vector-memory instructions.  A compiler-made scratch spill or reload, a rematerialised load or
an extra store in the loop body changes that count and turns the wait into a silent race (or a stall).

For each wait under test the analysis tracks, per program point, the range [min, max] over all paths of the number of
vector-memory instructions issued since the last "boundary" event (a load for the load-covering waits, or the previous
chunk's closing wait for the store-publishing waits).  Paths on which the boundary has already been waited for by an
earlier wait of the compiler or the source (nothing left to cover) are dropped.  The check: min == N (no path leaves
a covered operation among the N youngest, and the wait does not also cover one of the operations meant to stay in
flight) and max <= N + slack.

usage: python scripts/isa_vmcnt.py <file.s> <kernel-symbol-substring> N boundary   (boundary: load | chunk)
"""
import re
import sys

CAP = 400  # counts above this are "many" (loops of stores): only min matters for them


def function_lines(path, sym):
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and sym in l.split(":")[0])
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    return lines[start + 1:end]


def kernel_meta(path, sym):
    """The kernel's .amdhsa / metadata resource fields (private segment, spills) by symbol substring."""
    text = open(path).read()
    out = {}
    # the per-kernel .set directives of the listing: <sym>.private_seg_size etc.
    for key in ("private_seg_size", "num_vgpr", "num_agpr"):
        mm = re.search(r"\.set\s+(_Z\S*" + re.escape(sym) + r"\S*)\." + key + r",\s*(\d+)", text)
        if mm:
            out[key] = int(mm.group(2))
    # metadata block: vgpr_spill_count / sgpr_spill_count / private_segment_fixed_size
    md = re.search(r"\.name:\s+_Z\S*" + re.escape(sym) + r"\S*\n", text)
    if md:
        blk_start = text.rfind("  - ", 0, md.start())
        blk_end = text.find("\n  - ", md.end())
        blk = text[blk_start:blk_end if blk_end > 0 else len(text)]
        for key in ("private_segment_fixed_size", "vgpr_spill_count", "sgpr_spill_count", "vgpr_count"):
            mm = re.search(r"\." + key + r":\s+(\d+)", blk)
            if mm:
                out[key] = int(mm.group(1))
    return out


def parse(lines, asm_marks=None):
    """Instructions as (op, text) and label -> index; asm_marks (a list) collects the indices of instructions that
    come from the source's inline asm (between the listing's ;;#ASMSTART / ;;#ASMEND markers)."""
    ins, labels = [], {}
    in_asm = False
    for l in lines:
        ls = l.strip()
        if ls.startswith(";;#ASMSTART"):
            in_asm = True
            continue
        if ls.startswith(";;#ASMEND"):
            in_asm = False
            continue
        t = l.split(";")[0].strip()
        if not t:
            continue
        m = re.match(r"^(\.LBB[\w_]+):", t)
        if m:
            labels[m.group(1)] = len(ins)
            continue
        if t.startswith("."):
            continue
        if in_asm and asm_marks is not None:
            asm_marks.append(len(ins))
        ins.append((t.split()[0], t))
    return ins, labels


def is_vm(op):
    return op.startswith(("buffer_", "global_", "flat_", "scratch_"))


def is_load(op):
    return is_vm(op) and ("load" in op or "atomic" in op)


def vmcnt_of(text):
    m = re.search(r"vmcnt\((\d+)\)", text)
    return int(m.group(1)) if m and text.startswith("s_waitcnt") else None


def succs(ins, labels, i):
    op, t = ins[i]
    if op == "s_endpgm":
        return []
    if op == "s_branch":
        return [labels[t.split()[1]]]
    if op.startswith("s_cbranch"):
        return [labels[t.split()[1]], i + 1]
    if op in ("s_setpc_b64", "s_swappc_b64"):
        raise ValueError("calls / indirect branches are not analysed")
    return [i + 1] if i + 1 < len(ins) else []


def analyse(ins, labels, boundary):
    """State before each instruction: None (no path with an uncovered boundary) or (min, max)."""
    n = len(ins)
    state = [None] * n
    work = [0]
    seen = [False] * n
    seen[0] = True

    def merge(a, b):
        if a is None:
            return b
        if b is None:
            return a
        return (min(a[0], b[0]), max(a[1], b[1]))

    def transfer(i, s):
        op, t = ins[i]
        if boundary(op, t):
            return (0, 0)
        if s is None:
            return None
        k = vmcnt_of(t)
        if k is not None:
            # everything older than the k youngest has completed: the boundary op is covered on every path
            # with at least k ops after it (those paths have nothing left to cover)
            if s[0] >= k:
                return None
            return s
        if is_vm(op):
            return (min(s[0] + 1, CAP), min(s[1] + 1, CAP))
        return s

    # entry: nothing outstanding
    inq = set(work)
    while work:
        i = work.pop()
        inq.discard(i)
        out = transfer(i, state[i])
        for j in succs(ins, labels, i):
            nj = merge(state[j], out) if seen[j] else out
            if not seen[j] or nj != state[j]:
                seen[j] = True
                state[j] = nj
                if j not in inq:
                    inq.add(j)
                    work.append(j)
    return state


BOUNDARIES = {
    # the covered operations are loads (and LDS-DMA): the last load issued before the wait
    "load": lambda op, t: is_load(op),
    # the covered operations are everything issued before the current chunk began, which starts after the previous
    # chunk's closing wait (vmcnt(56) / vmcnt(24)) or a full drain
    "chunk": lambda op, t: t.startswith("s_waitcnt") and vmcnt_of(t) in (0, 24, 56),
}


def check_wait(path, sym, N, boundary, slack=None, lines=None):
    """[(index, (min, max))] for every hand-written (inline asm) `s_waitcnt vmcnt(N)` of the kernel, and the failures
    (min != N, or max > N + slack when slack is given).  lines: the function's listing lines (default: from path)."""
    marks = []
    ins, labels = parse(lines if lines is not None else function_lines(path, sym), marks)
    st = analyse(ins, labels, BOUNDARIES[boundary])
    res, bad = [], []
    for i in marks:
        op, t = ins[i]
        if op == "s_waitcnt" and vmcnt_of(t) == N:
            res.append((i, st[i]))
            if st[i] is None or st[i][0] != N or (slack is not None and st[i][1] > N + slack):
                bad.append((i, st[i]))
    return res, bad


def vm_inventory(path, sym):
    ins, _ = parse(function_lines(path, sym))
    inv = {}
    for op, _t in ins:
        if is_vm(op):
            inv[op] = inv.get(op, 0) + 1
    return inv


if __name__ == "__main__":
    p, s, N, b = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    res, bad = check_wait(p, s, N, b, slack=int(sys.argv[5]) if len(sys.argv) > 5 else None)
    print("waits:", res)
    print("failures:", bad)
    print("meta:", kernel_meta(p, s))
    print("vm inventory:", vm_inventory(p, s))
