"""CPU tier: the hand-counted vector-memory waits of the product kernels, checked on the compiled gfx950 code.

k_sdt_run (the C4 headline kernel) starts each row with `s_waitcnt vmcnt(5)`: its inputs were loaded during the
previous row, and the only younger vector-memory operations must be that row's five output stores.  k_pinf_recur_ws
(the single-subproblem C1-C3 kernel) publishes a chunk after `vmcnt(8)` (all but the next chunk's first 8 stores)
and completes the next chunk's LDS-DMAs with `vmcnt(56)` (all but the 56 stores issued after them).  Each count is
right only if the compiler emits exactly the vector-memory instructions the source issues there: a scratch spill, a
rematerialised load or one more store turns the wait into a silent race (wrong R or U) or a stall.  So:

  * the kernels have no scratch and no VGPR spills (hipcc -S metadata; no scratch_ instruction);
  * every hand-written counted wait is checked by dataflow over the kernel's control-flow graph
    (scripts/isa_vmcnt.py): on every path, exactly N vector-memory instructions lie between the operations the wait
    must cover and the wait;
  * the check itself is shown to fail when one vector-memory instruction is injected into the loop body.

Sources: mioc_sdt.hip (k_sdt_run), mioc_pinf.hip (k_pinf_recur_ws), compiled with the library's own flags.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mixed-integer-optimal-control---algorithm-tools_amd", "csrc")
sys.path.insert(0, os.path.join(ROOT, "scripts"))
import isa_vmcnt as iv  # noqa: E402

HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", "--offload-arch=gfx950"]
SDT_RUN = "k_sdt_runILi4"
WS = [f"k_pinf_recur_wsILi{cb}" for cb in range(2, 9)]

pytestmark = pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not available")


@pytest.fixture(scope="module")
def listings(tmp_path_factory):
    d = tmp_path_factory.mktemp("isa")
    out = {}
    procs = {}
    for src in ("mioc_sdt.hip", "mioc_pinf.hip"):
        o = str(d / (src + ".s"))
        procs[src] = (subprocess.Popen([HIPCC] + FLAGS + ["-S", "--cuda-device-only", "-o", o, src], cwd=CSRC,
                                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT), o)
    for src, (p, o) in procs.items():
        log = p.communicate(timeout=600)[0]
        assert p.returncode == 0, log.decode()[-2000:]
        out[src] = o
    return out


@pytest.mark.parametrize("sym", [SDT_RUN] + WS)
def test_no_scratch_no_vgpr_spills(listings, sym):
    path = listings["mioc_sdt.hip" if sym == SDT_RUN else "mioc_pinf.hip"]
    meta = iv.kernel_meta(path, sym)
    assert meta.get("private_segment_fixed_size") == 0, meta
    assert meta.get("vgpr_spill_count") == 0, meta
    ins, _ = iv.parse(iv.function_lines(path, sym))
    assert not [t for op, t in ins if op.startswith("scratch_")], "scratch access"


def test_sdt_run_row_start_wait(listings):
    """vmcnt(5) at a row's start: on every path exactly the previous row's 5 stores lie between the last load and the
    wait (6 on wave 0's path through the `done` flag store, which the wait then also covers: safe)."""
    res, bad = iv.check_wait(listings["mioc_sdt.hip"], SDT_RUN, 5, "load", slack=1)
    assert len(res) == 1, res
    assert not bad, bad


@pytest.mark.parametrize("sym", WS)
def test_pinf_ws_chunk_waits(listings, sym):
    path = listings["mioc_pinf.hip"]
    # the next chunk's LDS-DMAs (and the poll) are followed by exactly the chunk's 56 remaining stores
    res, bad = iv.check_wait(path, sym, 56, "load")
    assert len(res) == 1 and not bad, (res, bad)
    # the previous chunk is published once all but this chunk's first 8 stores have landed
    res, bad = iv.check_wait(path, sym, 8, "chunk")
    assert len(res) == 1 and not bad, (res, bad)


def _inject(lines, new, after_op=None, before_wait=None):
    """The listing with `new` inserted after the first instruction whose opcode is after_op, or just before the
    hand-written `s_waitcnt vmcnt(before_wait)`."""
    out, done = [], False
    for q, l in enumerate(lines):
        t = l.split(";")[0].strip()
        if (not done and before_wait is not None and l.strip().startswith(";;#ASMSTART")
                and q + 1 < len(lines) and lines[q + 1].strip() == f"s_waitcnt vmcnt({before_wait})"):
            out.append("\t" + new)
            done = True
        out.append(l)
        if not done and after_op is not None and t.split() and t.split()[0] == after_op:
            out.append("\t" + new)
            done = True
    assert done
    return out


@pytest.mark.parametrize("extra", ["global_load_dword v0, v[0:1], off", "buffer_store_dwordx4 v[0:3], v0, s[0:3], 0 offen"])
def test_guard_catches_one_extra_vm_instruction(listings, extra):
    """One more vector-memory instruction (a load or a store) in k_sdt_run's row body (after its first output store)
    or in k_pinf_recur_ws's unrolled chunk (just before either counted wait) makes the check fail; HEAD passes."""
    lines = iv.function_lines(listings["mioc_sdt.hip"], SDT_RUN)
    assert not iv.check_wait(None, SDT_RUN, 5, "load", slack=1, lines=lines)[1]
    _, bad = iv.check_wait(None, SDT_RUN, 5, "load", slack=1, lines=_inject(lines, extra, after_op="buffer_store_dwordx4"))
    assert bad
    lines = iv.function_lines(listings["mioc_pinf.hip"], WS[1])
    for n, b in ((56, "load"), (8, "chunk")):
        assert not iv.check_wait(None, WS[1], n, b, lines=lines)[1]
        _, bad = iv.check_wait(None, WS[1], n, b, lines=_inject(lines, extra, before_wait=n))
        assert bad, (n, extra)
