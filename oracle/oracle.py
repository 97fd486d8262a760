"""CPU oracle for the bellman_TRM! hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module.  The product (``libmioc.so`` and the ``mioc`` host package) never imports, links or calls it.

Two independent restatements of the reference's algorithm live here:

* ``OracleC``  -- ctypes binding of ``mioc_oracle.c`` (faithful C loops, built by ``oracle/Makefile``);
* ``bellman_py`` / ``backtrack_py`` -- a pure-Python scalar twin of the same loops.

plus an exhaustive-enumeration known-answer generator (``enumerate_kat``) that does not run any DP.

Parity status: **unpinned by the reference itself** -- the reference is Julia 1.10 (Manifest.toml:3),
no Julia toolchain exists in this image and the reference holds no tests or fixtures for this path.
The chain that pins this oracle instead: enumeration KAT (exact rational arithmetic on dyadic
inputs) == Python twin == C oracle, plus the TV_p docstring vectors (HelpFunctions.jl:235-249).

Reference citations (paths relative to the reference root):
  bellman_TRM!        HelpFunctions.jl:20-83
  eval_u_TRM!         HelpFunctions.jl:98-124
  TV_p                HelpFunctions.jl:251-268
  pred (int_val, TV)  multi-trust.jl:117-126;  ared / step decision  multi-trust.jl:127-158
  product_iterator    julia_opt/AdmissibleIterators.jl:9-18
  bounded_sum_iterator/check_sum  julia_opt/AdmissibleIterators.jl:26-49
"""
from __future__ import annotations

import ctypes
import itertools
import math
import os
import subprocess
from fractions import Fraction

import numpy as np

P_INF, P_ONE, P_INTLUT, P_TABLE = 0, 1, 2, 3

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "build", "liboracle.so")


# ----------------------------------------------------------------------------------------------
# admissible-level iterators (restated from julia_opt/AdmissibleIterators.jl)
# ----------------------------------------------------------------------------------------------
def product_tuples(nu):
    """Iterators.product(1:|V_1|, ..., 1:|V_M|): first index fastest (AdmissibleIterators.jl:9-18)."""
    ranges = [range(1, len(v) + 1) for v in nu]
    for t in itertools.product(*reversed(ranges)):
        yield tuple(reversed(t))


def bounded_sum_tuples(nu, lb, ub):
    """Generator filter of product_iterator by lb <= sum nu[m][l[m]] <= ub (AdmissibleIterators.jl:26-49)."""
    for t in product_tuples(nu):
        s = sum(nu[m][t[m] - 1] for m in range(len(nu)))
        if lb <= s <= ub:
            yield t


class Levels:
    """Flattened level table: the iterator's tuples in iteration order (1-based level indices)."""

    def __init__(self, nu, tuples):
        self.nu = [list(map(int, v)) for v in nu]
        self.M = len(self.nu)
        self.counts = np.array([len(v) for v in self.nu], dtype=np.int64)
        self.values = np.array([x for v in self.nu for x in v], dtype=np.int64)
        self.tuples = np.ascontiguousarray(np.array(list(tuples), dtype=np.int32).reshape(-1, self.M))
        self.L = self.tuples.shape[0]
        self.Lgrid = int(np.prod(self.counts))
        strides = np.cumprod(np.concatenate([[1], self.counts[:-1]]))
        self.gidx = ((self.tuples - 1) * strides).sum(axis=1).astype(np.int64)
        self.nuval = np.array([[self.nu[m][t[m] - 1] for m in range(self.M)] for t in self.tuples],
                              dtype=np.int64)

    @staticmethod
    def product(nu):
        return Levels(nu, product_tuples(nu))

    @staticmethod
    def bounded_sum(nu, lb, ub):
        return Levels(nu, bounded_sum_tuples(nu, lb, ub))


# ----------------------------------------------------------------------------------------------
# C oracle (ctypes)
# ----------------------------------------------------------------------------------------------
class _OrLevels(ctypes.Structure):
    _fields_ = [("M", ctypes.c_int64), ("counts", ctypes.c_void_p), ("values", ctypes.c_void_p),
                ("L", ctypes.c_int64), ("tuples", ctypes.c_void_p)]


def build_oracle():
    if not os.path.exists(_LIB) or os.path.getmtime(_LIB) < os.path.getmtime(
            os.path.join(_HERE, "mioc_oracle.c")):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else ctypes.c_void_p(0)


class OracleC:
    def __init__(self):
        self.lib = ctypes.CDLL(build_oracle())
        L = self.lib
        L.oracle_bellman.restype = ctypes.c_int
        L.oracle_bellman.argtypes = [ctypes.POINTER(_OrLevels), ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_int64,
                                     ctypes.c_double, ctypes.c_void_p, ctypes.c_int64, ctypes.c_double,
                                     ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_bellman_mt.restype = ctypes.c_int
        L.oracle_bellman_mt.argtypes = L.oracle_bellman.argtypes + [ctypes.c_int]
        L.oracle_backtrack.restype = ctypes.c_int
        L.oracle_backtrack.argtypes = [ctypes.POINTER(_OrLevels), ctypes.c_void_p, ctypes.c_int64,
                                       ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                       ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
        L.oracle_tv_p.restype = ctypes.c_double
        L.oracle_tv_p.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                  ctypes.c_double]
        L.oracle_bellman_steps.restype = ctypes.c_double
        L.oracle_bellman_steps.argtypes = [ctypes.POINTER(_OrLevels), ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_int64, ctypes.c_int64, ctypes.c_int, ctypes.c_double,
                                           ctypes.c_double, ctypes.c_int64, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_bellman_steps_mt.restype = ctypes.c_double
        L.oracle_bellman_steps_mt.argtypes = L.oracle_bellman_steps.argtypes + [ctypes.c_int]

    @staticmethod
    def _lv(lv):
        s = _OrLevels(lv.M, lv.counts.ctypes.data, lv.values.ctypes.data, lv.L, lv.tuples.ctypes.data)
        return s

    def bellman(self, lv, df, u_old, B, p_kind, beta, dt, p_int=1, wtab=None, threads=1):
        """Returns (phi, U) in the reference layouts: phi (B+1, Lgrid, 2), U (B+1, Lgrid, n-1) (Fortran).
        threads > 1: the target levels of each step split over OpenMP threads (bit-identical result)."""
        df = np.asfortranarray(df, dtype=np.float64)
        u_old = np.asfortranarray(u_old, dtype=np.float64)
        M, n = df.shape
        R = B + 1
        phi = np.zeros((R, lv.Lgrid, 2), dtype=np.float64, order="F")
        U = np.full((R, lv.Lgrid, max(n - 1, 0)), -1, dtype=np.int32, order="F")
        wt = None if wtab is None else np.ascontiguousarray(wtab, dtype=np.float64)
        args = (ctypes.byref(self._lv(lv)), _ptr(df), _ptr(u_old), n, B, p_kind, p_int, beta, _ptr(wt),
                0 if wt is None else wt.size, dt, _ptr(phi), _ptr(U))
        rc = self.lib.oracle_bellman_mt(*args, int(threads)) if threads > 1 else self.lib.oracle_bellman(*args)
        if rc != 0:
            raise OracleError(rc)
        return phi, U

    def backtrack(self, lv, u_old, phi, U, B, Bp):
        u_old = np.asfortranarray(u_old, dtype=np.float64)
        M, n = u_old.shape
        u = np.zeros((M, n), dtype=np.float64, order="F")
        ps = ctypes.c_double(0)
        cs = ctypes.c_int64(0)
        gs = ctypes.c_int64(0)
        rc = self.lib.oracle_backtrack(ctypes.byref(self._lv(lv)), _ptr(u_old), n, B, Bp, _ptr(phi),
                                       _ptr(U), _ptr(u), ctypes.byref(ps), ctypes.byref(cs),
                                       ctypes.byref(gs))
        if rc != 0:
            raise OracleError(rc)
        return u, ps.value

    def tv_p(self, u, p):
        u = np.asfortranarray(u, dtype=np.float64)
        kind = P_INF if p == math.inf else P_ONE
        return self.lib.oracle_tv_p(_ptr(u), u.shape[0], u.shape[1], kind, float(p))

    def bellman_steps(self, lv, df, u_old, B, p_kind, beta, dt, steps, threads=1):
        """Timing leg for bench.py's cpu_baseline (p in {1, Inf}); returns the checksum of the last front.
        threads > 1: OpenMP over the target levels of each step (same result)."""
        df = np.asfortranarray(df, dtype=np.float64)
        u_old = np.asfortranarray(u_old, dtype=np.float64)
        M, n = df.shape
        R = B + 1
        fa = np.empty(R * lv.L, dtype=np.float64)
        fb = np.empty(R * lv.L, dtype=np.float64)
        Us = np.zeros(R * lv.L, dtype=np.uint16)
        args = (ctypes.byref(self._lv(lv)), _ptr(df), _ptr(u_old), n, B, p_kind, beta, dt, steps, _ptr(fa),
                _ptr(fb), _ptr(Us))
        if threads > 1:
            return self.lib.oracle_bellman_steps_mt(*args, int(threads))
        return self.lib.oracle_bellman_steps(*args)


class OracleError(RuntimeError):
    pass


# ----------------------------------------------------------------------------------------------
# pure-Python scalar twin (independent transcription of the same reference loops)
# ----------------------------------------------------------------------------------------------
def _weight(lv, rl, rj, p_kind, p_int, wtab):
    if p_kind == P_INF:
        return 1.0                              # HelpFunctions.jl:63-67 with p = Inf: x^0.0 == 1.0
    if p_kind == P_TABLE:
        return float(wtab[rl * lv.L + rj])
    d = [abs(int(lv.nuval[rj, m]) - int(lv.nuval[rl, m])) for m in range(lv.M)]
    if p_kind == P_ONE:
        s = 0.0
        for x in d:
            s += float(x)
        return s
    return float(wtab[sum(x ** p_int for x in d)])


def bellman_py(lv, df, u_old, B, p_kind, beta, dt, p_int=1, wtab=None):
    """HelpFunctions.jl:20-83 as plain Python loops; same layouts as OracleC.bellman."""
    M, n = df.shape
    R = B + 1
    phi = np.zeros((R, lv.Lgrid, 2))
    U = np.full((R, lv.Lgrid, max(n - 1, 0)), -1, dtype=np.int32)
    buf = (n + 1) % 2
    phi[:, :, buf] = math.inf
    for rl in range(lv.L):
        b, t1 = 0, 0.0
        for m in range(M):
            numl = int(lv.nuval[rl, m])
            t1 += dt * float(df[m, n - 1]) * float(numl)
            x = abs(float(numl) - float(u_old[m, n - 1]))
            if x != math.floor(x):
                raise OracleError(-2)
            b += int(x)
        if b <= B:
            phi[b, lv.gidx[rl], buf] = t1
    for i in range(n - 1, 0, -1):
        w, r = (i + 1) % 2, i % 2
        phi[:, :, w] = math.inf
        for rl in range(lv.L):
            t1, bt = 0.0, 0
            for m in range(M):
                numl = int(lv.nuval[rl, m])
                t1 += dt * float(df[m, i - 1]) * float(numl)
                x = abs(float(numl) - float(u_old[m, i - 1]))
                if x != math.floor(x):
                    raise OracleError(-2)
                bt += int(x)
            gl = lv.gidx[rl]
            for rj in range(lv.L):
                t2 = t1 + beta * _weight(lv, rl, rj, p_kind, p_int, wtab)
                gj = lv.gidx[rj]
                for b in range(0, B - bt + 1):
                    val = t2 + phi[b, gj, r]
                    if phi[b + bt, gl, w] > val:
                        U[b + bt, gl, i - 1] = rj
                        phi[b + bt, gl, w] = val
    return phi, U


def _jl_key(v):
    """Julia findmin order: NaN first, then isless (-0.0 before +0.0)."""
    if math.isnan(v):
        return (0, 0.0, 0)
    return (1, v, 0 if math.copysign(1.0, v) < 0 else 1)


def backtrack_py(lv, u_old, phi, U, B, Bp):
    """HelpFunctions.jl:98-124."""
    M, n = u_old.shape
    best = None
    for g in range(lv.Lgrid):
        for c in range(Bp + 1):
            k = _jl_key(phi[c, g, 0])
            if best is None or k < best[0]:
                best = (k, c, g)
    _, c, g = best
    phistar = phi[c, g, 0]
    if not phistar < math.inf:
        raise OracleError(-5)
    rank_of_g = {int(gg): k for k, gg in enumerate(lv.gidx)}
    q = rank_of_g[g]
    u = np.zeros((M, n))
    u[:, 0] = lv.nuval[q]
    b = c
    for i in range(n - 1):
        q = int(U[b, lv.gidx[q], i])
        u[:, i + 1] = lv.nuval[q]
        b = int(b - sum(abs(u[m, i] - u_old[m, i]) for m in range(M)))
    return u, phistar


def tv_p_py(u, p):
    """TV_p, HelpFunctions.jl:251-268."""
    u = np.asarray(u, dtype=np.float64)
    val = 0.0
    for i in range(1, u.shape[1]):
        d = [abs(float(u[m, i]) - float(u[m, i - 1])) for m in range(u.shape[0])]
        if p == math.inf:
            val += max(d)
        elif p > 0:
            val += sum(x ** p for x in d) ** (1.0 / p)
        else:
            raise ValueError("Only positive integer valued `p` are accepted!")
    return val


def tv_p_kind(u, p_kind, p_int=1, wtab=None, lv=None):
    """TV_p (HelpFunctions.jl:251-268) under mioc_set_cost's weight conventions: p = 1 / Inf computed, integer
    p >= 2 as wtab[sum |d|^p] (Julia's Float64(S)^(1/p), host-supplied), MIOC_P_TABLE as wtab[r_{i-1} L + r_i].
    Summed over i = 2..n in order from 0.0, as the reference's loop."""
    u = np.asarray(u, dtype=np.float64)
    M, n = u.shape
    rank = None
    if p_kind == P_TABLE:
        rank = {tuple(float(x) for x in lv.nuval[r]): r for r in range(lv.L)}
    val = 0.0
    for i in range(1, n):
        d = [abs(float(u[m, i]) - float(u[m, i - 1])) for m in range(M)]
        if p_kind == P_INF:
            t = max(d)
        elif p_kind == P_ONE:
            t = 0.0
            for x in d:
                t += x
        elif p_kind == P_INTLUT:
            t = float(wtab[sum(int(x) ** p_int for x in d)])
        else:
            ra = rank[tuple(float(x) for x in u[:, i - 1])]
            rb = rank[tuple(float(x) for x in u[:, i])]
            t = float(wtab[ra * lv.L + rb])
        val += t
    return val


def _fma(a, b, c):
    """fl(a*b + c) with one rounding (Fraction -> float rounds correctly)."""
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def pred_py(df, u_old, u, dt, beta, tv_old, tv_new, fma=False):
    """multi-trust.jl:117-126: int_val = Δt·Σ_j ∇f[:,j]'(u_old[:,j] − u[:,j]) (j in order, each dot a left-to-right
    sum of products as BLAS ddot's tail loop; fma=True: an FMA-contracted ddot), pred = int_val + β(TV_old − TV_new).
    Returns (int_val, pred)."""
    M, n = df.shape
    int_val = 0.0
    for j in range(n):
        s = 0.0
        for m in range(M):
            v = float(u_old[m, j]) - float(u[m, j])
            s = _fma(float(df[m, j]), v, s) if fma else s + float(df[m, j]) * v
        int_val += s
    int_val *= dt
    return int_val, int_val + beta * (tv_old - tv_new)


def trm_decide_py(J_old, J_new, tv_old, tv_new, pred, beta, sigma):
    """multi-trust.jl:127-158: ared and the decision (2 stop, 1 halve Δ, 0 accept)."""
    ared = J_old - J_new + beta * (tv_old - tv_new)
    return ared, (2 if pred <= 0 else 1 if ared < sigma * pred else 0)


# ----------------------------------------------------------------------------------------------
# exhaustive-enumeration known answers (no DP involved)
# ----------------------------------------------------------------------------------------------
def enumerate_kat(lv, df, u_old, B, Bp, p_kind, beta, dt, p_int=1, wtab=None):
    """Brute-force the trust-region subproblem in exact rational arithmetic.

    Objective of a level sequence r_0..r_{n-1} (what Φ_0 accumulates along a path):
        sum_i Δt·<df_i, ν(r_i)>  +  β · sum_{i<n-1} w(r_i, r_{i+1}),
    subject to the exact budget c = sum_i ||ν(r_i) - u_old_i||_1 <= Bp.
    The DP's pick is the minimiser that is lexicographically smallest in
        (value, grid_index(r_0), c, rank(r_1), ..., rank(r_{n-1}))
    (argmin column-major at HelpFunctions.jl:106, strict `>` over iterator order at :73).
    Valid as a known answer when the inputs are dyadic so the float DP is exact.
    """
    M, n = df.shape
    T1 = [[sum(Fraction(dt) * Fraction(float(df[m, i])) * lv.nuval[r, m] for m in range(M))
           for r in range(lv.L)] for i in range(n)]
    bt = [[int(sum(abs(lv.nuval[r, m] - u_old[m, i]) for m in range(M))) for r in range(lv.L)]
          for i in range(n)]
    W = [[Fraction(beta) * Fraction(_weight(lv, a, b, p_kind, p_int, wtab)) for b in range(lv.L)]
         for a in range(lv.L)]
    best = None
    for seq in itertools.product(range(lv.L), repeat=n):
        c = sum(bt[i][seq[i]] for i in range(n))
        if c > Bp:
            continue
        v = sum(T1[i][seq[i]] for i in range(n)) + sum(W[seq[i]][seq[i + 1]] for i in range(n - 1))
        key = (v, int(lv.gidx[seq[0]]), c) + tuple(seq[1:])
        if best is None or key < best:
            best = key
    seq = (lv.rank_of_grid(best[1]),) + tuple(best[3:])
    u = np.array([[float(lv.nuval[r, m]) for r in seq] for m in range(M)])
    return u, best[0]


def _rank_of_grid(self, g):
    return int(np.nonzero(self.gidx == g)[0][0])


Levels.rank_of_grid = _rank_of_grid
