"""ctypes binding of ``libmioc.so`` (the C ABI declared in ``include/mioc.h``).

This is the product path.  There is no CPU fallback: if the HIP library is missing or no GPU is
visible, every entry point raises ``MiocNativeError``.
"""
from __future__ import annotations

import atexit
import ctypes
import math
import os
import sys
import weakref

import numpy as np

from .iterators import LevelTable

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(_PKG_ROOT, "lib", "libmioc.so")

MIOC_OK = 0
MIOC_EINVAL = -1
MIOC_EINEXACT = -2
MIOC_ENOMEM = -3
MIOC_EHIP = -4
MIOC_EINFEASIBLE = -5
MIOC_ESTATE = -6
MIOC_ENONFINITE = -7

MIOC_P_INF, MIOC_P_ONE, MIOC_P_INTLUT, MIOC_P_TABLE = 0, 1, 2, 3
MIOC_OPT_ALGO, MIOC_OPT_TIMING, MIOC_OPT_PERSIST, MIOC_OPT_PRED_FMA = 1, 2, 3, 4
MIOC_OPT_SPIN_LIMIT, MIOC_OPT_SDT_BUFFERS, MIOC_OPT_FSEP_SEGMENTS, MIOC_OPT_PINF_WALK = 5, 6, 7, 8
MIOC_ALGO_AUTO, MIOC_ALGO_GENERIC, MIOC_ALGO_PINF, MIOC_ALGO_PYRAMID, MIOC_ALGO_SEPARABLE = 0, 1, 2, 3, 4
MIOC_ALGO_FUSED, MIOC_ALGO_FUSED_SEPARABLE = 5, 6
MIOC_ODE_FISHING, MIOC_ODE_DOUBLETANK, MIOC_ODE_VANDERPOL = 1, 2, 3

EXPORTED = [
    "mioc_version", "mioc_create", "mioc_destroy", "mioc_last_error", "mioc_set_option", "mioc_set_levels",
    "mioc_set_cost", "mioc_bellman", "mioc_backtrack", "mioc_bellman_batch_device",
    "mioc_backtrack_batch_device", "mioc_synchronize", "mioc_stream", "mioc_kernel_stats",
    "mioc_reset_stats", "mioc_last_algo", "mioc_diagnostics", "mioc_get_argmin_table", "mioc_get_ranks_device",
    "mioc_pred", "mioc_pred_batch_device", "mioc_tv_device", "mioc_trm_decide_device", "mioc_batch_multi",
    "mioc_ode_eval_device", "mioc_rand_start_device", "mioc_backtrack_batch_budgets_device",
    "mioc_heat_setup", "mioc_heat_eval_device", "mioc_heat_eval",
    "mioc_trm_state_bytes", "mioc_trm_attach", "mioc_trm_outer_begin_device", "mioc_trm_inner_end_device",
    "mioc_trm_poll",
]


class MiocNativeError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"mioc error {code}: {msg}")
        self.code = code


class InexactError(MiocNativeError):
    """Non-integral |ν - u_old| -- the reference's InexactError (HelpFunctions.jl:37,57)."""


_lib = None


def load_library(path=None):
    """Load libmioc.so; raise loudly if it is missing (no silent fallback)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("MIOC_LIB") or LIB_PATH
    if not os.path.exists(p):
        raise MiocNativeError(MIOC_EHIP, f"HIP library not built: {p} (run __graft_entry__.build())")
    # One HIP runtime per process: torch ships its own libamdhip64.so (soname libamdhip64.so.7).
    # Loading torch first makes the dynamic linker bind libmioc's DT_NEEDED libamdhip64.so.7 to that
    # same runtime, so torch tensors / torch.distributed and libmioc share devices and streams.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = ctypes.CDLL(p)
    vp, i32, i64, dbl = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_double
    sig = {
        "mioc_version": (ctypes.c_char_p, []),
        "mioc_create": (i32, [i32, ctypes.POINTER(vp)]),
        "mioc_destroy": (i32, [vp]),
        "mioc_last_error": (ctypes.c_char_p, [vp]),
        "mioc_set_option": (i32, [vp, i32, i64]),
        "mioc_set_levels": (i32, [vp, i64, vp, vp, i64, vp]),
        "mioc_set_cost": (i32, [vp, i32, i64, dbl, i64, vp]),
        "mioc_bellman": (i32, [vp, vp, vp, i64, i64, i64, dbl]),
        "mioc_backtrack": (i32, [vp, i64, vp, ctypes.POINTER(dbl), vp]),
        "mioc_bellman_batch_device": (i32, [vp, i64, vp, vp, i64, i64, i64, dbl]),
        "mioc_backtrack_batch_device": (i32, [vp, i64, vp, vp, vp]),
        "mioc_synchronize": (i32, [vp]),
        "mioc_stream": (vp, [vp]),
        "mioc_kernel_stats": (i32, [vp, i32, ctypes.POINTER(dbl), ctypes.POINTER(i64),
                                    ctypes.POINTER(ctypes.c_char_p)]),
        "mioc_reset_stats": (i32, [vp]),
        "mioc_last_algo": (i32, [vp]),
        "mioc_diagnostics": (i32, [vp, vp, i32]),
        "mioc_get_argmin_table": (i32, [vp, i64, i64, vp]),
        "mioc_get_ranks_device": (i32, [vp, vp]),
        "mioc_pred": (i32, [vp, ctypes.POINTER(dbl), ctypes.POINTER(dbl), ctypes.POINTER(dbl),
                            ctypes.POINTER(dbl)]),
        "mioc_pred_batch_device": (i32, [vp, vp, vp, vp, vp]),
        "mioc_tv_device": (i32, [vp, i64, vp, i64, i64, vp]),
        "mioc_trm_decide_device": (i32, [vp, i64, vp, vp, vp, vp, vp, dbl, vp, vp]),
        "mioc_batch_multi": (i32, [vp, i32, i64, vp, vp, i64, i64, i64, dbl, i64, vp, vp, vp]),
        "mioc_ode_eval_device": (i32, [vp, i32, i64, vp, i64, i64, dbl, dbl, vp, i32, vp, vp]),
        "mioc_rand_start_device": (i32, [vp, i64, i64, i64, ctypes.c_uint64, vp]),
        "mioc_backtrack_batch_budgets_device": (i32, [vp, vp, vp, vp, vp]),
        "mioc_heat_setup": (i32, [vp, i64, i64, i64, dbl, dbl, dbl, vp, vp, vp, vp, vp]),
        "mioc_heat_eval_device": (i32, [vp, i64, vp, vp, vp]),
        "mioc_heat_eval": (i32, [vp, i64, vp, vp, vp]),
        "mioc_trm_state_bytes": (i64, [i64]),
        "mioc_trm_attach": (i32, [vp, vp]),
        "mioc_trm_outer_begin_device": (i32, [vp, i64, vp, vp, dbl, i64, vp]),
        "mioc_trm_inner_end_device": (i32, [vp, i64, vp, dbl, i64, dbl, i64, vp, vp, vp, vp, vp, vp, vp, vp, i64, vp,
                                            vp, vp]),
        "mioc_trm_poll": (i32, [vp, vp, vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    if path is None:
        _lib = lib
    return lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def cost_spec(p, L=None, levels=None):
    """Map the reference's ``p`` (Int, Float64 or Inf; multi-trust.jl:28) to (p_kind, p_int, table).

    p = Inf and p = 1 are exact on the device.  For other p the weight (sum |d|^p)^(1/p) uses
    Julia's own ``^`` in the reference; here the host supplies it (computed with Python's pow unless a
    caller passes Julia's values) -- parity for p not in {1, Inf} is unpinned.
    """
    if p == math.inf:
        return MIOC_P_INF, 1, None
    if float(p) == 1.0:
        return MIOC_P_ONE, 1, None
    if float(p) == int(p) and 2 <= int(p) <= 8:
        pi = int(p)
        maxkey = sum(int(max(v) - min(v)) ** pi for v in levels.nu)
        return MIOC_P_INTLUT, pi, np.array([float(s) ** (1.0 / pi) for s in range(maxkey + 1)])
    if not p > 0:
        raise ValueError("Only positive integer valued `p` are accepted!")
    nv = levels.nuval
    d = np.abs(nv[:, None, :] - nv[None, :, :]) ** float(p)
    return MIOC_P_TABLE, 1, np.ascontiguousarray((d.sum(axis=2) ** (1.0 / float(p))).reshape(-1))


_LIVE = weakref.WeakSet()  # contexts not yet closed


@atexit.register
def _close_live_contexts():
    """Destroy every context still open while the HIP runtime is alive: atexit handlers run before the C
    runtime's exit() tears down libamdhip64's static state, whereas a __del__ reached during interpreter
    finalisation (or from a garbage cycle collected then) can run after it ('What's weak' 5)."""
    for c in list(_LIVE):
        try:
            c.close()
        except Exception:
            pass


class Context:
    """One device context: levels + cost + the resident DP (fronts / argmin table / class tables).

    Close it explicitly (``close()`` or ``with Context(0) as ctx:``); contexts left open are closed by an atexit
    handler, never from ``__del__`` during interpreter shutdown."""

    def __init__(self, device=0):
        self.h = None
        self.lib = load_library()
        h = ctypes.c_void_p()
        rc = self.lib.mioc_create(int(device), ctypes.byref(h))
        if rc != MIOC_OK:
            raise MiocNativeError(rc, f"mioc_create(device={device}) failed (no visible HIP device?)")
        self.h = h
        self.device = int(device)
        self.levels = None
        self.M = None
        self.nt = None
        self.B = None
        _LIVE.add(self)

    def close(self):
        if self.h:
            h, self.h = self.h, None
            _LIVE.discard(self)
            self.lib.mioc_destroy(h)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def __del__(self, _finalizing=sys.is_finalizing):
        # an unreferenced context is destroyed while the program runs; at shutdown the atexit handler has
        # already closed it, and a HIP call from a finaliser that runs after the runtime's teardown is unsafe
        # (the default argument keeps the check usable after the sys module is torn down)
        if _finalizing():
            return
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != MIOC_OK:
            msg = self.lib.mioc_last_error(self.h).decode()
            if rc == MIOC_EINEXACT:
                raise InexactError(rc, msg)
            raise MiocNativeError(rc, msg)

    def set_option(self, option, value):
        self._check(self.lib.mioc_set_option(self.h, option, int(value)))

    def set_levels(self, levels: LevelTable):
        self.levels = levels
        self.M = levels.M
        self._check(self.lib.mioc_set_levels(self.h, levels.M, _p(levels.counts), _p(levels.values),
                                             levels.L, _p(levels.tuples)))

    def set_cost(self, p, beta, table=None, p_int=None, p_kind=None):
        if p_kind is None:
            p_kind, p_int, tab = cost_spec(p, levels=self.levels)
            if table is not None:
                tab = np.ascontiguousarray(table, dtype=np.float64)
        else:
            tab = None if table is None else np.ascontiguousarray(table, dtype=np.float64)
            p_int = p_int or 1
        self._tab = tab
        self._check(self.lib.mioc_set_cost(self.h, p_kind, int(p_int), float(beta),
                                           0 if tab is None else tab.size,
                                           None if tab is None else _p(tab)))

    # -- host-buffer API (Julia-style: ∇f and u_old are nx x nt, column-major) --------------
    def bellman(self, df, u_old, B, dt):
        df = np.asfortranarray(df, dtype=np.float64)
        u_old = np.asfortranarray(u_old, dtype=np.float64)
        if df.shape != u_old.shape:
            raise ValueError("df and u_old must have the same shape (nx, nt)")
        nx, nt = df.shape
        self.nt, self.B = nt, int(B)
        self._check(self.lib.mioc_bellman(self.h, _p(df), _p(u_old), nx, nt, int(B), float(dt)))

    def backtrack(self, B_use=None):
        if self.nt is None:  # no DP yet: let the library report the state error (MIOC_ESTATE)
            dummy = np.zeros(1, dtype=np.float64)
            self._check(self.lib.mioc_backtrack(self.h, 0 if B_use is None else int(B_use), _p(dummy),
                                                None, None))
        B_use = self.B if B_use is None else int(B_use)
        u = np.zeros((self.M, self.nt), dtype=np.float64, order="F")
        ps = ctypes.c_double(0.0)
        sw = np.zeros(self.nt, dtype=np.uint8)
        self._check(self.lib.mioc_backtrack(self.h, B_use, _p(u), ctypes.byref(ps), _p(sw)))
        return u, ps.value, sw.astype(bool)

    # -- device-resident batch API (pointers are device addresses, e.g. torch .data_ptr()) ----
    def bellman_batch_device(self, K, df_ptr, uold_ptr, nx, nt, B, dt):
        self.nt, self.B = nt, int(B)
        self._check(self.lib.mioc_bellman_batch_device(self.h, int(K), ctypes.c_void_p(df_ptr),
                                                       ctypes.c_void_p(uold_ptr), int(nx), int(nt), int(B),
                                                       float(dt)))

    def backtrack_batch_device(self, B_use, u_ptr, phi_ptr=0, status_ptr=0):
        self._check(self.lib.mioc_backtrack_batch_device(self.h, int(B_use), ctypes.c_void_p(u_ptr),
                                                         ctypes.c_void_p(phi_ptr or None),
                                                         ctypes.c_void_p(status_ptr or None)))

    # -- the same, from torch tensors (shape/contiguity checked: the raw-pointer API cannot check) --
    def bellman_batch_tensors(self, df, u_old, B, dt):
        """df, u_old: float64 CUDA tensors of shape (K, nt, nx), C-contiguous (each subproblem's nx x nt
        column-major block, the layout of mioc_bellman_batch_device)."""
        for name, t in (("df", df), ("u_old", u_old)):
            if t.dim() != 3 or not t.is_contiguous() or not t.is_cuda or str(t.dtype) != "torch.float64":
                raise ValueError(f"{name} must be a contiguous float64 CUDA tensor of shape (K, nt, nx)")
        if tuple(df.shape) != tuple(u_old.shape):
            raise ValueError("df and u_old must have the same shape (K, nt, nx)")
        K, nt, nx = df.shape
        self.bellman_batch_device(K, df.data_ptr(), u_old.data_ptr(), nx, nt, B, dt)

    def backtrack_batch_tensors(self, B_use, u, phi=None, status=None):
        """u: float64 CUDA tensor (K, nt, nx), contiguous; phi: (K,) float64; status: (K,) int32."""
        if u.dim() != 3 or not u.is_contiguous() or not u.is_cuda or str(u.dtype) != "torch.float64":
            raise ValueError("u must be a contiguous float64 CUDA tensor of shape (K, nt, nx)")
        for name, t, dt_ in (("phi", phi, "torch.float64"), ("status", status, "torch.int32")):
            if t is not None and (not t.is_contiguous() or str(t.dtype) != dt_ or t.numel() != u.shape[0]):
                raise ValueError(f"{name} must be a contiguous {dt_} tensor with K entries")
        self.backtrack_batch_device(B_use, u.data_ptr(), 0 if phi is None else phi.data_ptr(),
                                    0 if status is None else status.data_ptr())

    def backtrack_batch_budgets_tensors(self, budgets, u, phi=None, status=None):
        """eval_u_TRM! with one budget per subproblem: budgets (K,) int32 CUDA tensor (each <= B); u (K, nt, nx)
        float64 CUDA tensor; phi, status optional (mioc_backtrack_batch_budgets_device)."""
        if u.dim() != 3 or not u.is_contiguous() or not u.is_cuda or str(u.dtype) != "torch.float64":
            raise ValueError("u must be a contiguous float64 CUDA tensor of shape (K, nt, nx)")
        if not budgets.is_cuda or str(budgets.dtype) != "torch.int32" or not budgets.is_contiguous() or \
                budgets.numel() != u.shape[0]:
            raise ValueError("budgets must be a contiguous int32 CUDA tensor with K entries")
        for name, t, dt_ in (("phi", phi, "torch.float64"), ("status", status, "torch.int32")):
            if t is not None and (not t.is_contiguous() or str(t.dtype) != dt_ or t.numel() != u.shape[0]):
                raise ValueError(f"{name} must be a contiguous {dt_} tensor with K entries")
        self._check(self.lib.mioc_backtrack_batch_budgets_device(
            self.h, ctypes.c_void_p(budgets.data_ptr()), ctypes.c_void_p(u.data_ptr()),
            ctypes.c_void_p(phi.data_ptr()) if phi is not None else None,
            ctypes.c_void_p(status.data_ptr()) if status is not None else None))

    def ranks_tensor(self, out):
        """Level ranks (iterator order) of the last backtrack into `out`, an int32 CUDA tensor (K, nt)."""
        if not out.is_cuda or str(out.dtype) != "torch.int32" or not out.is_contiguous():
            raise ValueError("out must be a contiguous int32 CUDA tensor (K, nt)")
        self._check(self.lib.mioc_get_ranks_device(self.h, ctypes.c_void_p(out.data_ptr())))

    # -- trust-region quantities of the last backtrack (multi-trust.jl:117-158) -------------------
    def pred(self):
        """(int_val, TV_p(u_old), TV_p(u), pred) of the last single-subproblem backtrack, on the device."""
        out = [ctypes.c_double(0.0) for _ in range(4)]
        self._check(self.lib.mioc_pred(self.h, *[ctypes.byref(x) for x in out]))
        return tuple(x.value for x in out)

    def pred_batch_tensors(self, int_val=None, tv_old=None, tv_new=None, pred=None):
        """Per-subproblem int_val / TV_p(u_old) / TV_p(u) / pred of the last batch backtrack into (K,) float64
        CUDA tensors (each optional); enqueued on the context's stream."""
        for name, t in (("int_val", int_val), ("tv_old", tv_old), ("tv_new", tv_new), ("pred", pred)):
            if t is not None and (not t.is_cuda or not t.is_contiguous() or str(t.dtype) != "torch.float64"):
                raise ValueError(f"{name} must be a contiguous float64 CUDA tensor (K,)")
        ptr = [ctypes.c_void_p(t.data_ptr()) if t is not None else None for t in (int_val, tv_old, tv_new, pred)]
        self._check(self.lib.mioc_pred_batch_device(self.h, *ptr))

    def tv_tensors(self, u, out):
        """TV_p of controls u (K, nt, nx) float64 CUDA tensor into out (K,) float64; enqueued."""
        if u.dim() != 3 or not u.is_contiguous() or not u.is_cuda or str(u.dtype) != "torch.float64":
            raise ValueError("u must be a contiguous float64 CUDA tensor of shape (K, nt, nx)")
        if not out.is_cuda or not out.is_contiguous() or str(out.dtype) != "torch.float64" or \
                out.numel() != u.shape[0]:
            raise ValueError("out must be a contiguous float64 CUDA tensor (K,)")
        K, nt, nx = u.shape
        self._check(self.lib.mioc_tv_device(self.h, K, ctypes.c_void_p(u.data_ptr()), nx, nt,
                                            ctypes.c_void_p(out.data_ptr())))

    # ---- device-resident TRM control (multi-trust.jl:92-163; include/mioc.h) ----------------------------------
    def trm_state_tensor(self, K):
        """A zero-initialised device state block for K restarts (uint8 CUDA tensor)."""
        import torch
        n = int(self.lib.mioc_trm_state_bytes(int(K)))
        if n < 0:
            raise ValueError("K must be in [1, 4096]")
        return torch.zeros(n, dtype=torch.uint8, device=f"cuda:{self.device}")

    def trm_attach(self, state):
        """Gate the inner-loop kernels by the state's gate word (None detaches)."""
        self._check(self.lib.mioc_trm_attach(self.h, ctypes.c_void_p(state.data_ptr()) if state is not None else None))

    def trm_outer_begin(self, state, tv_u, D0, B, budgets):
        K = tv_u.numel()
        self._check(self.lib.mioc_trm_outer_begin_device(self.h, K, ctypes.c_void_p(state.data_ptr()),
                                                          ctypes.c_void_p(tv_u.data_ptr()), float(D0), int(B),
                                                          ctypes.c_void_p(budgets.data_ptr())))

    def trm_inner_end(self, state, sigma, kmax, tau, B, int_val, tv_new, J_new, J_old, J, tv_u, budgets, trial, u,
                      u_old, decision=None):
        K = J.numel()
        p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        self._check(self.lib.mioc_trm_inner_end_device(
            self.h, K, p(state), float(sigma), int(kmax), float(tau), int(B), p(int_val), p(tv_new), p(J_new),
            p(J_old), p(J), p(tv_u), p(budgets), p(decision) if decision is not None else None,
            u[0].numel(), p(trial), p(u), p(u_old)))

    def trm_state_arrays(self, state, K):
        """The state block on the host: Δᵏ, TV_old, k, flags (1 inner, 2 halved, 4 stopped), outer iterations."""
        self.synchronize()
        b = state.cpu().numpy()
        o = 16
        out = {}
        for name, dt in (("Dk", np.float64), ("tv_old", np.float64), ("k", np.int32), ("flags", np.int32),
                         ("iters", np.int32)):
            n = K * np.dtype(dt).itemsize
            out[name] = b[o:o + n].view(dt).copy()
            o += n
        return out

    def trm_poll(self, state):
        """Synchronise once; (any restart inside its inner loop, any restart not stopped)."""
        out = np.zeros(2, dtype=np.int32)
        self._check(self.lib.mioc_trm_poll(self.h, ctypes.c_void_p(state.data_ptr()), _p(out)))
        return bool(out[0]), bool(out[1])

    def trm_decide_tensors(self, J_old, J_new, tv_old, tv_new, pred, sigma, decision, ared=None):
        """multi-trust.jl:127-158 per subproblem: decision (K,) int32 = 2 stop / 1 halve / 0 accept."""
        ts = (J_old, J_new, tv_old, tv_new, pred)
        K = decision.numel()
        for t in ts + ((ared,) if ared is not None else ()):
            if not t.is_cuda or not t.is_contiguous() or str(t.dtype) != "torch.float64" or t.numel() != K:
                raise ValueError("J_old / J_new / tv_old / tv_new / pred / ared: contiguous float64 (K,)")
        if not decision.is_cuda or str(decision.dtype) != "torch.int32" or not decision.is_contiguous():
            raise ValueError("decision must be a contiguous int32 CUDA tensor (K,)")
        self._check(self.lib.mioc_trm_decide_device(
            self.h, K, *[ctypes.c_void_p(t.data_ptr()) for t in ts], float(sigma),
            ctypes.c_void_p(ared.data_ptr()) if ared is not None else None, ctypes.c_void_p(decision.data_ptr())))

    def ode_eval_tensors(self, problem, x, T0, T1, J=None, df=None, params=None):
        """eval_f! / eval_df! of an ODE example for K controls x (K, nt, 3) float64 CUDA tensor: J (K,) and df
        (K, nt, 3) float64 CUDA tensors (each optional); enqueued (mioc_ode_eval_device)."""
        if x.dim() != 3 or not x.is_contiguous() or not x.is_cuda or str(x.dtype) != "torch.float64":
            raise ValueError("x must be a contiguous float64 CUDA tensor of shape (K, nt, nx)")
        K, nt, nx = x.shape
        for name, t, n in (("J", J, K), ("df", df, x.numel())):
            if t is not None and (not t.is_cuda or not t.is_contiguous() or str(t.dtype) != "torch.float64" or
                                  t.numel() != n):
                raise ValueError(f"{name} must be a contiguous float64 CUDA tensor with {n} entries")
        par = None if params is None else np.ascontiguousarray(params, dtype=np.float64)
        self._check(self.lib.mioc_ode_eval_device(
            self.h, int(problem), K, ctypes.c_void_p(x.data_ptr()), nx, nt, float(T0), float(T1),
            None if par is None else _p(par), 0 if par is None else par.size,
            ctypes.c_void_p(J.data_ptr()) if J is not None else None,
            ctypes.c_void_p(df.data_ptr()) if df is not None else None))

    def heat_setup(self, M_invA, M_invF, mass, state0, yd, T0, T1, gamma):
        """Hand the heat objective's matrices to the device (mioc_heat_setup; example_heat.jl:101-115): M_invA, mass
        (N, N), M_invF (N, nx), state0 (N,), yd (N, nt+1) as numpy arrays; nt = yd.shape[1] - 1."""
        f = lambda a: np.asfortranarray(a, dtype=np.float64)  # noqa: E731  (column-major, Julia's layout)
        A, F, Mm, y0, Yd = f(M_invA), f(M_invF), f(mass), f(state0), f(yd)
        N, nx = F.shape
        nt = Yd.shape[1] - 1
        if A.shape != (N, N) or Mm.shape != (N, N) or y0.shape != (N,) or Yd.shape[0] != N:
            raise ValueError("heat matrices: M_invA, mass (N, N); M_invF (N, nx); state0 (N,); yd (N, nt+1)")
        self._check(self.lib.mioc_heat_setup(self.h, N, nx, nt, float(T0), float(T1), float(gamma),
                                             _p(A), _p(F), _p(Mm), _p(y0), _p(Yd)))
        self.heat_shape = (N, nx, nt)

    def heat_eval_tensors(self, x, J=None, df=None):
        """eval_f / eval_df of the heat objective for K controls x (K, nt, nx) float64 CUDA tensor into J (K,) and
        df (K, nt, nx) float64 CUDA tensors (each optional); enqueued (mioc_heat_eval_device)."""
        if x.dim() != 3 or not x.is_contiguous() or not x.is_cuda or str(x.dtype) != "torch.float64":
            raise ValueError("x must be a contiguous float64 CUDA tensor of shape (K, nt, nx)")
        K, nt, nx = x.shape
        if getattr(self, "heat_shape", None) is None or self.heat_shape[1:] != (nx, nt):
            raise ValueError("x does not match the (nx, nt) given to heat_setup")
        for name, t, n in (("J", J, K), ("df", df, x.numel())):
            if t is not None and (not t.is_cuda or not t.is_contiguous() or str(t.dtype) != "torch.float64" or
                                  t.numel() != n):
                raise ValueError(f"{name} must be a contiguous float64 CUDA tensor with {n} entries")
        self._check(self.lib.mioc_heat_eval_device(
            self.h, K, ctypes.c_void_p(x.data_ptr()),
            ctypes.c_void_p(J.data_ptr()) if J is not None else None,
            ctypes.c_void_p(df.data_ptr()) if df is not None else None))

    def heat_eval(self, xs):
        """Host entry (mioc_heat_eval): xs (K, nx, nt) numpy controls (Julia's per-restart layout) -> J (K,),
        df (K, nx, nt)."""
        x = np.ascontiguousarray(np.asarray(xs, dtype=np.float64).transpose(0, 2, 1))  # K x (nx x nt col-major)
        K, nt, nx = x.shape
        if getattr(self, "heat_shape", None) is None or self.heat_shape[1:] != (nx, nt):
            raise ValueError("xs does not match the (nx, nt) given to heat_setup")
        J = np.empty(K)
        df = np.empty_like(x)
        self._check(self.lib.mioc_heat_eval(self.h, K, _p(x), _p(J), _p(df)))
        return J, df.transpose(0, 2, 1)

    def rand_start_tensor(self, out, seed, jumps=-1):
        """rand_func_int (HelpFunctions.jl:204-225) for K restarts into out, a (K, nt, M) float64 CUDA tensor;
        jumps < 0: floor(nt / 10).  Enqueued (mioc_rand_start_device)."""
        if out.dim() != 3 or not out.is_contiguous() or not out.is_cuda or str(out.dtype) != "torch.float64":
            raise ValueError("out must be a contiguous float64 CUDA tensor of shape (K, nt, M)")
        K, nt, M = out.shape
        if M != self.M:
            raise ValueError("out's last dimension must be the levels' M")
        self._check(self.lib.mioc_rand_start_device(self.h, K, nt, int(jumps), ctypes.c_uint64(int(seed)),
                                                    ctypes.c_void_p(out.data_ptr())))

    def synchronize(self):
        self._check(self.lib.mioc_synchronize(self.h))

    def stream(self):
        return self.lib.mioc_stream(self.h)

    def kernel_stats(self, which=0):
        ms = ctypes.c_double(0)
        n = ctypes.c_int64(0)
        name = ctypes.c_char_p()
        self._check(self.lib.mioc_kernel_stats(self.h, int(which), ctypes.byref(ms), ctypes.byref(n),
                                               ctypes.byref(name)))
        return ms.value, n.value, (name.value or b"").decode()

    def reset_stats(self):
        self._check(self.lib.mioc_reset_stats(self.h))

    def last_algo(self):
        return self.lib.mioc_last_algo(self.h)

    def argmin_table(self, step, k=0):
        """U of step `step` in the reference layout: int32 (B+1, Lgrid), rank of the minimising source
        (mioc_get_argmin_table; cells with Φ = +Inf are -1 below b̃ and unspecified above)."""
        lg = int(np.prod(self.levels.counts))
        out = np.empty((lg, self.B + 1), dtype=np.int32)
        self._check(self.lib.mioc_get_argmin_table(self.h, int(k), int(step), _p(out)))
        return out.T

    def diagnostics(self):
        """[value-collision targets scanned, multi-level targets scanned, p=Inf walk fallbacks or U-table walk
        run-ahead rounds, errors,
        hash-overflow rows, targets whose value was not found, values flagged colliding (persistent / segmented DPs
        redone), occupancy, fused separable row segments, p=Inf segmented walk: subproblems walked serially]
        (include/mioc.h)."""
        out = np.zeros(10, dtype=np.int64)
        self._check(self.lib.mioc_diagnostics(self.h, _p(out), 10))
        return out.tolist()


def batch_multi(ctxs, df, u_old, B, dt, B_use=None):
    """mioc_batch_multi: K subproblems (host float64 arrays of shape (K, nt, nx), C-contiguous) split over the
    contexts (one per device, levels and cost set), each block solved from its own host thread.
    Returns (u (K, nt, nx), phi_star (K,), status (K,))."""
    df = np.ascontiguousarray(df, dtype=np.float64)
    u_old = np.ascontiguousarray(u_old, dtype=np.float64)
    if df.ndim != 3 or df.shape != u_old.shape:
        raise ValueError("df and u_old must have the same shape (K, nt, nx)")
    K, nt, nx = df.shape
    u = np.empty_like(df)
    phi = np.empty(K, dtype=np.float64)
    st = np.empty(K, dtype=np.int32)
    arr = (ctypes.c_void_p * len(ctxs))(*[c.h.value for c in ctxs])
    lib = ctxs[0].lib
    rc = lib.mioc_batch_multi(arr, len(ctxs), K, _p(df), _p(u_old), nx, nt, int(B), float(dt),
                              int(B if B_use is None else B_use), _p(u), _p(phi), _p(st))
    ctxs[0]._check(rc)
    return u, phi, st


def pyramid_eligible(levels: LevelTable):
    """Mirror of the library's L1-ball pyramid domain test (mioc_set_levels)."""
    if levels.L != int(np.prod(levels.counts)) or not (2 <= levels.M <= 6) or levels.L > 4096:
        return False
    if int(levels.counts[0]) not in (4, 8) or levels.L // int(levels.counts[0]) > 512:
        return False
    strides = np.cumprod(np.concatenate([[1], levels.counts[:-1]]))
    if not np.array_equal(((levels.tuples - 1) * strides).sum(axis=1), np.arange(levels.L)):
        return False
    return all(list(v) == list(range(v[0], v[0] + len(v))) for v in levels.nu)


def fused_eligible(L, B):
    """Mirror of the library's fused small-state domain (mioc_fused.hip fused_supported): L <= 64 levels, at
    most 192 (64-row block, target) tasks per step, and front + per-step tables within one CU's 160 KiB LDS."""
    if not (1 <= L <= 64) or B < 0:
        return False
    LP = next(x for x in (4, 8, 16, 24, 32, 36, 48, 64) if L <= x)
    R = B + 1
    nrb = (R + 63) // 64
    if nrb * L > 8 * 24:
        return False
    o = (R * (LP + 2) * 8 + 15) // 16 * 16 + 2 * L * LP * 8 + 2 * LP * 4 + 2 * 8 * 24 * 2
    return (o + 15) // 16 * 16 + 16 + L * 8 * 8 <= 160 * 1024


def fused_separable_eligible(levels: LevelTable, B):
    """Mirror of the library's fused separable domain (p = 1 and beta > 0 are checked by the library): a 2-D
    product grid of consecutive integer levels of shape 6x6, 4x4, 8x8 or 8x4, both fronts in one CU's LDS."""
    if levels.M != 2 or not (0 <= B < 512) or levels.L != int(np.prod(levels.counts)):
        return False
    n0, n1 = int(levels.counts[0]), int(levels.counts[1])
    if (n0, n1) not in ((6, 6), (4, 4), (8, 8), (8, 4)):
        return False
    FS = (n0 * n1 + 1) | 1  # two fronts of (B+1) rows + the per-step K table (double-buffered) in 160 KiB of LDS
    if 2 * (((B + 1) * FS * 8 + 15) // 16 * 16) + 2 * n0 * n1 * (n0 + n1 - 1) * 8 > 160 * 1024:
        return False
    strides = np.cumprod(np.concatenate([[1], levels.counts[:-1]]))
    if not np.array_equal(((levels.tuples - 1) * strides).sum(axis=1), np.arange(levels.L)):
        return False
    return all(list(v) == list(range(v[0], v[0] + len(v))) for v in levels.nu)


def separable_eligible(levels: LevelTable):
    """Mirror of the library's separable-transform domain (p = 1 and beta > 0 are checked by the library):
    the pyramid domain restricted to 8^3 and 8^4 grids."""
    return pyramid_eligible(levels) and levels.M in (3, 4) and all(int(c) == 8 for c in levels.counts)
