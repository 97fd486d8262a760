"""CPU: host-side mirror of the reference interface, the C-ABI library's exports, and the TRM driver
plumbing (config C1 fishing) with the oracle standing in for the GPU solver."""
import ctypes
import math
import os
import re

import numpy as np
import pytest

from conftest import ROOT
import mioc
from mioc import native
from mioc.iterators import LevelTable, bounded_sum_iterator, product_iterator


def test_iterators_mirror_reference():
    assert list(product_iterator([[0, 1], [0, 1, 2]])) == [(1, 1), (2, 1), (1, 2), (2, 2), (1, 3), (2, 3)]
    it = bounded_sum_iterator([[0, 1]] * 3, 1, 1)
    assert list(it) == [(2, 1, 1), (1, 2, 1), (1, 1, 2)]
    assert list(it) == [(2, 1, 1), (1, 2, 1), (1, 1, 2)]  # re-iterable like a Julia iterator
    lt = LevelTable([[0, 1]] * 3, it)
    assert lt.L == 3 and lt.nuval.tolist() == [[1, 0, 0], [0, 1, 0], [0, 0, 1]]


def test_tv_p_docstring():
    u = np.array([[1, -1, 1], [3, 3, 0], [2, 2, 1]], dtype=np.float64)
    assert mioc.TV_p(u, 1) == 8 and mioc.TV_p(u, math.inf) == 5
    assert mioc.TV_p(u, 2) == 5.741657386773941
    assert mioc.TV_p(None, 1) == 0.0
    with pytest.raises(ValueError):
        mioc.TV_p(u, 0)


def test_trm_parameters_defaults_and_aliases():
    par = mioc.TRM_parameters()
    assert (par.beta, par.p, par.Delta0, par.sigma, par.kmax, par.maxiter, par.log) == (0.001, 1, 1.0, 0.5, 40,
                                                                                       1000, False)
    par = mioc.TRM_parameters(**{"β": 1e-4, "Δ⁰": 2, "p": math.inf})
    assert par.beta == 1e-4 and par.Delta0 == 2.0 and par.p == math.inf


def test_cost_spec():
    lt = LevelTable([list(range(6))] * 2)
    assert native.cost_spec(math.inf, levels=lt)[0] == native.MIOC_P_INF
    assert native.cost_spec(1, levels=lt)[0] == native.MIOC_P_ONE
    k, pi, tab = native.cost_spec(2, levels=lt)
    assert k == native.MIOC_P_INTLUT and pi == 2 and len(tab) == 51 and tab[4] == 2.0
    k, _, tab = native.cost_spec(1.5, levels=lt)
    assert k == native.MIOC_P_TABLE and tab.size == 36 * 36


def test_library_exports_every_header_symbol():
    hdr = open(os.path.join(ROOT, "include", "mioc.h")).read()
    declared = set(re.findall(r"\b(mioc_[a-z_]+)\s*\(", hdr))
    assert declared == set(native.EXPORTED), declared ^ set(native.EXPORTED)
    lib = ctypes.CDLL(native.LIB_PATH)
    for name in declared:
        assert hasattr(lib, name), name
    assert b"gfx950" in native.load_library().mioc_version()


def test_create_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(native.MiocNativeError):
        native.Context(0)


def test_synthetic_inputs_shapes():
    from mioc.synth import CONFIGS, make_inputs
    cfg = CONFIGS["C4"]
    assert cfg.B == 256
    lv, df, uo = make_inputs(cfg, nt=1000)
    assert lv.L == 4096 and df.shape == (4, 1000) and uo.shape == (4, 1000)
    rows = {tuple(r) for r in lv.nuval.astype(int)}
    assert all(tuple(c) in rows for c in uo.T.astype(int))
    assert CONFIGS["C2"].B == 819 and CONFIGS["C3"].B == 819 and CONFIGS["C1"].B == 85


class OracleSolver:
    """Test double: the CPU oracle behind the SubproblemSolver interface (bellman / backtrack)."""

    def __init__(self, levels, p, beta):
        from oracle.oracle import OracleC, Levels, P_INF, P_ONE
        self.oc = OracleC()
        self.lv = Levels(levels.nu, [tuple(t) for t in levels.tuples])
        self.pk = P_INF if p == math.inf else P_ONE
        self.beta = beta

    def bellman(self, df, u_old, B, dt):
        self.df, self.dt = np.array(df, copy=True), dt
        self.uo = np.array(u_old, order="F", copy=True)
        self.B = B
        self.phi, self.U = self.oc.bellman(self.lv, df, u_old, B, self.pk, self.beta, dt)

    def backtrack(self, B_use):
        self.u, phi = self.oc.backtrack(self.lv, self.uo, self.phi, self.U, self.B, B_use)
        return self.u, phi

    def pred(self):
        from oracle.oracle import pred_py, tv_p_kind
        to, tn = tv_p_kind(self.uo, self.pk), tv_p_kind(self.u, self.pk)
        iv, pr = pred_py(self.df, self.uo, self.u, self.dt, self.beta, to, tn)
        return iv, to, tn, pr


def test_trm_fishing_plumbing_with_oracle():
    """Config C1: TRM on the fishing problem (main("fishing") presets, multi-trust.jl:181-183)."""
    from mioc.ode import LVMObj
    obj = LVMObj(nt=128)
    par = mioc.TRM_parameters(beta=1e-4, Delta0=2, p=math.inf)
    x0 = mioc.rand_func(obj, rng=7)
    J0 = mioc.eval_f(obj, x0) + par.beta * mioc.TV_p(x0, par.p)
    solver = OracleSolver(LevelTable(obj.V, obj.iterator), par.p, par.beta)
    J = mioc.TRM(obj, par, x0=x0, solver=solver)
    assert J < J0
    assert obj.f_evals > 1 and obj.df_evals >= 1
    assert np.all(obj.x.sum(axis=0) == 1)  # SOS1 admissibility
    assert np.isfinite(J)


def test_ode_gradient_matches_finite_differences():
    """ODEObjective adjoint gradient vs finite differences (the reference's test_df, example_fishing.jl:94-123)."""
    from mioc.ode import DTMObj, LVMObj, VPOObj
    for cls in (LVMObj, DTMObj, VPOObj):
        obj = cls(nt=200)
        rng = np.random.default_rng(3)
        obj.x[:, :] = mioc.rand_func(obj, rng=3)
        mioc.eval_f_(obj)
        mioc.eval_df_(obj)
        h = rng.standard_normal(obj.x.shape)
        t = 1e-6
        fp = mioc.eval_f(obj, obj.x + t * h)
        fm = mioc.eval_f(obj, obj.x - t * h)
        fd = (fp - fm) / (2 * t)
        an = float(np.sum(obj.df * h)) * obj.tau  # (∇f, h)_{L²} (README "Modelling problems")
        assert abs(fd - an) <= 1e-5 * max(1.0, abs(an)), (cls.__name__, fd, an)


def test_latex_dat_round_trip_reference_file(tmp_path):
    """pgfplots .dat I/O (HelpFunctions.jl:401-446) on the reference's own data_files/example.dat (a committed
    fixture): reading it back and writing it again reproduces the file byte for byte; the reference's importer
    chokes on its own header, and so does ours unless told to skip it."""
    from mioc.latex_io import import_from_latex_format, julia_float, save_latex_format
    src = os.path.join(os.path.dirname(__file__), "golden", "data_files")
    with pytest.raises(ValueError, match="Could not parse"):
        import_from_latex_format("example", directory=src)
    x, u = import_from_latex_format("example", directory=src, skip_header=True)
    assert x.size == 1024 and x[1] == 0.009765625 and u[0] == 5.0
    save_latex_format(x, u, "example", directory=str(tmp_path))
    assert (tmp_path / "example.dat").read_bytes() == open(os.path.join(src, "example.dat"), "rb").read()
    # Julia's print spelling: plain for -4 < pt <= 16, else d.ddde±x without padding
    cases = {1e-05: "1.0e-5", 1.5e16: "1.5e16", 1e16: "1.0e16", 1e15: "1000000000000000.0",
             0.0001: "0.0001", -0.0: "-0.0", 123456789.0: "123456789.0", 2.5e-7: "2.5e-7", float("inf"): "Inf",
             float("nan"): "NaN", 5.0: "5.0"}
    for v, want in cases.items():
        assert julia_float(v) == want, (v, julia_float(v))
