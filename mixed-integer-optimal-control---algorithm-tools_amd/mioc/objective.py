"""The objective plugin surface the TRM driver consumes.

Mirrors ``julia_opt/AbstractObjective.jl`` (reference):
  AbstractObjective{T}           :7        AbstractObjectiveAAO{T}      :15
  AbstractObjectiveLazy{T}       :70
  eval_f / eval_f! / eval_df! / eval_fdf!  (AAO :18-59, Lazy :74-110)
  user hooks eval_fdf_helper (:62), eval_f_helper / eval_df_helper (:113-114)

Julia's mutating ``eval_f!`` is spelled ``eval_f_`` here (likewise ``eval_df_``, ``eval_fdf_``).
Required fields of a concrete objective (README "Modelling problems"):
  nt, nx, tau, V (the reference's 𝓥 -- Python NFKC-normalises ``obj.𝓥`` to ``obj.V``), iterator,
  x (nx x nt), df (nx x nt), f, df_valid, f_evals, df_evals.
"""
from __future__ import annotations

import numpy as np


class AbstractObjective:
    """Abstract type for optimization problems (AbstractObjective.jl:7)."""

    def _init_fields(self, nx, nt):
        self.x = np.zeros((nx, nt), dtype=np.float64, order="F")
        self.df = np.zeros((nx, nt), dtype=np.float64, order="F")
        self.f = 0.0
        self.df_valid = False
        self.f_evals = 0
        self.df_evals = 0
        self.fdf_evals = 0


class AbstractObjectiveAAO(AbstractObjective):
    """Objective and gradient evaluated all at once (AbstractObjective.jl:15); implement
    ``eval_fdf_helper(x, df)`` returning f and filling ``df`` when it is not None."""

    def eval_fdf_helper(self, x, df):  # AbstractObjective.jl:62
        raise NotImplementedError


class AbstractObjectiveLazy(AbstractObjective):
    """Objective and gradient evaluated separately (AbstractObjective.jl:70); implement
    ``eval_f_helper(x, cache)`` and ``eval_df_helper()``."""

    def eval_f_helper(self, x, cache):  # AbstractObjective.jl:113
        raise NotImplementedError

    def eval_df_helper(self):  # AbstractObjective.jl:114
        raise NotImplementedError


def eval_f(obj, x):
    """Evaluate the objective at x without caching (AbstractObjective.jl:18-22, :74-78)."""
    if isinstance(obj, AbstractObjectiveAAO):
        obj.fdf_evals += 1
        return obj.eval_fdf_helper(x, None)
    obj.f_evals += 1
    return obj.eval_f_helper(x, False)


def eval_f_(obj):
    """eval_f!(obj): objective at obj.x, cached; invalidates df (AbstractObjective.jl:25-35, :81-91)."""
    if isinstance(obj, AbstractObjectiveAAO):
        f = eval_f(obj, obj.x)
    else:
        obj.f_evals += 1
        f = obj.eval_f_helper(obj.x, True)
    obj.f = f
    obj.df_valid = False
    return f


def eval_df_(obj):
    """eval_df!(obj): gradient at obj.x unless cached (AbstractObjective.jl:38-47, :94-102)."""
    if not obj.df_valid:
        if isinstance(obj, AbstractObjectiveAAO):
            obj.fdf_evals += 1
            obj.eval_fdf_helper(obj.x, obj.df)
        else:
            obj.df_evals += 1
            obj.eval_df_helper()
        obj.df_valid = True
    return None


def eval_fdf_(obj):
    """eval_fdf!(obj) (AbstractObjective.jl:50-59, :105-110)."""
    if isinstance(obj, AbstractObjectiveAAO):
        obj.fdf_evals += 1
        f = obj.eval_fdf_helper(obj.x, obj.df)
        obj.f = f
        obj.df_valid = True
        return f
    f = eval_f_(obj)
    eval_df_(obj)
    return f
