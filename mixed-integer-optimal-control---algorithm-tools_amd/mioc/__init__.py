"""mioc -- MI355X-native drop-in for the DP trust-region subproblem of
Jonas477/mixed-integer-optimal-control---algorithm-tools (``bellman_TRM!`` / ``eval_u_TRM!``).

Host-side mirror of the reference's interface for that path; the DP itself runs in ``libmioc.so``
(hand-written gfx950 HIP kernels behind the C ABI of ``include/mioc.h``).
"""
from .iterators import LevelTable, bounded_sum_iterator, check_sum, product_iterator
from .native import Context, InexactError, MiocNativeError, load_library
from .objective import (AbstractObjective, AbstractObjectiveAAO, AbstractObjectiveLazy, eval_df_, eval_f,
                        eval_f_, eval_fdf_)
from .trm import (TRM, SubproblemSolver, TRM_parameters, TV_p, bellman_TRM_, eval_u_TRM_, rand_func,
                  rand_func_int)

__all__ = [
    "LevelTable", "product_iterator", "bounded_sum_iterator", "check_sum", "Context", "MiocNativeError",
    "InexactError", "load_library", "AbstractObjective", "AbstractObjectiveAAO", "AbstractObjectiveLazy", "eval_f",
    "eval_f_", "eval_df_", "eval_fdf_", "TRM", "TRM_parameters", "TV_p", "SubproblemSolver", "bellman_TRM_",
    "eval_u_TRM_", "rand_func", "rand_func_int",
]
