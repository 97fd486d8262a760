"""Admissible-level iterators and their flattened device level table.

Mirrors ``julia_opt/AdmissibleIterators.jl`` (reference):
  product_iterator(nu)                    AdmissibleIterators.jl:9-18
  bounded_sum_iterator(nu, lb, ub)        AdmissibleIterators.jl:26-34
  check_sum(l, nu, nx, lb, ub)            AdmissibleIterators.jl:41-49

Tuples are 1-based level indices, first index fastest (Julia's ``Iterators.product`` order).
``LevelTable`` is what ``mioc_set_levels`` receives: the iterator flattened once, in order.
"""
from __future__ import annotations

import itertools

import numpy as np


class _Reiterable:
    """A re-iterable view (Julia iterators can be traversed repeatedly; Python generators cannot)."""

    def __init__(self, factory, nu):
        self._factory = factory
        self.nu = nu

    def __iter__(self):
        return self._factory()


def product_iterator(nu):
    """All tuples of indices of the ragged array ``nu`` (AdmissibleIterators.jl:9-18)."""
    nu = [list(v) for v in nu]
    ranges = [range(1, len(v) + 1) for v in nu]

    def gen():
        for t in itertools.product(*reversed(ranges)):
            yield tuple(reversed(t))

    return _Reiterable(gen, nu)


def check_sum(l, nu, nx, lb, ub):
    """lb <= sum_i nu[i][l[i]] <= ub (AdmissibleIterators.jl:41-49)."""
    val = 0
    for i in range(nx):
        val += nu[i][l[i] - 1]
    return lb <= val <= ub


def bounded_sum_iterator(nu, lower_bound, upper_bound):
    """Tuples of product_iterator(nu) whose level sum lies in [lb, ub] (AdmissibleIterators.jl:26-34)."""
    nu = [list(v) for v in nu]
    nx = len(nu)
    prod = product_iterator(nu)

    def gen():
        return (l for l in prod if check_sum(l, nu, nx, lower_bound, upper_bound))

    return _Reiterable(gen, nu)


class LevelTable:
    """The iterator flattened to arrays in iteration order (the device level table)."""

    def __init__(self, nu, iterator=None):
        self.nu = [[int(x) for x in v] for v in nu]
        self.M = len(self.nu)
        if self.M < 1:
            raise ValueError("need at least one integer control")
        it = product_iterator(self.nu) if iterator is None else iterator
        tuples = [tuple(int(x) for x in t) for t in it]
        if not tuples:
            raise ValueError("the admissible iterator is empty")
        self.counts = np.array([len(v) for v in self.nu], dtype=np.int64)
        self.values = np.array([x for v in self.nu for x in v], dtype=np.int64)
        self.tuples = np.ascontiguousarray(np.array(tuples, dtype=np.int32).reshape(-1, self.M))
        self.L = int(self.tuples.shape[0])
        self.nuval = np.array([[self.nu[m][t[m] - 1] for m in range(self.M)] for t in tuples],
                              dtype=np.float64)

    def __repr__(self):
        return f"LevelTable(M={self.M}, L={self.L}, counts={self.counts.tolist()})"
