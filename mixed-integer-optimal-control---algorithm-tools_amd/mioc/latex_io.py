"""pgfplots .dat files, as the reference writes and reads them.

  save_latex_format(x, y, name)        HelpFunctions.jl:401-410
  import_from_latex_format(name)       HelpFunctions.jl:417-446

The reference prints each Float64 with Julia's `print`: the shortest decimal that round-trips, in plain form when
the decimal point position pt satisfies -4 < pt <= 16, else as `d.ddde±x` with no `+` and no zero padding
(`1.0e-5`, `1.5e16`), and `Inf` / `NaN`.  Python's repr picks the same digits and the same plain range; only the
exponent form is spelled differently, which `julia_float` converts.
"""
from __future__ import annotations

import math
import os

import numpy as np


def julia_float(v) -> str:
    """Julia's `print(::Float64)` spelling of v."""
    v = float(v)
    if math.isnan(v):
        return "NaN"
    if math.isinf(v):
        return "Inf" if v > 0 else "-Inf"
    r = repr(v)
    if "e" not in r:
        return r
    mant, exp = r.split("e")
    if "." not in mant:
        mant += ".0"
    return f"{mant}e{int(exp)}"


def save_latex_format(x, y, name, directory="data_files"):
    """Write `name`.dat with the header `x    y` and one `x[i] y[i]` line per point (HelpFunctions.jl:401-410)."""
    with open(os.path.join(directory, name + ".dat"), "w") as io:
        io.write("x    y\n")
        for a, b in zip(np.asarray(x).ravel(), np.asarray(y).ravel()):
            io.write(f"{julia_float(a)} {julia_float(b)}\n")


def import_from_latex_format(name, directory="data_files", skip_header=False):
    """Read `name`.dat back into (x, u) Float64 vectors (HelpFunctions.jl:417-446): lines with fewer than two
    columns are skipped, and a line whose first two columns do not parse raises.  Like the reference, that includes
    the `x    y` header save_latex_format writes (Julia's parse(Float64, "x") throws), so the reference cannot read
    its own files back; skip_header=True skips that one line instead."""
    xs, us = [], []
    with open(os.path.join(directory, name + ".dat")) as f:
        for n, line in enumerate(f):
            cols = line.split()
            if len(cols) < 2 or (skip_header and n == 0 and cols[:2] == ["x", "y"]):
                continue
            try:
                xi, ui = float(cols[0]), float(cols[1])
            except ValueError:
                raise ValueError("Could not parse entries of the following line to Float64:\n" + line) from None
            xs.append(xi)
            us.append(ui)
    return np.array(xs), np.array(us)
