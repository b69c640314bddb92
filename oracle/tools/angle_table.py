#!/usr/bin/env python3
"""cos/sin of NEWUOA's fixed trial angles i·(2π/50), i = 0..49 (TRSAPP / BIGLAG / BIGDEN angle
searches: `ang = i*dang`, `dang = twopi/(iu+1)`, iu = 49), as OptimPackNextGen — pure Julia —
computes them: with Julia Base's cos/sin, i.e. the shared restatement gpd_jlmath.h that the
oracle also calls (evaluated here through liboracle.so).  Emits the C++ table of gpd_newuoa.hpp,
so the device NEWUOA reads the very values the oracle computes instead of evaluating 98 fp64
sin/cos per angle search."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402  (checker library; build tool only)

TWO_PI = 6.283185307179586476925286766559  # kTwoPi of gpd_newuoa.hpp / oracle
dang = TWO_PI / float(49 + 1)
ang = np.array([float(i) * dang for i in range(50)])


def table():
    return [float(v) for v in oracle.jl_eval("cos", ang)], [float(v) for v in oracle.jl_eval("sin", ang)]


def rows(v):
    out = []
    for k in range(0, 50, 4):
        out.append("    " + ", ".join(x.hex() for x in v[k:k + 4]) + ",")
    return "\n".join(out)


if __name__ == "__main__":
    cs, sn = table()
    print("constexpr double kAngCos[50] = {\n" + rows(cs) + "\n};")
    print("constexpr double kAngSin[50] = {\n" + rows(sn) + "\n};")
