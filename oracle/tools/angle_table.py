#!/usr/bin/env python3
"""cos/sin of NEWUOA's fixed trial angles i·(2π/50), i = 0..49 (TRSAPP / BIGLAG / BIGDEN angle
searches: `ang = i*dang`, `dang = twopi/(iu+1)`, iu = 49), as the oracle's libm (glibc, which
CPython's math module calls) computes them.  Emits the C++ table of gpd_newuoa.hpp, so the
device NEWUOA reads the very values the oracle computes instead of evaluating 98 fp64 sin/cos
per angle search."""
import math

TWO_PI = 6.283185307179586476925286766559  # kTwoPi of gpd_newuoa.hpp / oracle
dang = TWO_PI / float(49 + 1)
cs = [math.cos(float(i) * dang) for i in range(50)]
sn = [math.sin(float(i) * dang) for i in range(50)]


def rows(v):
    out = []
    for k in range(0, 50, 4):
        out.append("    " + ", ".join(x.hex() for x in v[k:k + 4]) + ",")
    return "\n".join(out)


print("constexpr double kAngCos[50] = {\n" + rows(cs) + "\n};")
print("constexpr double kAngSin[50] = {\n" + rows(sn) + "\n};")
