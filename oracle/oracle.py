"""ctypes binding of the CPU oracle (oracle/liboracle.so).

ORACLE — TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module, and only as the checker.  The product library never
loads it.  PARITY UNPINNED (see oracle/oracle.h).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")

PARAM_DTYPE = np.dtype(
    [("c", np.complex128), ("a", np.complex128), ("b", np.float64), ("phi", np.float64),
     ("chi2", np.float64), ("nfev", np.int32), ("status", np.int32)], align=True)
assert PARAM_DTYPE.itemsize == 64

FIT_OFFSETS, RECENTER, ONLY_HIGH = 1, 2, 4
M_2PI = 6.283185  # src/Modulation.jl:11

_lib = None


def build(force: bool = False) -> str:
    srcs = ("newuoa_oracle.c", "demod_oracle.c", "oracle.h", "Makefile",
            "../gppupildemodulation.jl_amd/csrc/gpd_jlmath.h")
    stale = not os.path.exists(_LIB) or any(
        os.path.getmtime(os.path.join(_HERE, f)) > os.path.getmtime(_LIB) for f in srcs)
    if force or stale:
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB)
        P = ctypes.c_void_p
        L.oracle_fit_batch.argtypes = [ctypes.c_int64, ctypes.c_int64, P, P, ctypes.c_int64, P,
                                       ctypes.c_int64, P, P, ctypes.c_double, P, ctypes.c_uint32,
                                       ctypes.c_int, P, P, ctypes.c_int64, ctypes.c_int,
                                       ctypes.c_uint64, ctypes.c_double]
        L.oracle_fit_batch.restype = ctypes.c_int
        L.oracle_chi2.argtypes = [ctypes.c_int64, P, P, P, P, ctypes.c_double, ctypes.c_int,
                                  ctypes.c_double, ctypes.c_double, P]
        L.oracle_chi2.restype = ctypes.c_double
        L.oracle_buildstates.argtypes = [ctypes.c_int64, P, ctypes.c_int64, P, ctypes.c_int64, P,
                                         ctypes.c_int8, ctypes.c_int8, ctypes.c_double,
                                         ctypes.c_double, P]
        L.oracle_buildstates.restype = ctypes.c_int
        L.oracle_mean_var_power.argtypes = [ctypes.c_int64, P, P, P, P]
        L.oracle_mean_var_power.restype = None
        L.oracle_mean_var_power_series.argtypes = [ctypes.c_int64, P, P, ctypes.c_uint32, P, P]
        L.oracle_mean_var_power_series.restype = None
        L.oracle_mean_var_power_fused.argtypes = [ctypes.c_int64, P, P, ctypes.c_uint32, P, P]
        L.oracle_mean_var_power_fused.restype = None
        L.oracle_phi_grid.argtypes = [P]
        L.oracle_phi_grid.restype = None
        OBJ = ctypes.CFUNCTYPE(ctypes.c_double, ctypes.c_void_p, ctypes.c_int,
                               ctypes.POINTER(ctypes.c_double))
        L.oracle_newuoa.argtypes = [ctypes.c_int, ctypes.c_int, P, ctypes.c_double,
                                    ctypes.c_double, ctypes.c_int, OBJ, P, P]
        L.oracle_newuoa.restype = ctypes.c_int
        L._OBJ = OBJ
        L.oracle_jl_eval.argtypes = [ctypes.c_int, ctypes.c_int64, P, P, P]
        L.oracle_jl_eval.restype = ctypes.c_int
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def newuoa(f, x0, rhobeg, rhoend, maxfun=None, npt=None):
    """Powell NEWUOA on a Python callable (test helper). Returns (x, fx, nfev)."""
    L = lib()
    x = np.ascontiguousarray(x0, dtype=np.float64).copy()
    n = x.size
    npt = 2 * n + 1 if npt is None else npt
    maxfun = 30 * n if maxfun is None else maxfun
    cb = L._OBJ(lambda ctx, nn, xp: float(f(np.ctypeslib.as_array(xp, shape=(nn,)).copy())))
    fx = np.zeros(1)
    nf = L.oracle_newuoa(n, npt, _ptr(x), rhobeg, rhoend, maxfun, cb, None, _ptr(fx))
    if nf < 0:
        raise ValueError("bad NEWUOA arguments")
    return x, float(fx[0]), nf


def fit_batch(t, d, fc, fc_of_pixel, state=None, omega=M_2PI, xinit=None, flags=RECENTER,
              maxfun=60, want_output=False, nthreads=0, perturb_seed=0, perturb_ulps=1.0,
              order=0):
    """Oracle batch fit.  d: (n_pixels, n_samples) complex128 (row k = pixel column k),
    fc: (n_fc, n_samples) complex128, fc_of_pixel: (n_pixels,) int32.  order: the cost's
    summation order — 0 = CR8 (the product's canonical order), 1 = sequential, 16 / 32 = a
    vectorised loop with 16 / 32 accumulators (AVX2 / AVX-512 × 4 unroll): the orders Julia's
    @simd loops and BLAS zdotc may take on a CPU (demod_oracle.c red_slot; the reference-ceiling
    probe of bench.py)."""
    if order not in (0, 1, 16, 32):
        raise ValueError(f"order {order}: 0, 1, 16 or 32")
    flags = int(flags) | (int(order) << 16)
    L = lib()
    t = np.ascontiguousarray(t, dtype=np.float64)
    d = np.ascontiguousarray(d, dtype=np.complex128)
    fc = np.ascontiguousarray(fc, dtype=np.complex128)
    fop = np.ascontiguousarray(fc_of_pixel, dtype=np.int32)
    P, N = d.shape
    st = None if state is None else np.ascontiguousarray(state, dtype=np.int8)
    xi = None if xinit is None else np.ascontiguousarray(xinit, dtype=np.float64)
    params = np.zeros(P, dtype=PARAM_DTYPE)
    out = np.zeros_like(d) if want_output else None
    rc = L.oracle_fit_batch(N, P, _ptr(t), _ptr(d), N, _ptr(fc), N, _ptr(fop), _ptr(st),
                            float(omega), _ptr(xi), int(flags), int(maxfun), _ptr(params),
                            _ptr(out), N, int(nthreads), int(perturb_seed),
                            float(perturb_ulps))
    if rc != 0:
        raise RuntimeError(f"oracle_fit_batch failed: {rc}")
    return (params, out) if want_output else params


def chi2(t, d, p, b, phi, w=None, omega=M_2PI, offsets=False):
    L = lib()
    t = np.ascontiguousarray(t, dtype=np.float64)
    d = np.ascontiguousarray(d, dtype=np.complex128)
    p = np.ascontiguousarray(p, dtype=np.complex128)
    w = None if w is None else np.ascontiguousarray(w, dtype=np.float64)
    rec = np.zeros(1, dtype=PARAM_DTYPE)
    v = L.oracle_chi2(t.size, _ptr(t), _ptr(d), _ptr(w), _ptr(p), float(omega), int(offsets),
                      float(b), float(phi), _ptr(rec))
    return v, rec[0]


def buildstates(t, timer1, timer2, state1=3, state2=1, preswitchdelay=0.0, postwitchdelay=0.0):
    L = lib()
    t = np.ascontiguousarray(t, dtype=np.float64)
    t1 = np.ascontiguousarray(timer1, dtype=np.float64)
    t2 = np.ascontiguousarray(timer2, dtype=np.float64)
    out = np.zeros(t.size, dtype=np.int8)
    rc = L.oracle_buildstates(t.size, _ptr(t), t1.size, _ptr(t1), t2.size, _ptr(t2), state1,
                              state2, preswitchdelay, postwitchdelay, _ptr(out))
    if rc != 0:
        raise ValueError("buildstates: need ≥2 samples and ≥1 timer each")
    return out


def mean_var_power(states, d):
    L = lib()
    s = np.ascontiguousarray(states, dtype=np.int8)
    d = np.ascontiguousarray(d, dtype=np.complex128)
    m = np.zeros(d.size)
    w = np.zeros(d.size)
    L.oracle_mean_var_power(d.size, _ptr(s), _ptr(d), _ptr(m), _ptr(w))
    return m, w


def mean_var_power_series(states, d, onlyhigh=False):
    """Per-state (m, w) of one whole series as demodulateall computes them (valid mask applied,
    sums over the original sample indices): arrays of 5, index = MetState code + 1."""
    L = lib()
    s = np.ascontiguousarray(states, dtype=np.int8)
    d = np.ascontiguousarray(d, dtype=np.complex128)
    m5 = np.zeros(5)
    w5 = np.zeros(5)
    L.oracle_mean_var_power_series(d.size, _ptr(s), _ptr(d), ONLY_HIGH if onlyhigh else 0,
                                   _ptr(m5), _ptr(w5))
    return m5, w5


def mean_var_power_fused(states, d, onlyhigh=False):
    """The one-pass shifted-sum form of mean_var_power_series (the device's fused statistics,
    r4): arrays of 5, index = MetState code + 1, NaN for states without samples."""
    L = lib()
    s = np.ascontiguousarray(states, dtype=np.int8)
    d = np.ascontiguousarray(d, dtype=np.complex128)
    m5 = np.zeros(5)
    w5 = np.zeros(5)
    L.oracle_mean_var_power_fused(d.size, _ptr(s), _ptr(d), ONLY_HIGH if onlyhigh else 0,
                                  _ptr(m5), _ptr(w5))
    return m5, w5


JL_FN = {"sin": 0, "cos": 1, "sincos": 2, "atan": 3, "atan2": 4, "hypot": 5, "rem_pio2": 6, "hypot_nb": 7,
         "sin_sel": 8, "sincos_sel": 9, "sin_ph_shift": 10}


def jl_eval(fn, x, y=None):
    """The shared Julia-Base libm restatement (gpd_jlmath.h) on the host, elementwise.
    sincos → (n, 2) [s, c]; rem_pio2 → (n, 3) [quadrant, hi, lo]; atan2(x=y_coord, y=x_coord)
    takes (x, y) = (imaginary, real) like Julia's atan(y, x)."""
    code = JL_FN[fn]
    x = np.ascontiguousarray(x, dtype=np.float64).ravel()
    yy = None if y is None else np.ascontiguousarray(y, dtype=np.float64).ravel()
    width = {2: 2, 6: 3, 9: 2}.get(code, 1)
    out = np.empty(x.size * width)
    if lib().oracle_jl_eval(code, x.size, _ptr(x), _ptr(yy), _ptr(out)) != 0:
        raise ValueError(fn)
    return out.reshape(-1, width) if width > 1 else out


def fc_phasor(fc):
    """exp.(im .* angle.(fc)) (src/Modulation.jl:388) with Julia Base's atan(y, x) and sincos
    (the shared restatement): p = (cos θ, sin θ), θ = atan(im, re); θ == 0 → (1, θ)."""
    fc = np.asarray(fc, dtype=np.complex128)
    th = jl_eval("atan2", fc.imag.ravel(), fc.real.ravel())
    sc = jl_eval("sincos", th)
    p = sc[:, 1] + 1j * sc[:, 0]
    zero = th == 0
    p[zero] = 1.0 + 1j * th[zero]
    return p.reshape(fc.shape)


def phi_grid():
    out = np.zeros(8)
    lib().oracle_phi_grid(_ptr(out))
    return out
