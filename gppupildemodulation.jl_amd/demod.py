"""Host-side mirror of the reference API for the demodulation hot path.

Mirrors FerreolS/GPPupilDemodulation.jl @ 2024-10-16:
  * enums Side {FT=0, SC=16}, Diode {D1..D4, FC}, MetState, idx()   (src/Modulation.jl:9-22, src/Faint.jl:1)
  * ModulationWithOffsets / ModulationNoOffsets records              (src/Modulation.jl:24-55)
  * FaintStates + buildstates                                        (src/Faint.jl:3-73)
  * demodulateall(timestamp, data; init, recenter, faintparam, onlyhigh, fitoffsets,
                  preswitchdelay, postwitchdelay) -> (output, param, likelihood)
                                                                     (src/Modulation.jl:344-435)
The diode loop runs on the GPU through ONE gpd_fit_batch call (include/gpdemod.h); there is no
CPU fallback.
"""
from __future__ import annotations

import ctypes
import enum
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import (GPD_FIT_OFFSETS, GPD_FP32, GPD_METHOD_EXACT, GPD_METHOD_HARMONIC,
                   GPD_ONLY_HIGH, GPD_RECENTER, PARAM_DTYPE, check, load, ptr)

M_2PI = 6.283185  # src/Modulation.jl:11 (not 2π)


class Side(enum.IntEnum):  # src/Modulation.jl:9
    FT = 0
    SC = 16


class Diode(enum.IntEnum):  # src/Modulation.jl:10
    D1 = 1
    D2 = 2
    D3 = 3
    D4 = 4
    FC = 5


class MetState(enum.IntEnum):  # src/Faint.jl:1
    OFF = 0
    LOW = 1
    NORMAL = 2
    HIGH = 3
    TRANSIENT = -1


def idx(side: Side, telescope: int, diode: Diode) -> int:
    """1-based column of (side, telescope, diode) in the N×40 matrix (src/Modulation.jl:17-22)."""
    if diode == Diode.FC:
        return 32 + int(side) // 4 + (telescope - 1) + 1
    return int(side) + (int(diode) - 1) + (telescope - 1) * 4 + 1


def fc_column_of(col: int) -> int:
    """1-based FC column used by the 1-based diode column `col` ∈ 1..32 (src/Modulation.jl:388)."""
    side = Side.FT if col <= 16 else Side.SC
    tel = ((col - 1) % 16) // 4 + 1
    return idx(side, tel, Diode.FC)


@dataclass
class ModulationNoOffsets:  # src/Modulation.jl:34-39
    a: complex
    b: float
    ϕ: float
    ω: float = M_2PI


@dataclass
class ModulationWithOffsets:  # src/Modulation.jl:26-32
    c: complex
    a: complex
    b: float
    ϕ: float
    ω: float = M_2PI


@dataclass
class FaintStates:  # src/Faint.jl:3-19
    timer1: np.ndarray
    timer2: np.ndarray
    voltage1: float
    voltage2: float
    state1: MetState = MetState.HIGH
    state2: MetState = MetState.LOW

    @classmethod
    def make(cls, timer1, timer2, voltage1, voltage2):
        """Outer constructor: the higher-voltage timer is the LOW one (src/Faint.jl:12-19)."""
        t1 = np.asarray(timer1, dtype=np.float64)
        t2 = np.asarray(timer2, dtype=np.float64)
        if voltage1 > voltage2:
            return cls(t2, t1, voltage2, voltage1, MetState.HIGH, MetState.LOW)
        return cls(t1, t2, voltage1, voltage2, MetState.HIGH, MetState.LOW)


MJD_1970_1_1 = 40587.0  # src/GPPupilDemodulation.jl:15
DAY_TO_SEC = 24 * 60 * 60  # :16


def buildfaintparameters(hdr) -> FaintStates:
    """FaintStates from the exposure header (src/GPPupilDemodulation.jl:64-81): timer_i =
    TIMERi + MJD(1970-01-01)·86400 + RATEi·(0:REPEATi-1), ordered by VOLTAGEi.  `hdr` is any
    mapping with the ESO keywords (e.g. the primary header from fits.read_fits)."""
    timers = []
    for i in (1, 2):
        start = hdr[f"ESO INS ANLO3 TIMER{i}"] + MJD_1970_1_1 * DAY_TO_SEC
        rate = hdr[f"ESO INS ANLO3 RATE{i}"]
        timers.append(start + rate * np.arange(int(hdr[f"ESO INS ANLO3 REPEAT{i}"])))
    return FaintStates.make(timers[0], timers[1], hdr["ESO INS ANLO3 VOLTAGE1"],
                            hdr["ESO INS ANLO3 VOLTAGE2"])


def metrology_times(time_us, mjd_obs):
    """Float64.(table["TIME"]) .* 1e-6 .+ DAY_TO_SEC * mjd (src/GPPupilDemodulation.jl:139)."""
    return np.asarray(time_us).astype(np.float64) * 1e-6 + (DAY_TO_SEC * float(mjd_obs))


def buildstates(faintstates: FaintStates, timestamp, lag: int = 0, preswitchdelay=0.0,
                postwitchdelay=0.0) -> np.ndarray:
    """src/Faint.jl:21-73 → int8 MetState codes (host C++ in libgpdemod)."""
    t = np.ascontiguousarray(timestamp, dtype=np.float64)
    if t.size < 2:
        raise ValueError("buildstates needs at least 2 timestamps")
    step = t[1] - t[0]
    t1 = np.ascontiguousarray(faintstates.timer1 + lag * step, dtype=np.float64)
    t2 = np.ascontiguousarray(faintstates.timer2 + lag * step, dtype=np.float64)
    if t1.size < 1 or t2.size < 1:
        raise ValueError("popfirst! on an empty timer list")  # src/Faint.jl:33-34
    out = np.empty(t.size, dtype=np.int8)
    rc = load().gpd_buildstates(t.size, ptr(t), t1.size, ptr(t1), t2.size, ptr(t2),
                                float(preswitchdelay), float(postwitchdelay), ptr(out))
    check(rc)
    return out


def mean_var_power_batch(states, d, *, onlyhigh=False, device=0):
    """Per-state faint power m and weight w of every series (rows of d) as the fit computes them
    on the GPU (gpd_mean_var_power): two (P, 5) arrays indexed by MetState code + 1."""
    L = load()
    d = np.ascontiguousarray(np.atleast_2d(d), dtype=np.complex128)
    st = np.ascontiguousarray(states, dtype=np.int8)
    P, N = d.shape
    if st.shape != (N,):
        raise ValueError("states and data must have the same length")
    out = np.empty((P, 10))
    err = ctypes.create_string_buffer(512)
    check(L.gpd_mean_var_power(N, P, ptr(d), N, ptr(st), GPD_ONLY_HIGH if onlyhigh else 0,
                               ptr(out), int(device), err, len(err)), err)
    return out[:, :5], out[:, 5:]


def compute_mean_var_power(states, data):
    """compute_mean_var_power(states, data) → (m, w) per sample (src/Faint.jl:89-100), for one
    series, on the GPU.  Every sample counts (the reference function has no mask; demodulateall
    passes it the valid samples only, src/Modulation.jl:391-395)."""
    st = np.asarray(states, dtype=np.int8)
    if np.any(st == MetState.TRANSIENT):
        # TRANSIENT samples are not part of any statistic the fit uses (dropped by the valid
        # mask before the call, src/Modulation.jl:380-382)
        raise ValueError("compute_mean_var_power: TRANSIENT samples must be masked by the caller")
    m5, w5 = mean_var_power_batch(st, np.asarray(data)[None, :])
    return m5[0][st + 1], w5[0][st + 1]


def _method_flags(method: str) -> int:
    if method == "auto":
        return 0
    if method == "exact":
        return GPD_METHOD_EXACT
    if method == "harmonic":
        return GPD_METHOD_HARMONIC
    if method == "fp32":  # the exact evaluator in Float32 per-sample arithmetic (GPD_FP32)
        return GPD_FP32
    raise ValueError(f"method must be auto|exact|harmonic|fp32, got {method!r}")


def _storage(d, fc):
    """Series and FC rows in their stored precision: both complex64 (Matrix{ComplexF32}, the
    FITS VOLT precision) → the Float32-storage entry points, which widen on load and compute in
    Float64; anything else → complex128."""
    d = np.asarray(d)
    fc = np.asarray(fc)
    if d.dtype == np.complex64 and fc.dtype == np.complex64:
        return np.ascontiguousarray(d), np.ascontiguousarray(fc), True
    return (np.ascontiguousarray(d, dtype=np.complex128),
            np.ascontiguousarray(fc, dtype=np.complex128), False)


def fit_batch(t, d, fc, fc_of_pixel, *, state=None, omega=M_2PI, xinit=None, recenter=True,
              fitoffsets=False, onlyhigh=False, maxfun=60, want_output=False, method="auto",
              n_gpus=1, out=None):
    """Batch fit of P series on the GPU.

    t: (N,) float64; d: (P, N) complex (row k = series k); fc: (G, N) complex raw FC
    columns; fc_of_pixel: (P,) int (0-based row of fc).  complex64 d and fc are kept in Float32
    in device memory (gpd_fit_batch_c32), anything else is taken as complex128.  Returns a
    PARAM_DTYPE record array (and the (P, N) complex128 demodulated series when want_output;
    `out`, a caller-owned (P, N) complex128 array with contiguous rows, receives them in place).
    """
    L = load()
    t = np.ascontiguousarray(t, dtype=np.float64)
    d, fc, c32 = _storage(d, fc)
    fop = np.ascontiguousarray(fc_of_pixel, dtype=np.int32)
    if d.ndim != 2 or fc.ndim != 2 or d.shape[1] != t.size or fc.shape[1] != t.size:
        raise ValueError("voltage and time must have the same number of lines")  # src/Modulation.jl:258
    P, N = d.shape
    if fop.shape != (P,):
        raise ValueError("fc_of_pixel must have one entry per series")
    st = None
    if state is not None:
        st = np.ascontiguousarray(state, dtype=np.int8)
        if st.shape != (N,):
            raise ValueError("state and time must have the same number of lines")
    xi = None
    if xinit is not None:
        xi = np.ascontiguousarray(xinit, dtype=np.float64)
        if xi.shape != (2,):
            raise ValueError("init must be a 2-vector [b, ϕ]")
    flags = _method_flags(method)
    if recenter:
        flags |= GPD_RECENTER
    if fitoffsets:
        flags |= GPD_FIT_OFFSETS
    if onlyhigh:
        flags |= GPD_ONLY_HIGH
    params = np.zeros(P, dtype=PARAM_DTYPE)
    ldo = N
    if out is not None:
        want_output = True
        if (out.dtype != np.complex128 or out.ndim != 2 or out.shape != (P, N)
                or out.strides[1] != 16 or out.strides[0] % 16 or out.strides[0] < 16 * N):
            raise ValueError("out must be a (P, N) complex128 array with contiguous rows")
        ldo = out.strides[0] // 16
    elif want_output:
        out = np.zeros((P, N), dtype=np.complex128)
    err = ctypes.create_string_buffer(512)
    fn = L.gpd_fit_batch_c32 if c32 else L.gpd_fit_batch
    rc = fn(N, P, ptr(t), ptr(d), N, ptr(fc), fc.shape[0], N, ptr(fop), ptr(st), float(omega),
            ptr(xi), flags, int(maxfun), ptr(params), ptr(out), ldo, int(n_gpus), err, len(err))
    check(rc, err)
    return (params, out) if want_output else params


def chi2_batch(t, d, fc, fc_of_pixel, bphi, *, state=None, omega=M_2PI, fitoffsets=False,
               onlyhigh=False, method="auto", n_gpus=1):
    """χ²(b_k, ϕ_k) per series — the Chi2CostFunction functor lkl(b, ϕ) (src/Modulation.jl:318-330)
    evaluated on the GPU for a batch.  bphi: (P, 2).  Returns a PARAM_DTYPE record array with chi2
    and the closed-form a (and c) at each point."""
    L = load()
    t = np.ascontiguousarray(t, dtype=np.float64)
    d = np.ascontiguousarray(d, dtype=np.complex128)
    fc = np.ascontiguousarray(fc, dtype=np.complex128)
    fop = np.ascontiguousarray(fc_of_pixel, dtype=np.int32)
    P, N = d.shape
    bp = np.ascontiguousarray(bphi, dtype=np.float64).reshape(P, 2)
    st = None if state is None else np.ascontiguousarray(state, dtype=np.int8)
    flags = _method_flags(method)
    if fitoffsets:
        flags |= GPD_FIT_OFFSETS
    if onlyhigh:
        flags |= GPD_ONLY_HIGH
    params = np.zeros(P, dtype=PARAM_DTYPE)
    err = ctypes.create_string_buffer(512)
    rc = L.gpd_chi2_batch(N, P, ptr(t), ptr(d), N, ptr(fc), fc.shape[0], N, ptr(fop), ptr(st),
                          float(omega), ptr(bp), flags, ptr(params), int(n_gpus), err, len(err))
    check(rc, err)
    return params


def demodulateall(timestamp, data, *, init="auto", recenter=True, faintparam=None,
                  onlyhigh=False, fitoffsets=False, preswitchdelay=0.01, postwitchdelay=0.3,
                  method="auto", n_gpus=1):
    """GPU drop-in for demodulateall (src/Modulation.jl:344-435).

    timestamp: (N,) float; data: (N, 40) complex (columns in idx() order, 1..32 diodes,
    33..40 FC).  Returns (output (N, 40) complex, param: list of 32 Modulation records,
    likelihood: (32,) float).  One gpd_demodulateall call: the library fills a fresh
    column-major output (the demodulated diodes and the FC columns as given), so no host copy
    of the exposure runs here.  `data` column-major (np.asfortranarray, a Julia Matrix's
    layout) is passed without a copy; a row-major array is converted first.
    """
    t = np.ascontiguousarray(timestamp, dtype=np.float64)
    data = np.asarray(data)
    if not np.iscomplexobj(data):
        raise TypeError("data must be a complex matrix (AbstractMatrix{Complex{T}})")
    if data.dtype != np.complex64:  # Matrix{ComplexF32} stays Float32 in device memory
        data = data.astype(np.complex128, copy=False)
    if data.ndim != 2 or data.shape[1] != 40:
        raise ValueError("data must be N×40 (32 diodes + 8 FC columns)")
    N = data.shape[0]
    if t.shape != (N,):
        raise ValueError("voltage and time must have the same number of lines")
    # (40, N): column k contiguous, like Julia's Matrix (no copy when `data` is column-major,
    # np.asfortranarray — the layout a Julia caller hands over)
    cols = np.ascontiguousarray(data.T)  # (40, N): no copy when data is column-major
    state = None
    if faintparam is not None:
        if isinstance(faintparam, FaintStates):
            state = buildstates(faintparam, t, preswitchdelay=preswitchdelay,
                                postwitchdelay=postwitchdelay)  # src/Modulation.jl:366-367
        else:
            state = np.asarray(faintparam, dtype=np.int8)
            if state.shape != (N,):
                raise ValueError("faintparam must have one MetState per sample")
        state = np.ascontiguousarray(state, dtype=np.int8)
    xinit = None
    if not (isinstance(init, str) and init == "auto"):
        xinit = np.ascontiguousarray(init, dtype=np.float64)
        if xinit.shape != (2,):
            raise ValueError("init must be a 2-vector [b, ϕ]")
    flags = _method_flags(method) | (GPD_RECENTER if recenter else 0) | \
        (GPD_FIT_OFFSETS if fitoffsets else 0) | (GPD_ONLY_HIGH if onlyhigh else 0)
    # output = copy(data) with the diodes demodulated (src/Modulation.jl:353, 417-425): a fresh
    # column-major (N, 40) array of data's element type, every column written by the library
    out_cols = np.empty((40, N), dtype=cols.dtype)
    params = np.zeros(32, dtype=PARAM_DTYPE)
    err = ctypes.create_string_buffer(512)
    L = load()
    fn = L.gpd_demodulateall_c32 if cols.dtype == np.complex64 else L.gpd_demodulateall
    check(fn(N, ptr(t), ptr(cols), N, ptr(state), ptr(xinit), flags, 60, ptr(params),
             ptr(out_cols), N, int(n_gpus), err, len(err)), err)
    output = out_cols.T  # (N, 40), column-major like the Julia Matrix
    param = []
    for p in params:
        if fitoffsets:
            param.append(ModulationWithOffsets(complex(p["c"]), complex(p["a"]), float(p["b"]),
                                               float(p["phi"])))
        else:
            param.append(ModulationNoOffsets(complex(p["a"]), float(p["b"]), float(p["phi"])))
    likelihood = params["chi2"].copy()
    return output, param, likelihood


def fit_windows(t, d, fc, fc_of_col, nwindow, *, state=None, omega=M_2PI, xinit=None,
                recenter=True, fitoffsets=False, onlyhigh=False, maxfun=60, want_output=False,
                method="auto", n_gpus=1, out=None):
    """Every window of `nwindow` samples (Iterators.partition, the last one shorter) fitted as its
    own demodulateall call (src/GPPupilDemodulation.jl:204-205), all windows in one GPU call.

    t: (N,); d: (C, N) complex (row k = column k); fc: (G, N) raw FC rows; fc_of_col: (C,);
    complex64 d and fc stay Float32 in device memory (gpd_fit_windows_c32).
    method: "auto" (harmonic moments per window; exact with fitoffsets), "exact", "harmonic".
    Returns params shaped (n_windows, C) (and the (C, N) demodulated rows when want_output)."""
    L = load()
    t = np.ascontiguousarray(t, dtype=np.float64)
    d, fc, c32 = _storage(d, fc)
    fop = np.ascontiguousarray(fc_of_col, dtype=np.int32)
    if d.ndim != 2 or fc.ndim != 2 or d.shape[1] != t.size or fc.shape[1] != t.size:
        raise ValueError("voltage and time must have the same number of lines")
    C, N = d.shape
    nwindow = int(nwindow)
    if nwindow < 1:
        raise ValueError("window must span at least one sample")
    if fop.shape != (C,):
        raise ValueError("fc_of_col must have one entry per column")
    st = None if state is None else np.ascontiguousarray(state, dtype=np.int8)
    if st is not None and st.shape != (N,):
        raise ValueError("state and time must have the same number of lines")
    xi = None if xinit is None else np.ascontiguousarray(xinit, dtype=np.float64).reshape(2)
    flags = _method_flags(method) | (GPD_RECENTER if recenter else 0) | \
        (GPD_FIT_OFFSETS if fitoffsets else 0) | (GPD_ONLY_HIGH if onlyhigh else 0)
    nwin = -(-N // nwindow)
    params = np.zeros(nwin * C, dtype=PARAM_DTYPE)
    ldo = N
    if out is not None:  # caller-owned (C, N) complex128 rows, written in place
        want_output = True
        if (out.dtype != np.complex128 or out.ndim != 2 or out.shape != (C, N)
                or out.strides[1] != 16 or out.strides[0] % 16 or out.strides[0] < 16 * N):
            raise ValueError("out must be a (C, N) complex128 array with contiguous rows")
        ldo = out.strides[0] // 16
    elif want_output:
        out = np.zeros((C, N), dtype=np.complex128)
    err = ctypes.create_string_buffer(512)
    fn = L.gpd_fit_windows_c32 if c32 else L.gpd_fit_windows
    rc = fn(N, nwindow, C, ptr(t), ptr(d), N, ptr(fc), fc.shape[0], N, ptr(fop), ptr(st),
            float(omega), ptr(xi), flags, int(maxfun), ptr(params), ptr(out), ldo, int(n_gpus), err,
            len(err))
    check(rc, err)
    params = params.reshape(nwin, C)
    return (params, out) if want_output else params


def window_length(timestamp, window):
    """nwindow = round(Int, window / (times[2] - times[1])) (src/GPPupilDemodulation.jl:191)."""
    t = np.asarray(timestamp, dtype=np.float64)
    return int(round(window / (t[1] - t[0])))


def demodulate_windows(timestamp, data, window, *, faintparam=None, onlyhigh=False,
                       fitoffsets=False, preswitchdelay=0.01, postwitchdelay=0.3, method="auto",
                       n_gpus=1):
    """processmetrology's windowed branch (src/GPPupilDemodulation.jl:191-225) on the GPU:
    window (seconds) → nwindow samples; every window demodulated with its own fit.

    Returns (output (N, 40), params (n_windows, 32) records, tables) where tables holds the
    per-sample Float32 parameter columns ABSA, ARGA, B, PHI (and X0, Y0 with fitoffsets),
    each (32, N) in idx() order, as the reference writes them (:209-224, :239-244)."""
    t = np.asarray(timestamp, dtype=np.float64)
    data = np.asarray(data)
    if data.dtype != np.complex64:
        data = data.astype(np.complex128, copy=False)
    if data.ndim != 2 or data.shape[1] != 40 or data.shape[0] != t.size:
        raise ValueError("data must be N×40 with one row per timestamp")
    N = t.size
    nwindow = window_length(t, window)
    if nwindow < 1:
        raise ValueError("window shorter than half a sample interval")
    state = None
    if faintparam is not None:
        state = buildstates(faintparam, t, preswitchdelay=preswitchdelay,
                            postwitchdelay=postwitchdelay) \
            if isinstance(faintparam, FaintStates) else np.asarray(faintparam, dtype=np.int8)
    cols = np.ascontiguousarray(data.T)
    fop = np.array([fc_column_of(c) - 1 for c in range(1, 33)], dtype=np.int32)
    out_cols = cols.copy()  # output = copy(data), written in place as in demodulateall
    inplace = out_cols.dtype == np.complex128
    params, out = fit_windows(t, cols[:32], cols, fop, nwindow, state=state, fitoffsets=fitoffsets,
                              onlyhigh=onlyhigh, want_output=True, method=method, n_gpus=n_gpus,
                              out=out_cols[:32] if inplace else None)
    if not inplace:
        out_cols[:32] = out
    output = out_cols.T
    return output, params, window_tables(params, N, nwindow, fitoffsets=fitoffsets)


def window_tables(params, n_samples, nwindow, *, fitoffsets=False):
    """Broadcast per-window parameters to per-sample Float32 columns (32, N)
    (src/GPPupilDemodulation.jl:209-224; b ≥ 0 already, :427-430 normalised it)."""
    nwin, C = params.shape
    counts = np.full(nwin, nwindow)
    counts[-1] = n_samples - nwindow * (nwin - 1)

    def per_sample(v):  # (nwin, C) per-window values → (C, N) Float32 rows, one pass
        return np.repeat(np.ascontiguousarray(v.T, dtype=np.float32), counts, axis=1)

    tables = {"ABSA": per_sample(np.abs(params["a"])),
              "ARGA": per_sample(np.angle(params["a"])),
              "B": per_sample(params["b"]),
              "PHI": per_sample(params["phi"])}
    if fitoffsets:
        tables["X0"] = per_sample(params["c"].real)
        tables["Y0"] = per_sample(params["c"].imag)
    return tables


def read_stefan_file(filename):
    """Column centres from a Stefan calibration file (src/GPPupilDemodulation.jl:84-104): every
    `avg` row names (side, telescope, diode) and gives VX, VY in mV; centre = 1e-3·(VX + i·VY)
    at idx(side, telescope, diode).  Returns (40,) complex128 (unset columns stay 0)."""
    offsets = np.zeros(40, dtype=np.complex128)
    with open(filename) as f:
        for line in f:
            if not line.startswith("avg"):
                continue
            values = line.split()
            name = values[1]
            side = Side[name[0:2]]
            telescope = int(name[3])
            diode = Diode[name[4:6]]
            offsets[idx(side, telescope, diode) - 1] = 1e-3 * (float(values[2]) + 1j * float(values[4]))
    return offsets


def process_volt(timestamp, volt, *, offsets=None, window=None, faintparam=None, onlyhigh=False,
                 preswitchdelay=0.01, postwitchdelay=0.3, init="auto", method="auto", device=0):
    """processmetrology's numeric core (src/GPPupilDemodulation.jl:137-171, 191-244) straight from
    the FITS VOLT column on the GPU.

    volt: (N, 80) float32 rows [re1 im1 … re40 im40].  offsets: (40,) complex centres subtracted
    first (a Stefan file, read_stefan_file), False → no centring and fitoffsets (:151-157), None →
    no centring.  window: seconds (None = one fit per diode over the exposure).
    Returns (volt_out (N, 80) float32 demodulated rows, params, tables) — params (32,) or
    (n_windows, 32); tables = per-sample Float32 parameter columns in window mode, else None."""
    L = load()
    t = np.ascontiguousarray(timestamp, dtype=np.float64)
    v = np.ascontiguousarray(volt, dtype=np.float32)
    if v.ndim != 2 or v.shape[1] != 80 or v.shape[0] != t.size:
        raise ValueError("VOLT must be N×80 Float32 rows")
    N = t.size
    fitoffsets = offsets is False
    if offsets is True:
        raise NotImplementedError("compute_offsets (circle fit) is outside the hot path")
    cen = None
    if offsets is not None and offsets is not False:
        cen = np.ascontiguousarray(offsets, dtype=np.complex128)
        if cen.shape != (40,):
            raise ValueError("offsets must hold 40 complex centres")
    state = None
    if faintparam is not None:
        state = buildstates(faintparam, t, preswitchdelay=preswitchdelay,
                            postwitchdelay=postwitchdelay) \
            if isinstance(faintparam, FaintStates) else np.asarray(faintparam, dtype=np.int8)
        state = np.ascontiguousarray(state, dtype=np.int8)
    xi = None if (isinstance(init, str) and init == "auto") else \
        np.ascontiguousarray(init, dtype=np.float64).reshape(2)
    nwindow = 0 if window is None else window_length(t, window)
    if window is not None and nwindow < 1:
        raise ValueError("window shorter than half a sample interval")
    flags = _method_flags(method) | GPD_RECENTER | (GPD_FIT_OFFSETS if fitoffsets else 0) | \
        (GPD_ONLY_HIGH if onlyhigh else 0)
    nrec = 32 * (-(-N // nwindow) if nwindow else 1)
    params = np.zeros(nrec, dtype=PARAM_DTYPE)
    out = np.zeros((N, 80), dtype=np.float32)
    err = ctypes.create_string_buffer(512)
    rc = L.gpd_process_volt(N, ptr(t), ptr(v), 80, ptr(cen), ptr(state), float(M_2PI), ptr(xi),
                            flags, 60, nwindow, ptr(params), ptr(out), 80, int(device), err,
                            len(err))
    check(rc, err)
    if nwindow:
        params = params.reshape(-1, 32)
        return out, params, window_tables(params, N, nwindow, fitoffsets=fitoffsets)
    return out, params, None


def _diode_order():
    """(side, telescope, diode) in the order of Iterators.product((D1,D2,D3,D4), 1:4, (FT,SC))
    (src/GPPupilDemodulation.jl:171,212): diode fastest, then telescope, then side."""
    return [(side, tel, diode) for side in (Side.FT, Side.SC) for tel in range(1, 5)
            for diode in (Diode.D1, Diode.D2, Diode.D3, Diode.D4)]


def processmetrology(table, header, *, window=None, faintparam=None, keepraw=False,
                     onlyhigh=False, offsets=None, method="auto", device=0, mjd=None):
    """processmetrology (src/GPPupilDemodulation.jl:128-255) on the GPU, minus FITS I/O.

    table: mapping of the METROLOGY columns with at least "TIME" (µs, N) and "VOLT" (N×80
    Float32 rows); header: mapping of its header (the "MJD-OBS" key gives mjd, :139).  faintparam:
    FaintStates (e.g. buildfaintparameters(primary header)).  offsets: (40,) complex centres, or
    False → fitoffsets (a circle fit, offsets=True, is not restated).
    Returns (table, header) as new dicts: VOLT replaced by the Float32 demodulated rows (80 per
    row, or 144 with keepraw: raw rows then the 32 demodulated columns), in window mode the
    per-sample Float32 columns ABSA, ARGA, B, PHI (+ X0, Y0) as (N, 32) rows and STATE (Int8) with
    faint states; otherwise the header gains the per-diode DEMODULATION keywords (:172-189);
    PROCSOFT = "GPPupilDemodulation.jl" in both modes (:253).  mjd: the reference's argument
    (the primary header's MJD-OBS); default header["MJD-OBS"]."""
    mjd = float(header["MJD-OBS"] if mjd is None else mjd)  # the reference's mjd argument
    times = metrology_times(table["TIME"], mjd)
    state = None
    if faintparam is not None:
        state = buildstates(faintparam, times)  # default delays of buildstates (:144)
    volt = np.ascontiguousarray(table["VOLT"], dtype=np.float32)
    if offsets is True:
        raise NotImplementedError("compute_offsets (circle fit) is outside the hot path")
    fitoffsets = offsets is False
    vout, params, tabs = process_volt(times, volt, offsets=None if fitoffsets else offsets,
                                      window=window, faintparam=state, onlyhigh=onlyhigh,
                                      method=method, device=device)
    tab = dict(table)
    hdr = dict(header)
    N = times.size
    if keepraw:  # s[1:80,:] = volt; s[81:2:end,:] = real(output[:,1:32])' … (:162-167, :228-233)
        s = np.empty((N, 144), dtype=np.float32)
        s[:, :80] = volt
        s[:, 80:] = vout[:, :64]
        vout = s
    if window is None:
        for side, tel, diode in _diode_order():
            p = params[idx(side, tel, diode) - 1]
            b, phi = float(p["b"]), float(p["phi"])
            if b < 0:  # rem2pi(ϕ+π, RoundNearest) (:175-178; b ≥ 0 already, :427-430)
                b = -b
                phi = float(np.remainder(phi + np.pi + np.pi, 2 * np.pi) - np.pi)
            name = f"{side.name} T{tel} {diode.name}"
            if fitoffsets:
                hdr[f"DEMODULATION CENTER X0 {name}"] = float(p["c"].real)
                hdr[f"DEMODULATION CENTER Y0 {name}"] = float(p["c"].imag)
            hdr[f"DEMODULATION AMPLITUDE ABS {name}"] = float(abs(p["a"]))
            hdr[f"DEMODULATION AMPLITUDE ARG {name}"] = float(np.angle(p["a"]))
            hdr[f"DEMODULATION SIN AMPLITUDE {name}"] = b
            hdr[f"DEMODULATION SIN PHASE {name}"] = phi
    else:
        order = ["X0", "Y0"] if fitoffsets else []
        for key in order + ["ABSA", "ARGA", "B", "PHI"]:
            tab[key] = np.ascontiguousarray(tabs[key].T)  # (N, 32): Julia's 32×N column per row
        if state is not None:
            tab["STATE"] = state.astype(np.int8)
    hdr["PROCSOFT"] = "GPPupilDemodulation.jl"
    tab["VOLT"] = vout
    return tab, hdr


def process_exposure(filename, outname, *, offsets, window=None, keepraw=False, onlyhigh=False,
                     nofaint=False, method="auto", device=0):
    """One exposure file as the reference's main loop handles it (src/GPPupilDemodulation.jl:
    357-414, without the argument parsing and directory walk): skipped (returns False) unless the
    primary header has ESO INS PMC1 MODULATE = T and ESO INS MET MODE is not OFF; FAINT mode
    builds the faint states from the primary header unless `nofaint`; MJD-OBS gives mjd; the
    METROLOGY table goes through processmetrology and the file is copied to `outname` with that
    table and header replaced (FITScopy!, fits.fits_copy).  offsets: the 40 complex centres
    (Stefan's, or zeros for "uncentered") or False ("fit")."""
    from . import fits
    hdus = fits.read_fits(filename)
    prim = hdus[0][0]
    if not prim.get("ESO INS PMC1 MODULATE", False):
        return False
    metmode = prim.get("ESO INS MET MODE", "ON")
    if metmode == "OFF":
        return False
    faint = buildfaintparameters(prim) if metmode == "FAINT" and not nofaint else None
    met = next(((h, d) for h, d in hdus if h.get("EXTNAME") == "METROLOGY"), None)
    if met is None:
        raise KeyError(f"{filename}: no METROLOGY table")
    table, hdr = processmetrology(met[1], met[0], window=window, faintparam=faint,
                                  keepraw=keepraw, onlyhigh=onlyhigh, offsets=offsets,
                                  method=method, device=device, mjd=float(prim["MJD-OBS"]))
    fits.fits_copy(outname, filename, {"METROLOGY": table}, {"METROLOGY": hdr})
    return True
