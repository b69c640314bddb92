"""ctypes binding of libgpdemod.so (include/gpdemod.h).

The product path has no CPU fallback: if the HIP library is missing this module raises on
import, and every compute entry point returns GPD_E_NODEV when no GPU is visible.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# GPD_LIB=<name>: load libgpdemod_<name>.so instead — "diag" is the diagnostics build
# (moment-kernel timing variants, build.py --diag); other names are A/B builds of another revision
LIB_PATH = os.path.join(HERE, f"libgpdemod_{os.environ['GPD_LIB']}.so" if os.environ.get("GPD_LIB")
                        else "libgpdemod.so")

GPD_ABI_VERSION = 1
GPD_FIT_OFFSETS = 0x1
GPD_RECENTER = 0x2
GPD_ONLY_HIGH = 0x4
GPD_METHOD_EXACT = 0x10
GPD_METHOD_HARMONIC = 0x20
GPD_FP32 = 0x40  # Float32 per-sample arithmetic (exact evaluator), include/gpdemod.h

GPD_ST_REFIT = 0x1
GPD_ST_MAXFUN = 0x2
GPD_ST_NAN = 0x4
GPD_ST_EXACT = 0x8
GPD_ST_FALLBACK = 0x10
GPD_ST_SYNC = 0x20

GPD_OK = 0
GPD_E_ARG = -1
GPD_E_HIP = -2
GPD_E_NODEV = -3
GPD_E_OOM = -4
GPD_E_UNSAFE = -5

PARAM_DTYPE = np.dtype(
    [("c", np.complex128), ("a", np.complex128), ("b", np.float64), ("phi", np.float64),
     ("chi2", np.float64), ("nfev", np.int32), ("status", np.int32)], align=True)
assert PARAM_DTYPE.itemsize == 64

# every symbol declared in include/gpdemod.h
EXPORTS = ("gpd_version", "gpd_strerror", "gpd_device_count", "gpd_fit_batch",
           "gpd_fit_batch_dev", "gpd_chi2_batch", "gpd_chi2_batch_dev", "gpd_buildstates",
           "gpd_synth_fill_dev", "gpd_last_timings", "gpd_fit_windows", "gpd_fit_windows_dev",
           "gpd_process_volt", "gpd_fit_batch_c32", "gpd_fit_batch_c32_dev", "gpd_fit_windows_c32",
           "gpd_fit_windows_c32_dev", "gpd_buildstates_dev", "gpd_release", "gpd_libm_eval",
           "gpd_mean_var_power", "gpd_build_id", "gpd_last_faint_stats", "gpd_set_option",
           "gpd_get_option", "gpd_reset_options", "gpd_option_name", "gpd_demodulateall",
           "gpd_demodulateall_c32")


class GpdError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"gpdemod error {code}: {msg}")
        self.code = code


_lib = None


def _warn_legacy_env():
    """The library reads no environment variable (r5); the GPD_* variables earlier rounds' A/B
    scripts set (GPD_MOMENTS, GPD_FIT_PROF, GPD_COHORTS, …) now do nothing.  Say so once, so a run
    that sets one does not silently measure the default path (advisor r5).  GPD_LIB (library
    variant) and GPD_OPTS (options_from_env, the A/B tools) are still read on the Python side."""
    import warnings
    legacy = sorted(k for k in os.environ
                    if k.startswith("GPD_") and k not in ("GPD_LIB", "GPD_OPTS"))
    if legacy:
        warnings.warn(f"environment variables {legacy} are ignored: the library reads no "
                      "environment; set options with gpd_set_option / GPD_OPTS=name=value,… "
                      "(tools) instead", RuntimeWarning, stacklevel=3)


def load():
    """Load libgpdemod.so (built in-tree by __graft_entry__.build() / build.py)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} not found: the HIP extension is not built "
            "(run `python -c 'import __graft_entry__ as g; g.build()'`). No CPU fallback exists.")
    _warn_legacy_env()
    L = ctypes.CDLL(LIB_PATH)
    V, I64, I32, U32, D = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, ctypes.c_uint32, ctypes.c_double
    L.gpd_version.restype = ctypes.c_int
    L.gpd_version.argtypes = []
    L.gpd_strerror.restype = ctypes.c_char_p
    L.gpd_strerror.argtypes = [ctypes.c_int]
    L.gpd_device_count.restype = ctypes.c_int
    L.gpd_device_count.argtypes = []
    L.gpd_release.restype = ctypes.c_int
    L.gpd_release.argtypes = [ctypes.c_int]
    common = [I64, I64, V, V, I64, V, I64, I64, V, V, D, V, U32, I32, V, V, I64]
    L.gpd_fit_batch.restype = ctypes.c_int
    L.gpd_fit_batch.argtypes = common + [I32, ctypes.c_char_p, ctypes.c_size_t]
    L.gpd_fit_batch_dev.restype = ctypes.c_int
    L.gpd_fit_batch_dev.argtypes = common + [ctypes.c_int, V, ctypes.c_char_p, ctypes.c_size_t]
    chi = [I64, I64, V, V, I64, V, I64, I64, V, V, D, V, U32, V]
    L.gpd_chi2_batch.restype = ctypes.c_int
    L.gpd_chi2_batch.argtypes = chi + [I32, ctypes.c_char_p, ctypes.c_size_t]
    L.gpd_chi2_batch_dev.restype = ctypes.c_int
    L.gpd_chi2_batch_dev.argtypes = chi + [ctypes.c_int, V, ctypes.c_char_p, ctypes.c_size_t]
    win = [I64, I64] + common[1:]  # n_samples, window, n_cols, ... (same tail as gpd_fit_batch)
    L.gpd_fit_windows.restype = ctypes.c_int
    L.gpd_fit_windows.argtypes = win + [I32, ctypes.c_char_p, ctypes.c_size_t]
    L.gpd_fit_windows_dev.restype = ctypes.c_int
    L.gpd_fit_windows_dev.argtypes = win + [ctypes.c_int, V, ctypes.c_char_p, ctypes.c_size_t]
    # Float32-storage variants: same argument lists (d / fc are ComplexF32 arrays)
    for name, base in (("gpd_fit_batch_c32", "gpd_fit_batch"),
                       ("gpd_fit_batch_c32_dev", "gpd_fit_batch_dev"),
                       ("gpd_fit_windows_c32", "gpd_fit_windows"),
                       ("gpd_fit_windows_c32_dev", "gpd_fit_windows_dev")):
        getattr(L, name).restype = ctypes.c_int
        getattr(L, name).argtypes = getattr(L, base).argtypes
    L.gpd_process_volt.restype = ctypes.c_int
    L.gpd_process_volt.argtypes = [I64, V, V, I64, V, V, D, V, U32, I32, I64, V, V, I64,
                                   ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t]
    L.gpd_buildstates.restype = ctypes.c_int
    L.gpd_buildstates.argtypes = [I64, V, I64, V, I64, V, D, D, V]
    L.gpd_buildstates_dev.restype = ctypes.c_int
    L.gpd_buildstates_dev.argtypes = [I64, V, I64, V, I64, V, I64, D, D, V, ctypes.c_int, V]
    L.gpd_synth_fill_dev.restype = ctypes.c_int
    L.gpd_synth_fill_dev.argtypes = [I64, I64, I64, ctypes.c_uint64, D, D, D, ctypes.c_int, D, V, V,
                                     I64, V, I64, V, V, ctypes.c_int, V]
    L.gpd_mean_var_power.restype = ctypes.c_int
    L.gpd_mean_var_power.argtypes = [I64, I64, V, I64, V, U32, V, ctypes.c_int, ctypes.c_char_p,
                                     ctypes.c_size_t]
    L.gpd_libm_eval.restype = ctypes.c_int
    L.gpd_libm_eval.argtypes = [ctypes.c_int, I64, V, V, V, ctypes.c_int]
    L.gpd_build_id.restype = ctypes.c_char_p
    L.gpd_build_id.argtypes = []
    L.gpd_last_faint_stats.restype = ctypes.c_int
    L.gpd_last_faint_stats.argtypes = [ctypes.c_int, V, I64]
    L.gpd_last_timings.restype = ctypes.c_int
    L.gpd_last_timings.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                   ctypes.POINTER(ctypes.c_double), ctypes.c_int]
    # (entry points added in r5: an A/B library of an older revision, GPD_LIB, may lack them)
    for name in ("gpd_demodulateall", "gpd_demodulateall_c32"):
        if hasattr(L, name):
            getattr(L, name).restype = ctypes.c_int
            getattr(L, name).argtypes = [I64, V, V, I64, V, V, U32, I32, V, V, I64, I32,
                                         ctypes.c_char_p, ctypes.c_size_t]
    if hasattr(L, "gpd_set_option"):
        L.gpd_set_option.restype = ctypes.c_int
        L.gpd_set_option.argtypes = [ctypes.c_char_p, I64]
        L.gpd_get_option.restype = ctypes.c_int
        L.gpd_get_option.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64)]
        L.gpd_reset_options.restype = None
        L.gpd_reset_options.argtypes = []
        L.gpd_option_name.restype = ctypes.c_char_p
        L.gpd_option_name.argtypes = [ctypes.c_int]
    if L.gpd_version() != GPD_ABI_VERSION:
        raise ImportError(f"libgpdemod ABI {L.gpd_version()} != {GPD_ABI_VERSION}")
    _lib = L
    return L


def ptr(a) -> ctypes.c_void_p | None:
    if a is None:
        return None
    if isinstance(a, int):
        return ctypes.c_void_p(a)
    return a.ctypes.data_as(ctypes.c_void_p)


def check(rc: int, errbuf=None):
    if rc != GPD_OK:
        L = load()
        msg = errbuf.value.decode(errors="replace") if errbuf is not None else ""
        raise GpdError(rc, f"{L.gpd_strerror(rc).decode()}: {msg}")


LIBM_FN = {"sin": 0, "cos": 1, "sincos": 2, "atan": 3, "atan2": 4, "hypot": 5, "rem_pio2": 6, "hypot_nb": 7,
           "sin_sel": 8, "sincos_sel": 9, "sin_ph_shift": 10}


def libm_eval(fn: str, x, y=None, device: int = 0):
    """Julia Base's sin/cos/sincos/atan/atan(y,x)/hypot/rem_pio2 as the device evaluates them
    (gpd_jlmath.h).  sincos → (n, 2) [s, c]; rem_pio2 → (n, 3) [quadrant, hi, lo]."""
    code = LIBM_FN[fn]
    x = np.ascontiguousarray(x, dtype=np.float64).ravel()
    yy = None if y is None else np.ascontiguousarray(y, dtype=np.float64).ravel()
    width = {2: 2, 6: 3, 9: 2}.get(code, 1)
    out = np.empty(x.size * width)
    check(load().gpd_libm_eval(code, x.size, ptr(x), ptr(yy), ptr(out), device))
    return out.reshape(-1, width) if width > 1 else out


def build_id() -> str:
    """Id of the sources the loaded library was built from (build.tree_id at build time)."""
    return load().gpd_build_id().decode()


def last_faint_stats(n_series: int, device: int = 0):
    """The faint statistics the last fit call on `device` used (gpd_last_faint_stats): m and w
    as (n, 5) arrays indexed by MetState code + 1, and (n, 3) [Σw|d|², Σw m² n, Σ(w m)²|d|²]."""
    out = np.empty((n_series, 16))
    check(load().gpd_last_faint_stats(device, ptr(out), n_series))
    return out[:, :5], out[:, 5:10], out[:, 10:13]


def timings(device: int = 0):
    """Per-kernel HIP-event timings (ms) of the last gpd_fit_batch_dev call on `device`; a stage
    that ran once per series cohort (the pipelined harmonic path) is summed over its cohorts."""
    L = load()
    cap = 160  # >= kMaxTimers (gpd_engine.hip)
    names = (ctypes.c_char_p * cap)()
    ms = (ctypes.c_double * cap)()
    n = L.gpd_last_timings(device, names, ms, cap)
    out = {}
    for i in range(n):
        k = names[i].decode()
        out[k] = out.get(k, 0.0) + ms[i]
    return out


# ---- test and diagnostics controls (gpd_set_option; the library reads no environment) --------
def set_option(name: str, value: int):
    """Set one of the library's process-wide test/diagnostics options (include/gpdemod.h)."""
    check(load().gpd_set_option(name.encode(), int(value)))


def get_option(name: str) -> int:
    v = ctypes.c_int64(0)
    check(load().gpd_get_option(name.encode(), ctypes.byref(v)))
    return v.value


def reset_options():
    """Every option back to its production default."""
    load().gpd_reset_options()


def option_names():
    L, out, i = load(), [], 0
    while (n := L.gpd_option_name(i)) is not None:
        out.append(n.decode())
        i += 1
    return out


class options:
    """Context manager: `with options(mix=0, faint_stats=1): ...` sets the options for the block
    and restores their previous values afterwards."""

    def __init__(self, **kw):
        self.kw = kw
        self.old = {}

    def __enter__(self):
        for k, v in self.kw.items():
            self.old[k] = get_option(k)
            set_option(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.old.items():
            set_option(k, v)
        return False


def options_from_env(var: str = "GPD_OPTS"):
    """For the A/B tools only (never called by the package): apply "name=value,..." from the
    environment variable `var` through set_option, and return the dict applied."""
    spec = os.environ.get(var, "")
    applied = {}
    for item in filter(None, (x.strip() for x in spec.split(","))):
        k, v = item.split("=", 1)
        set_option(k.strip(), int(v))
        applied[k.strip()] = int(v)
    return applied
