"""gpdemod — MI355X-native drop-in for the demodulateall hot path of
FerreolS/GPPupilDemodulation.jl (src/Modulation.jl:344-435).

The package directory name contains a dot, so load it by path, e.g.::

    import importlib.util, sys
    spec = importlib.util.spec_from_file_location(
        "gpdemod", "gppupildemodulation.jl_amd/__init__.py",
        submodule_search_locations=["gppupildemodulation.jl_amd"])
    gpdemod = importlib.util.module_from_spec(spec); sys.modules["gpdemod"] = gpdemod
    spec.loader.exec_module(gpdemod)

(`gpdemod_loader.load()` at the repo root does exactly this.)
"""
from ._lib import (GPD_FIT_OFFSETS, GPD_FP32, GPD_METHOD_EXACT, GPD_METHOD_HARMONIC, GPD_ONLY_HIGH,
                   GPD_RECENTER, GPD_ST_EXACT, GPD_ST_FALLBACK, GPD_ST_MAXFUN, GPD_ST_NAN,
                   GPD_ST_REFIT, GPD_ST_SYNC, PARAM_DTYPE, GpdError, build_id, get_option,
                   last_faint_stats, libm_eval, load, option_names, options, options_from_env,
                   reset_options, set_option, timings)
from .demod import (DAY_TO_SEC, M_2PI, MJD_1970_1_1, Diode, FaintStates, MetState,
                    ModulationNoOffsets, ModulationWithOffsets, Side, buildfaintparameters,
                    buildstates, chi2_batch, compute_mean_var_power, demodulate_windows,
                    mean_var_power_batch, metrology_times, process_exposure, processmetrology,
                    demodulateall, fc_column_of, fit_batch, fit_windows, idx, process_volt,
                    read_stefan_file, window_length, window_tables)
from . import fits  # processmetrology's FITS output (host I/O)

__all__ = [
    "fits", "process_exposure",
    "GPD_FIT_OFFSETS", "GPD_FP32", "GPD_METHOD_EXACT", "GPD_METHOD_HARMONIC", "GPD_ONLY_HIGH", "GPD_RECENTER",
    "GPD_ST_EXACT", "GPD_ST_FALLBACK", "GPD_ST_MAXFUN", "GPD_ST_NAN", "GPD_ST_REFIT",
    "GPD_ST_SYNC",
    "PARAM_DTYPE", "GpdError", "build_id", "get_option", "last_faint_stats", "option_names",
    "options", "options_from_env", "reset_options", "set_option", "libm_eval", "load", "timings", "M_2PI", "Diode", "FaintStates", "MetState",
    "ModulationNoOffsets", "ModulationWithOffsets", "Side", "buildstates", "chi2_batch",
    "demodulate_windows", "demodulateall", "fc_column_of", "fit_batch", "fit_windows", "idx",
    "window_length", "window_tables", "process_volt", "read_stefan_file", "DAY_TO_SEC",
    "MJD_1970_1_1", "buildfaintparameters", "metrology_times", "processmetrology",
    "compute_mean_var_power", "mean_var_power_batch",
]
