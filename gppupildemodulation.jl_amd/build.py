"""In-tree build of libgpdemod.so for gfx950 (hipcc; no JIT cache, travels with the repo)."""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libgpdemod.so")
# diagnostics build: the production library plus the moment kernel's timing variants
# (GPD_MOMENTS=ws_nomfma|ws_noload|ws_nof0|ws_noq|ws_mfmaonly|ws_prof; results invalid),
# loaded instead of libgpdemod.so when GPD_LIB=diag (tools/pmc_variants.sh)
OUT_DIAG = os.path.join(HERE, "libgpdemod_diag.so")
SOURCES = ["gpd_engine.hip"]
HEADERS = ["gpd_kernels.hpp", "gpd_device.hpp", "gpd_newuoa.hpp", "gpd_states.hpp", "gpd_jlmath.h"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
         # the exact evaluator and NEWUOA must not fuse a*b+c (Julia does not contract);
         # the moment kernel asks for FMAs explicitly with fma().
         "-ffp-contract=off", "-Wall", "-Wno-unused-function"]


def _stale(out: str) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(HERE, "..", "include", "gpdemod.h"))
    return any(os.path.getmtime(p) > t for p in deps if os.path.exists(p))


def build(force: bool = False, verbose: bool = False, diag: bool = False) -> str:
    out = OUT_DIAG if diag else OUT
    if not force and not _stale(out):
        return out
    cmd = [HIPCC, *FLAGS, *(["-DGPD_DIAG"] if diag else []), "-o", out + ".tmp",
           *[os.path.join(CSRC, s) for s in SOURCES]]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed ({r.returncode}):\n{r.stderr[-4000:]}")
    if verbose and r.stderr:
        print(r.stderr)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    import sys

    print(build(force=True, verbose=True, diag="--diag" in sys.argv))
