"""In-tree build of libgpdemod.so for gfx950 (hipcc; no JIT cache, travels with the repo)."""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libgpdemod.so")
SOURCES = ["gpd_engine.hip"]
HEADERS = ["gpd_kernels.hpp", "gpd_device.hpp", "gpd_newuoa.hpp", "gpd_states.hpp", "gpd_jlmath.h"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
         # the exact evaluator and NEWUOA must not fuse a*b+c (Julia does not contract);
         # the moment kernel asks for FMAs explicitly with fma().
         "-ffp-contract=off", "-Wall", "-Wno-unused-function"]


def _stale() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(HERE, "..", "include", "gpdemod.h"))
    return any(os.path.getmtime(p) > t for p in deps if os.path.exists(p))


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return OUT
    cmd = [HIPCC, *FLAGS, "-o", OUT + ".tmp", *[os.path.join(CSRC, s) for s in SOURCES]]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed ({r.returncode}):\n{r.stderr[-4000:]}")
    if verbose and r.stderr:
        print(r.stderr)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force=True, verbose=True))
