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
# translation units compiled in parallel and linked into one library (gpd_kernels.hpp GPD_OWNS:
# unit 0 = host code + light kernels, the others = the heavy kernel instances)
# the slowest units first (the exact path's instances), so the pool's tail is short
SOURCES = ["gpd_part3.hip", "gpd_part4.hip", "gpd_part7.hip", "gpd_part8.hip", "gpd_part12.hip",
           "gpd_part13.hip", "gpd_part14.hip", "gpd_part15.hip", "gpd_part16.hip", "gpd_part17.hip",
           "gpd_part18.hip", "gpd_part19.hip", "gpd_part5.hip", "gpd_part9.hip",
           "gpd_part10.hip", "gpd_part11.hip", "gpd_part2.hip", "gpd_part6.hip", "gpd_part1.hip",
           "gpd_engine.hip"]
HEADERS = ["gpd_kernels.hpp", "gpd_device.hpp", "gpd_newuoa.hpp", "gpd_states.hpp", "gpd_jlmath.h"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
         # the exact evaluator and NEWUOA must not fuse a*b+c (Julia does not contract);
         # the moment kernel asks for FMAs explicitly with fma().
         "-ffp-contract=off", "-Wall", "-Wno-unused-function"]


def tree_id() -> str:
    """Build id of the sources in this tree: sha256 (first 16 hex digits) over the contents of
    every translation unit and header, include/gpdemod.h, and the compiler flags — compiled into
    the library (gpd_build_id) so that a run can show which sources its .so was built from."""
    import hashlib

    h = hashlib.sha256()
    for f in sorted(SOURCES + HEADERS):
        h.update(f.encode() + b"\0")
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
    with open(os.path.join(HERE, "..", "include", "gpdemod.h"), "rb") as fh:
        h.update(fh.read())
    h.update(" ".join(FLAGS).encode())
    return h.hexdigest()[:16]


ID_MARKER = b"GPD_BUILD_ID="


def unit_deps(src: str) -> list:
    """`src` and every unit it #includes, transitively (gpd_part6.hip includes gpd_part2.hip,
    gpd_part9-11.hip gpd_part5.hip, …): an edit to an included unit must change the key of
    every unit that compiles it."""
    import re

    seen, todo = [], [src]
    while todo:
        f = todo.pop(0)
        if f in seen:
            continue
        seen.append(f)
        with open(os.path.join(CSRC, f)) as fh:
            todo += re.findall(r'^\s*#\s*include\s+"(gpd_part\d+\.hip)"', fh.read(), re.M)
    return seen


def unit_key(src: str, extra=(), bid: str = "") -> str:
    """Content key of one translation unit's object: its source and every unit it includes, the
    headers, include/gpdemod.h, the compiler and its flags (and the build id for unit 0)."""
    import hashlib

    h = hashlib.sha256()
    for f in unit_deps(src) + HEADERS:
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    with open(os.path.join(HERE, "..", "include", "gpdemod.h"), "rb") as fh:
        h.update(fh.read())
    h.update(" ".join([HIPCC, *FLAGS, *extra, bid if src == "gpd_engine.hip" else ""]).encode())
    return h.hexdigest()


def lib_id(path: str) -> str | None:
    """The build id embedded in a built library (read from its bytes, without loading it)."""
    try:
        with open(path, "rb") as fh:
            data = fh.read()
    except OSError:
        return None
    i = data.find(ID_MARKER)
    if i < 0:
        return None
    return data[i + len(ID_MARKER):i + len(ID_MARKER) + 16].decode(errors="replace")


def _stale(out: str) -> bool:
    # content, not mtimes: a library whose embedded id differs from the tree's is rebuilt
    return not os.path.exists(out) or lib_id(out) != tree_id()


def build(force: bool = False, verbose: bool = False, diag: bool = False, jobs: int = 0,
          variant: str | None = None, defines: tuple = (), only: tuple = (),
          flags: tuple = ()) -> str:
    """variant: an A/B build libgpdemod_<variant>.so with extra -D `defines` and compiler
    `flags` (loaded with GPD_LIB=<variant>, tools/ab_*.sh); `only`: compile just these units for
    the variant and link the other units' objects of the release build; diag: the diagnostics
    build."""
    out = (os.path.join(HERE, f"libgpdemod_{variant}.so") if variant
           else OUT_DIAG if diag else OUT)
    if not force and not _stale(out):
        return out
    objdir = os.path.join(HERE, "build", variant or ("diag" if diag else "release"))
    os.makedirs(objdir, exist_ok=True)
    extra = (["-DGPD_DIAG"] if diag else []) + [f"-D{d}" for d in defines] + list(flags)
    # the build id is compiled into unit 0 only (gpd_build_id); an object whose inputs (the
    # headers, its unit, the flags) are unchanged since its last compile is reused (.key file)
    bid = f'-DGPD_BUILD_ID="{tree_id()}"'
    jobs = jobs or max(1, min(len(SOURCES), os.cpu_count() or 1))
    procs, objs, errs = [], [], []
    pending = [u for u in SOURCES if not only or u in only]
    if only:  # the other units from the release build
        rel = os.path.join(HERE, "build", "release")
        reuse = [u for u in SOURCES if u not in only]
        # every kernel takes Problem & co. by value: a release object built from other sources
        # or headers would link silently against another struct layout (advisor r3) — refuse
        # any whose content key is not the current release key of its unit (advisor r4: keys,
        # not mtimes, so a touched but unchanged header does not refuse valid objects)
        rbid = f'-DGPD_BUILD_ID="{tree_id()}"'
        stale = []
        for u in reuse:
            o = os.path.join(rel, u.replace(".hip", ".o"))
            try:
                with open(o + ".key") as fh:
                    ok = os.path.exists(o) and fh.read() == unit_key(u, [], rbid)
            except OSError:
                ok = False
            if not ok:
                stale.append(os.path.basename(o))
        if stale:
            raise RuntimeError("--only: release objects not built from this tree (rebuild the "
                               "release library first): " + ", ".join(stale))
        objs += [os.path.join(rel, u.replace(".hip", ".o")) for u in reuse]
    keys = {}
    while pending or procs:
        while pending and len(procs) < jobs:
            src = pending.pop(0)
            obj = os.path.join(objdir, src.replace(".hip", ".o"))
            objs.append(obj)
            keys[src] = unit_key(src, extra, bid)
            try:
                with open(obj + ".key") as fh:
                    if fh.read() == keys[src] and os.path.exists(obj):
                        continue  # unchanged inputs: reuse the object
            except OSError:
                pass
            ex = extra + ([bid] if src == "gpd_engine.hip" else [])
            cmd = [HIPCC, *FLAGS, *ex, "-c", "-o", obj + ".tmp", os.path.join(CSRC, src)]
            procs.append((src, obj, subprocess.Popen(cmd, stdout=subprocess.PIPE,
                                                     stderr=subprocess.PIPE, text=True)))
        if not procs:
            continue
        src, obj, p = procs.pop(0)
        _, err = p.communicate()
        if p.returncode != 0:
            errs.append(f"{src}: hipcc failed ({p.returncode}):\n{err[-4000:]}")
        else:
            if verbose and err:
                print(err)
            os.replace(obj + ".tmp", obj)
            with open(obj + ".key", "w") as fh:
                fh.write(keys[src])
    if errs:
        raise RuntimeError("\n".join(errs))
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out + ".tmp", *objs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed ({r.returncode}):\n{r.stderr[-4000:]}")
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    import sys

    # build.py [--diag] [--variant NAME -DDEF ... --flag=-mllvm --flag=-opt ...]
    argv = sys.argv[1:]
    var = argv[argv.index("--variant") + 1] if "--variant" in argv else None
    defs = tuple(a[2:] for a in argv if a.startswith("-D"))
    only = tuple(argv[argv.index("--only") + 1].split(",")) if "--only" in argv else ()
    flg = tuple(a[len("--flag="):] for a in argv if a.startswith("--flag="))
    print(build(force=True, verbose=True, diag="--diag" in argv, variant=var, defines=defs,
                only=only, flags=flg))
