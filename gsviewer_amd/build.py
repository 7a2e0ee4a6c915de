"""Build the in-tree HIP shared library ``gsviewer_amd/libgsr.so`` for gfx950.

Usage: ``python -m gsviewer_amd.build [--jobs N] [--debug]``.  The library is
plain hipcc output (no torch extension machinery): a C-ABI ``.so`` whose
entry points are declared in ``include/gsr.h``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INCLUDE = os.path.join(ROOT, "include")
BUILD = os.path.join(ROOT, "build", "gsr")
LIB = os.path.join(PKG, "libgsr.so")
ARCH = os.environ.get("GSR_OFFLOAD_ARCH", "gfx950")

SOURCES = ["api.hip", "scene.hip", "scan.hip", "radix_sort.hip", "preprocess.hip", "composite.hip",
           "export.hip",
           "ply.cpp"]
# The per-Gaussian stage must evaluate exactly like the oracle: no contraction.
EXTRA_FLAGS = {"preprocess.hip": ["-ffp-contract=off"]}


def hipcc():
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (set HIPCC)")


def _compile(src, debug, bdir=BUILD, defines=()):
    obj = os.path.join(bdir, os.path.basename(src) + ".o")
    deps = [os.path.join(CSRC, src), os.path.join(CSRC, "gsr_internal.h"), os.path.join(INCLUDE, "gsr.h"),
            os.path.join(INCLUDE, "gsr_io.h")]
    if os.path.exists(obj) and all(os.path.getmtime(obj) >= os.path.getmtime(d) for d in deps):
        return obj
    # -fno-slp-vectorize: plain -O3 packs adjacent f32 adds/muls into
    # v_pk_*_f32, which costs more issue than the scalar pair on gfx950
    # (MI355X_MICROARCH.md, packed f32 VALU row)
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", "-c", "-fno-slp-vectorize",
           "-fhip-fp32-correctly-rounded-divide-sqrt", "-Wall", "-Wno-unused-function", "-Wno-bitwise-instead-of-logical",
           "-I", INCLUDE, "-I", CSRC, os.path.join(CSRC, src), "-o", obj]
    cmd += ["-O0", "-g"] if debug else ["-O3"]
    cmd += EXTRA_FLAGS.get(src, [])
    cmd += ["-D" + d for d in defines]
    # experiment builds only (never the product): extra flags for one source, "file.hip:-flag,-flag"
    extra = os.environ.get("GSR_BUILD_EXTRA", "")
    if extra and defines and extra.split(":", 1)[0] == src:
        cmd += extra.split(":", 1)[1].split(",")
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    if r.stderr.strip():
        sys.stderr.write(r.stderr)
    return obj


def build(jobs=None, debug=False, verbose=True, defines=(), out=None):
    """Compile and link libgsr.so.  `defines`/`out` build an experiment
    variant (extra -D flags) into a separate .so; the default build is the
    product library."""
    out = out or LIB
    bdir = BUILD if not defines else BUILD + "_" + "_".join(d.replace("=", "") for d in defines)
    os.makedirs(bdir, exist_ok=True)
    jobs = jobs or min(len(SOURCES), os.cpu_count() or 4, 8)
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, debug, bdir, defines), SOURCES))
    if os.path.exists(out) and all(os.path.getmtime(out) >= os.path.getmtime(o) for o in objs):
        return out
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", out + ".tmp"] + objs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(out + ".tmp", out)
    if verbose:
        print("built", out)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--debug", action="store_true")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="experiment define (variant build)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    build(a.jobs, a.debug, defines=a.defines, out=a.out)
