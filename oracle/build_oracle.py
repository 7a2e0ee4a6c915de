"""Build the C oracle (test infrastructure) into oracle/_build/libgl_oracle.so.

gcc, -O2, -ffp-contract=off (same evaluation order as oracle/gl_oracle.py and
the HIP preprocess), OpenMP for the multithreaded CPU baseline.  No reference
sources are compiled: the reference has no C/C++ code,
so there is no oracle/_ref build.
"""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "_build", "libgl_oracle.so")
SRC = os.path.join(HERE, "gl_oracle.c")


def build(verbose=False):
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    if os.path.exists(OUT) and os.path.getmtime(OUT) >= os.path.getmtime(SRC):
        return OUT
    cmd = ["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math", "-fopenmp", "-shared", "-fPIC", "-std=c11",
           "-Wall", SRC, "-o", OUT + ".tmp", "-lm"]
    subprocess.run(cmd, check=True)
    os.replace(OUT + ".tmp", OUT)
    if verbose:
        print("built", OUT)
    return OUT


if __name__ == "__main__":
    build(verbose=True)
