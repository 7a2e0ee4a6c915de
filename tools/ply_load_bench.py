"""Load time of a 1M-Gaussian degree-3 PLY into a device scene (tooling):
the host path (native parse + NumPy activations + scale_data + points_center +
upload/repack) against gsr_scene_load_ply (chunked parse into pinned buffers
overlapped with the copies, activations / rescale / mean on the GPU).
usage: python tools/ply_load_bench.py [N] [OUT.json]"""
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

from oracle import ply_oracle as P  # noqa: E402  (test infrastructure: writes the file)
from test_ply import vertex_array  # noqa: E402


def main():
    import torch

    from gsviewer_amd.ply import load_ply
    from gsviewer_amd.rasterizer import HipScene
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    path = os.path.join(tempfile.mkdtemp(), "bench.ply")
    with open(path, "wb") as f:
        f.write(P.ply_bytes(vertex_array(n, deg=3, seed=0), "binary_little_endian"))
    torch.cuda.init()
    HipScene.from_ply(path).close()  # warm-up (page cache, code objects)
    res = {"n": n, "file_bytes": os.path.getsize(path)}
    for name in ("host", "device"):
        ts = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if name == "host":
                g = load_ply(path)
                g.scale_data(5.0)
                _ = g.points_center
                sc = HipScene.from_gaussian_data(g)
            else:
                sc = HipScene.from_ply(path, 5.0)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
            sc.close()
        res[f"{name}_ms"] = 1e3 * min(ts)
    print(json.dumps(res))
    if len(sys.argv) > 2:
        json.dump(res, open(sys.argv[2], "w"))


if __name__ == "__main__":
    main()
