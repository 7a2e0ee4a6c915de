"""Throughput with K independent views in flight (tooling): host time per
render call vs wall time per frame.  usage: python tools/inflight_probe.py K [K ...]"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gsviewer_amd import _lib  # noqa: E402
from gsviewer_amd.gaussian_data import garden_standin  # noqa: E402
from gsviewer_amd.multiview import view_of  # noqa: E402
from gsviewer_amd.rasterizer import HipContext, HipScene, RenderSettings, camera_from, render_into  # noqa: E402

_lib.load()
g = garden_standin(1_000_000, seed=1)
scene = HipScene.from_gaussian_data(g)
H, W = 1080, 1920
for K in [int(a) for a in sys.argv[1:]]:
    ctxs = [HipContext() for _ in range(K)]
    streams = [torch.cuda.Stream() for _ in range(K)]
    outs = [torch.empty((3, H, W), dtype=torch.float32, device="cuda") for _ in range(K)]
    cams = [camera_from(view_of(k, H, W)) for k in range(K)]
    st = RenderSettings(t_min=1e-4, out_layout=0)
    host = []

    def step(i):
        k = i % K
        t = time.perf_counter()
        with torch.cuda.stream(streams[k]):
            render_into(ctxs[k], scene, cams[k], st, outs[k])
        host.append(time.perf_counter() - t)

    for i in range(40):
        step(i)
    torch.cuda.synchronize()
    host.clear()
    t0 = time.perf_counter()
    n = 400
    for i in range(n):
        step(i)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    h = np.array(host) * 1e3
    print(f"K={K}: {dt * 1e3:.4f} ms per frame; host per call mean {h.mean():.4f} ms, median {np.median(h):.4f}, "
          f"p90 {np.percentile(h, 90):.4f}", flush=True)
    import ctypes
    for k in range(K):
        ms = (ctypes.c_double * 3)()
        fr = ctypes.c_int64()
        _lib.load().gsr_debug_host_times(ctxs[k].handle, ms, ctypes.byref(fr))
        print(f"   view {k}: per frame enqueue-before {ms[0] / fr.value * 1e3:.1f} us, wait {ms[1] / fr.value * 1e3:.1f} us, "
              f"enqueue-after {ms[2] / fr.value * 1e3:.1f} us", flush=True)
    # one host thread per view (ctypes releases the GIL inside gsr_render)
    import threading

    def worker(k, frames):
        with torch.cuda.stream(streams[k]):
            for _ in range(frames):
                render_into(ctxs[k], scene, cams[k], st, outs[k])

    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ths = [threading.Thread(target=worker, args=(k, n // K)) for k in range(K)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / (K * (n // K))
    print(f"K={K} threads: {dt * 1e3:.4f} ms per frame", flush=True)
    for c in ctxs:
        c.close()
