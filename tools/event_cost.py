"""Throughput of the 4-view pipeline with and without one cross-stream
event (record on the view stream, wait on another stream) per frame:
the price of the event hand-offs a shared scene pass needs (tooling)."""
import os
import sys
import time

os.environ.setdefault("GPU_MAX_HW_QUEUES", "8")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from gsviewer_amd.gaussian_data import garden_standin  # noqa: E402
from gsviewer_amd.multiview import ViewPipeline, view_of  # noqa: E402
from gsviewer_amd.rasterizer import HipContext, HipScene, RenderSettings, camera_from, render_finish  # noqa: E402


def run(mode, steps=100):
    g = garden_standin(1_000_000, seed=1, sh_degree=3)
    scene = HipScene.from_gaussian_data(g)
    K = 4
    ctxs = [HipContext() for _ in range(K)]
    streams = [torch.cuda.Stream() for _ in range(K)]
    other = torch.cuda.Stream()
    outs = [torch.empty((3, 1080, 1920), dtype=torch.float32, device="cuda") for _ in range(K)]
    cams = [camera_from(view_of(k, 1080, 1920)) for k in range(K)]
    st = RenderSettings(t_min=1e-4, out_layout=0)
    pipe = ViewPipeline(ctxs, streams, scene, cams, st, outs)

    def step():
        k = pipe.next
        pipe.step()
        if mode == "event":
            ev = torch.cuda.Event()
            ev.record(streams[k])
            other.wait_event(ev)
            ev2 = torch.cuda.Event()
            ev2.record(other)
            streams[k].wait_event(ev2)
    for _ in range(20):
        step()
    pipe.drain()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    pipe.drain()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(mode, "ms/frame", round(1e3 * dt / steps, 4), flush=True)


if __name__ == "__main__":
    run("plain")
    run("event")
    run("plain")
