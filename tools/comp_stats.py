"""Compositor work statistics on the bench workload (GSR_COMP_STATS build):
slice evaluations, those spent on already-saturated slices, records visited.
    python -m gsviewer_amd.build -D GSR_COMP_STATS --out gsviewer_amd/libgsr_stats.so
    GSR_LIB_PATH=gsviewer_amd/libgsr_stats.so python tools/comp_stats.py [--views] [--c3]
(--c3: the 6M-Gaussian frame of BASELINE config C3, seed 2)"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gsviewer_amd import _lib  # noqa: E402
from gsviewer_amd.camera import Camera  # noqa: E402
from gsviewer_amd.gaussian_data import garden_standin  # noqa: E402
from gsviewer_amd.rasterizer import HipContext, HipScene, RenderSettings, camera_from, render_into  # noqa: E402


def main():
    lib = _lib.load()
    g = garden_standin(6_000_000, seed=2) if "--c3" in sys.argv else garden_standin(1_000_000, seed=1)
    scene = HipScene.from_gaussian_data(g)
    ctx = HipContext()
    out = torch.empty((3, 1080, 1920), dtype=torch.float32, device="cuda")
    buf = (ctypes.c_ulonglong * 5)()
    # --views: the group path (gsr_render_finish_views: GSR_CHUNK_VIEWS, first-major order), one group of
    # the bench's first 5 views (stats summed over them)
    views = "--views" in sys.argv
    k = 5 if views else 1
    from gsviewer_amd.multiview import view_of
    ctxs = [ctx] + [HipContext() for _ in range(k - 1)]
    outs = [out] + [torch.empty_like(out) for _ in range(k - 1)]

    def frame(st):
        if not views:
            render_into(ctx, scene, camera_from(Camera(1080, 1920)), st, out)
            return
        from gsviewer_amd.rasterizer import render_begin_sorts, render_begin_views, render_finish_views
        cams = [camera_from(view_of(v, 1080, 1920)) for v in range(k)]
        s = torch.cuda.current_stream()
        render_begin_views(ctxs, scene, cams, st, outs, stream=s)
        render_begin_sorts(ctxs, s)
        render_finish_views(ctxs, s)

    for t_min in (1e-4, 0.0):
        st = RenderSettings(t_min=t_min, out_layout=0)
        frame(st)
        lib.gsr_debug_comp_stats(buf)  # discard warm-up frame
        frame(st)
        torch.cuda.synchronize()
        lib.gsr_debug_comp_stats(buf)
        ev, wasted, recs, inst, empty = list(buf)
        print(f"t_min={t_min}: instances {inst} records visited {recs} ({recs / inst:.3f}), slice evals {ev} "
              f"({ev / max(recs, 1):.2f} per record), on saturated slices {wasted} ({wasted / max(ev, 1):.3f}), "
              f"with no kept fragment {empty} ({empty / max(ev, 1):.3f})", flush=True)


if __name__ == "__main__":
    main()
