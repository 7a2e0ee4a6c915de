"""Per-wave timeline of the composite kernel (tooling, not product code).

Needs the trace build:
    python -m gsviewer_amd.build -D GSR_COMP_TRACE --out gsviewer_amd/libgsr_trace.so
then on a GPU:
    GSR_LIB_PATH=gsviewer_amd/libgsr_trace.so python tools/comp_trace.py [--n 1000000]

Prints the launch span, per-wave duration quantiles, resident waves per SIMD
over time (occupancy), how long the tail runs after 50/90/99 % of the waves
have retired, and the per-XCD finish times.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--seed", type=int, default=1, help="garden stand-in seed (C3: --n 6000000 --seed 2)")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--frames", type=int, default=5)
    ap.add_argument("--t-min", type=float, default=1e-4)
    ap.add_argument("--dump", default=None, help="write the raw trace (.npy)")
    a = ap.parse_args()
    assert os.environ.get("GSR_LIB_PATH"), "set GSR_LIB_PATH to the GSR_COMP_TRACE build"

    import torch

    from gsviewer_amd import _lib
    from gsviewer_amd.camera import view_for_rank
    from gsviewer_amd.gaussian_data import garden_standin
    from gsviewer_amd.rasterizer import HipContext, HipScene, RenderSettings, camera_from, render_into

    lib = _lib.load()
    fn = lib.gsr_debug_comp_trace
    fn.restype = ctypes.c_int64
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]

    g = garden_standin(a.n, seed=a.seed, sh_degree=3)
    scene = HipScene(*[torch.from_numpy(np.ascontiguousarray(getattr(g, f))).cuda()
                       for f in ("xyz", "rot", "scale", "opacity", "sh")])
    ctx = HipContext()
    cam = view_for_rank(a.height, a.width, 0)
    st = RenderSettings()
    st.t_min = a.t_min
    out = torch.empty((3, a.height, a.width), dtype=torch.float32, device="cuda")
    for _ in range(a.frames):
        render_into(ctx, scene, camera_from(cam), st, out)
    torch.cuda.synchronize()
    stats = ctx.stats()
    nt = stats["tiles_x"] * stats["tiles_y"]

    buf = np.zeros((1 << 16, 2, 4), np.uint32)
    got = fn(buf.ctypes.data, buf.shape[0])
    assert got > 0
    tr = buf[:got]
    used = tr[:, 1, 0] != 0
    # waves traced this frame: slots 0 .. num_tiles + extra chunks - 1
    slot = tr[:, 0, 0]
    live = used & (slot == np.arange(got))
    tr = tr[live]
    hw, work = tr[:, 0, 1], tr[:, 0, 2].astype(np.int64)
    xcc, evals = tr[:, 0, 3] & 15, (tr[:, 0, 3] >> 4).astype(np.int64)  # (record, slice) evaluations
    t0 = tr[:, 1, 0].astype(np.int64)
    t1 = tr[:, 1, 1].astype(np.int64)
    r0 = tr[:, 1, 2].astype(np.int64)
    r1 = tr[:, 1, 3].astype(np.int64)
    # 100 MHz realtime counter -> us; shader clock counts -> cycles (per-XCD clocks are not synchronized)
    base = r0.min()
    s_us = (r0 - base) / 100.0
    e_us = (r1 - base) / 100.0
    dur_cyc = (t1 - t0) % (1 << 32)
    dur_us = e_us - s_us
    span = e_us.max()
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    se = (hw >> 13) & 7
    simd_key = ((xcc.astype(np.int64) * 8 + se) * 16 + cu) * 4 + simd
    n_simd = len(np.unique(simd_key))

    # occupancy timeline (1 us bins): resident waves per SIMD
    bins = np.arange(0, span + 1.0, 1.0)
    occ = np.zeros(len(bins))
    for s_, e_ in zip(s_us, e_us):
        i0, i1 = int(s_), int(np.ceil(e_))
        occ[i0:i1] += 1
    occ /= max(n_simd, 1)
    order = np.sort(e_us)
    q = lambda f: float(order[min(len(order) - 1, int(f * len(order)))])
    mhz = float(np.median(dur_cyc / np.maximum(dur_us, 1e-3)))
    res = dict(
        waves=int(len(tr)), tiles=int(nt), simds_seen=int(n_simd), span_us=float(span),
        shader_clock_mhz_est=mhz,
        wave_us_quantiles={str(p): float(np.quantile(dur_us, p)) for p in (0.1, 0.5, 0.9, 0.99, 1.0)},
        work_quantiles={str(p): float(np.quantile(work, p)) for p in (0.1, 0.5, 0.9, 0.99, 1.0)},
        retire_us={"50%": q(0.5), "90%": q(0.9), "99%": q(0.99), "100%": float(span)},
        start_us_quantiles={str(p): float(np.quantile(s_us, p)) for p in (0.5, 0.9, 0.99, 1.0)},
        mean_resident_waves_per_simd=float(occ[: int(span)].mean()) if span >= 1 else None,
        occupancy_by_10pct=[round(float(occ[int(i * span / 10): int((i + 1) * span / 10)].mean()), 2)
                            for i in range(10)],
        xcc_finish_us={int(x): float(e_us[xcc == x].max()) for x in np.unique(xcc)},
        us_per_record_median=float(np.median(dur_us[work > 0] / work[work > 0])),
        empty_wave_us_median=float(np.median(dur_us[work == 0])) if (work == 0).any() else None,
        total_wave_us=float(dur_us.sum()), total_work=int(work.sum()), total_evals=int(evals.sum()),
        evals_quantiles={str(p): float(np.quantile(evals, p)) for p in (0.1, 0.5, 0.9, 0.99, 1.0)},
        # how much of a wave's duration its instance count and its slice evaluations explain
        corr_dur_instances=float(np.corrcoef(dur_us, work)[0, 1]) if len(tr) > 2 else None,
        corr_dur_evals=float(np.corrcoef(dur_us, evals)[0, 1]) if len(tr) > 2 else None,
        us_per_eval_median=float(np.median(dur_us[evals > 0] / evals[evals > 0])) if (evals > 0).any() else None,
    )
    # the waves that retire last (after 90 % of them): what they carry against the rest
    late = e_us >= q(0.9)
    full = work == work.max()
    res["late_waves"] = dict(
        n=int(late.sum()), start_us_median=float(np.median(s_us[late])), dur_us_median=float(np.median(dur_us[late])),
        evals_median=float(np.median(evals[late])), instances_median=float(np.median(work[late])))
    res["full_chunks"] = dict(
        n=int(full.sum()), instances=int(work.max()),
        dur_us_quantiles={str(p): float(np.quantile(dur_us[full], p)) for p in (0.1, 0.5, 0.9, 1.0)},
        evals_quantiles={str(p): float(np.quantile(evals[full], p)) for p in (0.1, 0.5, 0.9, 1.0)},
        corr_dur_evals=float(np.corrcoef(dur_us[full], evals[full])[0, 1]) if full.sum() > 2 else None)
    # a wave's duration fitted as a + b * evals + c * instances (least squares): the residual is what neither explains
    A = np.stack([np.ones(len(tr)), evals, work], 1).astype(np.float64)
    coef, *_ = np.linalg.lstsq(A, dur_us, rcond=None)
    res["fit_us"] = dict(const=float(coef[0]), per_eval=float(coef[1]), per_instance=float(coef[2]),
                         r2=float(1 - ((A @ coef - dur_us) ** 2).sum() / ((dur_us - dur_us.mean()) ** 2).sum()))
    print(json.dumps(res, indent=1))
    if a.dump:
        np.save(a.dump, np.stack([s_us, e_us, work, xcc, simd_key, evals], 1))


if __name__ == "__main__":
    main()
