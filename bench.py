"""Benchmark: forward Gaussian-splat rasterization on MI355X.

Metric (BASELINE.json): rendered splats/s (N Gaussians x frames/s) at 1080p on
a 1M-Gaussian SH-degree-3 scene.  One "step" = one full frame of the hot path
(cull + project + SH, depth radix sort, tile binning + sort, compositing) for
one camera, inputs resident in HBM.  With --gpus N (torchrun, one process per
GPU) the scene is generated on rank 0, broadcast once over RCCL/xGMI (untimed)
and rank k renders view k (default camera yawed by k*45 deg):
weak scaling, no per-frame collective.

Prints ONE JSON line on rank 0.  Stage timings come from HIP events recorded
by libgsr on the render stream during the timed region.

Launch: ``python bench.py --gpus N`` with N > 1 and no WORLD_SIZE in the
environment starts ``torch.distributed.run`` (N ranks, 127.0.0.1) as a CHILD
process before anything touches the GPU, and exits with its status; under
torchrun (WORLD_SIZE set) the process is one rank and checks that the world
size equals --gpus.  ``--dry-run`` runs the same launch, rendezvous, scene
broadcast, view assignment and max-over-ranks timing on CPU over gloo, with
no rendering (a CPU test of the launcher: tests/test_bench_launch.py).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
CUS = 256
SIMDS = CUS * 4        # MI355X CUs x SIMDs
CLOCK_GHZ = 2.4        # MI355X max clock (the chip holds less under load: issue fractions are lower bounds)
# VALU issue per SIMD with several waves resident: a wave64 instruction every 2 cycles (SIMD-32,
# MI355X_MICROARCH.md "Wave scheduling"; a transcendental twice that, its 8-cycle one-wave cost against 4);
# round 4's marginal test on the compositor measured 0.73 ns per added VALU (profiles/r4_s16: 1.75 cycles)
VALU_NS = 2.0 / CLOCK_GHZ
TRANS_NS = 4.0 / CLOCK_GHZ
REPEATS = 3            # instrumented repeats of the timed region (compositor busy union: the median)

CONFIGS = {
    # name: (N, sh_degree, width, height, description)
    "c1": (100_000, 0, 640, 480, "100k random Gaussians, SH deg 0, 640x480"),
    "c2": (1_000_000, 3, 1920, 1080, "1M Gaussians, SH deg 3, 1920x1080 (garden stand-in)"),
    "c3": (6_000_000, 3, 1920, 1080, "6M Gaussians synthetic, SH deg 3, 1920x1080"),
    "c5": (1_000_000, 3, 3840, 2160, "1M Gaussians, SH deg 3, 3840x2160"),
    # stress scene beside C2: heavy-tailed splat sizes
    "c2h": (1_000_000, 3, 1920, 1080, "1M heavy-splat garden stand-in (scale exp(N(-3.5, 0.8))), SH deg 3, "
                                      "1920x1080 (stress)"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_scene(cfg, n, deg):
    from gsviewer_amd.gaussian_data import garden_standin, random_scene
    if cfg == "c1":
        return random_scene(n, sh_degree=deg, seed=0), "synthetic: random uniform (seed 0)"
    seed = 2 if cfg == "c3" else 1
    if cfg == "c2h":
        return (garden_standin(n, seed=seed, sh_degree=deg, log_scale=(-3.5, 0.8)),
                f"synthetic: heavy-splat garden stand-in (seed {seed}, log-scale N(-3.5, 0.8)), no PLY offline")
    return garden_standin(n, seed=seed, sh_degree=deg), f"synthetic: garden stand-in (seed {seed}), no PLY offline"


def morton_order(xyz, bits=10):
    """Permutation putting Gaussians in 3D Morton (Z-curve) order of their
    positions (experiment: record gathers of spatially coherent scenes)."""
    lo, hi = xyz.min(axis=0), xyz.max(axis=0)
    q = ((xyz - lo) / np.maximum(hi - lo, 1e-12) * ((1 << bits) - 1)).astype(np.uint64)
    code = np.zeros(len(xyz), np.uint64)
    for b in range(bits):
        for d in range(3):
            code |= ((q[:, d] >> np.uint64(b)) & np.uint64(1)) << np.uint64(3 * b + d)
    return np.argsort(code, kind="stable")


def box_settings(g, kind):
    """SURVEY.md 8d C5 box cull settings (RenderSettings fields)."""
    if kind == "aabb":
        lo, hi, _ = g.compute_aabb
        return dict(enable_aabb=1, cube_min=[float(v) for v in np.float32(lo) * np.float32(0.5)],
                    cube_max=[float(v) for v in np.float32(hi) * np.float32(0.5)],
                    points_center=[float(v) for v in g.points_center.astype(np.float32)])
    from gsviewer_amd.camera import euler_to_rotation_matrix
    return dict(enable_obb=1, cube_rotation=euler_to_rotation_matrix([30.0, 15.0, 0.0]).tolist(),
                cube_min=[-1.5, -1.5, -1.5], cube_max=[1.5, 1.5, 1.5],
                points_center=[float(v) for v in g.points_center.astype(np.float32)])


def host_cpu():
    """CPU model and the cores this process may run on (cpu_baseline context)."""
    model = None
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count()
    return dict(cpu_model=model, nproc=os.cpu_count(), affinity_cpus=usable, cgroup_quota_cpus=cgroup_cpus())


def cgroup_cpus():
    """CPUs this process's cgroup may use (cpu.max quota / period), or None."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            quota, period = open(path).read().split()[:2]
            if quota != "max":
                return max(1, int(int(quota) // int(period)))
        except (OSError, ValueError):
            pass
    return None


def baseline_threads():
    """Threads for the CPU baseline: every host core this process may use
    (OpenMP over all host cores), i.e. its CPU affinity capped by
    its cgroup's CPU quota, unless OMP_NUM_THREADS says otherwise (the GPU
    pool sets 16: its boxes grant one GPU's share of a 256-CPU host, and
    threads beyond a quota only time-slice).  Returns (threads, reason)."""
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    quota = cgroup_cpus()
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if env > 0:
        return env, (f"OMP_NUM_THREADS={env} (the environment's CPU share; affinity {usable} CPUs, "
                     f"cgroup quota {quota if quota else 'none'})")
    if quota and quota < usable:
        return quota, f"all CPUs the cgroup quota grants ({quota}; affinity {usable})"
    return usable, f"all CPUs in this process's affinity ({usable})"


def cpu_baseline(g, cam, seconds):
    """The C restatement of the reference OGL path (oracle/gl_oracle.c), full
    frames of the same workload on the host cores, bounded to ~`seconds`.
    One untimed frame first (thread pool start-up, first-touch of the
    buffers).  Also times the depth sort alone: the C port's parallel radix
    sort on all threads and on one, and the reference's own NumPy expression
    of _sort_gaussian_cpu (renderer_ogl.py:16-26: view-z dot + argsort)."""
    from oracle import c_oracle as C
    from oracle import gl_oracle as O
    threads, why = baseline_threads()
    U = O.default_uniforms(cam.get_view_matrix(), cam.get_project_matrix(),
                           np.asarray(cam.get_htanfovxy_focal(), np.float32), cam.position, cam.w, cam.h)
    flat = g.flat()
    C.render(flat, g.sh_dim, U, threads=threads)  # warm-up, untimed
    frames, t_total, per = 0, 0.0, []
    while True:
        t0 = time.perf_counter()
        C.render(flat, g.sh_dim, U, threads=threads)
        per.append(time.perf_counter() - t0)
        t_total += per[-1]
        frames += 1
        if t_total >= seconds or frames >= 50:
            break

    def best_of(fn, reps=3):
        fn()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return 1e3 * min(ts)

    V = np.asarray(U["view"], np.float32)
    xyz = np.ascontiguousarray(g.xyz, np.float32)
    sort_mt = best_of(lambda: C.sort_depth(xyz, V, threads=threads))
    sort_1t = best_of(lambda: C.sort_depth(xyz, V, threads=1))
    # renderer_ogl.py:16-26 as written: xyz_view = view @ xyz_h; argsort of z
    xyz_h = np.concatenate([xyz, np.ones((len(xyz), 1), np.float32)], axis=1)
    sort_np = best_of(lambda: np.argsort((V @ xyz_h.T)[2]))
    out = dict(value=len(g) * frames / t_total, unit="splats/s", cores=threads, kind="port",
               sample=f"{frames} full frames of the same workload ({len(g)} Gaussians, {cam.w}x{cam.h}) "
                      f"through oracle/gl_oracle.c (OGL-path restatement: vertex stage, parallel radix depth "
                      f"sort, rect raster + fragment + blend), {threads} OpenMP threads, after one untimed frame",
               ms_per_frame=1e3 * t_total / frames,
               ms_per_frame_spread={"min": 1e3 * min(per), "median": 1e3 * float(np.median(per)),
                                    "max": 1e3 * max(per)},
               host_variance="the GPU pool grants a CPU quota on a shared many-core host: the same sample has "
                             "measured 327 and 404 ms/frame on two boxes (profiles/r3_s37, BENCH_r03), so "
                             "this figure carries ~25 % host-to-host spread; it is context, not the target",
               threads_reason=why,
               sort_ms={f"port_radix_{threads}threads": sort_mt, "port_radix_1thread": sort_1t,
                        "reference_numpy_argsort_1thread": sort_np})
    out.update(host_cpu())
    return out


# stage name -> kernel symbol in rocprofv3 summaries
JSON_OUT = sys.stdout  # main() points it at the real stdout before routing fd 1 to stderr

KERNEL_SYMBOL = {"composite": "k_composite<0, false>", "preprocess": "k_preprocess_fc_views<3, true>",
                 "merge": "k_merge"}
PMC_PROFILE = os.path.join(ROOT, "profiles", "LATEST")


def pmc_counters(kernel, args):
    """Per-dispatch PMC counters of `kernel` from the committed rocprofv3 --pmc
    summary of this same bench command (profiles/<LATEST>/pmc_summary.csv,
    written by tools/gpu_round.sh; FETCH_SIZE already doubled per the gfx950
    correction).  PMC collection needs its own profiler passes, so the values
    are read back here rather than measured inside the timed region."""
    if kernel is None or args.config != "c2" or args.n or args.width or args.height or args.box != "none":
        return None, None
    import csv
    try:
        d = open(PMC_PROFILE).read().strip()
        with open(os.path.join(ROOT, "profiles", d, "pmc_summary.csv")) as fh:
            rows = list(csv.reader(fh))[1:]  # (kernel names hold commas: "k_composite<0, false>")
    except OSError:
        return None, None
    return {r[1]: float(r[4]) for r in rows if r[0] == kernel}, f"profiles/{d}/pmc_summary.csv ({kernel})"


def rocprof_avg_ms(kernel, args):
    """Average duration (ms) of `kernel` in the committed rocprofv3 --stats
    summary of this same bench command (profiles/<LATEST>/kernel_stats.csv),
    the cross-check of the live launch time."""
    if args.config != "c2" or args.n or args.width or args.height or args.box != "none":
        return None
    import csv
    try:
        d = open(PMC_PROFILE).read().strip()
        with open(os.path.join(ROOT, "profiles", d, "kernel_stats.csv")) as fh:
            for row in csv.DictReader(fh):
                if kernel in row["Name"]:
                    return {"ms": float(row["AverageNs"]) * 1e-6, "calls": int(row["Calls"]),
                            "source": f"profiles/{d}/kernel_stats.csv"}
    except (OSError, KeyError, ValueError):
        return None
    return None


def pmc_traffic(kernel, args):
    """HBM bytes per launch (FETCH_SIZE + WRITE_SIZE) of `kernel`."""
    got, src = pmc_counters(kernel, args)
    if not got or "FETCH_SIZE" not in got or "WRITE_SIZE" not in got:
        return None
    return got["FETCH_SIZE"] + got["WRITE_SIZE"], src


def default_shape(args):
    """The committed profiles describe the default C2 command only."""
    return args.config == "c2" and not (args.n or args.width or args.height) and args.box == "none"


def latest():
    return open(PMC_PROFILE).read().strip()


def committed_json(name, args):
    """A JSON file of the committed profile of this same bench command
    (profiles/<LATEST>/name), or None."""
    if not default_shape(args):
        return None
    try:
        return json.load(open(os.path.join(ROOT, "profiles", latest(), name)))
    except (OSError, ValueError):
        return None


def stage_bytes(n, nvis, inst, ntiles, W, H, rec_bytes, share=1, depth_passes=2):
    """Each stage's own algorithmic bytes per frame (DESIGN.md "Kernels of a
    frame"): the scene read once per group of `share` views (SoA: 16-B
    position of every Gaussian, the rest of the record for the visible ones),
    12 B key + rect per slot and a 48-B record per visible splat out; per radix
    pass 12 B in + 12 B out per key (key, slot, payload); the binning's rect
    and slot in, 8 B per instance out; the tile sort's pass 8 + 8 B per
    instance; the compositor's 48-B record + 4-B slot per instance, the tile
    ranges and the image."""
    attrs = rec_bytes - 16 + 4  # SoA planes: 240 B per Gaussian at SH 3 (pos+opacity 16, rot 16, scale 16, SH 192)
    return {
        "preprocess": (n * 16 + nvis * attrs) / share + n * 12 + nvis * 48,
        "depth_sort": n * 12 + nvis * 12 + (depth_passes - 1) * nvis * 24,
        "binning": nvis * 8 + inst * 8,
        "tile_sort": inst * 16,
        "tile_ranges": inst * 4 + ntiles * 8,
        "composite": inst * (48 + 4) + ntiles * 8 + W * H * 12,
        "merge": W * H * 12,
    }


# kernels of the timed region (groups of views) -> the stage whose bytes they move
REGION_STAGE = {
    "k_preprocess_fc_views<3, false>": "preprocess",
    "k_rs_scatter_views<8, true, 8>": "depth_sort",
    "k_bin_scatter_views<true, 8>": "binning",
    "k_rs_scatter_views<8, false, 8>": "tile_sort",
    "k_tile_ranges_views<false>": "tile_ranges",
    "k_composite_views<0>": "composite",
}


def per_kernel_table(region, n, nvis, inst, ntiles, W, H, rec_bytes, share):
    """Per kernel of the timed region: its own algorithmic bytes per frame
    (stage_bytes; a group's depth sort runs 4 exact passes) over its busy time
    per frame in the committed rocprofv3 trace of this command (the union of
    its launches, tools/region_kernels.py).  The four group streams overlap,
    so busy times add up to more than the frame (concurrency ~2)."""
    by = stage_bytes(n, nvis, inst, ntiles, W, H, rec_bytes, share=share, depth_passes=4)
    rows = {}
    for k, v in region["timed_region"]["kernels"].items():
        st = REGION_STAGE.get(k)
        row = {"busy_us_per_frame": round(v["busy_us_per_frame"], 2), "launches": v["launches"]}
        if st:
            gbps = by[st] / (v["busy_us_per_frame"] * 1e-6) / 1e9
            row.update(stage=st, alg_bytes_per_frame=int(by[st]), GBps=round(gbps, 1),
                       frac=round(gbps / HBM_PEAK_GBS, 4))
        rows[k] = row
    return {"kernels": rows, "region_span_us_per_frame": region["timed_region"]["span_us_per_frame"],
            "region_busy_us": region["timed_region"]["busy_us"],
            "source": f"profiles/{latest()}/region_kernels.json",
            "note": "radix upsweeps, offsets scans, histograms and chunk kernels move few bytes (counts): "
                    "listed with their busy time only"}


def frame_resources(args, share, ms_per_frame, b_frame, fps):
    """Demand of the frame in flight on each chip resource, as a fraction of
    what the chip offers over the frame time, from the committed PMC summary
    of this same command (every *_views kernel, per view-frame):
    VALU issue (wave64 instructions at 2 cycles per SIMD, transcendentals 4,
    MI355X_MICROARCH.md; 1024 SIMDs at 2.4 GHz: a lower bound under DVFS),
    LDS (SQ_LDS_IDX_ACTIVE LDS-array cycles per CU, 256 CUs), the L2's
    fabric traffic (FETCH x 2 + WRITE bytes: HBM and Infinity Cache hits
    alike, MI355X_MICROARCH.md) and SURVEY 8(d)'s B_frame, both against the
    8 TB/s HBM peak."""
    if share <= 1 or not default_shape(args):
        return None
    import csv
    try:
        with open(os.path.join(ROOT, "profiles", latest(), "pmc_summary.csv")) as fh:
            rows = list(csv.reader(fh))[1:]  # (kernel names hold commas: "k_rs_scatter_views<8, true, 8>")
    except OSError:
        return None
    tot, disp = {}, {}
    for r in rows:
        k, c = r[0], r[1]
        if "_views" not in k or k.endswith(", true>"):  # the group kernels (not the frame alone's preprocess)
            continue
        tot[c] = tot.get(c, 0.0) + float(r[4]) * int(r[2])
        if k == "k_composite_views<0>":
            disp[c] = int(r[2])
    groups = disp.get("SQ_INSTS_VALU") or disp.get("FETCH_SIZE")
    if not groups:
        return None
    per = {c: v / groups / share for c, v in tot.items()}  # per view-frame
    t = ms_per_frame * 1e-3
    fr, raw = {}, {}
    if "SQ_INSTS_VALU" in per:
        trans = per.get("SQ_INSTS_VALU_TRANS_F32", 0.0)
        issue = (VALU_NS * (per["SQ_INSTS_VALU"] - trans) + TRANS_NS * trans) * 1e-9 / SIMDS
        fr["VALU issue"] = issue / t
        raw.update(valu_instr=per["SQ_INSTS_VALU"], trans_instr=trans, valu_issue_us=issue * 1e6)
    if "SQ_LDS_IDX_ACTIVE" in per:
        lds = per["SQ_LDS_IDX_ACTIVE"] / (CUS * CLOCK_GHZ * 1e9)
        fr["LDS"] = lds / t
        raw.update(lds_array_cycles=per["SQ_LDS_IDX_ACTIVE"], lds_us=lds * 1e6)
    if "FETCH_SIZE" in per and "WRITE_SIZE" in per:
        by = per["FETCH_SIZE"] + per["WRITE_SIZE"]
        fr["fabric traffic (FETCH x 2 + WRITE, Infinity Cache hits included)"] = by / t / (HBM_PEAK_GBS * 1e9)
        raw.update(traffic_bytes=by)
    fr["HBM (B_frame)"] = b_frame * fps / 1e9 / HBM_PEAK_GBS
    return {"fractions": {k: round(v, 4) for k, v in fr.items()}, "per_view_frame": raw,
            "frame_us": ms_per_frame * 1e3, "prices": {"valu_ns": VALU_NS, "trans_ns": TRANS_NS,
                                                       "clock_ghz": CLOCK_GHZ},
            "source": f"profiles/{latest()}/pmc_summary.csv (*_views kernels)"}


def busy_union_ms(spans):
    """Union of [start, end) intervals in 100 MHz ticks, in ms: the time the
    kernel was executing, launches that overlap counted once."""
    tot, cur = 0, None
    for a, b in sorted(spans):
        if cur is None or a > cur[1]:
            if cur is not None:
                tot += cur[1] - cur[0]
            cur = [a, b]
        else:
            cur[1] = max(cur[1], b)
    if cur is not None:
        tot += cur[1] - cur[0]
    return tot * 1e-5


def _free_port():
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def measured_copy_gbps(dev, nbytes=1 << 31, reps=5):
    """This box's device-to-device copy rate (read + write bytes / s) over a
    2 GiB buffer, 8x the Infinity Cache, so it streams from HBM (SURVEY 8(d):
    record the measured stream copy beside the 8 TB/s spec peak)."""
    import torch
    src = torch.ones(nbytes // 4, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    for _ in range(2):
        dst.copy_(src)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        dst.copy_(src)
    e1.record()
    e1.synchronize()
    gbps = 2.0 * nbytes * reps / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del src, dst
    torch.cuda.empty_cache()
    return gbps


def launch_ranks(n, argv):
    """Start n ranks of this script under torch.distributed.run as a child
    process (one process per GPU, rendezvous on 127.0.0.1) and return its
    exit status.  Nothing before this touches the GPU, so no process that
    initialised HIP is ever replaced."""
    env = dict(os.environ)
    env["MASTER_ADDR"] = "127.0.0.1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    log("bench.py: launching", n, "ranks:", " ".join(cmd[1:]))
    return subprocess.call(cmd, env=env)


def dry_run(args):
    """The multi-rank skeleton of the GPU run, on CPU over gloo: rendezvous,
    the one scene broadcast, view assignment and the barrier-bracketed
    max-over-ranks timed region, with a no-op frame.  Rank 0 prints one JSON
    line listing every rank; nothing is measured."""
    import torch.distributed as dist

    from gsviewer_amd.multiview import broadcast_scene, gather_objects, timed_region, view_of

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    if world > 1:
        dist.init_process_group("gloo")
    _, deg, W, H, desc = CONFIGS[args.config]
    n = args.n or 1000
    k_coef = (deg + 1) ** 2
    g = make_scene(args.config, n, deg)[0] if rank == 0 else None
    packed, bcast = broadcast_scene(g, n, k_coef, "cpu")
    views = [rank + world * j for j in range(max(1, args.inflight))]
    cam0 = view_of(views[0], H, W)
    elapsed = timed_region(lambda: None, args.steps, "cpu")
    c4_view = rank  # the C4 sub-record: view k on GPU k, one view per GPU
    c4_elapsed = timed_region(lambda: None, args.steps, "cpu")
    me = dict(rank=rank, world=dist.get_world_size() if world > 1 else 1, views=views, c4_view=c4_view,
              view0_row2=[float(x) for x in cam0.get_view_matrix()[2]],
              c4_view_row2=[float(x) for x in view_of(c4_view, H, W).get_view_matrix()[2]],
              scene_sum=float(packed.double().sum()), elapsed=elapsed)
    ranks = gather_objects(me, world)
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "backend": "gloo" if world > 1 else None,
                          "workload": desc, "n_gaussians": n, "steps": args.steps, "broadcast": bcast,
                          "views_batched": {"views_per_gpu": max(1, args.inflight), "elapsed_max_s": elapsed},
                          "c4_one_view_per_gpu": None if world == 1 else
                          {"views": [r["c4_view"] for r in ranks], "elapsed_max_s": c4_elapsed},
                          "ranks": ranks}), file=JSON_OUT, flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--n", type=int, default=None)
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--t-min", type=float, default=1e-4)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--inflight", type=int, default=20,
                    help="independent views in flight per GPU (own context each, pipelined with "
                         "gsr_render_begin[_views]/finish); 1 = one at a time.  Default 20: 4 groups of 5 "
                         "(tools/short_region_sweep2.sh: 0.204 ms/frame over 100 frames and 0.215 over the "
                         "driver's 20, against 0.209 / 0.230 for 16 as 4 x 4), and 20 frames are then exactly "
                         "one begin + finish of every group")
    ap.add_argument("--group-sizes", default=None,
                    help="with --share > 1: explicit group sizes in step order, e.g. 2,6,6,6 (each <= 8, summing "
                         "to --inflight); default: groups of --share")
    ap.add_argument("--share", type=int, default=None,
                    help="views per shared scene pass (gsr_render_begin_views): the views in flight form "
                         "inflight/share groups, one stream each, whose cull + preprocess read the scene once "
                         "per group; 1 = off (one stream per view).  Default: --inflight / 4 (four group streams) "
                         "when --inflight is a multiple of 4 in [8, 32], else 1")
    ap.add_argument("--no-batched-sorts", action="store_true",
                    help="with --share > 1: one depth sort per view instead of one batched sort per group")
    ap.add_argument("--no-batched-finish", action="store_true",
                    help="with --share > 1: finish each view's frame alone instead of one launch per stage "
                         "for the group")
    ap.add_argument("--lookahead", type=int, default=None,
                    help="with --share > 1: at most this many groups begun and not yet finished (default: all "
                         "groups; a group is finished when it is begun again or drained)")
    ap.add_argument("--priorities", default=None,
                    help="experiment: comma-separated HIP stream priorities of the group streams (lower = "
                         "higher priority; torch.cuda.Stream.priority_range()), cycled over the streams")
    ap.add_argument("--host-threads", action="store_true",
                    help="with --share > 1: one host thread per group drives its stream (parallel enqueue)")
    ap.add_argument("--no-profile", action="store_true", help="do not record per-stage HIP events")
    ap.add_argument("--render-mod", type=int, default=6,
                    help="render_mod uniform (experiments; 6 = SH:0~3, the reference default)")
    ap.add_argument("--box", default="none", choices=["none", "aabb", "obb"],
                    help="boundary-box cull (SURVEY.md 8d C5): aabb = compute_aabb min/max x 0.5 around "
                         "points_center; obb = euler(30, 15, 0) deg, +-1.5")
    ap.add_argument("--scene-order", default="given", choices=["given", "morton"],
                    help="experiment: render the scene with its Gaussians permuted into 3D Morton order")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU rehearsal of the multi-rank launch over gloo (no GPU, no rendering)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    # Libraries below (gloo, RCCL, HIP) may write to file descriptor 1; the
    # driver reads ONE JSON line from stdout.  Route fd 1 to stderr and keep
    # a private handle on the real stdout for that line.
    global JSON_OUT
    JSON_OUT = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    if args.dry_run:
        return dry_run(args)

    # One hardware queue per in-flight view stream (+ torch's own): HIP maps
    # streams round-robin onto GPU_MAX_HW_QUEUES queues (4 by default), and two
    # view streams sharing a queue serialise.  Must be set before HIP starts.
    share = args.share if args.share is not None else (
        args.inflight // 4 if args.inflight % 4 == 0 and 8 <= args.inflight <= 32 else 1)
    share = max(1, share)
    want_q = min(32, max(8, -(-args.inflight // share) + 2))  # one stream per view (share 1) or per group
    if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < want_q:
        os.environ["GPU_MAX_HW_QUEUES"] = str(want_q)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
    # Rehearsal of the multi-rank GPU path on a one-GPU box (GSR_BENCH_SHARED_GPU=1):
    # every rank renders on device 0 and the process group is gloo (RCCL refuses
    # two ranks on one GPU).  Launch, broadcast, per-rank views and the
    # max-over-ranks timing are the driver's N-GPU run; the rate is not.
    shared_gpu = world > 1 and os.environ.get("GSR_BENCH_SHARED_GPU", "0") == "1"
    if shared_gpu:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if shared_gpu:
        dist.init_process_group("gloo")
    elif world > 1:
        dist.init_process_group("nccl", device_id=dev)  # RCCL over xGMI on ROCm
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"bench.py: process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")

    from gsviewer_amd import _lib
    from gsviewer_amd.multiview import (ThreadedViewBatchPipeline, ViewBatchPipeline, ViewPipeline, broadcast_scene,
                                        timed_region, view_of)
    from gsviewer_amd.rasterizer import HipContext, HipScene, RenderSettings, camera_from, render_into

    _lib.load()
    n, deg, W, H, desc = CONFIGS[args.config]
    n = args.n or n
    W = args.width or W
    H = args.height or H
    k_coef = (deg + 1) ** 2

    # ---- scene: generated on rank 0, broadcast once (RCCL over xGMI), untimed
    t_gen = time.perf_counter()
    g, data_desc = make_scene(args.config, n, deg) if rank == 0 else (None, None)
    if g is not None and args.scene_order == "morton":  # experiment: spatially coherent Gaussian order
        g = g[morton_order(g.xyz)]
        data_desc += ", Gaussians in 3D Morton order"
    t_gen = time.perf_counter() - t_gen
    packed, bcast = broadcast_scene(g, n, k_coef, dev)  # one RCCL broadcast of the packed scene at load (world > 1)
    scene = HipScene.from_flat(packed, 3 * k_coef)
    del packed
    cam = view_of(rank, H, W)
    camc = camera_from(cam)
    st = RenderSettings(t_min=args.t_min, out_layout=0)
    st.render_mod = args.render_mod
    if args.box != "none":
        box = box_settings(g, args.box) if rank == 0 else None
        if world > 1:
            obj = [box]
            dist.broadcast_object_list(obj, src=0)
            box = obj[0]
        for k, v in box.items():
            setattr(st, k, v)
    lib = _lib.load()
    # K independent views in flight on K streams (one context and output per
    # view): frame i renders view i mod K.  Rank r's views are r + world*j.
    K = max(1, args.inflight)
    ctxs = [HipContext() for _ in range(K)]
    for c in ctxs:  # workspace sized up front: no device allocation inside any frame
        c.reserve(n, W, H)
    if args.priorities:
        pri = [int(x) for x in args.priorities.split(",")]
        print(f"bench: stream priority range {torch.cuda.Stream.priority_range()}, using {pri}", file=sys.stderr)
        streams = [torch.cuda.Stream(device=dev, priority=pri[i % len(pri)]) for i in range(K)]
    else:
        streams = [torch.cuda.Stream(device=dev) for _ in range(K)]
    outs = [torch.empty((3, H, W), dtype=torch.float32, device=dev) for _ in range(K)]
    cams = [cam] + [view_of(rank + world * j, H, W) for j in range(1, K)]
    camcs = [camera_from(c) for c in cams]
    ctx = ctxs[0]
    if share == 1:
        pipe = ViewPipeline(ctxs, streams, scene, camcs, st, outs)
    else:
        # groups of `share` views (the last one may be smaller), one stream each
        starts = list(range(0, K, share))
        if args.group_sizes:
            sizes_req = [int(x) for x in args.group_sizes.split(",")]
            if sum(sizes_req) != K or not all(1 <= x <= 8 for x in sizes_req):
                raise SystemExit(f"--group-sizes {args.group_sizes}: sizes in 1..8 summing to --inflight {K}")
            starts = [sum(sizes_req[:i]) for i in range(len(sizes_req))]
        bounds = starts + [K]
        groups = [(ctxs[a:b], camcs[a:b], outs[a:b], streams[gi])
                  for gi, (a, b) in enumerate(zip(bounds[:-1], bounds[1:]))]
        if args.host_threads:
            pipe = ThreadedViewBatchPipeline(groups, scene, st, batched_sorts=not args.no_batched_sorts,
                                             batched_finish=not args.no_batched_finish)
        else:
            pipe = ViewBatchPipeline(groups, scene, st, batched_sorts=not args.no_batched_sorts,
                                     batched_finish=not args.no_batched_finish, lookahead=args.lookahead)

    def serial_frame():
        render_into(ctx, scene, camc, st, outs[0])

    for _ in range(max(args.warmup // share, 2 * ((K + share - 1) // share))):
        pipe.step()
    pipe.drain()
    torch.cuda.synchronize()

    # barrier + synchronize on both sides; MAX over ranks.  No instrumentation
    # inside: every HIP event record stalls the stream for several us.  Every
    # begun frame is finished (drain) before the closing synchronize.
    host_step_s = []  # host time of each step() call in the timed region (perf_counter only: no GPU effect)

    def pipelined(steps):
        for _ in range(steps):
            h = time.perf_counter()
            pipe.step()
            host_step_s.append(time.perf_counter() - h)
        h = time.perf_counter()
        pipe.drain()
        host_step_s.append(time.perf_counter() - h)

    own = []
    if share == 1:
        elapsed = timed_region(lambda: pipelined(args.steps), 1, dev, own)
    else:
        # a step renders one group's frames (groups in round-robin order from
        # group 0 after the drain): time the whole steps covering args.steps
        # frames -- exactly args.steps when the group sizes add up to it (the
        # defaults do for multiples of --inflight), else normalised to it
        sizes = [len(gr[0]) for gr in groups]
        calls, timed_frames = 0, 0
        while timed_frames < args.steps:
            timed_frames += sizes[calls % len(sizes)]
            calls += 1
        pipe.next = 0
        elapsed = timed_region(lambda: pipelined(calls), 1, dev, own) * args.steps / timed_frames
        own[0] *= args.steps / timed_frames
    host_steps = list(host_step_s)  # (the timed region's calls only)
    # single-view latency: the same number of frames of view 0, one at a time
    latency = timed_region(serial_frame, args.steps, dev) if K > 1 else elapsed
    # SURVEY 8(d)'s GPU timing: the median of per-frame times, one frame at a
    # time, each bracketed by device synchronizes (so it includes one host
    # round trip per frame)
    per_frame = []
    for _ in range(max(args.steps, 20)):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        serial_frame()
        torch.cuda.synchronize(dev)
        per_frame.append(time.perf_counter() - t0)
    latency_median_ms = 1e3 * float(np.median(per_frame))
    copy_gbps = measured_copy_gbps(dev)

    import ctypes
    # The compositing launch the timed region runs (k_composite_views, one per
    # group): a fourth region, the same pipeline again with HIP events around
    # every group's compositing launch on the group's stream.
    group_comp = None
    if not args.no_profile and share > 1:
        leads = [gr[0][0] for gr in groups]
        for c in leads:
            _lib.check(lib.gsr_context_set_profiling(c.handle, 2), "set_profiling")
        # REPEATS repeats of the timed region (one busy union each, the median
        # is the figure: a single region's union spans +-10 % run to run)
        gp_elapsed = []
        for _ in range(REPEATS):
            pipe.next = 0
            gp_elapsed.append(timed_region(lambda: pipelined(calls), 1, dev))
        tot_ms, tot_l, tot_v, tot_span = 0.0, 0, 0, 0.0
        spans = []  # per lead context: its launches' in-kernel (start, end), 100 MHz ticks, device-wide clock
        for c in leads:
            cms, cl, cv, csp = ctypes.c_double(), ctypes.c_int64(), ctypes.c_int64(), ctypes.c_double()
            _lib.check(lib.gsr_context_group_times(c.handle, ctypes.byref(cms), ctypes.byref(cl), ctypes.byref(cv),
                                                   ctypes.byref(csp)), "group_times")
            tot_ms, tot_l, tot_v, tot_span = tot_ms + cms.value, tot_l + cl.value, tot_v + cv.value, tot_span + csp.value
            buf = (ctypes.c_uint64 * 128)()
            got = lib.gsr_context_group_spans(c.handle, buf, 64)
            _lib.check(0 if got >= 0 else int(got), "group_spans")
            spans.append([(buf[2 * i], buf[2 * i + 1]) for i in range(min(int(got), 64))])
            _lib.check(lib.gsr_context_set_profiling(c.handle, 0), "set_profiling")
        # region r's launches: the r-th of every lead's REPEATS equal runs of its launches (a lead leads
        # one launch per region and step of its group: 1 at --steps 20, 5 at 100)
        per_region = []
        for r in range(REPEATS):
            iv = []
            for sp in spans:
                m = len(sp) // REPEATS
                iv += sp[r * m:(r + 1) * m]
            per_region.append(busy_union_ms(iv))
        vstats = [c.stats() for c in ctxs]
        group_comp = dict(launches=tot_l, views=tot_v, ms_per_launch=tot_span / max(tot_l, 1),
                          event_ms_per_launch=tot_ms / max(tot_l, 1), views_per_launch=tot_v / max(tot_l, 1),
                          busy_ms_regions=per_region, busy_ms=float(np.median(per_region)),
                          launches_per_region=tot_l / REPEATS, views_per_region=tot_v / REPEATS,
                          span_launches=sum(len(sp) for sp in spans),
                          mean_instances=float(np.mean([v["n_instances"] for v in vstats])),
                          instrumented_ms_per_frame=1e3 * float(np.median(gp_elapsed)) / timed_frames)

    # Per-stage times: a third region (view 0, one at a time) with libgsr's
    # HIP events recorded on the render stream between the stages.
    if not args.no_profile:
        _lib.check(lib.gsr_context_set_profiling(ctx.handle, 1), "set_profiling")
        prof_elapsed = timed_region(serial_frame, args.steps, dev)

    stats = ctx.stats()
    # tile-list length distribution of the last frame (load balance of the compositor)
    nt = stats["tiles_x"] * stats["tiles_y"]
    rb = torch.empty(2 * nt, dtype=torch.int32, device=dev)
    lib.gsr_debug_copy(ctx.handle, _lib.GSR_DEBUG_TILE_RANGES, ctypes.c_void_p(rb.data_ptr()), 8 * nt, None)
    torch.cuda.synchronize()
    rr = rb.cpu().numpy().reshape(nt, 2).astype(np.int64)
    lens = rr[:, 1] - rr[:, 0]
    stats["tile_len_max"] = int(lens.max())
    stats["tile_len_p99"] = int(np.percentile(lens, 99))
    stats["tile_len_mean"] = float(lens.mean())
    stats["instances_per_visible"] = stats["n_instances"] / max(stats["n_visible"], 1)
    stage = {}
    if not args.no_profile:
        ms = (ctypes.c_double * len(_lib.STAGES))()
        frames = ctypes.c_int64()
        _lib.check(lib.gsr_context_stage_times(ctx.handle, ms, ctypes.byref(frames)), "stage_times")
        stage = {name: ms[i] / max(frames.value, 1) for i, name in enumerate(_lib.STAGES)}
        stage["instrumented_ms_per_frame"] = 1e3 * prof_elapsed / args.steps

    # every rank's own rate (validation of the weak-scaling line; outside the timed regions)
    from gsviewer_amd.multiview import gather_objects
    per_rank = gather_objects(dict(rank=rank, local_rank=local, views=[rank + world * j for j in range(K)],
                                   elapsed_s=own[0], splats_per_s=n * args.steps / own[0],
                                   n_visible=stats["n_visible"], n_instances=stats["n_instances"]), world)
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return

    for c in ctxs[1:]:
        c.close()
    ms_per_step = 1e3 * elapsed / args.steps
    fps = args.steps / elapsed
    value = n * args.steps * world / elapsed
    rec_bytes = 4 * (11 + 3 * k_coef)
    b_frame = n * rec_bytes + W * H * 12

    roof = None
    if stage:
        inst = stats["n_instances"]
        ntiles = stats["tiles_x"] * stats["tiles_y"]
        nvis = stats["n_visible"]
        # each stage's own algorithmic bytes per frame alone (DESIGN.md "Kernels of a frame")
        alg = stage_bytes(n, nvis, inst, ntiles, W, H, rec_bytes, share=1)
        kernels = {k: v for k, v in stage.items() if k in alg}
        dom = max(kernels, key=kernels.get)
        achieved = alg[dom] / (stage[dom] * 1e-3) / 1e9
        roof = {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS, "traffic": None, "alg_bytes_per_launch": alg[dom],
                "ms_per_launch": stage[dom], "traffic_source": None,
                "frame": {"bytes": b_frame, "GBps": b_frame * fps / 1e9, "frac": b_frame * fps / 1e9 / HBM_PEAK_GBS,
                          "basis": "SURVEY 8(d) B_frame = N*R + W*H*12 per frame, at the timed region's frame rate"},
                "measured_copy_GBps": copy_gbps}
        traffic = pmc_traffic(KERNEL_SYMBOL.get(dom), args)
        if traffic:
            roof["traffic"], roof["traffic_source"] = traffic
        if group_comp is not None and group_comp["launches"] > 0 and group_comp["busy_ms"] > 0:
            # The timed region's dominant kernel: k_composite_views<0>, one launch per group of
            # `vpl` views.  Bytes: its OWN algorithmic bytes (the records and slots of its instances,
            # the tile ranges, the image; the scene read is the preprocess's).  Time:
            # the union of the launches' in-kernel spans over a repeat of the timed region (the four
            # groups' launches overlap: a launch's own span counts waits for CUs the others hold),
            # the median of REPEATS repeats, per launch; beside it the same union from the committed
            # rocprofv3 kernel trace of this command (profiles/LATEST/region_kernels.json).
            vpl = group_comp["views_per_launch"]
            busy_ms = group_comp["busy_ms"]
            us_view = 1e3 * busy_ms / group_comp["views_per_region"]
            ms_launch = busy_ms / group_comp["launches_per_region"]
            alg_view = group_comp["mean_instances"] * (48 + 4) + ntiles * 8 + W * H * 12
            ach = alg_view * vpl / (ms_launch * 1e-3) / 1e9
            single = {k: roof.pop(k) for k in ("kernel", "achieved", "frac", "traffic", "alg_bytes_per_launch",
                                               "ms_per_launch", "traffic_source") if k in roof}
            single["kernel"] = f"{KERNEL_SYMBOL.get(dom, dom)} (one view at a time, gsr_render: {dom} stage)"
            gt = pmc_traffic("k_composite_views<0>", args)
            prof = rocprof_avg_ms("k_composite_views<0>", args)
            region = committed_json("region_kernels.json", args)
            rk = None
            if region:
                kk = region["timed_region"]["kernels"].get("k_composite_views<0>")
                rk = {"us_per_view": kk["busy_us_per_frame"] if kk else None,
                      "source": f"profiles/{latest()}/region_kernels.json (tools/region_kernels.py)"}
            # The printed time is the profiler's (recomputable from profiles/LATEST): the
            # union of the launches' [start, end) in the committed rocprofv3 trace of `bench.py --steps 20
            # --warmup 5`, per view of its timed region.  It counts a launch from its dispatch, also while its
            # first blocks wait for CUs other streams hold; the live in-kernel union below counts from the
            # first block's start, so it reads lower (the two differ by definition, not by noise).
            live_us = us_view
            live_ach = ach
            use_rp = bool(rk and rk["us_per_view"])
            if use_rp:
                us_view = rk["us_per_view"]
                ms_launch = us_view * vpl * 1e-3
                ach = alg_view * vpl / (ms_launch * 1e-3) / 1e9
            roof.update({"kernel": f"k_composite_views<0> (the timed region's compositing, one launch per group "
                                   f"of {vpl:g} views)",
                         "basis": "the kernel's own algorithmic bytes per view: instances x (48-B record + 4-B slot) "
                                  "+ tiles x 8 (ranges) + W*H*12 (image)",
                         "achieved": ach, "frac": ach / HBM_PEAK_GBS, "alg_bytes_per_launch": alg_view * vpl,
                         "alg_bytes_per_view": alg_view, "ms_per_launch": ms_launch, "us_per_view": us_view,
                         "timing": ("rocprofv3: union of the k_composite_views launches' [start, end) in the timed "
                                    f"region of the committed kernel trace ({rk['source']}), per view"
                                    if use_rp else "live (no committed profile for this command): see live"),
                         "live": {"us_per_view": live_us, "achieved": live_ach, "frac": live_ach / HBM_PEAK_GBS,
                                  "timing": f"union of the in-kernel spans (first block start to last wave end, "
                                            f"100 MHz s_memrealtime) of the k_composite_views launches of a repeat "
                                            f"of the timed region, median of {REPEATS} repeats "
                                            f"({[round(x, 4) for x in group_comp['busy_ms_regions']]} ms; "
                                            f"{group_comp['instrumented_ms_per_frame']:.4f} ms/frame instrumented)"},
                         "cross_check": {"us_per_view_le_ms_per_step": us_view <= 1e3 * ms_per_step,
                                         "ms_per_step_us": 1e3 * ms_per_step,
                                         "achieved_le_peak": ach <= HBM_PEAK_GBS,
                                         "live_over_rocprof": live_us / rk["us_per_view"] if use_rp else None,
                                         "printed": "achieved / frac / us_per_view: the committed rocprofv3 trace "
                                                    "(recomputable from profiles/LATEST); live: this run's own "
                                                    "in-kernel figure"},
                         "views_per_launch": vpl,
                         "traffic": gt[0] if gt else None, "traffic_per_view": gt[0] / vpl if gt else None,
                         "traffic_source": gt[1] if gt else None,
                         "rocprof_stats_avg_launch": prof,
                         "contended_span": {
                             "ms_per_launch": group_comp["ms_per_launch"],
                             "event_ms_per_launch": group_comp["event_ms_per_launch"],
                             "timing": "each launch's own in-kernel span, averaged (overlapping launches each count "
                                       "the others' time: not the kernel's cost); event_ms_per_launch: HIP events "
                                       "around the same launches on the group's stream"},
                         "single_view": single})
            if region:
                roof["per_kernel"] = per_kernel_table(region, n, nvis, group_comp["mean_instances"], ntiles, W, H,
                                                      rec_bytes, vpl)
        res_fr = frame_resources(args, share, ms_per_step, b_frame, fps)
        if res_fr:
            roof["resources"] = res_fr
            top = max(res_fr["fractions"], key=res_fr["fractions"].get)
            roof["binding_resource"] = {
                "name": top, "frac": res_fr["fractions"][top],
                "basis": "the frame in flight's demand on each resource over the timed region's frame time "
                         "(resources.fractions); the largest is named",
                "reading": ("no resource saturates: the frame is latency-bound (dependent record and LDS waits, "
                            "launch floors and dispatch tails under four group streams)"
                            if res_fr["fractions"][top] < 0.6 else "saturating")}

    cpu = None
    if not args.no_cpu_baseline and world == 1 and g is not None:
        cpu = cpu_baseline(g, cam, args.cpu_seconds)

    res = {
        "metric": "rendered splats/sec/GPU + frames/sec at 1080p, 1M Gaussians" if args.config == "c2"
        else f"rendered splats/sec ({desc})",
        "value": value,
        "unit": "splats/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "fps_per_gpu": fps,
        "latency_ms_per_frame": 1e3 * latency / args.steps,
        "host_ms_per_call": {"calls": len(host_steps), "mean": 1e3 * sum(host_steps) / max(1, len(host_steps)),
                             "max": 1e3 * max(host_steps, default=0.0),
                             "note": "host time of each pipeline step (one group's finish + begin) and of the "
                                     "closing drain in the timed region"},
        "latency_ms_median": latency_median_ms,
        "views_in_flight": K,
        "splats_per_s_per_gpu": value / world,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": data_desc,
        "config": {"workload": desc + ("" if args.box == "none" else f", {args.box.upper()} box cull")
                   + (f", {K} views in flight per GPU" if K > 1 else ""),
                   "n_gaussians": n, "sh_degree": deg, "width": W, "height": H,
                   "views": f"view v = default camera yawed v*45 deg; rank r renders v = r + {world}*j, j < {K}, "
                            f"round-robin, one stream per view",
                   "t_min": args.t_min,
                   "parallelism": f"replicated scene, {world * K} independent views ({K} per GPU in flight)"
                                  + (f", cull + preprocess shared by groups of {share} views (one scene pass "
                                     f"per group; the last group {K - share * ((K - 1) // share)})"
                                     if share > 1 else "")},
        "frame_stats": stats,
        "stage_ms": stage,
        "roofline": roof,
        "cpu_baseline": cpu,
        "c4_one_view_per_gpu": None if world == 1 else {
            "definition": "SURVEY 8d C4: view k = default camera yawed k*45 deg on GPU k, one view per GPU, "
                          "frames one at a time (gsr_render); barrier + synchronize around the region, max over ranks",
            "value": n * args.steps * world / latency, "unit": "splats/s", "ms_per_frame": 1e3 * latency / args.steps,
            "views": list(range(world))},
        "broadcast": bcast,
        "process_group": {"backend": dist.get_backend() if world > 1 else None,
                          "world_size": dist.get_world_size() if world > 1 else 1,
                          "rehearsal_shared_gpu": shared_gpu},
        "per_rank": per_rank,
        "scene_gen_s": t_gen,
    }
    print(json.dumps(res), file=JSON_OUT, flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
