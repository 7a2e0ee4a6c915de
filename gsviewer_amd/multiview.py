"""Multi-GPU path: independent camera views, one process per GPU.

SURVEY.md §8(e): the path shards over independent units (camera views).
Every rank holds the whole scene and renders its own view, and nothing is
exchanged per frame.  The only collective is ONE broadcast of the scene from
rank 0 at load.  On MI355X the backend is "nccl" (RCCL over xGMI).  The CPU
tests run the same code over gloo.

bench.py and the world_size-2 gloo tests (tests/test_multiview_gloo.py) both
use these helpers, so the tested code is the benchmarked code.
"""
from __future__ import annotations

import queue
import threading
import time
from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from .camera import Camera, view_for_rank

SCENE_FIELDS = ("xyz", "rot", "scale", "opacity", "sh")


def record_floats(k_coef: int) -> int:
    """Floats per Gaussian of the packed scene record, ``GaussianData.flat()``
    (util_gau.py:40-42): xyz, rot, scale, opacity, sh = 11 + 3 k_coef."""
    return 11 + 3 * k_coef


def broadcast_scene(g, n: int, k_coef: int, device, src: int = 0) -> Tuple[torch.Tensor, Optional[dict]]:
    """Replicate the scene on every rank as ONE packed buffer.

    Rank `src` passes its GaussianData `g` and packs it into the record
    layout the reference uploads as its SSBO (``flat()``, [n, 11 + 3 k_coef]
    float32); the other ranks pass None and allocate a receive buffer of that
    shape.  One ``broadcast`` of the whole buffer (RCCL over xGMI on the GPU
    pool) replicates it; ``HipScene.from_flat`` then repacks it on each device.
    Returns the buffer on `device` and the broadcast's size/time (None when
    single-process).
    """
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    shape = (n, record_floats(k_coef))
    if rank == src:
        if g is None:
            raise ValueError("broadcast_scene: the source rank must pass the scene")
        flat = np.ascontiguousarray(g.flat(), dtype=np.float32)
        if flat.shape != shape:
            raise ValueError(f"broadcast_scene: packed scene {flat.shape} != expected {shape}")
        buf = torch.from_numpy(flat).to(device)
    else:
        buf = torch.empty(shape, dtype=torch.float32, device=device)
    if world == 1:
        return buf, None
    _sync(device)
    dist.barrier()
    t0 = time.perf_counter()
    dist.broadcast(buf, src=src)
    _sync(device)
    dt = time.perf_counter() - t0
    nbytes = buf.numel() * buf.element_size()
    return buf, dict(bytes=nbytes, seconds=dt, GBps=nbytes / max(dt, 1e-12) / 1e9, collectives=1)


def unpack_scene(buf: torch.Tensor, k_coef: int):
    """The five field views (xyz, rot, scale, opacity, sh) of a packed buffer."""
    cuts = np.cumsum([0, 3, 4, 3, 1, 3 * k_coef])
    return [buf[:, cuts[i]:cuts[i + 1]] for i in range(5)]


def view_of(rank: int, height: int, width: int) -> Camera:
    """Camera of rank k: the default camera yawed by k*45 degrees."""
    return view_for_rank(height, width, rank)


def timed_region(step: Callable[[], None], steps: int, device, local_out: Optional[list] = None) -> float:
    """Time exactly `steps` calls of `step`.

    The region is bracketed by a barrier and a device synchronize on both
    sides.  Returns the MAX elapsed seconds over all ranks (this rank's own
    time is appended to `local_out` when given).
    """
    world = dist.get_world_size() if dist.is_initialized() else 1
    if world > 1:
        dist.barrier()
    _sync(device)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    _sync(device)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if local_out is not None:
        local_out.append(elapsed)
    if world > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
        elapsed = float(e.item())
    return elapsed


def gather_objects(obj, world: int) -> Sequence:
    """All-gather a small picklable object (validation only, outside timed regions)."""
    if world == 1:
        return [obj]
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def _sync(device) -> None:
    dev = torch.device(device)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


class ViewPipeline:
    """Several independent views in flight on one GPU, one context and stream
    each.  step() renders the next frame round-robin: it finishes that view's
    previous frame (gsr_render_finish: host wait for its counts, then the
    binning, tile sort and compositing launches) and begins its next one
    (gsr_render_begin: culling, preprocess, depth sort).  A view's counts are
    therefore waited on only after the other views' frames have been
    enqueued, so the GPU always has work queued.  drain() finishes every
    pending frame; a frame counts once begun, and is complete after drain()
    and a device synchronize."""

    def __init__(self, ctxs, streams, scene, cams, settings, outs):
        assert len(ctxs) == len(streams) == len(cams) == len(outs) >= 1
        self.ctxs, self.streams, self.scene, self.cams = ctxs, streams, scene, cams
        self.settings, self.outs = settings, outs
        self.pending = [False] * len(ctxs)
        self.next = 0

    def step(self):
        from .rasterizer import render_begin, render_finish
        k = self.next
        self.next = (k + 1) % len(self.ctxs)
        s = self.streams[k]
        if self.pending[k]:
            render_finish(self.ctxs[k], s)
        render_begin(self.ctxs[k], self.scene, self.cams[k], self.settings, self.outs[k], stream=s)
        self.pending[k] = True

    def drain(self):
        from .rasterizer import render_finish
        for k, p in enumerate(self.pending):
            if p:
                render_finish(self.ctxs[k], self.streams[k])
                self.pending[k] = False


class ViewBatchPipeline:
    """Views in flight in groups whose cull + preprocess share one pass over
    the scene (gsr_render_begin_views).

    `groups`: list of (ctxs, cams, outs, stream), k views each.  Everything of
    a group runs on the group's stream, so no cross-stream event is needed
    (each costs the frame ~50 us here: tools/event_cost.py): step() finishes
    the next group's pending frames (gsr_render_finish_views: the host waits
    for the views' counts, then enqueues their binning, tile sort and
    compositing, one launch per stage for the group), then begins the group's
    next frames: the shared cull + preprocess of its k views, then their depth
    sorts, batched into one launch per radix step (gsr_render_begin_sorts).
    The groups' streams overlap one another, as the views of ViewPipeline do.
    batched_sorts / batched_finish=False use the per-view calls instead.  drain() finishes every pending frame.  Images
    are identical to rendering each view alone (tests/test_gpu_multiview.py)."""

    def __init__(self, groups, scene, settings, batched_sorts=True, batched_finish=True, lookahead=None):
        assert len(groups) >= 1
        self.groups = groups
        self.scene, self.settings = scene, settings
        self.batched_sorts = batched_sorts  # the group's depth sorts in one launch per radix step
        self.batched_finish = batched_finish  # the group's second halves in one launch per stage
        # at most `lookahead` groups begun and not finished: a step that begins a
        # group finishes the oldest pending ones beyond that (None: all groups,
        # i.e. a group is finished only when it is begun again or drained; 0: every
        # group is finished in the step that begins it, the host waiting for its counts)
        self.lookahead = len(groups) if lookahead is None else max(0, min(int(lookahead), len(groups)))
        self.pending = [False] * len(groups)
        self.order = []  # pending groups, oldest first
        self.next = 0

    @property
    def frames_per_step(self):
        return len(self.groups[self.next][0])

    def _finish(self, gi):
        from .rasterizer import render_finish, render_finish_views
        ctxs, _, _, stream = self.groups[gi]
        if self.batched_finish:
            render_finish_views(ctxs, stream)
        else:
            for c in ctxs:
                render_finish(c, stream)
        self.pending[gi] = False
        self.order.remove(gi)

    def step(self):
        from .rasterizer import render_begin_sort, render_begin_sorts, render_begin_views
        gi = self.next
        self.next = (gi + 1) % len(self.groups)
        ctxs, cams, outs, stream = self.groups[gi]
        if self.pending[gi]:
            self._finish(gi)
        render_begin_views(ctxs, self.scene, cams, self.settings, outs, stream=stream)
        if self.batched_sorts:
            render_begin_sorts(ctxs, stream)
        else:
            for c in ctxs:
                render_begin_sort(c, stream)
        self.pending[gi] = True
        self.order.append(gi)
        while len(self.order) > self.lookahead:
            self._finish(self.order[0])

    def drain(self):
        while self.order:
            self._finish(self.order[0])


class _GroupWorker(threading.Thread):
    """One host thread driving one group's stream (ThreadedViewBatchPipeline)."""

    def __init__(self, device):
        super().__init__(daemon=True)
        self.q = queue.Queue()
        self.error = None
        self.device = device
        self.start()

    def run(self):
        if self.device is not None:  # HIP's current device is per thread: the group stream's own
            torch.cuda.set_device(self.device)
        while True:
            fn = self.q.get()
            if fn is None:
                self.q.task_done()
                return
            try:
                if self.error is None:
                    fn()
            except BaseException as e:  # re-raised by the pipeline's wait()
                self.error = e
            finally:
                self.q.task_done()


class ThreadedViewBatchPipeline(ViewBatchPipeline):
    """ViewBatchPipeline with one host thread per group: a group's finish
    (which waits on the host for its frames' counts) and begin calls run on
    its own thread, so the groups' launch sequences are enqueued in parallel
    instead of one after the other (ctypes releases the GIL during each call;
    the library's calls for different contexts and streams are independent).
    step() hands the group's next step to its thread and returns; drain()
    finishes every pending frame and waits for all threads.  Images are
    identical to ViewBatchPipeline's (tests/test_gpu_multiview.py)."""

    def __init__(self, groups, scene, settings, batched_sorts=True, batched_finish=True):
        super().__init__(groups, scene, settings, batched_sorts, batched_finish)
        self.workers = [_GroupWorker(getattr(g[3], "device", None)) for g in groups]

    def _group_step(self, gi):
        from .rasterizer import render_begin_sort, render_begin_sorts, render_begin_views
        ctxs, cams, outs, stream = self.groups[gi]
        if self.pending[gi]:
            self._finish_group(gi)
        render_begin_views(ctxs, self.scene, cams, self.settings, outs, stream=stream)
        if self.batched_sorts:
            render_begin_sorts(ctxs, stream)
        else:
            for c in ctxs:
                render_begin_sort(c, stream)
        self.pending[gi] = True

    def _finish_group(self, gi):
        from .rasterizer import render_finish, render_finish_views
        ctxs, _, _, stream = self.groups[gi]
        if self.batched_finish:
            render_finish_views(ctxs, stream)
        else:
            for c in ctxs:
                render_finish(c, stream)
        self.pending[gi] = False

    def step(self):
        gi = self.next
        self.next = (gi + 1) % len(self.groups)
        self.workers[gi].q.put(lambda gi=gi: self._group_step(gi))

    def wait(self):
        for w in self.workers:
            w.q.join()
        for w in self.workers:
            if w.error is not None:
                e, w.error = w.error, None
                raise e

    def drain(self):
        for gi, w in enumerate(self.workers):
            w.q.put(lambda gi=gi: self._finish_group(gi) if self.pending[gi] else None)
        self.wait()

    def close(self):
        for w in self.workers:
            w.q.put(None)
        for w in self.workers:
            w.join()
