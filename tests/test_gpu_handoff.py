"""The tail merge's cross-XCD hand-off, under forced orderings.

A group's tile of several chunks is folded inside the compositing launch by
the chunk whose counter add comes last: it reads the other chunks' partials
(stored `sc1`) and the slices' saturation words (agent-scope atomics).
Round 3 changed two of those reads after a run-to-run mismatch that appeared
only when dispatch timing happened to line up (f4e3b53: the partials, then
plain loads, now `sc1` loads; 8352f97: the saturation words, then an
agent-scope load, now an atomic read); neither change is confirmed as the
cause (below).  Here the context's test knob GSR_DEBUG_HANDOFF forces the
orderings every time (composite_chunk):

* bit 0: chunk 0 of every multi-chunk tile adds last (it waits for the other
  chunks' adds), so the fold always runs on chunk 0's CU;
* bit 1: chunk 0 polls its tile's saturation words first, so its XCD's L2
  holds that line before any later chunk saturates a slice;
* bit 2: chunk 0 plain-loads the other chunks' partial slots first, so its
  XCD's L2 holds them with the previous frame's contents.

The same contexts render two different views alternately (the partial slots
then hold another frame's values), with small chunks and t_min > 0 on a dense,
opaque scene (many multi-chunk tiles; later chunks saturate slices).  Every
frame must equal the k_merge path's (GSR_TAIL_MERGE=0) bit for bit.

What this does NOT show: the verification builds -DGSR_TAIL_REVERT_SAT_ATOMIC
and -DGSR_TAIL_REVERT_SC1_LOADS (the code before each round-3 fix) PASS these
checks too (profiles/r4_s6/README.md), and a microbenchmark found the XCD L2
coherent for exactly these accesses (profiles/r4_s5).  So the tests guard the
fold's logic under forced orderings (chunk order, the saturation bound, slots
holding another frame's values), not the two memory-visibility forms; round
3's run-to-run mismatch has no confirmed cause ("Tail merge:
determinism").
"""
import numpy as np
import pytest
import torch

from gsviewer_amd.camera import Camera
from gsviewer_amd.gaussian_data import random_scene

pytestmark = pytest.mark.gpu

H, W = 180, 320
GROUP = 3


def _render_alternating(monkeypatch, env, scene, cam_sets, rounds):
    """The same GROUP contexts render cam_sets[0], cam_sets[1], ... in turn,
    `rounds` times; returns the images of every render."""
    from gsviewer_amd.multiview import ViewBatchPipeline
    from gsviewer_amd.rasterizer import HipContext, RenderSettings, camera_from
    for k in ("GSR_TAIL_MERGE", "GSR_DEBUG_HANDOFF", "GSR_CHUNK_VIEWS", "GSR_FIRST_MAJOR"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    ctxs = [HipContext() for _ in range(GROUP)]
    outs = [torch.empty((3, H, W), dtype=torch.float32, device="cuda") for _ in range(GROUP)]
    stream = torch.cuda.Stream()
    st = RenderSettings(t_min=1e-4, out_layout=0)
    images = []
    for _ in range(rounds):
        for cams in cam_sets:
            pipe = ViewBatchPipeline([(ctxs, [camera_from(c) for c in cams], outs, stream)], scene, st)
            pipe.step()
            pipe.drain()
            torch.cuda.synchronize()
            images.append([o.permute(1, 2, 0).contiguous().cpu().numpy() for o in outs])
    multi = ctxs[0].stats()
    for c in ctxs:
        c.close()
    return images, multi


@pytest.fixture(scope="module")
def scene_and_views():
    from gsviewer_amd.rasterizer import HipScene
    g = random_scene(60_000, sh_degree=1, seed=7, scale_range=(0.01, 0.06))
    g.opacity[:] = np.maximum(g.opacity, 0.6).astype(np.float32)   # opaque: slices saturate mid-list
    scene = HipScene.from_gaussian_data(g)
    cam_sets = [[Camera(H, W).yaw(30.0 * v) for v in range(GROUP)],
                [Camera(H, W).yaw(30.0 * v + 100.0) for v in range(GROUP)]]
    yield scene, cam_sets
    scene.close()


@pytest.mark.parametrize("knob", ["3", "5", "7"])
def test_forced_handoff_equals_merge_launch(gpu, monkeypatch, scene_and_views, knob):
    scene, cam_sets = scene_and_views
    small = {"GSR_CHUNK_VIEWS": "64", "GSR_FIRST_MAJOR": "1"}
    ref, stats = _render_alternating(monkeypatch, dict(small, GSR_TAIL_MERGE="0"), scene, cam_sets, 1)
    assert stats["n_instances"] > 60_000, stats  # ~50 tiles of 65 to 5000 instances: 64-instance chunks
    got, _ = _render_alternating(monkeypatch, dict(small, GSR_TAIL_MERGE="1", GSR_DEBUG_HANDOFF=knob), scene,
                                 cam_sets, 3)
    for i, frame in enumerate(got):
        want = ref[i % len(cam_sets)]
        for v in range(GROUP):
            np.testing.assert_array_equal(frame[v], want[v], err_msg=f"knob {knob} render {i} view {v}")


def test_alternating_groups_equal_merge_launch(gpu, monkeypatch, scene_and_views):
    """Without the knob: different frames through the same contexts (the
    partial slots hold the other frame's values) still fold exactly."""
    scene, cam_sets = scene_and_views
    small = {"GSR_CHUNK_VIEWS": "64"}
    ref, _ = _render_alternating(monkeypatch, dict(small, GSR_TAIL_MERGE="0"), scene, cam_sets, 1)
    got, _ = _render_alternating(monkeypatch, dict(small, GSR_TAIL_MERGE="1"), scene, cam_sets, 4)
    for i, frame in enumerate(got):
        want = ref[i % len(cam_sets)]
        for v in range(GROUP):
            np.testing.assert_array_equal(frame[v], want[v], err_msg=f"render {i} view {v}")
