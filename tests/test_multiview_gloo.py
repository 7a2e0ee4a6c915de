"""World-size-2 tests of the multi-GPU path (gsviewer_amd/multiview.py) over
gloo on CPU: the one-time scene broadcast, the view
assignment, and the barrier-bracketed, max-over-ranks timing that bench.py
uses.  The rendering check uses the CPU oracle (test infrastructure), since
there is no GPU here; the GPU renders the same views in bench.py."""
import hashlib
import os
import socket
import time

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gsviewer_amd.gaussian_data import random_scene
from gsviewer_amd.multiview import broadcast_scene, gather_objects, timed_region, unpack_scene, view_of
from oracle import gl_oracle as O

WORLD = 2
N, DEG = 400, 1
H, W = 48, 64


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _digest(tensors):
    h = hashlib.sha256()
    for t in tensors:
        h.update(t.contiguous().numpy().tobytes())
    return h.hexdigest()


def _oracle_image(flat, k_coef, cam):
    """CPU oracle render of the packed scene buffer, for one camera."""
    flat = np.ascontiguousarray(flat, np.float32)
    U = O.default_uniforms(cam.get_view_matrix(), cam.get_project_matrix(),
                           np.asarray(cam.get_htanfovxy_focal(), np.float32), cam.position, cam.w, cam.h)
    return O.render(flat, 3 * k_coef, U)[0]


def _worker(rank, port, out_dir):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=WORLD)
    try:
        k_coef = (DEG + 1) ** 2
        g = random_scene(N, sh_degree=DEG, seed=5) if rank == 0 else None
        calls = []
        real_broadcast = dist.broadcast

        def counting_broadcast(*a, **kw):  # every collective the scene load issues
            calls.append(tuple(a[0].shape))
            return real_broadcast(*a, **kw)

        dist.broadcast = counting_broadcast
        try:
            packed, info = broadcast_scene(g, N, k_coef, "cpu")
        finally:
            dist.broadcast = real_broadcast
        fields = unpack_scene(packed, k_coef)
        digests = gather_objects(_digest([packed]), WORLD)
        collectives = gather_objects(calls, WORLD)

        cam = view_of(rank, H, W)
        img = _oracle_image(packed.numpy(), k_coef, cam)
        assert [tuple(f.shape) for f in fields] == [(N, 3), (N, 4), (N, 3), (N, 1), (N, 3 * k_coef)]
        images = gather_objects(img, WORLD)

        # rank 1 is slower: both ranks must report the same (max) elapsed time
        delay = 0.05 if rank == 1 else 0.0
        elapsed = timed_region(lambda: time.sleep(delay), 2, "cpu")
        times = gather_objects(elapsed, WORLD)

        if rank == 0:
            src = torch.from_numpy(np.ascontiguousarray(g.flat(), dtype=np.float32))
            np.savez(os.path.join(out_dir, "result.npz"),
                     src_digest=_digest([src]), digests=np.array(digests), bytes=info["bytes"],
                     collectives=np.array([len(c) for c in collectives]), info_collectives=info["collectives"],
                     collective_shapes=np.array([list(c[0]) for c in collectives]),
                     img0=images[0], img1=images[1], times=np.array(times),
                     ref0=_oracle_image(g.flat(), k_coef, view_of(0, H, W)),
                     ref1=_oracle_image(g.flat(), k_coef, view_of(1, H, W)))
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def result(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("mv"))
    mp.spawn(_worker, args=(_free_port(), out), nprocs=WORLD, join=True)
    return np.load(os.path.join(out, "result.npz"))


def test_broadcast_replicates_scene(result):
    # every rank holds a bit-identical copy of rank 0's packed scene (GaussianData.flat()) after ONE broadcast
    assert len(set(result["digests"].tolist())) == 1
    assert result["digests"][0] == result["src_digest"]
    assert int(result["bytes"]) == N * 4 * (3 + 4 + 3 + 1 + 3 * (DEG + 1) ** 2)


def test_scene_load_is_one_collective(result):
    # one broadcast of the packed scene buffer, on every rank, and nothing else
    assert result["collectives"].tolist() == [1] * WORLD
    assert int(result["info_collectives"]) == 1
    assert result["collective_shapes"].tolist() == [[N, 11 + 3 * (DEG + 1) ** 2]] * WORLD


def test_views_are_independent_per_rank(result):
    # rank k renders view k (default camera yawed by k*45 deg) of the replicated scene
    np.testing.assert_array_equal(result["img0"], result["ref0"])
    np.testing.assert_array_equal(result["img1"], result["ref1"])
    assert not np.array_equal(result["img0"], result["img1"])


def test_timed_region_reports_max_over_ranks(result):
    t = result["times"]
    assert t[0] == t[1]          # the same (max-reduced) value on every rank
    assert t[0] >= 0.1           # includes the slow rank's 2 x 50 ms


def test_view_assignment_matches_bench_contract():
    # view k = default camera yawed by k*45 degrees
    from gsviewer_amd.camera import Camera
    v0, v2 = view_of(0, H, W), view_of(2, H, W)
    np.testing.assert_allclose(v0.get_view_matrix(), Camera(H, W).get_view_matrix())
    np.testing.assert_allclose(v2.get_view_matrix(), Camera(H, W).yaw(90.0).get_view_matrix())
