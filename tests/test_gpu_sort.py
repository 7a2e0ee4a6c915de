"""The frame's radix sort on its own (C-ABI test hook gsr_debug_sort_pairs):
stable (key, index) order must equal NumPy's stable argsort exactly, across
sizes from one tile to ~1800 tiles (both tile sizes: 2048 items for wider
digits, 4096 for <= 8-bit digits), digit widths 6..11 bits and exact ties.
The depth-sort service and the in-frame sorts are checked against the
reference in test_gpu_scale.py; this isolates the sort itself."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def gpu_sort(ctx, keys, bits, passes):
    import torch

    from gsviewer_amd import _lib
    n = len(keys)
    kd = torch.from_numpy(keys.view(np.int32)).cuda()
    ko = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")
    vo = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")
    _lib.check(_lib.load().gsr_debug_sort_pairs(ctx.handle, ctypes.c_void_p(kd.data_ptr()), n, bits, passes,
                                                ctypes.c_void_p(ko.data_ptr()), ctypes.c_void_p(vo.data_ptr()), None),
               "gsr_debug_sort_pairs")
    torch.cuda.synchronize()
    return ko.cpu().numpy()[:n].view(np.uint32), vo.cpu().numpy()[:n].view(np.uint32)


@pytest.fixture(scope="module")
def ctx(gpu):
    from gsviewer_amd.rasterizer import HipContext
    c = HipContext()
    yield c
    c.close()


@pytest.mark.parametrize("n", [1, 100, 1024, 1025, 2049, 4097, 70_001, 300_000, 1_817_600])
@pytest.mark.parametrize("bits,passes", [(9, 1), (13, 2), (32, 3)])
def test_sort_matches_stable_argsort(ctx, n, bits, passes):
    rng = np.random.default_rng(n * 31 + bits)
    keys = rng.integers(0, 1 << bits, n, dtype=np.uint64).astype(np.uint32)
    if n > 10:
        keys[rng.integers(0, n, n // 10)] = keys[0]  # many exact ties
    want = np.argsort(keys, kind="stable").astype(np.uint32)
    ko, vo = gpu_sort(ctx, keys, bits, passes)
    np.testing.assert_array_equal(vo, want)
    np.testing.assert_array_equal(ko, keys[want])


def test_sort_all_equal_and_presorted(ctx):
    for keys in (np.full(50_000, 7, np.uint32), np.arange(50_000, dtype=np.uint32),
                 np.arange(50_000, dtype=np.uint32)[::-1].copy()):
        ko, vo = gpu_sort(ctx, keys, 16, 2)
        want = np.argsort(keys, kind="stable").astype(np.uint32)
        np.testing.assert_array_equal(vo, want)
