"""The test model of the coarse depth order (helpers.frame_depth_order), on CPU.

The GPU tests compare a frame's GSR_DEBUG_DEPTH_ORDER with this model and its
tile lists with the exact GL order (tests/test_gpu_coarse_depth.py).  Here:
the model with 0 coarse bits is the exact front-to-back order; with a coarse
width it is sorted by coarse key, equal coarse keys in descending id, and it
differs from the exact order only inside groups of equal coarse keys -- the
groups k_tile_ranges' run repair reorders per tile.
"""
import numpy as np
import pytest

from helpers import frame_depth_order
from oracle import gl_oracle as O


def _stage(n, seed):
    rng = np.random.default_rng(seed)
    z = rng.uniform(-8.0, -1.0, n).astype(np.float32)
    z[rng.integers(0, n, n // 10)] = np.float32(-3.0)          # exact ties
    near = rng.integers(0, n, n // 10)
    z[near] = np.nextafter(np.float32(-2.0), np.float32(0.0))  # neighbours in the low key bits
    vis = rng.random(n) > 0.2
    return {"view_z": z, "visible": vis}


def _keys(z):
    b = (-z.astype(np.float32)).view(np.uint32).astype(np.uint64)
    return np.where(b & 0x80000000, ~b & 0xFFFFFFFF, b | 0x80000000)


@pytest.mark.parametrize("seed", [0, 1])
def test_exact_model_is_the_gl_order(seed):
    vs = _stage(20_000, seed)
    exact = O.sort_back_to_front(vs["view_z"], vs["visible"])[::-1]
    np.testing.assert_array_equal(frame_depth_order(vs, 0), exact)


@pytest.mark.parametrize("coarse", [8, 16, 22, 24])
def test_coarse_model_refines_to_exact(coarse):
    vs = _stage(20_000, coarse)
    exact = O.sort_back_to_front(vs["view_z"], vs["visible"])[::-1]
    got = frame_depth_order(vs, coarse)
    assert sorted(got.tolist()) == sorted(exact.tolist())
    key = _keys(vs["view_z"])
    # ascending coarse keys (a stable sort's output), equal coarse keys in descending id
    gid = np.nonzero(vs["visible"])[0]
    kmin = int(key[gid].min())
    s0 = max(0, int(key[gid].max() - kmin).bit_length() - coarse)
    ck = (key[got] - kmin) >> np.uint64(s0)
    assert np.all(np.diff(ck.astype(np.int64)) >= 0)
    same = ck[1:] == ck[:-1]
    assert np.all(got[1:][same] < got[:-1][same])
    # a key range no wider than the coarse bits: nothing was dropped, the order is exact
    if s0 == 0:
        np.testing.assert_array_equal(got, exact)
    else:
        # the exact order moves instances only inside groups of equal coarse keys
        ck_exact = (key[exact] - kmin) >> np.uint64(s0)
        np.testing.assert_array_equal(ck_exact, ck)
        if coarse <= 16:  # 8+ dropped bits over 20k random depths: some groups are out of key order
            assert not np.array_equal(got, exact)
