"""The oracle against the reference's own shaders run on a real GL driver.

``tests/golden/llvmpipe_golden.npz`` holds framebuffers that Mesa llvmpipe
rendered from ``/root/reference/shaders/gau_vert.glsl`` + ``gau_frag.glsl``
with the reference's draw call, blend state, uniforms and depth order
(``tests/golden/make_gl_golden.py``, ``oracle/gl_ref/llvmpipe_gl.c``).  This
pins the restatement in ``oracle/gl_oracle.py``: the vertex stage, the GL
coverage (8 sub-pixel bits), the fragment stage, and both blend modes.

Stated tolerances (what remains is llvmpipe's own exp/rcp approximations: a
fragment whose alpha sits on the 1/255 discard threshold or an 8-bit rounding
boundary can land on the other side):
* float (RGBA32F target, fragment colour clamped): every channel within
  ``TOL_FLOAT`` = 2e-5 on >= 99.95 % of pixels, and within ``TOL_MAX`` = 8e-3
  everywhere (tests/helpers.py: two threshold flips in one pixel);
* gl8 (RGBA8 target): identical on >= 99.9 % of pixels, never more than 1/255.
"""
import os

import numpy as np
import pytest

import gl_cases as GC
from helpers import TOL_MAX
from oracle import gl_oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "llvmpipe_golden.npz")
TOL_FLOAT = 2e-5
FRAC_FLOAT = 0.9995
FRAC_GL8 = 0.999


@pytest.fixture(scope="module")
def golden():
    return np.load(GOLDEN)


def test_fixture_covers_every_case(golden):
    assert list(golden["cases"]) == list(GC.CASES)
    assert "llvmpipe" in str(golden["renderer"])


def oracle_frames(golden, name):
    g = GC.scene(GC.CASES[name][0])
    assert str(golden[f"{name}/sha"]) == GC.flat_sha(g), "scene generator changed: regenerate the fixture"
    _, U = GC.uniforms(name, g)
    vs = O.vertex_stage(g.flat(), g.sh_dim, U)
    order = golden[f"{name}/order"]
    order = order[vs["visible"][order]]   # the instances the vertex stage keeps, in the reference's draw order
    return vs, U, order


def _frames(golden, name):
    """(float image, gl8 image) of the oracle for a case: the NumPy restatement
    in the reference's own draw order, or for the large cases the C one
    (oracle/gl_oracle.c, pinned against the NumPy one by tests/test_oracle_c.py)
    in its own depth order."""
    if name in GC.LARGE:
        from oracle import c_oracle as C
        g = GC.scene(GC.CASES[name][0])
        assert str(golden[f"{name}/sha"]) == GC.flat_sha(g), "scene generator changed: regenerate the fixture"
        _, U = GC.uniforms(name, g)
        return (C.render(g.flat(), g.sh_dim, U, mode="float", threads=8),
                C.render(g.flat(), g.sh_dim, U, mode="gl8", threads=8))
    vs, U, order = oracle_frames(golden, name)
    return O.composite(vs, U, "float", order=order), O.composite(vs, U, "gl8", order=order)


@pytest.mark.parametrize("name", list(GC.CASES))
def test_oracle_matches_llvmpipe(golden, name):
    f, q8 = _frames(golden, name)
    ref = golden[f"{name}/float"]
    d = np.abs(f - ref).max(-1)
    assert (d <= TOL_FLOAT).mean() >= FRAC_FLOAT, (name, int((d > TOL_FLOAT).sum()))
    assert d.max() <= TOL_MAX, (name, float(d.max()))

    q = np.rint(q8 * 255).astype(np.int32)
    d8 = np.abs(q - golden[f"{name}/rgba8"].astype(np.int32)).max(-1)
    assert (d8 == 0).mean() >= FRAC_GL8, (name, int((d8 > 0).sum()))
    assert d8.max() <= 1, (name, int(d8.max()))


def test_reference_order_is_the_oracle_order_up_to_near_ties(golden):
    """The reference's _sort_gaussian_cpu order (stored) against the oracle's
    depth order: the same up to swaps of Gaussians whose view z differ by a few
    ulps (the reference's float32 matmul sums in another order)."""
    for name in ("sh3_m6", "sh0_m6", "big_close"):
        vs, U, order = oracle_frames(golden, name)
        z = vs["view_z"][order]
        assert np.all(np.diff(z) >= -1e-6 * np.maximum(1.0, np.abs(z[1:]))), name
