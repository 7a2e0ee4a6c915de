"""The pipeline's alternative stage forms give identical frames:

* GSR_BIN_FUSED (default 1): the binning with the tile sort's first radix
  pass fused in (k_bin_hist + k_bin_scatter) against the separate binning and
  full tile sort (k_bin_reduce + k_bin_write, then every radix pass): integer
  index work;
* GSR_TAIL_MERGE (groups, default 1) / GSR_TAIL_MERGE_ALONE (a frame alone,
  default 0): a multi-chunk tile folded by its last chunk to finish, inside
  the compositing launch, against the k_merge launch: the same fold in the
  same chunk order;
* GSR_FUSED_CULL (default 1): culling inside the preprocess, uncompacted
  slots, culled keys dropped by the depth sort's first pass, against k_cull +
  the compaction scan + k_preprocess (tests/helpers.grab_debug maps the
  uncompacted slots to the compacted ones by rank);
* GSR_CHUNK_SINGLE (default 0): a frame alone's chunk descriptors, dispatch
  order and class totals written by one block (k_chunk_single) against the
  count + write launches.

Images, records, depth order, tile lists and tile ranges must be bit-identical, on a frame rendered alone (gsr_render) and on a group of
views (gsr_render_finish_views), for frame sizes whose tile ids take one
radix pass (<= 2048 tiles) and two, plus the full-size C2 frame."""
import numpy as np
import pytest

from gsviewer_amd.camera import Camera
from gsviewer_amd.gaussian_data import garden_standin
from helpers import batched_frames, gpu_frame

pytestmark = pytest.mark.gpu

VARIANTS = [{}, {"GSR_BIN_FUSED": "0"}, {"GSR_TAIL_MERGE": "0", "GSR_TAIL_MERGE_ALONE": "1"},
            {"GSR_FUSED_CULL": "0"}, {"GSR_CHUNK_SINGLE": "1"}]


def _settings(**kw):
    from gsviewer_amd.rasterizer import RenderSettings
    return RenderSettings(**kw)


def _frames(monkeypatch, env, g, scene, cams):
    for k in ("GSR_BIN_FUSED", "GSR_TAIL_MERGE", "GSR_TAIL_MERGE_ALONE", "GSR_FUSED_CULL", "GSR_DEPTH_COARSE",
              "GSR_CHUNK_SINGLE"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    alone = gpu_frame(g, cams[0], _settings(), with_debug=True)
    group = batched_frames(scene, cams, _settings(), group=len(cams), debug_views=(0,))
    return alone, group


@pytest.mark.parametrize("h,w,n", [(360, 640, 60_000), (720, 1280, 200_000), (1080, 1920, 1_000_000)])
def test_stage_variants_identical(gpu, monkeypatch, h, w, n):
    from gsviewer_amd.rasterizer import HipScene
    g = garden_standin(n, seed=1, sh_degree=0 if n < 1_000_000 else 3)
    scene = HipScene.from_gaussian_data(g)
    cams = [Camera(h, w).yaw(45.0 * v) for v in range(3)]
    ref = None
    for env in VARIANTS:
        alone, group = _frames(monkeypatch, env, g, scene, cams)
        got = (alone, group)
        if ref is None:
            ref = got
            assert alone["stats"]["n_instances"] > 0
            continue
        for a, b in ((ref[0], alone), (ref[1][0], group[0])):
            for key in ("tile_list", "ranges", "depth_order", "records"):
                if key == "depth_order" and a["depth_coarse"] != b["depth_coarse"]:
                    continue  # (GSR_BIN_FUSED=0 sorts exactly: the repair needs the fused binning's keys)
                np.testing.assert_array_equal(a[key], b[key], err_msg=f"{env} {key}")
            np.testing.assert_array_equal(a["image"], b["image"], err_msg=f"{env} image")
        for v in range(1, len(cams)):
            np.testing.assert_array_equal(ref[1][v]["image"], group[v]["image"], err_msg=f"{env} view {v}")
    scene.close()


def test_group_frames_repeatable(gpu):
    """The same group rendered again gives bit-identical images.  A group's
    tiles of several chunks are folded in-kernel by the chunk that finishes
    last (the tail merge), reading the other chunks' partials across XCDs;
    a stale read there shows as a few pixels (single-splat footprints) that
    differ from one render to the next, at the bench's 1080p / 1M size."""
    from gsviewer_amd.rasterizer import HipScene
    h, w = 1080, 1920
    g = garden_standin(1_000_000, seed=1, sh_degree=3)
    scene = HipScene.from_gaussian_data(g)
    cams = [Camera(h, w).yaw(45.0 * v) for v in range(3)]
    ref = [f["image"] for f in batched_frames(scene, cams, _settings(), group=3)]
    for it in range(6):
        got = batched_frames(scene, cams, _settings(), group=3)
        for v in range(3):
            np.testing.assert_array_equal(got[v]["image"], ref[v], err_msg=f"repeat {it} view {v}")
    scene.close()


def test_chunk_single_deep_form(gpu, monkeypatch):
    """The deep form's chunking (longer chunks, first chunks dispatched
    first, published maxima initialised) by one block and by the count +
    write launches: identical frames at t_min = 0 (the bound then never
    stops a chunk, so the images depend on the descriptors only)."""
    g = garden_standin(300_000, seed=1, sh_degree=1)
    cam = Camera(720, 1280)
    monkeypatch.setenv("GSR_CHUNK_TARGET", "256")  # D / 256 chunks: longer than 192, the deep form
    got = {}
    for single in ("1", "0"):
        monkeypatch.setenv("GSR_CHUNK_SINGLE", single)
        got[single] = gpu_frame(g, cam, _settings(t_min=0.0), with_debug=True)
    for key in ("tile_list", "ranges", "image"):
        np.testing.assert_array_equal(got["1"][key], got["0"][key], err_msg=key)

