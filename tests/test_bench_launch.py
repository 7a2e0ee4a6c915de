"""bench.py's multi-GPU launch, rehearsed on CPU.

`python bench.py --gpus N` must start N ranks by itself (the driver's
scaling command) and, under torchrun, check that the world size equals
--gpus.  `--dry-run` runs the same launch, rendezvous (gloo), scene
broadcast, view assignment and max-over-ranks timing without a GPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=ROOT)


def _json_line(out):
    # stdout is exactly the one JSON line: library output on fd 1 (gloo's
    # connection messages, RCCL) goes to stderr (bench.py routes fd 1 there)
    lines = out.splitlines()
    assert len(lines) == 1 and lines[0].startswith("{"), out
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 3])
def test_gpus_flag_spawns_that_many_ranks(n):
    r = _run("--gpus", str(n), "--dry-run", "--steps", "2", "--inflight", "4")
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["dry_run"] and d["n_gpus"] == n and d["backend"] == "gloo"
    ranks = d["ranks"]
    assert [x["rank"] for x in ranks] == list(range(n))
    assert all(x["world"] == n for x in ranks)
    # rank r renders views r, r + n, r + 2n, ... (view k = default camera yawed k*45 deg)
    assert [x["views"][0] for x in ranks] == list(range(n))
    assert all(x["views"] == [x["rank"] + n * j for j in range(4)] for x in ranks)
    # one broadcast replicated the scene bit-for-bit
    assert len({x["scene_sum"] for x in ranks}) == 1
    assert d["broadcast"]["bytes"] == 1000 * 4 * (11 + 48)
    # the timed region reports the max over ranks on every rank
    assert len({x["elapsed"] for x in ranks}) == 1
    # distinct views per rank
    assert len({tuple(x["view0_row2"]) for x in ranks}) == n


def test_single_rank_dry_run():
    r = _run("--dry-run", "--steps", "1")
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 1 and d["broadcast"] is None and len(d["ranks"]) == 1


def test_world_size_must_match_gpus():
    r = _run("--gpus", "2", "--dry-run", "--steps", "1",
             env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=1 but --gpus 2" in r.stderr


def test_eight_rank_line_carries_c4_and_batched_views():
    """The driver's 8-GPU command: rank 0's line carries the batched-views
    record beside the C4 sub-record (view k on GPU k, one view
    per GPU), and every rank's view assignment."""
    r = _run("--gpus", "8", "--dry-run", "--steps", "1", timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 8 and len(d["ranks"]) == 8
    assert d["views_batched"]["views_per_gpu"] == 20
    assert all(x["views"] == [x["rank"] + 8 * j for j in range(20)] for x in d["ranks"])
    c4 = d["c4_one_view_per_gpu"]
    assert c4["views"] == list(range(8))
    assert [x["c4_view"] for x in d["ranks"]] == list(range(8))
    # eight distinct cameras: the default one yawed by k * 45 deg
    assert len({tuple(x["c4_view_row2"]) for x in d["ranks"]}) == 8
