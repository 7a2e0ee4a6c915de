"""The C-ABI library loads, exports every symbol include/*.h declares, and the
ctypes struct layouts match the C headers (no GPU calls)."""
import ctypes
import os
import re
import subprocess

import pytest

from gsviewer_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in sorted(os.listdir(os.path.join(ROOT, "include")))
           if h.endswith(".h")]


def header_functions():
    names = set()
    for h in HEADERS:
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names |= set(re.findall(r"\b(gsr_[a-z0-9_]+)\s*\(", src))
    return sorted(names)


def test_header_declares_expected_entry_points():
    names = header_functions()
    for must in ("gsr_scene_create", "gsr_scene_create_flat", "gsr_scene_destroy", "gsr_context_create",
                 "gsr_render", "gsr_render_begin", "gsr_render_finish", "gsr_sort_depth", "gsr_debug_sort_pairs", "gsr_debug_host_times", "gsr_last_error", "gsr_settings_default",
                 "gsr_ply_probe", "gsr_ply_read", "gsr_ply_write_3dgs", "gsr_points_center", "gsr_export_select"):
        assert must in names


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    missing = [n for n in header_functions() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(header_functions()) == set(_lib.SIGNATURES), "ctypes signatures out of sync with include/*.h"


def test_abi_version_and_defaults():
    lib = _lib.load()
    assert lib.gsr_abi_version() == _lib.ABI_VERSION
    s = _lib.default_settings()
    assert s.render_mod == 6 and s.scale_modifier == 1.0 and list(s.rot_modifier) == [0, 0, 0, 1]
    assert list(s.cube_rotation) == [1, 0, 0, 0, 1, 0, 0, 0, 1]


def test_invalid_arguments_fail_loudly():
    lib = _lib.load()
    out = ctypes.c_void_p()
    rc = lib.gsr_scene_create(None, None, None, None, None, 10, 48, None, ctypes.byref(out))
    assert rc != 0 and b"null" in lib.gsr_last_error()
    rc = lib.gsr_scene_create_flat(None, 10, 7, None, ctypes.byref(out))
    assert rc != 0 and b"sh_dim" in lib.gsr_last_error()
    with pytest.raises(RuntimeError):
        _lib.check(rc, "gsr_scene_create_flat")


def test_struct_layout_matches_header(tmp_path):
    prog = tmp_path / "sz.c"
    prog.write_text(r'''
#include <stdio.h>
#include <stddef.h>
#include "gsr_io.h"
int main(void){
 printf("%zu %zu %zu\n", sizeof(gsr_camera), sizeof(gsr_settings), sizeof(gsr_frame_stats));
 printf("%zu %zu %zu %zu\n", sizeof(gsr_ply_info), offsetof(gsr_ply_info, body_offset), sizeof(gsr_box),
        offsetof(gsr_box, rot_inv));
 printf("%zu %zu %zu %zu\n", offsetof(gsr_settings, cube_rotation), offsetof(gsr_settings, bg),
        offsetof(gsr_settings, t_min), offsetof(gsr_settings, out_layout));
 printf("%zu %zu\n", offsetof(gsr_camera, hfovxy_focal), offsetof(gsr_camera, height));
 return 0;}
''')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(prog), "-o", str(exe)], check=True)
    got = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    S, C, FS = _lib.GsrSettings, _lib.GsrCamera, _lib.GsrFrameStats
    PI, B = _lib.GsrPlyInfo, _lib.GsrBox
    want = [ctypes.sizeof(C), ctypes.sizeof(S), ctypes.sizeof(FS),
            ctypes.sizeof(PI), PI.body_offset.offset, ctypes.sizeof(B), B.rot_inv.offset,
            S.cube_rotation.offset, S.bg.offset,
            S.t_min.offset, S.out_layout.offset, C.hfovxy_focal.offset, C.height.offset]
    assert [int(x) for x in got] == want


def test_workspace_size_needs_no_gpu():
    """gsr_workspace_size sizes a caller-provided workspace on the host alone:
    it grows with every bound and rejects bad arguments."""
    from gsviewer_amd.rasterizer import workspace_size
    base = workspace_size(100_000, 640, 480, 0)
    assert base > 100_000 * 48
    assert workspace_size(200_000, 640, 480, 0) > base
    assert workspace_size(100_000, 1920, 1080, 0) > base
    assert workspace_size(100_000, 640, 480, 1_000_000) > base
    assert workspace_size(100_000, 640, 480, 0) == base
    with pytest.raises(RuntimeError, match="context_reserve"):
        workspace_size(-1, 640, 480, 0)
    with pytest.raises(RuntimeError, match="context_reserve"):
        workspace_size(10, 0, 480, 0)


def test_context_knobs_read_at_creation(monkeypatch):
    """gsr_context_knob reports the stage forms a context read from the
    environment at creation (host only: creating a context makes no HIP call)."""
    from gsviewer_amd.rasterizer import HipContext
    a = HipContext()
    assert a.knob("rect_payload") == 1 and a.knob("chunk") == 192 and a.knob("frame_chunk") == 0
    monkeypatch.setenv("GSR_NO_RECT_PAYLOAD", "1")
    monkeypatch.setenv("GSR_CHUNK", "256")
    b = HipContext()
    assert b.knob("rect_payload") == 0 and b.knob("chunk") == 256
    assert a.knob("rect_payload") == 1  # read once, at creation
    with pytest.raises(RuntimeError, match="unknown knob"):
        a.knob("no_such_knob")
    a.close()
    b.close()


def test_stale_library_refused(monkeypatch):
    """The in-tree library carries the digest of its sources; a library built
    from other sources is refused (tools/gpu_round.sh loads, never builds)."""
    from gsviewer_amd import _srcid
    lib = _lib.load()
    assert lib.gsr_source_digest().decode() == _srcid.source_digest()

    class Stale:
        @staticmethod
        def gsr_source_digest():
            return b"0000000000000000"
    with pytest.raises(RuntimeError, match="built from other sources"):
        _lib.check_fresh(Stale())
