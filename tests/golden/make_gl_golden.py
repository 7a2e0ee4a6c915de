"""Golden framebuffers from the reference's own shaders on a real GL driver.

Run in the build container (needs /root/reference and Mesa's swrast_dri.so):

    python tests/golden/make_gl_golden.py

For every case of ``tests/gl_cases.py`` this

1. builds the scene and the camera, and orders the Gaussians with the
   reference's own ``renderer_ogl._sort_gaussian_cpu`` (imported as in
   ``make_golden.py``);
2. runs ``oracle/_ref/llvmpipe_gl`` (built here from
   ``oracle/gl_ref/llvmpipe_gl.c``), which compiles
   ``/root/reference/shaders/gau_vert.glsl`` and ``gau_frag.glsl`` as the
   reference's ``util.load_shaders`` does, sets the uniforms through the same
   calls, and draws the instanced quads into an RGBA8 framebuffer and into an
   RGBA32F one with fragment-colour clamping;
3. stores only data: the case name, the scene's SHA-256, the draw order, and
   the two framebuffers (RGB, rows flipped to top-down as ``Save Image`` does,
   gs_elements_control.py:192-196) in ``tests/golden/llvmpipe_golden.npz``.

The shader text is read at generation time and never written anywhere.
"""
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), HERE]

import gl_cases as GC  # noqa: E402
from make_golden import import_reference  # noqa: E402

REF = "/root/reference"
OUT = os.path.join(HERE, "llvmpipe_golden.npz")
SRC = os.path.join(ROOT, "oracle", "gl_ref", "llvmpipe_gl.c")
EXE = os.path.join(ROOT, "oracle", "_ref", "llvmpipe_gl")
F = np.float32


def build_harness():
    os.makedirs(os.path.dirname(EXE), exist_ok=True)
    if not os.path.exists(EXE) or os.path.getmtime(EXE) < os.path.getmtime(SRC):
        subprocess.run(["gcc", "-O2", "-std=gnu11", "-Wall", "-o", EXE, SRC, "-ldl"], check=True)
    return EXE


def frame_header(U, n, sh_dim):
    ints = np.array([U["width"], U["height"], n, sh_dim, U["render_mod"], U["enable_aabb"], U["enable_obb"], 0],
                    np.int32)
    floats = np.concatenate([
        np.asarray(U["view"], F).reshape(16), np.asarray(U["proj"], F).reshape(16),
        np.asarray(U["hfovxy_focal"], F), np.asarray(U["cam_pos"], F),
        np.array([U["gaussian_scale_factor"], U["screen_display_scale_factor"], U["dc_factor"],
                  U["extra_factor"]], F),
        np.asarray(U["color_scale_factors"], F), np.asarray(U["rot_modifier"], F),
        np.asarray(U["light_rotation"], F), np.asarray(U["points_center"], F),
        np.asarray(U["cube_rotation"], F).reshape(9), np.asarray(U["cubeMin"], F), np.asarray(U["cubeMax"], F),
    ]).astype(F)
    assert floats.size == 70
    return ints.tobytes() + floats.tobytes()


def run_gl(exe, U, flat, order, bits):
    n, rec = flat.shape
    with tempfile.TemporaryDirectory() as td:
        fin, fout = os.path.join(td, "in.bin"), os.path.join(td, "out.bin")
        with open(fin, "wb") as f:
            f.write(frame_header(U, n, rec - 11))
            f.write(np.ascontiguousarray(flat, F).tobytes())
            f.write(np.ascontiguousarray(order, np.int32).tobytes())
        env = dict(os.environ, LP_NUM_THREADS=os.environ.get("LP_NUM_THREADS", "4"))
        r = subprocess.run([exe, os.path.join(REF, "shaders", "gau_vert.glsl"),
                            os.path.join(REF, "shaders", "gau_frag.glsl"), fin, fout, str(bits)],
                           capture_output=True, text=True, env=env)
        if r.returncode != 0:
            raise RuntimeError(f"llvmpipe_gl failed ({r.returncode}): {r.stderr}")
        H, W = U["height"], U["width"]
        raw = np.fromfile(fout, np.uint8 if bits == 8 else F).reshape(H, W, 4)
        return raw[::-1, :, :3].copy(), r.stderr.strip()


def main():
    exe = build_harness()
    _, _, renderer_ogl = import_reference()
    out = {"cases": np.array(list(GC.CASES))}
    renderer = None
    for name in GC.CASES:
        g = GC.scene(GC.CASES[name][0])
        cam, U = GC.uniforms(name, g)
        # the reference's own sort (renderer_ogl.py:16-26) on the view matrix the shader gets
        order = renderer_ogl._sort_gaussian_cpu(g, cam.get_view_matrix())[:, 0].astype(np.int32)
        flat = g.flat()
        img8, info = run_gl(exe, U, flat, order, 8)
        imgf, _ = run_gl(exe, U, flat, order, 32)
        renderer = renderer or info
        out[f"{name}/sha"] = np.array(GC.flat_sha(g))
        out[f"{name}/order"] = order
        out[f"{name}/rgba8"] = img8
        out[f"{name}/float"] = imgf.astype(F)
        print(f"{name}: {U['width']}x{U['height']} n={len(order)} covered={int((img8 > 0).any(-1).sum())}")
    out["renderer"] = np.array(renderer)
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, os.path.getsize(OUT), "bytes;", renderer)


if __name__ == "__main__":
    main()
