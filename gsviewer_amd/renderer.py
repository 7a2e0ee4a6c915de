"""Renderer-plugin surface of the reference (``render/renderer_ogl.py:79-130``
``GaussianRenderBase``) with an MI355X backend, ``HIPRenderer``.

``HIPRenderer`` keeps the OpenGLRenderer setter names and argument meaning
(``renderer_ogl.py:235-318``) so the viewer's control code
(``main.py:128-137``, ``gui/*.py``) could drive it unchanged, and its ``draw()``
returns the frame as a CUDA tensor [H,W,3] instead of presenting it (MI355X has
no display; the CUDA->GL interop of ``renderer_cuda.py:250-277`` is out of
scope).  Differences from the OGL backend, by design:
  * every draw sorts for the camera it renders (the OGL backend draws with the
    last ``sort_and_update`` order unless "Auto Sort" is on,
    gs_elements_control.py:181-185), so ``sort_and_update`` is a no-op;
  * overlays (axes, boundary-box mesh) are UI decoration and not drawn.
"""
from __future__ import annotations

import numpy as np
import torch

from .camera import euler_to_quaternion, euler_to_rotation_matrix
from .gaussian_data import GaussianData
from .rasterizer import HipContext, HipScene, RenderSettings, camera_from, depth_order, render_into


class GaussianRenderBase:
    """renderer_ogl.py:79-130"""

    def __init__(self):
        self.gaussians = None
        self._reduce_updates = True

    @property
    def reduce_updates(self):
        return self._reduce_updates

    @reduce_updates.setter
    def reduce_updates(self, val):
        self._reduce_updates = val

    def update_gaussian_data(self, gaus: GaussianData):
        raise NotImplementedError()

    def sort_and_update(self):
        raise NotImplementedError()

    def set_scale_modifier(self, modifier: float):
        raise NotImplementedError()

    def set_render_mod(self, mod: int):
        raise NotImplementedError()

    def update_camera_pose(self):
        raise NotImplementedError()

    def update_camera_intrin(self):
        raise NotImplementedError()

    def set_enable_cube(self, enable_cube: int):
        raise NotImplementedError()

    def set_cube_rotation(self, cube_rotation: list):
        raise NotImplementedError()

    def set_point_cubeMin(self, point_cubeMin: list):
        raise NotImplementedError()

    def set_point_cubeMax(self, point_cubeMax: list):
        raise NotImplementedError()

    def draw(self):
        raise NotImplementedError()

    def set_render_reso(self, w, h):
        raise NotImplementedError()


class HIPRenderer(GaussianRenderBase):
    """MI355X backend with the OpenGLRenderer API (renderer_ogl.py:133-318)."""

    def __init__(self, w, h, camera):
        super().__init__()
        self.camera = camera
        self.w, self.h = int(w), int(h)
        self.settings = RenderSettings(out_layout=1)
        self._ctx = HipContext()
        self._scene = None
        self._cam = None
        self.need_rerender = True
        self.last_image = None

    # -- data -------------------------------------------------------------
    def update_gaussian_data(self, gaus: GaussianData):
        """renderer_ogl.py:235-242 / renderer_cuda.py:147-150"""
        self.gaussians = gaus
        g = gaus.astype32()
        self._scene = HipScene.from_gaussian_data(g)
        self.need_rerender = True

    def sort_and_update(self):
        """renderer_ogl.py:263-268: every draw sorts for its own camera."""
        self.need_rerender = True

    def depth_order(self):
        """The index buffer the OGL path uploads as SSBO 1 (renderer_ogl.py:264)."""
        return depth_order(self._scene, self.camera.get_view_matrix())

    # -- appearance (renderer_ogl.py:246-277) --------------------------------
    def adjust_dc_features(self, dc_factor):
        self.settings.dc_factor = float(dc_factor); self.need_rerender = True

    def adjust_extra_features(self, extra_factor):
        self.settings.extra_factor = float(extra_factor); self.need_rerender = True

    def update_color_factor(self, g_rgb_factor):
        self.settings.color_scale = [float(v) for v in g_rgb_factor]; self.need_rerender = True

    def set_rot_modifier(self, modifier):
        self.settings.rot_modifier = list(euler_to_quaternion(modifier[0], modifier[1], modifier[2]))
        self.need_rerender = True

    def set_light_rotation(self, light_rotation):
        self.settings.light_rotation = [float(v) for v in light_rotation]; self.need_rerender = True

    def set_scale_modifier(self, modifier):
        self.settings.scale_modifier = float(modifier); self.need_rerender = True

    def set_screen_scale_factor(self, factor):
        self.settings.screen_scale = float(factor); self.need_rerender = True

    def set_render_mod(self, mod: int):
        self.settings.render_mod = int(mod); self.need_rerender = True

    def set_render_reso(self, w, h):
        self.w, self.h = int(w), int(h)
        self.camera.update_resolution(self.h, self.w)
        self.need_rerender = True

    # -- camera (renderer_ogl.py:282-292) ------------------------------------
    def update_camera_pose(self, camera=None):
        if camera is not None:
            self.camera = camera
        self.need_rerender = True

    def update_camera_intrin(self, camera=None):
        if camera is not None:
            self.camera = camera
        self.need_rerender = True

    # -- boundary box (renderer_ogl.py:296-318) ------------------------------
    def set_points_center(self, points_center):
        self.settings.points_center = [float(v) for v in points_center]; self.need_rerender = True

    def set_enable_aabb(self, enable_aabb: int):
        self.settings.enable_aabb = int(enable_aabb); self.need_rerender = True

    def set_enable_obb(self, enable_obb: int):
        self.settings.enable_obb = int(enable_obb); self.need_rerender = True

    def set_enable_cube(self, enable_cube: int):
        self.set_enable_aabb(enable_cube)

    def set_cube_rotation(self, cube_rotation):
        self.settings.cube_rotation = euler_to_rotation_matrix(cube_rotation); self.need_rerender = True

    def set_point_cubeMin(self, point_cubeMin):
        self.settings.cube_min = [float(v) for v in point_cubeMin]; self.need_rerender = True

    def set_point_cubeMax(self, point_cubeMax):
        self.settings.cube_max = [float(v) for v in point_cubeMax]; self.need_rerender = True

    # -- frame ---------------------------------------------------------------
    def draw(self) -> torch.Tensor:
        """Render the current camera; returns [H, W, 3] float32 (row 0 = top).
        With reduce_updates, an unchanged state returns the previous frame
        (renderer_cuda.py:216-221)."""
        if self._scene is None:
            raise RuntimeError("update_gaussian_data() first")
        if self.reduce_updates and not self.need_rerender and self.last_image is not None \
                and not self.camera.is_pose_dirty and not self.camera.is_intrin_dirty:
            return self.last_image
        self.camera.h, self.camera.w = self.h, self.w
        cam = camera_from(self.camera)
        self.camera.is_pose_dirty = self.camera.is_intrin_dirty = False
        out = torch.empty((self.h, self.w, 3), dtype=torch.float32, device="cuda")
        render_into(self._ctx, self._scene, cam, self.settings, out)
        self.need_rerender = False
        self.last_image = out
        return out

    def frame_stats(self):
        return self._ctx.stats()
