"""gsviewer_amd -- MI355X-native forward rasterizer for 3D Gaussian splats.

Drop-in for the per-frame rasterization path of Lucasmogsan/GSViewer
(``render/renderer_cuda.py`` render() boundary, OpenGL-path semantics).
The compute path is ``libgsr.so`` (hand-written HIP for gfx950, C ABI in
``include/gsr.h``); Python only marshals device pointers and camera state.
"""
from .gaussian_data import GaussianData, naive_gaussian, random_scene, garden_standin  # noqa: F401
from .camera import Camera  # noqa: F401

__all__ = ["GaussianData", "naive_gaussian", "random_scene", "garden_standin", "Camera"]


def __getattr__(name):
    # GPU-facing modules import torch and the HIP library lazily.
    if name in ("HipScene", "HipContext", "RenderSettings", "render", "render_into", "GaussianRasterizer",
                "GaussianRasterizationSettings", "depth_order", "camera_from", "camera_struct"):
        from . import rasterizer
        return getattr(rasterizer, name)
    if name in ("HIPRenderer", "GaussianRenderBase"):
        from . import renderer
        return getattr(renderer, name)
    raise AttributeError(name)
