"""Scene container with the reference's field layout (``util_gau.GaussianData``,
``util_gau.py:10-147``) plus the scene generators used by tests and bench.

Arrays are float32 NumPy: xyz [N,3]; rot [N,4] (w,x,y,z, unit); scale [N,3]
(already exp-activated); opacity [N,1] (already sigmoid-activated); sh [N,3K]
coefficient-major, RGB-interleaved.  ``flat()`` is the per-Gaussian AoS record
the OGL path uploads as SSBO 0 (``util_gau.py:40-42``).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass
class GaussianData:
    xyz: np.ndarray
    rot: np.ndarray
    scale: np.ndarray
    opacity: np.ndarray
    sh: np.ndarray
    path: str | None = None
    # positions as constructed (the reference keeps a copy of its original
    # state, util_gau.py:18-36, and export_ply crops by it, :410-413)
    original_xyz: np.ndarray | None = None

    def __post_init__(self):
        if self.original_xyz is None:
            self.original_xyz = np.copy(self.xyz)

    def __len__(self):
        return len(self.xyz)

    def __getitem__(self, idx):
        # a fresh instance whose original state is the current subset (util_gau.py:31-38)
        return GaussianData(self.xyz[idx], self.rot[idx], self.scale[idx], self.opacity[idx], self.sh[idx])

    def flat(self) -> np.ndarray:
        """util_gau.py:40-42"""
        return np.ascontiguousarray(np.concatenate([self.xyz, self.rot, self.scale, self.opacity, self.sh], axis=-1))

    def scale_data(self, scale_to_interval: float):
        """util_gau.py:44-53: recentre on the bbox centre, max extent -> value,
        scales multiplied by the same factor, rotations renormalised.  The
        reference's pandas columns keep the input dtype, and under NumPy 2
        promotion the Python-float interval stays weak, so a float32 scene is
        rescaled in float32."""
        xyz = np.asarray(self.xyz)
        mn, mx = xyz.min(axis=0), xyz.max(axis=0)
        center = (mn + mx) / 2
        max_extent = (mx - mn).max()
        factor = scale_to_interval / max_extent
        self.xyz = (xyz - center) * factor
        self.rot = self.rot / np.linalg.norm(self.rot, axis=-1, keepdims=True)
        self.scale = self.scale * factor

    @property
    def sh_dim(self) -> int:
        return self.sh.shape[-1]

    @property
    def points_center(self):
        return np.mean(self.xyz, axis=0)

    @property
    def points_min(self):
        return np.min(self.xyz, axis=0)

    @property
    def points_max(self):
        return np.max(self.xyz, axis=0)

    @property
    def compute_aabb(self):
        """util_gau.py:96-111"""
        xmin, ymin, zmin = self.points_min
        xmax, ymax, zmax = self.points_max
        corners = np.array([[xmin, ymin, zmin], [xmax, ymin, zmin], [xmin, ymax, zmin], [xmax, ymax, zmin],
                            [xmin, ymin, zmax], [xmax, ymin, zmax], [xmin, ymax, zmax], [xmax, ymax, zmax]])
        return self.points_min, self.points_max, corners

    @property
    def compute_obb(self):
        """util_gau.py:114-138: the oriented box of the positions by PCA.
        Returns (obb_min, obb_max, U, corners): the box's extreme corners in
        world coordinates, the principal axes (columns of U from the SVD of the
        covariance) and the 8 corners in the reference's order.  Same float
        path as the reference: the float32 column means, float32 centring,
        np.cov in float64 (what DataFrame.cov runs on NaN-free data), the SVD,
        projections in float64.  Bit-exact against reference-run fixtures."""
        xyz = np.asarray(self.xyz)
        center = xyz.mean(axis=0)
        centered = xyz - center
        cov = np.cov(np.asarray(centered, np.float64).T)
        U, _, _ = np.linalg.svd(cov)
        proj = centered @ U
        obb_min = center + proj.min(axis=0) @ U.T
        obb_max = center + proj.max(axis=0) @ U.T
        lo, hi = obb_min, obb_max
        corners = np.array([[lo[0], lo[1], lo[2]], [hi[0], lo[1], lo[2]], [lo[0], hi[1], lo[2]],
                            [hi[0], hi[1], lo[2]], [lo[0], lo[1], hi[2]], [hi[0], lo[1], hi[2]],
                            [lo[0], hi[1], hi[2]], [hi[0], hi[1], hi[2]]])
        return obb_min, obb_max, U, corners

    def astype32(self) -> "GaussianData":
        return GaussianData(*(np.ascontiguousarray(np.asarray(a, np.float32))
                              for a in (self.xyz, self.rot, self.scale, self.opacity, self.sh)), path=self.path,
                            original_xyz=self.original_xyz)


def naive_gaussian() -> GaussianData:
    """The reference's built-in 4-Gaussian scene (util_gau.py:149-184)."""
    xyz = np.array([0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0, 1], np.float32).reshape(-1, 3)
    rot = np.array([1, 0, 0, 0] * 4, np.float32).reshape(-1, 4)
    s = np.array([.03, .03, .03, .2, .03, .03, .03, .2, .03, .03, .03, .2], np.float32).reshape(-1, 3)
    c = np.array([1, 0, 1, 1, 0, 0, 0, 1, 0, 0, 0, 1], np.float32).reshape(-1, 3)
    c = (c - 0.5) / 0.28209
    a = np.ones((4, 1), np.float32)
    return GaussianData(xyz, rot, s, a, c)


def _sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def random_scene(n: int, sh_degree: int = 0, seed: int = 0, extent: float = 2.0,
                 scale_range=(0.005, 0.05)) -> GaussianData:
    """BASELINE config 1 generator: xyz ~ U(-e,e)^3,
    rot = normalize(N(0,1)^4), scale = exp(U(ln a, ln b)), opacity =
    sigmoid(N(0,1.5)), sh ~ N(0,0.6)."""
    rng = np.random.default_rng(seed)
    k = (sh_degree + 1) ** 2
    xyz = rng.uniform(-extent, extent, (n, 3)).astype(np.float32)
    rot = rng.normal(0, 1, (n, 4)).astype(np.float32)
    rot /= np.linalg.norm(rot, axis=-1, keepdims=True)
    scale = np.exp(rng.uniform(np.log(scale_range[0]), np.log(scale_range[1]), (n, 3))).astype(np.float32)
    opacity = _sigmoid(rng.normal(0, 1.5, (n, 1))).astype(np.float32)
    sh = rng.normal(0, 0.6, (n, 3 * k)).astype(np.float32)
    return GaussianData(xyz, rot, scale, opacity, sh)


def garden_standin(n: int, seed: int = 1, sh_degree: int = 3, log_scale=(-4.6, 0.6)) -> GaussianData:
    """Seeded synthetic stand-in for the Mip-NeRF360 'garden' scene (SURVEY.md
    8d C2/C3): 70 % ground disc + 30 % blob, scale_data(5.0) applied as on PLY
    load (gs_elements_control.py:41-42), scale = exp(N(-4.6,0.6)) before the
    rescale (`log_scale` = (mean, std); the heavy-splat stress scene of
    bench.py --config c2h uses (-3.5, 0.8)), opacity = sigmoid(N(0,2)),
    sh0 ~ N(0,0.6), rest ~ N(0,0.1)."""
    rng = np.random.default_rng(seed)
    k = (sh_degree + 1) ** 2
    n_disc = int(round(0.7 * n))
    n_blob = n - n_disc
    r = 4.0 * np.sqrt(rng.uniform(0, 1, n_disc))
    th = rng.uniform(0, 2 * np.pi, n_disc)
    disc = np.stack([r * np.cos(th), rng.normal(-1.0, 0.05, n_disc), r * np.sin(th)], 1)
    blob = rng.normal(0, 1, (n_blob, 3)) * np.array([0.8, 0.6, 0.8]) + np.array([0.0, -0.2, 0.0])
    xyz = np.concatenate([disc, blob]).astype(np.float32)
    perm = rng.permutation(n)
    xyz = xyz[perm]
    rot = rng.normal(0, 1, (n, 4)).astype(np.float32)
    scale = np.exp(rng.normal(log_scale[0], log_scale[1], (n, 3))).astype(np.float32)
    opacity = _sigmoid(rng.normal(0, 2, (n, 1))).astype(np.float32)
    sh = np.empty((n, 3 * k), np.float32)
    sh[:, :3] = rng.normal(0, 0.6, (n, 3))
    if k > 1:
        sh[:, 3:] = rng.normal(0, 0.1, (n, 3 * k - 3))
    g = GaussianData(xyz, rot, scale, opacity, sh)
    g.scale_data(5.0)
    return g.astype32()
