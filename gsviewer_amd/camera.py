"""Camera math restated from the reference's ``util.Camera`` (``util.py:8-218``),
which needs PyGLM (absent here).  Only the frame-defining parts are restated:
view matrix (``get_view_matrix`` :61-76, glm.lookAt right-handed), projection
(``get_project_matrix`` :78-93, glm.perspective RH with z_ndc in [-1,1], or
glm.ortho), ``get_htanfovxy_focal`` (:181-185) and the free-rotation
quaternion (glm.quat / angleAxis / mat4_cast).  Interaction handlers
(:99-213) are UI and out of scope, except ``yaw``/``orbit`` helpers that apply
the same quaternion update as the mouse handler (:112-115).

Matrices are returned as row-major float32 NumPy "math" matrices, i.e. what the
reference's ``np.array(glm.mat4)`` yields and what GLSL sees after
``util.set_uniform_mat4`` (``util.py:364-375``).
"""
from __future__ import annotations

import math

import numpy as np

F = np.float32


def quat_mul(a, b):
    """Hamilton product of (w,x,y,z) quaternions (glm::quat operator*)."""
    aw, ax, ay, az = a
    bw, bx, by, bz = b
    return np.array([aw * bw - ax * bx - ay * by - az * bz,
                     aw * bx + ax * bw + ay * bz - az * by,
                     aw * by + ay * bw + az * bx - ax * bz,
                     aw * bz + az * bw + ax * by - ay * bx], np.float64)


def angle_axis(angle_rad, axis):
    """glm.angleAxis"""
    axis = np.asarray(axis, np.float64)
    s = math.sin(angle_rad * 0.5)
    return np.array([math.cos(angle_rad * 0.5), axis[0] * s, axis[1] * s, axis[2] * s])


def quat_normalize(q):
    q = np.asarray(q, np.float64)
    return q / np.sqrt(np.dot(q, q))


def mat3_cast(q):
    """glm.mat3_cast of a (w,x,y,z) quaternion as a row-major math matrix."""
    w, x, y, z = [float(v) for v in q]
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]], np.float32)


def _normalize(v):
    v = np.asarray(v, F)
    return (v * (F(1.0) / np.sqrt(np.dot(v, v)))).astype(F)


def look_at(eye, center, up):
    """glm.lookAt (right-handed) as a row-major math matrix."""
    eye, center, up = (np.asarray(a, F) for a in (eye, center, up))
    f = _normalize(center - eye)
    s = _normalize(np.cross(f, up).astype(F))
    u = np.cross(s, f).astype(F)
    M = np.eye(4, dtype=F)
    M[0, :3], M[1, :3], M[2, :3] = s, u, -f
    M[0, 3] = -np.dot(s, eye)
    M[1, 3] = -np.dot(u, eye)
    M[2, 3] = np.dot(f, eye)
    return M


def perspective(fovy, aspect, znear, zfar):
    """glm.perspective (RH, NO: z_ndc in [-1,1]) as a row-major math matrix."""
    fovy, aspect, znear, zfar = F(fovy), F(aspect), F(znear), F(zfar)
    t = F(np.tan(fovy / F(2)))
    M = np.zeros((4, 4), F)
    M[0, 0] = F(1) / (aspect * t)
    M[1, 1] = F(1) / t
    M[2, 2] = -(zfar + znear) / (zfar - znear)
    M[3, 2] = F(-1)
    M[2, 3] = -(F(2) * zfar * znear) / (zfar - znear)
    return M


def ortho(l, r, b, t, n, f):
    """glm.ortho (RH, NO) as a row-major math matrix."""
    l, r, b, t, n, f = (F(v) for v in (l, r, b, t, n, f))
    M = np.eye(4, dtype=F)
    M[0, 0] = F(2) / (r - l)
    M[1, 1] = F(2) / (t - b)
    M[2, 2] = -F(2) / (f - n)
    M[0, 3] = -(r + l) / (r - l)
    M[1, 3] = -(t + b) / (t - b)
    M[2, 3] = -(f + n) / (f - n)
    return M


class Camera:
    """Frame-defining state of ``util.Camera`` with the reference defaults
    (util.py:9-46): h, w, fovy = pi/2, znear 0.001, zfar 500, target 0,
    target_dist 5, free rotation with identity quaternion."""

    def __init__(self, h: int, w: int):
        self.znear = 0.001
        self.zfar = 500
        self.h = h
        self.w = w
        self.fovy = np.pi / 2
        self.position = np.array([0.0, 0.0, 5.0], dtype=F)
        self.target = np.array([0.0, 0.0, 0.0], dtype=F)
        self.up = np.array([0.0, -1.0, 0.0], dtype=F)
        self.target_dist = 5.0
        self.rotation = np.array([1.0, 0.0, 0.0, 0.0])  # glm.quat(1,0,0,0): (w,x,y,z)
        self.use_free_rotation = True
        self.rotation_center = np.array([0.0, 0.0, 0.0], dtype=F)
        self.use_custom_rotation_center = False
        self.use_orthographic = False
        self.ortho_scale = 5.0
        self.is_pose_dirty = True
        self.is_intrin_dirty = True

    def get_view_matrix(self):
        """util.py:61-76"""
        if self.use_free_rotation:
            R = mat3_cast(self.rotation)
            direction = (R @ np.array([0, 0, -1], F)).astype(F)
            up_direction = (R @ np.array([0, 1, 0], F)).astype(F)
            center = self.rotation_center if self.use_custom_rotation_center else self.target
            self.position = (np.asarray(center, F) - direction * F(self.target_dist)).astype(F)
            return look_at(self.position, self.target, up_direction)
        return look_at(self.position, self.target, self.up)

    def get_project_matrix(self):
        """util.py:78-93"""
        if self.use_orthographic:
            ar = self.w / self.h
            return ortho(-self.ortho_scale * ar, self.ortho_scale * ar, -self.ortho_scale, self.ortho_scale,
                         self.znear, self.zfar)
        return perspective(self.fovy, self.w / self.h, self.znear, self.zfar)

    def get_htanfovxy_focal(self):
        """util.py:181-185"""
        htany = np.tan(self.fovy / 2)
        htanx = htany / self.h * self.w
        focal = self.h / (2 * htany)
        return [htanx, htany, focal]

    def yaw(self, degrees: float):
        """Rotate the free-rotation quaternion about world +y, the left-drag
        update of util.py:112-115 (yaw_quat * rotation)."""
        q = angle_axis(math.radians(degrees), (0, 1, 0))
        self.rotation = quat_normalize(quat_mul(q, self.rotation))
        self.is_pose_dirty = True
        return self

    def update_resolution(self, height, width):
        self.h = max(height, 1)
        self.w = max(width, 1)
        self.is_intrin_dirty = True


def view_for_rank(h: int, w: int, k: int) -> Camera:
    """view k = default camera yawed by k*45 degrees."""
    return Camera(h, w).yaw(45.0 * k)


def euler_to_rotation_matrix(angles_deg):
    """util.convert_euler_angles_to_rotation_matrix (util.py:453-479):
    R = Rz @ Ry @ Rx, angles in degrees."""
    ax, ay, az = np.radians(angles_deg)
    sx, sy, sz = np.sin([ax, ay, az])
    cx, cy, cz = np.cos([ax, ay, az])
    Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    return np.dot(Rz, np.dot(Ry, Rx))


def euler_to_quaternion(roll, pitch, yaw):
    """util.euler_to_quaternion (util.py:481-492) returning the (x,y,z,w)
    order in which renderer_ogl.set_rot_modifier uploads it (renderer_ogl.py:257)."""
    r, p, y = math.radians(roll), math.radians(pitch), math.radians(yaw)
    qx = math.sin(r / 2) * math.cos(p / 2) * math.cos(y / 2) - math.cos(r / 2) * math.sin(p / 2) * math.sin(y / 2)
    qy = math.cos(r / 2) * math.sin(p / 2) * math.cos(y / 2) + math.sin(r / 2) * math.cos(p / 2) * math.sin(y / 2)
    qz = math.cos(r / 2) * math.cos(p / 2) * math.sin(y / 2) - math.sin(r / 2) * math.sin(p / 2) * math.cos(y / 2)
    qw = math.cos(r / 2) * math.cos(p / 2) * math.cos(y / 2) + math.sin(r / 2) * math.sin(p / 2) * math.sin(y / 2)
    return np.array([qx, qy, qz, qw], np.float32)


def _quat_from_matrix(m):
    """Unit quaternion (x, y, z, w) of a rotation matrix by the largest-pivot
    method (Markley: the diagonal entry or the trace that is largest picks
    the component computed from it), as scipy's Rotation.from_matrix does
    (scipy 1.15, the reference's util.py:498 dependency)."""
    m = np.asarray(m, np.float64)
    dec = (m[0, 0], m[1, 1], m[2, 2], m[0, 0] + m[1, 1] + m[2, 2])
    ch = int(np.argmax(dec))
    q = [0.0, 0.0, 0.0, 0.0]
    if ch != 3:
        i = ch
        j = (i + 1) % 3
        k = (j + 1) % 3
        q[i] = 1 - dec[3] + 2 * m[i, i]
        q[j] = m[j, i] + m[i, j]
        q[k] = m[k, i] + m[i, k]
        q[3] = m[k, j] - m[j, k]
    else:
        q = [m[2, 1] - m[1, 2], m[0, 2] - m[2, 0], m[1, 0] - m[0, 1], 1 + dec[3]]
    nrm = math.sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3])
    return [c / nrm for c in q]


def rotation_matrix_to_euler(R):
    """util.convert_rotation_matrix_to_euler_angles (util.py:494-501): the
    extrinsic 'xyz' Euler angles of R in degrees, the inverse of
    euler_to_rotation_matrix (R = Rz Ry Rx).  scipy's as_euler algorithm
    restated: the quaternion-based direct method of Bernardes & Viollet (2022)
    (angles from two half-angle atan2s; the middle angle within 1e-7 of 0 or
    pi is the gimbal-lock case, whose third angle is set to 0).  Bit-exact
    against the reference-run fixtures (tests/golden)."""
    q = _quat_from_matrix(R)
    i, j, k = 0, 1, 2  # extrinsic x, y, z: Tait-Bryan, even permutation
    sign = (i - j) * (j - k) * (k - i) // 2
    a = q[3] - q[j]
    b = q[i] + q[k] * sign
    c = q[j] + q[3]
    d = q[k] * sign - q[i]
    ang = [0.0, 2 * math.atan2(math.hypot(c, d), math.hypot(a, b)), 0.0]
    eps = 1e-7
    case = 1 if abs(ang[1]) <= eps else (2 if abs(ang[1] - math.pi) <= eps else 0)
    half_sum = math.atan2(b, a)
    half_diff = math.atan2(d, c)
    if case == 0:
        ang[0] = half_sum - half_diff
        ang[2] = half_sum + half_diff
    else:  # gimbal lock: the third angle is not determined
        ang[0] = 2 * half_sum if case == 1 else -2 * half_diff
    ang[2] *= sign
    ang[1] -= math.pi / 2
    for t in range(3):
        if ang[t] < -math.pi:
            ang[t] += 2 * math.pi
        elif ang[t] > math.pi:
            ang[t] -= 2 * math.pi
    return np.degrees(np.array(ang))
