"""Camera matrices, restated from the reference.

getWorld2View2 / getProjectionMatrix follow utils/graphics_utils.py:38-71 and the Camera /
MiniCam conventions follow scene/cameras.py:17-66: the rasterizer receives the *transposed*
(column-major flat) world-to-view matrix and full projection `world_view @ projection`, plus the
camera centre taken from the inverse of the world-to-view matrix.
"""
import math

import numpy as np
import torch


def get_world2view2(R, t, translate=np.array([0.0, 0.0, 0.0]), scale=1.0):
    """utils/graphics_utils.py:38-49: world->view with optional recentring, float32."""
    Rt = np.zeros((4, 4))
    Rt[:3, :3] = np.asarray(R).transpose()
    Rt[:3, 3] = t
    Rt[3, 3] = 1.0
    c2w = np.linalg.inv(Rt)
    c2w[:3, 3] = (c2w[:3, 3] + translate) * scale
    return np.float32(np.linalg.inv(c2w))


def get_projection_matrix(znear, zfar, fovX, fovY):
    """utils/graphics_utils.py:51-71: OpenGL-style perspective with z mapped to [0, 1]."""
    tan_y, tan_x = math.tan(fovY / 2), math.tan(fovX / 2)
    top, right = tan_y * znear, tan_x * znear
    bottom, left = -top, -right
    P = torch.zeros(4, 4)
    P[0, 0] = 2.0 * znear / (right - left)
    P[1, 1] = 2.0 * znear / (top - bottom)
    P[0, 2] = (right + left) / (right - left)
    P[1, 2] = (top + bottom) / (top - bottom)
    P[3, 2] = 1.0
    P[2, 2] = zfar / (zfar - znear)
    P[2, 3] = -(zfar * znear) / (zfar - znear)
    return P


def focal2fov(focal, pixels):
    return 2 * math.atan(pixels / (2 * focal))


def fov2focal(fov, pixels):
    return pixels / (2 * math.tan(fov / 2))


class Camera:
    """The fields of scene/cameras.py:Camera that render() reads (cameras.py:17-66)."""

    def __init__(self, R, T, FoVx, FoVy, width, height, time=0.0, znear=0.01, zfar=100.0,
                 trans=np.array([0.0, 0.0, 0.0]), scale=1.0):
        self.R, self.T, self.FoVx, self.FoVy = R, T, FoVx, FoVy
        self.image_width, self.image_height = int(width), int(height)
        self.time = time
        self.znear, self.zfar = znear, zfar
        self.world_view_transform = torch.tensor(get_world2view2(R, T, trans, scale)).transpose(0, 1)
        self.projection_matrix = get_projection_matrix(znear, zfar, FoVx, FoVy).transpose(0, 1)
        self.full_proj_transform = (self.world_view_transform.unsqueeze(0).bmm(
            self.projection_matrix.unsqueeze(0))).squeeze(0)
        self.camera_center = self.world_view_transform.inverse()[3, :3]

    def on_device(self, dev):
        """(world_view_transform, full_proj_transform, camera_center) on `dev`, copied once per device
        (render() of the reference copies them host->device on every call, gaussian_renderer:45-51)."""
        cache = self.__dict__.setdefault("_dev_cache", {})
        key = str(dev)
        if key not in cache:
            cache[key] = (self.world_view_transform.to(dev), self.full_proj_transform.to(dev),
                          self.camera_center.to(dev))
        return cache[key]

    @property
    def tanfovx(self):
        return math.tan(self.FoVx * 0.5)

    @property
    def tanfovy(self):
        return math.tan(self.FoVy * 0.5)
