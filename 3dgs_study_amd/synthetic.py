"""Seeded synthetic Gaussians and cameras (SURVEY.md §8d recipe).

Everything is generated on the CPU with a fixed ``torch.Generator`` and only
then moved to the device, so every box sees identical bits.

Camera conventions follow the reference exactly:
  * ``getWorld2View2`` (utils/graphics_utils.py:49-87): Rt[:3,:3] = R^T,
    Rt[:3,3] = t, computed in float64 and rounded to float32;
  * ``getProjectionMatrix`` (utils/graphics_utils.py:97-133): znear 0.01,
    zfar 100, P[3,2] = 1, P[2,2] = f/(f-n), P[2,3] = -fn/(f-n);
  * ``Camera`` (scene/cameras.py:103-121): world_view = W2C^T,
    full_proj = world_view @ proj^T, camera_center = inverse(world_view)[3,:3].
The Gaussian parameters mirror ``GaussianModel`` storage
(scene/gaussian_model.py:49-54) and its activations (:106-126).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

ZNEAR = 0.01
ZFAR = 100.0

# BASELINE.json configs (A..E); B..E use SH degree 3 (M = 16).
CONFIGS = {
    "A": dict(P=10_000, W=256, H=256, sh_degree=0, backward=False),
    "B": dict(P=100_000, W=800, H=800, sh_degree=3, backward=True),
    "C": dict(P=1_000_000, W=1920, H=1080, sh_degree=3, backward=True),
    "D": dict(P=1_000_000, W=1920, H=1080, sh_degree=3, backward=True),
    "E": dict(P=5_000_000, W=3840, H=2160, sh_degree=3, backward=False),
}


def get_world2view2(R: np.ndarray, t: np.ndarray, translate=np.array([0.0, 0.0, 0.0]), scale=1.0) -> np.ndarray:
    Rt = np.zeros((4, 4))
    Rt[:3, :3] = R.transpose()
    Rt[:3, 3] = t
    Rt[3, 3] = 1.0
    C2W = np.linalg.inv(Rt)
    cam_center = C2W[:3, 3]
    cam_center = (cam_center + translate) * scale
    C2W[:3, 3] = cam_center
    Rt = np.linalg.inv(C2W)
    return np.float32(Rt)


def get_projection_matrix(znear: float, zfar: float, fovX: float, fovY: float) -> torch.Tensor:
    tanHalfFovY = math.tan(fovY / 2)
    tanHalfFovX = math.tan(fovX / 2)
    top = tanHalfFovY * znear
    bottom = -top
    right = tanHalfFovX * znear
    left = -right
    P = torch.zeros(4, 4)
    z_sign = 1.0
    P[0, 0] = 2.0 * znear / (right - left)
    P[1, 1] = 2.0 * znear / (top - bottom)
    P[0, 2] = (right + left) / (right - left)
    P[1, 2] = (top + bottom) / (top - bottom)
    P[3, 2] = z_sign
    P[2, 2] = z_sign * zfar / (zfar - znear)
    P[2, 3] = -(zfar * znear) / (zfar - znear)
    return P


@dataclass
class SynthCamera:
    """Duck-types the attributes render() reads from a Camera/MiniCam."""
    image_width: int
    image_height: int
    FoVx: float
    FoVy: float
    world_view_transform: torch.Tensor
    projection_matrix: torch.Tensor
    full_proj_transform: torch.Tensor
    camera_center: torch.Tensor
    znear: float = ZNEAR
    zfar: float = ZFAR

    def to(self, device) -> "SynthCamera":
        return SynthCamera(self.image_width, self.image_height, self.FoVx, self.FoVy,
                           self.world_view_transform.to(device), self.projection_matrix.to(device),
                           self.full_proj_transform.to(device), self.camera_center.to(device), self.znear, self.zfar)


def yaw_rotation(theta: float) -> np.ndarray:
    c, s = math.cos(theta), math.sin(theta)
    return np.array([[c, 0.0, s], [0.0, 1.0, 0.0], [-s, 0.0, c]])


def make_camera(W: int, H: int, view: int = 0, distance: float = 6.0, fovx_deg: float = 60.0) -> SynthCamera:
    """Camera k: distance 6 from the origin, yaw k*45 deg, looking at the origin."""
    fovx = math.radians(fovx_deg)
    fovy = 2.0 * math.atan(math.tan(fovx / 2.0) * H / W)
    R = yaw_rotation(view * math.pi / 4.0)  # camera-to-world rotation (COLMAP-style R)
    T = np.array([0.0, 0.0, distance])  # world-to-camera translation
    wv = torch.tensor(get_world2view2(R, T)).transpose(0, 1)
    proj = get_projection_matrix(ZNEAR, ZFAR, fovx, fovy).transpose(0, 1)
    full = wv.unsqueeze(0).bmm(proj.unsqueeze(0)).squeeze(0)
    center = wv.inverse()[3, :3]
    return SynthCamera(W, H, fovx, fovy, wv.contiguous(), proj.contiguous(), full.contiguous(), center.contiguous())


@dataclass
class SynthGaussians:
    """Leaf parameters in GaussianModel storage layout (pre-activation)."""
    xyz: torch.Tensor  # [P,3]
    features_dc: torch.Tensor  # [P,1,3]
    features_rest: torch.Tensor  # [P,M-1,3]
    scaling: torch.Tensor  # [P,3] (log scale)
    rotation: torch.Tensor  # [P,4] (unnormalized quaternion)
    opacity: torch.Tensor  # [P,1] (logit)
    max_sh_degree: int
    active_sh_degree: int

    # GaussianModel getters (scene/gaussian_model.py:106-129)
    @property
    def get_xyz(self):
        return self.xyz

    @property
    def get_scaling(self):
        return torch.exp(self.scaling)

    @property
    def get_rotation(self):
        return torch.nn.functional.normalize(self.rotation)

    @property
    def get_opacity(self):
        return torch.sigmoid(self.opacity)

    @property
    def get_features(self):
        return torch.cat((self.features_dc, self.features_rest), dim=1)

    def params(self):
        return [self.xyz, self.features_dc, self.features_rest, self.opacity, self.scaling, self.rotation]

    def to(self, device, requires_grad=False) -> "SynthGaussians":
        t = [p.detach().to(device).contiguous().requires_grad_(requires_grad) for p in
             (self.xyz, self.features_dc, self.features_rest, self.scaling, self.rotation, self.opacity)]
        return SynthGaussians(*t, self.max_sh_degree, self.active_sh_degree)


def make_gaussians(P: int, sh_degree: int, seed: int = 0, radius: float = 2.0,
                   scale_range=(0.003, 0.03), active_sh_degree=None) -> SynthGaussians:
    g = torch.Generator().manual_seed(seed)
    M = (sh_degree + 1) ** 2
    d = torch.randn(P, 3, generator=g)
    d = d / d.norm(dim=1, keepdim=True).clamp_min(1e-12)
    r = radius * torch.rand(P, 1, generator=g).pow(1.0 / 3.0)
    xyz = d * r
    lo, hi = math.log(scale_range[0]), math.log(scale_range[1])
    scaling = lo + (hi - lo) * torch.rand(P, 3, generator=g)
    rotation = torch.randn(P, 4, generator=g)
    opacity = -2.0 + 4.0 * torch.rand(P, 1, generator=g)
    f_dc = 0.5 * torch.randn(P, 1, 3, generator=g)
    f_rest = 0.05 * torch.randn(P, M - 1, 3, generator=g)
    return SynthGaussians(xyz.contiguous(), f_dc.contiguous(), f_rest.contiguous(), scaling.contiguous(),
                          rotation.contiguous(), opacity.contiguous(), sh_degree,
                          sh_degree if active_sh_degree is None else active_sh_degree)


def make_target(W: int, H: int, seed: int = 1) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    return torch.rand(3, H, W, generator=g)
