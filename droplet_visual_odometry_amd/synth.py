"""Seeded synthetic mono8 frame streams for tests and the benchmark.

The reference runs on rosbag frames that are not in the repository
(SURVEY.md §4, §8d), so parity tests and bench.py use a ray-cast, non-planar,
textured scene instead: a closed room (floor, four walls) with boxes, every
surface carrying an integer-hashed two-scale mosaic (strong FAST corners on all
eight ORB pyramid levels) plus smooth shading, viewed by a camera moving on a
circle (10 cm per frame, always translating, so every pair has a well-posed
essential matrix and most depths stay inside recoverPose's 50-baseline cut).
A 0.10 m square "marker" at a fixed 3-D pose supplies the per-frame corner
arrays that the reference gets from STag detections
(scripts/traj_eval_ground_truth.py:303-311, float64[K,2]).

Rendering is plain torch on any device; the texture hash is integer-exact, so
frames differ across devices only where a ray lands within rounding of a cell
edge.  Parity tests always feed the *same bytes* to the GPU path and the oracle.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch

# Intrinsics per config.  640x480 uses the reference's own
# Parameters/rosbot_calibration.yaml:29 camera.
INTRINSICS = {
    (640, 480): (606.811009, 611.104701, 325.199941, 227.591593),
    (1280, 720): (1213.622, 1213.622, 640.0, 360.0),
    (1920, 1080): (1820.433, 1820.433, 960.0, 540.0),
}

ROOM = 5.5          # walls at x, y = +-ROOM
CEIL = 3.6
CAM_RADIUS = 3.0
CAM_HEIGHT = 1.1
STEP = 0.25         # metres per frame along the circle
HEADING_OFFSET = 45.0   # degrees the view is turned outward from the direction of travel
MARKER_LEN = 0.10
# (cx, cy, cz, hx, hy, hz) axis-aligned boxes (centre, half extents): an outer
# ring of pillars 1.5 m outside the camera circle and an inner ring of crates,
# so every view mixes 1.5-3 m structure with 5-9 m walls (well-conditioned E).
BOXES = [(4.1 * math.cos(a), 4.1 * math.sin(a), 1.2, 0.35, 0.35, 1.2)
         for a in [k * math.pi / 6 + 0.2 for k in range(12)]] + \
        [(2.0 * math.cos(a), 2.0 * math.sin(a), 0.4, 0.35, 0.35, 0.4)
         for a in [k * math.pi / 3 for k in range(6)]]


def intrinsics(w: int, h: int) -> np.ndarray:
    if (w, h) in INTRINSICS:
        fx, fy, cx, cy = INTRINSICS[(w, h)]
    else:
        fx = fy = 0.948 * w
        cx, cy = w / 2.0, h / 2.0
    return np.array([[fx, 0.0, cx], [0.0, fy, cy], [0.0, 0.0, 1.0]], np.float64)


def camera_pose(i: int):
    """World->camera rotation R (rows = camera axes in world) and centre C for frame i.

    The camera circles the room centre, heading along the tangent turned
    HEADING_OFFSET degrees outward, pitched down 10 degrees with a small wobble."""
    phi = STEP * i / CAM_RADIUS
    C = np.array([CAM_RADIUS * math.cos(phi), CAM_RADIUS * math.sin(phi), CAM_HEIGHT])
    tangent = phi + math.pi / 2
    psi = tangent - math.radians(HEADING_OFFSET)   # heading angle in the xy plane
    theta = math.radians(10.0 + 1.5 * math.sin(i / 9.0))
    f = np.array([math.cos(psi) * math.cos(theta), math.sin(psi) * math.cos(theta), -math.sin(theta)])
    r = np.array([math.sin(psi), -math.cos(psi), 0.0])
    d = np.cross(f, r)
    R = np.stack([r, d, f])                     # x right, y down, z forward
    return R, C


def marker_world_corners() -> np.ndarray:
    # A square on the +x wall, facing the room, 1.2 m up.
    c = np.array([ROOM - 1e-3, 2.5, 1.2])
    u = np.array([0.0, 1.0, 0.0]) * MARKER_LEN / 2
    v = np.array([0.0, 0.0, 1.0]) * MARKER_LEN / 2
    return np.stack([c - u + v, c + u + v, c + u - v, c - u - v])


def marker_corners(i: int, K: np.ndarray) -> np.ndarray:
    R, C = camera_pose(i)
    Xc = (marker_world_corners() - C) @ R.T
    uv = Xc[:, :2] / Xc[:, 2:3]
    return np.stack([K[0, 0] * uv[:, 0] + K[0, 2], K[1, 1] * uv[:, 1] + K[1, 2]], axis=1)


def relative_pose(i: int, j: int):
    """Ground-truth motion from frame i to frame j as (R, t) with X_j = R X_i + t."""
    Ri, Ci = camera_pose(i)
    Rj, Cj = camera_pose(j)
    R = Rj @ Ri.T
    t = -Rj @ (Cj - Ci)
    return R, t


def _hash(a: torch.Tensor, b: torch.Tensor, salt: int) -> torch.Tensor:
    """Integer hash of two int64 lattice coordinates -> [0, 1)."""
    m = (1 << 31) - 1
    x = (a * 73856093) ^ (b * 19349663) ^ (salt * 83492791)
    x = x & m
    x = (x ^ (x >> 13)) * 1274126177 & m
    x = (x ^ (x >> 16)) * 668265263 & m
    x = x ^ (x >> 15)
    return (x & 0xFFFF).to(torch.float32) / 65536.0


def _texture(s: torch.Tensor, t: torch.Tensor, sid: torch.Tensor) -> torch.Tensor:
    salt = sid.to(torch.int64)
    v = torch.zeros_like(s)
    for cell, amp, k in ((0.03, 0.25, 1), (0.08, 0.40, 2), (0.25, 0.30, 3), (0.9, 0.05, 4)):
        a = torch.floor(s / cell).to(torch.int64)
        b = torch.floor(t / cell).to(torch.int64)
        v = v + amp * _hash(a + salt * 1000003 * k, b, k)
    return v


@dataclass
class SceneStream:
    width: int
    height: int
    device: str = "cpu"
    noise_sigma: float = 2.0

    def __post_init__(self):
        self.K = intrinsics(self.width, self.height)

    def render(self, idx: int) -> torch.Tensor:
        """Frame `idx` as uint8 [H, W] on self.device."""
        dev = torch.device(self.device)
        w, h = self.width, self.height
        fx, fy, cx, cy = self.K[0, 0], self.K[1, 1], self.K[0, 2], self.K[1, 2]
        R, C = camera_pose(idx)
        Rt = torch.tensor(R.T, dtype=torch.float32, device=dev)   # camera -> world
        Cw = torch.tensor(C, dtype=torch.float32, device=dev)
        v, u = torch.meshgrid(torch.arange(h, device=dev, dtype=torch.float32),
                              torch.arange(w, device=dev, dtype=torch.float32), indexing="ij")
        dc = torch.stack([(u - cx) / fx, (v - cy) / fy, torch.ones_like(u)], -1)
        d = dc @ Rt.T                                                # world ray directions
        inf = torch.full_like(u, float("inf"))
        best_t = inf.clone()
        sid = torch.zeros_like(u, dtype=torch.int32)

        def plane(axis, value, surface):
            nonlocal best_t, sid
            den = d[..., axis]
            tt = (value - Cw[axis]) / torch.where(den.abs() > 1e-9, den, torch.full_like(den, 1e-9))
            ok = (tt > 1e-4) & (tt < best_t)
            best_t = torch.where(ok, tt, best_t)
            sid = torch.where(ok, torch.full_like(sid, surface), sid)

        plane(2, 0.0, 1)
        plane(2, CEIL, 2)
        plane(0, ROOM, 3)
        plane(0, -ROOM, 4)
        plane(1, ROOM, 5)
        plane(1, -ROOM, 6)
        for bi, (bx, by, bz, hx, hy, hz) in enumerate(BOXES):
            lo = torch.tensor([bx - hx, by - hy, bz - hz], device=dev)
            hi = torch.tensor([bx + hx, by + hy, bz + hz], device=dev)
            safe = torch.where(d.abs() > 1e-9, d, torch.full_like(d, 1e-9))
            t0 = (lo - Cw) / safe
            t1 = (hi - Cw) / safe
            tmin = torch.minimum(t0, t1).amax(-1)
            tmax = torch.maximum(t0, t1).amin(-1)
            ok = (tmax >= tmin) & (tmin > 1e-4) & (tmin < best_t)
            best_t = torch.where(ok, tmin, best_t)
            sid = torch.where(ok, torch.full_like(sid, 10 + bi), sid)
        P = Cw + d * best_t.unsqueeze(-1)
        X, Y, Z = P[..., 0], P[..., 1], P[..., 2]
        # surface parametrisation (s, t) and a per-orientation shade
        ax = (X.abs() > ROOM - 1e-3) | ((sid >= 10) & self._face_is(P, sid, 0))
        ay = (Y.abs() > ROOM - 1e-3) | ((sid >= 10) & self._face_is(P, sid, 1))
        s = torch.where(ax, Y, X)
        t = torch.where(ax | ay, Z, Y)
        shade = torch.where(ax, 0.85, torch.where(ay, 1.0, 0.7))
        tex = _texture(s + 0.37 * sid, t - 0.21 * sid, sid)
        img = 25.0 + 215.0 * tex * shade
        img = img * (0.85 + 0.15 * torch.cos(0.9 * s + 0.6 * t))
        gen = torch.Generator(device=dev).manual_seed(1000 + idx)
        img = img + self.noise_sigma * torch.randn(img.shape, generator=gen, device=dev)
        return img.clamp(0, 255).round().to(torch.uint8)

    @staticmethod
    def _face_is(P, sid, axis):
        out = torch.zeros(P.shape[:-1], dtype=torch.bool, device=P.device)
        for bi, (bx, by, bz, hx, hy, hz) in enumerate(BOXES):
            c = (bx, by, bz)[axis]
            hlf = (hx, hy, hz)[axis]
            on = (sid == 10 + bi) & (((P[..., axis] - c).abs() - hlf).abs() < 1e-3)
            out = out | on
        return out

    def frames(self, start: int, count: int) -> torch.Tensor:
        return torch.stack([self.render(start + i) for i in range(count)])

    def marker_corners(self, idx: int) -> np.ndarray:
        return marker_corners(idx, self.K)
