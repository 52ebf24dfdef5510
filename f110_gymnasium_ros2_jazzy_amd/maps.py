"""Track maps: ROS map_server yaml + grayscale image -> occupancy -> exact EDT.

Mirrors ScanSimulator2D.set_map (laser_models.py:383-427): the image is
flipped top/bottom, thresholded at 128 (<= 128 occupied), and the
distance transform is taken to the nearest occupied cell.  The EDT itself is
computed by libf110 (f110_edt_k) as exact squared distances ``k``; the scan
kernels read ``resolution * sqrt(k)``, which equals SciPy's
``resolution * distance_transform_edt(bitmap)`` bit for bit.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field

import numpy as np

from . import _lib

MAP_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "maps")


@dataclass
class TrackMap:
    free_mask: np.ndarray          # uint8 [H, W], 1 = free (after flip + threshold)
    resolution: float
    origin: tuple                  # (x, y, yaw)
    yaml_path: str = ""
    edt_k: np.ndarray = field(default=None, repr=False)  # uint32 [H, W]

    @property
    def shape(self):
        return self.free_mask.shape

    @property
    def height(self):
        return self.free_mask.shape[0]

    @property
    def width(self):
        return self.free_mask.shape[1]

    def ensure_edt(self) -> np.ndarray:
        if self.edt_k is None:
            self.edt_k = edt_k(self.free_mask)
        return self.edt_k

    def dt(self) -> np.ndarray:
        """resolution * EDT in metres (get_dt, laser_models.py:40-53)."""
        return self.resolution * np.sqrt(self.ensure_edt().astype(np.float64))

    @property
    def bounds(self):
        """F110Env's obs bounds (f110_env.py:224-232)."""
        x0, y0 = self.origin[0], self.origin[1]
        return (x0, x0 + self.width * self.resolution, y0, y0 + self.height * self.resolution)


def edt_k(free_mask: np.ndarray) -> np.ndarray:
    fm = np.ascontiguousarray(free_mask, dtype=np.uint8)
    H, W = fm.shape
    k = np.empty((H, W), np.uint32)
    _lib.check(_lib.load().f110_edt_k(fm.ctypes.data, H, W, k.ctypes.data), "f110_edt_k")
    return k


def resolve(map_path: str, map_ext: str = ".png") -> str:
    """Accept a yaml path, a map name in the bundled maps dir, or a path without extension."""
    if os.path.exists(map_path) and map_path.endswith((".yaml", ".yml")):
        return map_path
    for cand in (map_path + ".yaml", os.path.join(MAP_DIR, map_path + ".yaml"), os.path.join(MAP_DIR, map_path)):
        if os.path.exists(cand):
            return cand
    raise FileNotFoundError(f"map yaml not found: {map_path}")


def load_map(map_path: str, map_ext: str = ".png") -> TrackMap:
    import yaml
    from PIL import Image

    yaml_path = resolve(map_path, map_ext)
    img_path = os.path.splitext(yaml_path)[0] + map_ext
    img = np.array(Image.open(img_path).transpose(Image.FLIP_TOP_BOTTOM)).astype(np.float64)
    if img.ndim != 2:
        raise ValueError(f"map image must be single-channel grayscale: {img_path}")
    free = (img > 128.).astype(np.uint8)
    with open(yaml_path) as f:
        meta = yaml.safe_load(f)
    origin = tuple(float(v) for v in meta["origin"])
    return TrackMap(free_mask=free, resolution=float(meta["resolution"]), origin=origin, yaml_path=yaml_path)


def centerline_spawns(name: str = "Spielberg", n_agents: int = 1, gap: int = 40, stride: int = 1) -> np.ndarray:
    """Spawn-pose table [S, A, 3] from a bundled centerline: agent a sits a*gap
    points ahead of agent 0, heading = local segment tangent."""
    d = np.load(os.path.join(MAP_DIR, f"{name}_centerline.npz"))
    xy = d["xy"]
    n = xy.shape[0]
    idx = np.arange(0, n, stride)
    out = np.empty((idx.shape[0], n_agents, 3))
    for a in range(n_agents):
        j = (idx + a * gap) % n
        k = (j + 3) % n
        out[:, a, 0] = xy[j, 0]
        out[:, a, 1] = xy[j, 1]
        out[:, a, 2] = np.arctan2(xy[k, 1] - xy[j, 1], xy[k, 0] - xy[j, 0])
    return out
