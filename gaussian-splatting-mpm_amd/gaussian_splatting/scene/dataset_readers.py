"""CameraInfo / getNerfppNorm as upstream 3DGS scene/dataset_readers.py (extra.py:20,27,131-132)."""
from __future__ import annotations

from typing import NamedTuple

import numpy as np

from gaussian_splatting.utils.graphics_utils import getWorld2View2


class CameraInfo(NamedTuple):
    uid: int
    R: np.ndarray
    T: np.ndarray
    FovY: float
    FovX: float
    image: object
    image_path: str
    image_name: str
    width: int
    height: int


def getNerfppNorm(cam_info):
    centers = []
    for cam in cam_info:
        W2C = getWorld2View2(cam.R, cam.T)
        C2W = np.linalg.inv(W2C)
        centers.append(C2W[:3, 3:4])
    centers = np.hstack(centers)
    center = np.mean(centers, axis=1, keepdims=True)
    diagonal = np.max(np.linalg.norm(centers - center, axis=0, keepdims=True))
    radius = diagonal * 1.1
    return {"translate": -center.flatten(), "radius": radius}
