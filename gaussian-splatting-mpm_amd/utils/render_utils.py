"""Camera record and image quantisation (utils/render_utils.py:4-21)."""
import numpy as np
import torch


class TinyCam:
    def __init__(self, width, height, FovX, FovY, cam_center, view_mat, full_proj_mat):
        self.width = width
        self.height = height
        self.FovX = FovX
        self.FovY = FovY
        self.cam_center = cam_center
        self.view_mat = view_mat
        self.full_proj_mat = full_proj_mat

    def toCuda(self, device="cuda"):
        self.cam_center = torch.as_tensor(self.cam_center).to(device)
        self.view_mat = torch.as_tensor(self.view_mat).to(device)
        self.full_proj_mat = torch.as_tensor(self.full_proj_mat).to(device)


def to8b(x):
    """uint8(255 * clip(x, 0, 1)) -- truncation, as render_utils.py:20-21."""
    return (255 * np.clip(x, 0, 1)).astype(np.uint8)
