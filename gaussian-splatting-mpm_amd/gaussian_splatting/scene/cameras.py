"""Camera as upstream 3DGS scene/cameras.py (extra.py:28,141-146): R is the
transposed world->camera rotation (glm convention), T the world->camera
translation; world_view_transform / full_proj_transform are the transposed
matrices the rasterizer consumes, znear 0.01, zfar 100."""
from __future__ import annotations

import numpy as np
import torch

from gaussian_splatting.utils.graphics_utils import getProjectionMatrix, getWorld2View2


class Camera:
    def __init__(self, colmap_id, R, T, FoVx, FoVy, image, gt_alpha_mask, image_name, uid,
                 trans=np.array([0.0, 0.0, 0.0]), scale=1.0, data_device="cuda"):
        self.uid, self.colmap_id, self.image_name = uid, colmap_id, image_name
        self.R, self.T, self.FoVx, self.FoVy = R, T, FoVx, FoVy
        self.data_device = torch.device(data_device)
        self.original_image = image.clamp(0.0, 1.0).to(self.data_device)
        self.image_width = self.original_image.shape[2]
        self.image_height = self.original_image.shape[1]
        if gt_alpha_mask is not None:
            self.original_image *= gt_alpha_mask.to(self.data_device)
        self.zfar, self.znear = 100.0, 0.01
        self.trans, self.scale = trans, scale
        self.world_view_transform = torch.tensor(getWorld2View2(R, T, trans, scale)).transpose(0, 1).to(self.data_device)
        self.projection_matrix = getProjectionMatrix(znear=self.znear, zfar=self.zfar, fovX=FoVx,
                                                     fovY=FoVy).transpose(0, 1).to(self.data_device)
        self.full_proj_transform = (self.world_view_transform.unsqueeze(0).bmm(
            self.projection_matrix.unsqueeze(0))).squeeze(0)
        self.camera_center = self.world_view_transform.inverse()[3, :3]
