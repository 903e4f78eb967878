"""PILtoTorch as upstream 3DGS utils/general_utils.py (extra.py:29)."""
import numpy as np
import torch


def PILtoTorch(pil_image, resolution):
    resized = pil_image.resize(resolution)
    t = torch.from_numpy(np.array(resized)) / 255.0
    if t.dim() == 3:
        return t.permute(2, 0, 1)
    return t.unsqueeze(-1).permute(2, 0, 1)
