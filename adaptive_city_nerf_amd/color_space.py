"""sRGB <-> linear conversions used by the loss and the PSNR metric (reference interface:
nerfs/color_space.py:4-66).  Elementwise torch ops on whatever device the images live on."""
from __future__ import annotations

import torch


def linear_to_srgb(x: torch.Tensor) -> torch.Tensor:
    """color_space.py:4-10: clamp to [0,1], 12.92 x below 0.0031308, else 1.055 x^(1/2.4) - 0.055."""
    x = x.clamp(0, 1)
    return torch.where(x <= 0.0031308, 12.92 * x, 1.055 * x.pow(1 / 2.4) - 0.055)


def srgb_to_linear(x: torch.Tensor) -> torch.Tensor:
    """color_space.py:13-19: x / 12.92 below 0.04045, else ((x + 0.055) / 1.055)^2.4."""
    return torch.where(x <= 0.04045, x / 12.92, ((x + 0.055) / 1.055).pow(2.4))


def color_space_transformer(pred_linear: torch.Tensor, gt_tensor: torch.Tensor, color_space: str):
    """Bring prediction (linear) and ground truth (sRGB in [0,1]) into one space (color_space.py:22-66):
    'linear' converts the GT, 'srgb' converts the prediction, 'identity' takes both as they are."""
    cs = str(color_space).lower()
    pred = pred_linear.to(torch.float32)
    gt = gt_tensor.to(torch.float32).clamp(0, 1)
    if cs == "linear":
        pred, gt = pred.clamp(0, 1), srgb_to_linear(gt).clamp(0, 1)
    elif cs == "srgb":
        pred, gt = linear_to_srgb(pred).clamp(0, 1), gt.clamp(0, 1)
    elif cs == "identity":
        if (gt.max() > 1) or (gt.min() < 0):
            raise ValueError("GT out of [0,1]; identity mode assumes normalized linear GT.")
    else:
        raise ValueError(f"Invalid color_space={color_space!r}; use 'linear'|'srgb'|'identity'")
    return pred.to(pred_linear.dtype).to(pred_linear.device), gt.to(pred_linear.dtype).to(pred_linear.device)
