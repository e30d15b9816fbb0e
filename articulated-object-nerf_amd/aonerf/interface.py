"""Metric definitions and the eval frame-gather contract of the reference's LitModel
(models/interface.py:22-74)."""
import numpy as np
import torch


@torch.no_grad()
def psnr_each(preds, gts):
    """interface.py:54-62: per-image PSNR with both sides clipped to [0, 1]."""
    out = []
    for pred, gt in zip(preds, gts):
        mse = torch.mean((torch.clip(pred, 0, 1) - torch.clip(gt, 0, 1)) ** 2)
        out.append(-10.0 * torch.log(mse) / np.log(10))
    return torch.stack(out)


def mse(image_pred, image_gt, valid_mask=None, reduction="mean"):
    """interface.py:64-70."""
    value = (image_pred - image_gt) ** 2
    if valid_mask is not None:
        value = value[valid_mask]
    return torch.mean(value) if reduction == "mean" else value


@torch.no_grad()
def psnr_legacy(image_pred, image_gt, valid_mask=None, reduction="mean"):
    """interface.py:72-74: -10*log10(mse), no clipping."""
    return -10 * torch.log10(mse(image_pred, image_gt, valid_mask, reduction))


def split_images(flat, image_sizes):
    """The reshape half of LitModel.alter_gather_cat (interface.py:40-51): a flat (sum h*w, C)
    tensor -> list of (h, w, C) / (h, w) images.  The all_gather half is replaced by the
    tile-sharded frame gather of aonerf.parallel (the reference's rank interleave,
    interface.py:36-37, does not re-assemble frames correctly and is not reproduced)."""
    out, cur = [], 0
    for (h, w) in image_sizes:
        img = flat[cur:cur + h * w]
        out.append(img.reshape(h, w, -1) if img.dim() == 2 and img.shape[-1] > 1 else img.reshape(h, w))
        cur += h * w
    return out
