"""Evaluation side of the reference's LitModel / test epoch (models/interface.py:22-139,
models/utils.py:12-27, 62-73, 102-109, model.py:459-507), on the GPU.

* ``psnr_each`` / ``psnr`` / ``psnr_obj``: per-image clipped MSE (and its object-masked
  variant) from one aon_image_mse launch for all images; the dict layout of LitModel.psnr.
* ``split_images`` + aonerf.parallel.render_frame_sharded / gather_frame replace
  alter_gather_cat: frames are row bands gathered to rank 0 and assembled in pixel order,
  which the reference's all_gather + permute interleave (interface.py:34-37) only does at one
  rank.
* ``store_image`` (to8b on the device, aon_to8b; JPEG write with PIL on the host, as the
  reference) and ``write_stats`` (the same JSON).
SSIM / LPIPS need piqa's pretrained networks, absent offline: not provided.
"""
import json
import os

import numpy as np
import torch

from . import _lib as L


def _stack(images):
    imgs = [L.contig(i.reshape(-1, 3).float()) for i in images]
    P = imgs[0].shape[0]
    if any(i.shape[0] != P for i in imgs):
        raise ValueError("all images of one call must have the same pixel count")
    return torch.stack(imgs), P


def _image_mse(preds, gts, masks=None, clip=True):
    p, P = _stack(preds)
    g, Pg = _stack(gts)
    if Pg != P or p.shape[0] != g.shape[0]:
        raise ValueError("preds and gts differ in shape")
    L.require_gpu(p, g)
    m = None
    if masks is not None:
        m = torch.stack([L.contig(x.reshape(-1)).to(torch.uint8) for x in masks])
    n = p.shape[0]
    mse = torch.empty((n,), device=p.device)
    psnr = torch.empty((n,), device=p.device)
    L.call("aon_image_mse", L.ptr(p), L.ptr(g), n, P, L.ptr(m), int(clip), L.ptr(mse), L.ptr(psnr),
           L.stream(p.device))
    return mse, psnr


@torch.no_grad()
def psnr_each(preds, gts):
    """interface.py:54-62: per-image PSNR, both sides clipped to [0, 1]."""
    return _image_mse(preds, gts)[1]


@torch.no_grad()
def psnr(preds, gts, i_train=None, i_val=None, i_test=None):
    """interface.py:124-139: {"name": "PSNR", "mean": m, "test": m}."""
    m = psnr_each(preds, gts).mean().item()
    return {"name": "PSNR", "mean": m, "test": m}


@torch.no_grad()
def psnr_obj(preds, gts, instance_masks):
    """The object PSNR of the test epoch (model.py:475-480): psnr over the pixels of each
    image's segmentation mask (get_obj_rgbs_from_segmap, models/utils.py:102-109)."""
    m = _image_mse(preds, gts, masks=instance_masks)[1].mean().item()
    return {"name": "PSNR", "mean": m, "test": m}


@torch.no_grad()
def psnr_legacy(image_pred, image_gt, valid_mask=None, reduction="mean"):
    """interface.py:72-74: -10*log10(mse), no clipping (mean reduction)."""
    if reduction != "mean":
        raise ValueError("psnr_legacy implements the mean reduction")
    masks = None if valid_mask is None else [valid_mask]
    mse = _image_mse([image_pred], [image_gt], masks=masks, clip=False)[0]
    return -10 * torch.log10(mse[0])


def mse(image_pred, image_gt, valid_mask=None, reduction="mean"):
    """interface.py:64-70 (mean reduction on the GPU kernel)."""
    if reduction != "mean":
        raise ValueError("mse implements the mean reduction")
    masks = None if valid_mask is None else [valid_mask]
    return _image_mse([image_pred], [image_gt], masks=masks, clip=False)[0][0]


def split_images(flat, image_sizes):
    """The reshape half of LitModel.alter_gather_cat (interface.py:40-51): a flat (sum h*w, C)
    tensor -> list of (h, w, C) / (h, w) images."""
    out, cur = [], 0
    for (h, w) in image_sizes:
        img = flat[cur:cur + h * w]
        out.append(img.reshape(h, w, -1) if img.dim() == 2 and img.shape[-1] > 1 else img.reshape(h, w))
        cur += h * w
    return out


def to8b(x):
    """models/utils.py:12-13 on the device: uint8(255 * clip(x, 0, 1))."""
    x = L.contig(x.float())
    L.require_gpu(x)
    out = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    L.call("aon_to8b", L.ptr(x), x.numel(), L.ptr(out), L.stream(x.device))
    return out


def store_image(dirpath, rgbs, name):
    """models/utils.py:21-27: <name><iii>.jpg per image (PIL, as the reference)."""
    from PIL import Image

    os.makedirs(dirpath, exist_ok=True)
    for i, rgb in enumerate(rgbs):
        Image.fromarray(to8b(rgb).cpu().numpy()).save(os.path.join(dirpath, f"{name}{str(i).zfill(3)}.jpg"))


def write_stats(fpath, *stats):
    """models/utils.py:62-73 / interface.py:173-184."""
    d = {}
    for stat in stats:
        d[stat["name"]] = {k: float(w) for (k, w) in stat.items() if k not in ("name", "scene_wise")}
    with open(fpath, "w") as fp:
        json.dump(d, fp, indent=4, sort_keys=True)


@torch.no_grad()
def test_epoch(model, dataset, out_dir=None, group=None):
    """LitNeRF's test loop + test_epoch_end (model.py:329-348, 459-507) over a SapienDataset
    test/val split: every image is rendered in row bands across the ranks of `group`
    (aonerf.parallel, one RCCL gather per image), then on rank 0: PSNR, object PSNR over the
    images' instance masks, optional image store + results.json.  Returns the stats dicts on
    rank 0 (None elsewhere)."""
    import torch.distributed as dist

    from .parallel import render_frame_sharded

    rank = dist.get_rank(group) if dist.is_initialized() else 0
    w, h = dataset.img_wh
    rgbs, targets, masks = [], [], []
    for i in range(len(dataset.img_files_val)):
        f = dataset.img_files_val[i]
        c2w = torch.FloatTensor(np.array(dataset.meta["frames"][f.split(".")[0]]))[:3, :4]
        frame, _ = render_frame_sharded(model, c2w, h, w, dataset.focal, dataset.near, dataset.far,
                                        True, group=group)
        if rank == 0:
            sample = dataset[i]
            rgbs.append(frame[:, :3].reshape(h, w, 3))
            targets.append(sample["target"].reshape(h, w, 3))
            masks.append(sample["instance_mask"].reshape(h, w))
    if rank != 0:
        return None
    stats = (psnr(rgbs, targets), psnr_obj(rgbs, targets, masks))
    if out_dir is not None:
        store_image(out_dir, rgbs, "image")
        write_stats(os.path.join(out_dir, "results.json"), stats[0],
                    dict(stats[1], name="PSNR_obj"))
    return stats
