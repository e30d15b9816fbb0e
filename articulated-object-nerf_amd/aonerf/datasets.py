"""Data ingest of the reference datasets with the rays and
targets produced on the GPU.

``SapienDataset`` mirrors datasets/sapien.py:11-154 (transforms.json + RGBA PNGs alpha-blended
onto white): the same constructor, splits, ``focal``/``near``/``far``, ``__len__`` and
``__getitem__`` samples.  ``SapienMultiImage`` mirrors the per-image part of
datasets/sapien_multi.py (read_data :240-306, load_image_and_seg :156-168,
get_masked_img_seg :186-196, get_ray_batch :207-238).

What stays on the host is what the reference also does there and the GPU cannot: JSON parsing,
PNG decoding and the LANCZOS resize (PIL, same library and calls as the reference).  The
decoded images live on the device as uint8 (4 B/pixel instead of the reference's 44 B of
float rays + targets per pixel), and every ray batch -- the whole training set, a random
4096-ray batch, or a full validation image -- comes from one aon_sample_rays launch: camera
ray of the pixel (bit-identical to aon_frame_rays / the reference's get_rays) plus its
alpha-blended or mask-selected target.  That replaces the CPU DataLoader of run.py.
"""
import json
import os

import numpy as np
import torch
from PIL import Image

from . import _lib as L


def _load_rgba(path, img_wh):
    img = Image.open(path)
    img = img.resize(img_wh, Image.LANCZOS)  # sapien.py:95 / :143
    a = np.array(img)
    if a.ndim != 3 or a.shape[2] != 4:
        raise ValueError(f"{path}: expected an RGBA image (the reference blends its alpha)")
    return a


def _sample(poses, images, C, H, W, focal, idx, n, mode, bg, device):
    ro = torch.empty((n, 3), device=device)
    rd = torch.empty((n, 3), device=device)
    tgt = torch.empty((n, 3), device=device) if images is not None else None
    L.call("aon_sample_rays", L.ptr(poses), L.ptr(images), C, poses.shape[0], H, W, float(focal),
           L.ptr(idx), n, mode, float(bg), L.ptr(ro), L.ptr(rd), None, L.ptr(tgt),
           L.stream(device))
    return ro, rd, tgt


class SapienDataset:
    """reference datasets/sapien.py:11-154 (device-resident)."""

    def __init__(self, root_dir, split="train", img_wh=(320, 240), model_type=None,
                 white_back=None, eval_inference=None, device="cuda"):
        self.root_dir, self.split, self.img_wh = root_dir, split, tuple(img_wh)
        self.device = torch.device(device)
        self.read_meta()
        self.white_back = white_back
        w, h = self.img_wh
        n = len(self.img_files_val) if eval_inference is not None else 1
        self.image_sizes = np.array([[h, w] for _ in range(n)])

    def read_meta(self):
        w, h = self.img_wh
        if self.split == "train":
            base = os.path.join(self.root_dir, "train")
            files = os.listdir(os.path.join(base, "rgb"))  # listdir order, as the reference
        else:
            base = os.path.join(self.root_dir, "val" if self.split == "val" else "test")
            files = os.listdir(os.path.join(base, "rgb"))
            order = np.argsort([int(f.split("_")[1].split(".")[0]) for f in files])
            files = [files[i] for i in order]
            self.base_dir_val, self.img_files_val = base, files
        self.meta = json.load(open(os.path.join(base, "transforms.json")))
        cam_x = self.meta.get("camera_angle_x", False)
        if cam_x:
            self.focal = 0.5 * h / np.tan(0.5 * self.meta["camera_angle_x"])
            self.focal *= self.img_wh[0] / 320
        else:
            self.focal = self.meta.get("focal", None)
            if self.focal is None:
                raise ValueError("focal length not found in transforms.json")
        self.near, self.far = 2.0, 6.0
        self.bounds = np.array([self.near, self.far])
        if self.split == "train":
            poses, imgs = [], []
            for f in files:
                pose = np.array(self.meta["frames"][f.split(".")[0]])
                poses.append(torch.FloatTensor(pose)[:3, :4])
                imgs.append(_load_rgba(os.path.join(base, "rgb", f), self.img_wh))
            self.img_files_train = files
            self.poses = torch.stack(poses).contiguous().to(self.device)
            self.images = torch.from_numpy(np.stack(imgs)).to(self.device)  # (N, H, W, 4) u8

    def __len__(self):
        if self.split == "train":
            return self.poses.shape[0] * self.img_wh[0] * self.img_wh[1]
        if self.split == "val":
            return 1
        return len(self.img_files_val)

    def batch(self, idx):
        """The training samples of flat indices ``idx`` (device int64) as one batch dict
        {rays_o, rays_d, viewdirs, target} (sapien.py:131-135 for every index)."""
        w, h = self.img_wh
        idx = L.contig(torch.as_tensor(idx, dtype=torch.int64, device=self.device))
        ro, rd, tgt = _sample(self.poses, self.images, 4, h, w, self.focal, idx, idx.numel(), 1,
                              1.0, self.device)
        return {"rays_o": ro, "rays_d": rd, "viewdirs": rd, "target": tgt}

    def random_batch(self, n, generator=None):
        """A batch of n samples drawn uniformly WITH replacement (synthetic benches).  The
        reference's training loader (DataLoader(shuffle=True), model.py:228-236) visits every
        sample once per epoch: that is epoch_batches."""
        idx = torch.randint(0, len(self), (n,), device=self.device, generator=generator)
        return self.batch(idx)

    def epoch_batches(self, n, generator=None, drop_last=False):
        """One epoch of the reference's shuffled DataLoader (batch_size n, shuffle=True,
        drop_last False): a device permutation of every sample index, cut into batches of n
        (the last one ragged)."""
        perm = torch.randperm(len(self), device=self.device, generator=generator)
        for i in range(0, perm.numel(), n):
            if drop_last and i + n > perm.numel():
                break
            yield self.batch(perm[i:i + n])

    def __getitem__(self, idx):
        if self.split == "train":
            b = self.batch(torch.tensor([int(idx)]))
            return {k: v[0] for k, v in b.items()}
        f = self.img_files_val[idx]
        c2w = torch.FloatTensor(np.array(self.meta["frames"][f.split(".")[0]]))[:3, :4]
        img = torch.from_numpy(_load_rgba(os.path.join(self.base_dir_val, "rgb", f),
                                          self.img_wh)).to(self.device)
        w, h = self.img_wh
        poses = c2w[None].contiguous().to(self.device)
        ro, rd, tgt = _sample(poses, img, 4, h, w, self.focal, None, h * w, 1, 1.0, self.device)
        return {"rays_o": ro, "rays_d": rd, "viewdirs": rd,
                "instance_mask": (img[..., 3] > 0).reshape(-1),  # sapien.py:142
                "target": tgt}


class SapienMultiImage:
    """One (instance, degree, image) of datasets/sapien_multi.py's layout
    ``root/<instance>/train/<degree>/{rgb,seg}/<img>.png + transforms.json``: the masked image
    (background white or black, :186-196), its rays, and ray batches (:207-238)."""

    def __init__(self, root_dir, instance_id, degree_id, image_id, img_wh=(320, 240),
                 split="train", white_back=True, device="cuda"):
        self.img_wh, self.white_back = tuple(img_wh), white_back
        self.device = torch.device(device)
        base = os.path.join(root_dir, instance_id, "train", degree_id)  # every split: train dir
        files = os.listdir(os.path.join(base, "rgb"))
        if split != "train":
            order = np.argsort([int(f.split("_")[1].split(".")[0]) for f in files])
            files = [files[i] for i in order]
        poses = json.load(open(os.path.join(base, "transforms.json")))
        w, h = self.img_wh
        self.focal = 0.5 * h / np.tan(0.5 * poses["camera_angle_x"]) * (self.img_wh[0] / 320)
        f = files[image_id]
        c2w = torch.FloatTensor(np.array(poses["frames"][f.split(".")[0]]))[:3, :4]
        rgb = Image.open(os.path.join(base, "rgb", f)).convert("RGB").resize((w, h), Image.LANCZOS)
        seg = np.array(Image.open(os.path.join(base, "seg", f)).resize((w, h), Image.LANCZOS)) > 0
        if seg.ndim == 3:
            raise ValueError("segmentation masks are single-channel in the reference layout")
        packed = np.concatenate([np.array(rgb), seg[..., None].astype(np.uint8)], -1)
        self.image = torch.from_numpy(packed).to(self.device)  # (H, W, 4): rgb + mask
        self.pose = c2w[None].contiguous().to(self.device)
        self.mask = torch.from_numpy(seg.reshape(-1)).to(self.device)

    def ray_batch(self, idx=None):
        """rays_o, view_dirs (= rays_d), rgbs and mask of pixel indices ``idx`` (all pixels when
        None), as get_ray_batch (:207-238) returns them for the masked image."""
        w, h = self.img_wh
        n = h * w if idx is None else idx.numel()
        if idx is not None:
            idx = L.contig(torch.as_tensor(idx, dtype=torch.int64, device=self.device))
        ro, rd, tgt = _sample(self.pose, self.image, 4, h, w, self.focal, idx, n, 2,
                              1.0 if self.white_back else 0.0, self.device)
        msk = self.mask if idx is None else self.mask[idx]
        return {"rays_o": ro, "rays_d": rd, "viewdirs": rd, "target": tgt, "mask": msk}
