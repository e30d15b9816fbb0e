"""Data ingest: aonerf.datasets against the reference's SapienDataset /
SapienDatasetMulti outputs on the committed mini datasets (tests/golden/data, made by
tests/golden/make_golden.py:make_mini_datasets).  The reference's image order is os.listdir
order, which depends on the filesystem, so images are matched by file name."""
import os

import numpy as np
import pytest
import torch

from conftest import ROOT

DATA = os.path.join(ROOT, "tests", "golden", "data")
HW = 32 * 24


def test_host_meta_cpu(golden):
    """Host side (transforms.json, focal, splits, PIL decode + LANCZOS resize) on CPU."""
    from aonerf.datasets import SapienDataset

    g = golden("datasets.npz")
    ds = SapienDataset(os.path.join(DATA, "sapien_mini"), "train", img_wh=(32, 24), white_back=True,
                       device="cpu")
    assert ds.focal == float(g["train_focal"])
    assert len(ds) == 3 * HW and ds.near == 2.0 and ds.far == 6.0
    assert tuple(ds.images.shape) == (3, 24, 32, 4) and ds.images.dtype == torch.uint8
    assert sorted(ds.img_files_train) == sorted(str(f) for f in g["train_files"])
    dv = SapienDataset(os.path.join(DATA, "sapien_mini"), "val", img_wh=(32, 24), device="cpu")
    assert len(dv) == 1 and dv.img_files_val == ["r_0.png", "r_1.png"]


@pytest.mark.gpu
def test_train_batches_match_reference(golden):
    from aonerf.datasets import SapienDataset

    g = golden("datasets.npz")
    ds = SapienDataset(os.path.join(DATA, "sapien_mini"), "train", img_wh=(32, 24), white_back=True)
    for r, f in enumerate(g["train_files"]):
        k = ds.img_files_train.index(str(f))
        b = ds.batch(torch.arange(k * HW, (k + 1) * HW, device="cuda"))
        ref = slice(r * HW, (r + 1) * HW)
        np.testing.assert_array_equal(b["rays_o"].cpu().numpy(), g["train_rays"][ref, :3])
        np.testing.assert_allclose(b["viewdirs"].cpu().numpy(), g["train_rays"][ref, 3:6], rtol=0, atol=1e-6)
        np.testing.assert_allclose(b["rays_d"].cpu().numpy(), g["train_rays_d"][ref], rtol=0, atol=1e-6)
        np.testing.assert_array_equal(b["target"].cpu().numpy(), g["train_rgbs"][ref])
    # a random batch is drawn from the same table
    rb = ds.random_batch(4096, torch.Generator(device="cuda").manual_seed(0))
    assert rb["target"].shape == (4096, 3) and torch.isfinite(rb["rays_d"]).all()
    # one shuffled epoch (the reference's DataLoader(shuffle=True)) visits every sample once:
    # the union of its batches (ragged last one included) is the whole table, each row once
    full = ds.batch(torch.arange(len(ds), device="cuda"))
    seen = torch.cat([torch.cat([b["rays_d"], b["target"]], -1)
                      for b in ds.epoch_batches(1000, torch.Generator(device="cuda").manual_seed(1))])
    assert seen.shape[0] == len(ds)
    key = lambda x: x[torch.argsort(x[:, 0] * 1e4 + x[:, 1] * 1e2 + x[:, 2])]  # noqa: E731
    assert torch.equal(key(seen[:, :3]), key(full["rays_d"]))


@pytest.mark.gpu
def test_val_samples_match_reference(golden):
    from aonerf.datasets import SapienDataset

    g = golden("datasets.npz")
    dv = SapienDataset(os.path.join(DATA, "sapien_mini"), "val", img_wh=(32, 24), white_back=True)
    for i in range(2):
        s = dv[i]
        np.testing.assert_array_equal(s["rays_o"].cpu().numpy(), g[f"val{i}_rays_o"])
        np.testing.assert_allclose(s["rays_d"].cpu().numpy(), g[f"val{i}_rays_d"], rtol=0, atol=1e-6)
        np.testing.assert_allclose(s["viewdirs"].cpu().numpy(), g[f"val{i}_viewdirs"], rtol=0, atol=1e-6)
        np.testing.assert_array_equal(s["instance_mask"].cpu().numpy(), g[f"val{i}_instance_mask"])
        np.testing.assert_array_equal(s["target"].cpu().numpy(), g[f"val{i}_target"])


@pytest.mark.gpu
def test_multi_masked_batch_matches_reference(golden):
    from aonerf.datasets import SapienMultiImage

    g = golden("datasets.npz")
    ours = os.listdir(os.path.join(DATA, "multi_mini", "inst1", "train", "deg0", "rgb"))
    image_id = ours.index(str(g["multi_files"][1]))  # the reference read listdir()[1]
    im = SapienMultiImage(os.path.join(DATA, "multi_mini"), "inst1", "deg0", image_id,
                          img_wh=(32, 24), white_back=True)
    b = im.ray_batch(torch.from_numpy(g["multi_pix"]).cuda())
    np.testing.assert_array_equal(b["rays_o"].cpu().numpy(), g["multi_rays_o"])
    np.testing.assert_allclose(b["rays_d"].cpu().numpy(), g["multi_rays_d"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(b["viewdirs"].cpu().numpy(), g["multi_viewdirs"], rtol=0, atol=1e-6)
    np.testing.assert_array_equal(b["target"].cpu().numpy(), g["multi_rgbs"])
    np.testing.assert_array_equal(b["mask"].cpu().numpy(), g["multi_mask"].reshape(-1))


def test_tiled_layout_helpers():
    """aonerf/tiles.py: element (row, f) of a tiled (rows(n), W) buffer sits at
    (row // 16) 16 W + 256 (f // 16) + 16 (row % 16) + f % 16 (the layout
    csrc/mlp_f16x3_core.hpp act_base writes), and untile inverts tile on ragged sizes."""
    import torch
    from aonerf import tiles

    for n, W in ((37, 32), (16, 128), (2405, 256)):
        x = torch.arange(n * W, dtype=torch.int64).reshape(n, W)
        t = tiles.tile(x).reshape(-1)
        assert t.numel() == tiles.rows(n) * W
        for row in sorted(r for r in {0, 5, 15, 16, n - 1} if r < n):
            for f in sorted({0, 3, 7, 17, W - 1}):
                off = (row // 16) * 16 * W + 256 * (f // 16) + 16 * (row % 16) + f % 16
                assert t[off] == x[row, f]
        assert torch.equal(tiles.untile(t.reshape(-1, W), n), x)
