"""Evaluation metrics and image output against the reference's
definitions restated in the oracle (models/interface.py:54-74, models/utils.py:12-13, 102-109):
PSNR agreement 1e-4 dB (the GPU sums the squared errors in fp64, torch CPU in fp32 cascade
order), to8b bit-exact."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import nerf_oracle as O

pytestmark = pytest.mark.gpu


def _images(seed, n=3, h=24, w=32):
    g = torch.Generator().manual_seed(seed)
    preds = [torch.rand((h, w, 3), generator=g) * 1.2 - 0.1 for _ in range(n)]  # outside [0,1] too
    gts = [torch.rand((h, w, 3), generator=g) for _ in range(n)]
    masks = [torch.rand((h, w), generator=g) > 0.6 for _ in range(n)]
    return preds, gts, masks


def test_psnr_definitions():
    from aonerf import interface as I

    preds, gts, masks = _images(0)
    cu = lambda xs: [x.cuda() for x in xs]  # noqa: E731
    got = I.psnr_each(cu(preds), cu(gts)).cpu().numpy()
    ref = O.psnr_each(preds, gts).numpy()
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-4)
    d = I.psnr(cu(preds), cu(gts))
    assert d["name"] == "PSNR" and abs(d["test"] - float(ref.mean())) < 1e-4
    # object PSNR: pixels of each segmentation mask (get_obj_rgbs_from_segmap + psnr_each)
    obj_p = [p[m[..., None].repeat(1, 1, 3)] for p, m in zip(preds, masks)]
    obj_g = [g[m[..., None].repeat(1, 1, 3)] for g, m in zip(gts, masks)]
    ref_obj = O.psnr_each(obj_p, obj_g).mean().item()
    assert abs(I.psnr_obj(cu(preds), cu(gts), cu(masks))["test"] - ref_obj) < 1e-4
    # legacy PSNR (no clipping) with and without a valid mask
    ref_leg = O.psnr_legacy(preds[0], gts[0]).item()
    assert abs(I.psnr_legacy(preds[0].cuda(), gts[0].cuda()).item() - ref_leg) < 1e-4
    vm = masks[1].reshape(-1)
    ref_vm = -10 * torch.log10(torch.mean(((preds[1].reshape(-1, 3) - gts[1].reshape(-1, 3)) ** 2)[vm]))
    got_vm = I.psnr_legacy(preds[1].reshape(-1, 3).cuda(), gts[1].reshape(-1, 3).cuda(), vm.cuda())
    assert abs(got_vm.item() - ref_vm.item()) < 1e-4


def test_to8b_and_store(tmp_path):
    from aonerf import interface as I

    preds, _, _ = _images(1, n=2)
    for p in preds:
        ref = (255 * np.clip(p.numpy(), 0, 1)).astype(np.uint8)  # models/utils.py:12-13
        np.testing.assert_array_equal(I.to8b(p.cuda()).cpu().numpy(), ref)
    I.store_image(str(tmp_path), [p.cuda() for p in preds], "image")
    assert sorted(os.listdir(tmp_path)) == ["image000.jpg", "image001.jpg"]
    I.write_stats(str(tmp_path / "results.json"), {"name": "PSNR", "mean": 1.5, "test": 1.5})
    assert json.load(open(tmp_path / "results.json")) == {"PSNR": {"mean": 1.5, "test": 1.5}}


def test_epoch_on_mini_dataset(tmp_path):
    """The whole test epoch on the mini dataset (single rank): PSNR of the rendered views
    against the targets agrees with the oracle's render of the same views."""
    from aonerf.datasets import SapienDataset
    from aonerf.interface import test_epoch
    from aonerf.model import NeRF
    from oracle import weights as W
    from conftest import ROOT

    ds = SapienDataset(os.path.join(ROOT, "tests", "golden", "data", "sapien_mini"), "test"
                       if os.path.isdir(os.path.join(ROOT, "tests", "golden", "data", "sapien_mini", "test"))
                       else "val", img_wh=(32, 24), white_back=True)
    net = NeRF().cuda().requires_grad_(False)
    sd = W.nerf_state_dict(0)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    st_psnr, st_obj = test_epoch(net, ds, out_dir=str(tmp_path))
    assert os.path.exists(tmp_path / "results.json") and os.path.exists(tmp_path / "image000.jpg")
    # oracle: render the same views on CPU, same metric definitions
    params = O.split_state_dict(sd)
    ref = []
    for i, f in enumerate(ds.img_files_val):
        c2w = torch.FloatTensor(np.array(ds.meta["frames"][f.split(".")[0]]))[:3, :4]
        d = O.get_ray_directions(24, 32, ds.focal)
        ro, rv, rd = O.get_rays(d, c2w, True)
        out = O.nerf_forward(params, {"rays_o": ro, "rays_d": rd, "viewdirs": rv}, False, True, 2.0, 6.0)
        ref.append((out[1][0].reshape(24, 32, 3), ds[i]["target"].cpu().reshape(24, 32, 3)))
    ref_psnr = O.psnr_each([a for a, _ in ref], [b for _, b in ref]).mean().item()
    assert abs(st_psnr["test"] - ref_psnr) < 1e-3, (st_psnr, ref_psnr)
    assert np.isfinite(st_obj["test"])
