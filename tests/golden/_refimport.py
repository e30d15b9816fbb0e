"""Import the reference (/root/reference) with inert stand-ins for absent third-party modules.

Test infrastructure only; runs in the build container, never on the GPU box.  Only the
fixture generator (make_golden.py) uses it.  The one stub with semantics is
``kornia.create_meshgrid(H, W, normalized_coordinates=False)`` which must return (1,H,W,2)
with [...,0] = column index x in [0, W-1] and [...,1] = row index y (kornia 0.6.1,
pinned at reference requirements.txt:3; used at datasets/ray_utils.py:84).  The dataset
fixtures also need ``torchvision.transforms.ToTensor`` with its published semantics (PIL / HWC
ndarray -> CHW tensor; uint8 -> float32 / 255, other dtypes unchanged; used at
datasets/sapien.py:119 and sapien_multi.py:209-211); everything else is inert.
"""
import sys
import types

REF = "/root/reference"


class _LooseModule(types.ModuleType):
    """Module whose unknown attributes resolve to an inert callable (constants -> 0)."""

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return _Anything()


def _mod(name, **attrs):
    m = _LooseModule(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


def _create_meshgrid(height, width, normalized_coordinates=True, device=None, dtype=None):
    import torch

    xs = torch.linspace(0, width - 1, width)
    ys = torch.linspace(0, height - 1, height)
    if normalized_coordinates:
        xs = (xs / (width - 1) - 0.5) * 2
        ys = (ys / (height - 1) - 0.5) * 2
    gx, gy = torch.meshgrid(xs, ys, indexing="xy")
    return torch.stack([gx, gy], dim=-1)[None]


class _Anything:
    def __init__(self, *a, **k):
        pass

    def __call__(self, *a, **k):
        return _Anything()

    def __getattr__(self, name):
        return _Anything()


class _ToTensor:
    """torchvision.transforms.ToTensor (PIL.Image or HWC/HW ndarray -> CHW; uint8 -> /255)."""

    def __call__(self, pic):
        import numpy as np
        import torch

        a = np.array(pic, copy=True)
        if a.ndim == 2:
            a = a[:, :, None]
        t = torch.from_numpy(a).permute(2, 0, 1).contiguous()
        if t.dtype == torch.uint8:
            return t.to(dtype=torch.float32).div(255)
        return t


def install_stubs():
    import torch.nn as nn

    sys.dont_write_bytecode = True  # never write __pycache__ into /root/reference
    _mod("kornia", create_meshgrid=_create_meshgrid)
    _mod("numba", jit=lambda *a, **k: (lambda f: f))
    pl = _mod("pytorch_lightning", LightningModule=nn.Module, Trainer=_Anything,
              seed_everything=lambda *a, **k: None)
    _mod("pytorch_lightning.callbacks", ModelCheckpoint=_Anything, LearningRateMonitor=_Anything,
         TQDMProgressBar=_Anything)
    _mod("pytorch_lightning.loggers", WandbLogger=_Anything)
    _mod("pytorch_lightning.plugins", DDPPlugin=_Anything)
    pl.callbacks = sys.modules["pytorch_lightning.callbacks"]
    pl.loggers = sys.modules["pytorch_lightning.loggers"]
    pl.plugins = sys.modules["pytorch_lightning.plugins"]
    _mod("wandb", Image=_Anything, init=_Anything, log=_Anything)
    _mod("piqa")
    _mod("piqa.lpips", LPIPS=_Anything)
    _mod("piqa.ssim", SSIM=_Anything)
    _mod("cv2", COLORMAP_JET=2, COLORMAP_HOT=11)
    _mod("imageio")
    tv = _mod("torchvision", models=_Anything())
    _mod("torchvision.ops", masks_to_boxes=_Anything(), box_iou=_Anything())
    _mod("torchvision.transforms", Compose=_Anything, ToTensor=_ToTensor, Normalize=_Anything,
         Resize=_Anything)
    tv.transforms = sys.modules["torchvision.transforms"]
    _mod("torchvision.utils", make_grid=_Anything())
    _mod("torchvision.models", resnet34=_Anything(), resnet18=_Anything())
    tv.ops = sys.modules["torchvision.ops"]
    tv.utils = sys.modules["torchvision.utils"]
    _mod("torch_optimizer")
    if REF not in sys.path:
        sys.path.insert(0, REF)


def load_datasets():
    """Return the reference's datasets.sapien and datasets.sapien_multi modules."""
    import os

    install_stubs()
    argv, cwd = sys.argv, os.getcwd()
    try:
        sys.argv = ["x"]
        os.chdir(REF)
        import datasets.sapien as sapien
        import datasets.sapien_multi as sapien_multi
    finally:
        sys.argv = argv
        os.chdir(cwd)
    return sapien, sapien_multi


def load_articulated():
    """Return the reference's models/vanilla_nerf/model_autodecoder module (NeRF_AE_Art)."""
    import os

    install_stubs()
    argv, cwd = sys.argv, os.getcwd()
    try:
        sys.argv = ["x"]
        os.chdir(REF)
        import models.vanilla_nerf.model_autodecoder as mad
    finally:
        sys.argv = argv
        os.chdir(cwd)
    return mad


def load():
    """Return (helper, model_module, ray_utils, sapien_multi) reference modules."""
    import os

    install_stubs()
    argv = sys.argv
    cwd = os.getcwd()
    try:
        sys.argv = ["x"]
        os.chdir(REF)  # code_library.py appends "./" to sys.path for `from opt import get_opts`
        import models.vanilla_nerf.helper as helper
        import models.vanilla_nerf.model as model
        import datasets.ray_utils as ray_utils
        import datasets.sapien_multi as sapien_multi
    finally:
        sys.argv = argv
        os.chdir(cwd)
    return helper, model, ray_utils, sapien_multi
