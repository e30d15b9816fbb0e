"""Teacher-forced training steps of the reference, for the per-step training gates.

TEST INFRASTRUCTURE ONLY (oracle/__init__.py): tests/test_gpu_teacher_forced.py and the CPU
study tools/diag/tf_study.py use it as the checker.

A free-running training trajectory is a chaotic quantity (Adam on the reference's own
arithmetic parts from itself under one-ulp perturbations within ~10 steps at lr 1e-3,
tests/test_gpu_art_train_bf16.py), so it gates nothing past the first steps.  Teacher forcing
removes the chaos: the reference's fp32 run (torch autograd through the oracle + torch.optim.Adam,
reference model.py:256-282 / :386-389; model_autodecoder.py:395-477 / :599-601) records, at every
step k, its parameters theta_k and Adam moments (m_k, v_k); the implementation under test is
loaded with exactly that state, takes ONE step, and its update delta = theta' - theta_k is
compared with the reference's own update from the same state.  The reference's self-variance is
the same step re-evaluated in fp64 from the same (fp32) state: how far an equally valid
evaluation of the reference moves the update.
"""
import numpy as np
import torch

from . import nerf_oracle as O
from . import weights as W

BETAS = (0.9, 0.999)
EPS = 1e-8


def _vanilla_leaves(seed, dtype):
    out = {}
    for lv, pre in ((0, "coarse_mlp."), (1, "fine_mlp.")):
        for k, v in O.split_state_dict(W.nerf_state_dict(seed))[lv].items():
            out[pre + k] = v.to(dtype)
    return out


def _art_leaves(seed, dtype):
    out = {}
    for lv, pre in ((0, "coarse_mlp."), (1, "fine_mlp.")):
        for k, v in O.split_state_dict(W.art_state_dict(seed))[lv].items():
            out[pre + k] = v.to(dtype)
    for k, v in W.code_library_state_dict(seed).items():
        out["code_library." + k] = torch.from_numpy(v).to(dtype)
    return out


def _loss(kind, leaves, batch):
    """The reference's training loss on ``leaves`` (name -> tensor), eval sampling."""
    rays = {k: batch[k] for k in ("rays_o", "rays_d", "viewdirs")}
    if kind == "vanilla":
        params = [{k[len(pre):]: v for k, v in leaves.items() if k.startswith(pre)}
                  for pre in ("coarse_mlp.", "fine_mlp.")]
        ret = O.nerf_forward(params, rays, False, True, 2.0, 6.0)
        return O.img2mse(ret[1][0], batch["target"]) + O.img2mse(ret[0][0], batch["target"])
    params = [{k[len(pre):]: v for k, v in leaves.items() if k.startswith(pre)}
              for pre in ("coarse_mlp.", "fine_mlp.")]
    tables = {k[len("code_library."):]: v for k, v in leaves.items()
              if k.startswith("code_library.")}
    return O.art_training_loss(params, tables, rays, batch["target"], int(batch["instance_id"]),
                               int(batch["articulation_id"]), False, True, 2.0, 6.0)[0]


def one_step(kind, state, batch, lr, dtype=torch.float32):
    """One reference training step + torch.optim.Adam from ``state`` = dict(theta, m, v, step)
    (name -> fp32 tensors; step = Adam steps taken so far), evaluated in ``dtype``.  Returns
    (loss, new state (fp32 copies of dtype values), update theta' - theta in float64, grads)."""
    names = list(state["theta"])
    leaves = {n: state["theta"][n].to(dtype).clone().requires_grad_(True) for n in names}
    opt = torch.optim.Adam(list(leaves.values()), lr=lr, betas=BETAS, eps=EPS)
    if state["step"] > 0:
        for n in names:
            opt.state[leaves[n]] = {"step": torch.tensor(float(state["step"])),
                                    "exp_avg": state["m"][n].to(dtype).clone(),
                                    "exp_avg_sq": state["v"][n].to(dtype).clone()}
    b = {k: (v.to(dtype) if torch.is_tensor(v) and v.is_floating_point() else v)
         for k, v in batch.items()}
    loss = _loss(kind, leaves, b)
    loss.backward()
    grads = {n: leaves[n].grad.detach().double().clone() for n in names}
    opt.step()
    new = {"theta": {n: leaves[n].detach().float().clone() for n in names},
           "m": {n: opt.state[leaves[n]]["exp_avg"].float().clone() for n in names},
           "v": {n: opt.state[leaves[n]]["exp_avg_sq"].float().clone() for n in names},
           "step": state["step"] + 1}
    delta = {n: leaves[n].detach().double() - state["theta"][n].double() for n in names}
    return float(loss.detach()), new, delta, grads


def initial_state(kind, seed=0):
    theta = (_vanilla_leaves if kind == "vanilla" else _art_leaves)(seed, torch.float32)
    return {"theta": theta, "m": {n: torch.zeros_like(t) for n, t in theta.items()},
            "v": {n: torch.zeros_like(t) for n, t in theta.items()}, "step": 0}


def reference_run(kind, batch, steps, lr, seed=0, self_variance=True):
    """The fp32 reference's trajectory with its teacher-forcing record: per step k, the state
    it starts from, its loss, its update and (self_variance) the fp64 re-evaluation's update
    from the same state."""
    state = initial_state(kind, seed)
    rec = []
    for _ in range(steps):
        loss, nxt, delta, grads = one_step(kind, state, batch, lr)
        d64 = g64 = None
        if self_variance:
            _, _, d64, g64 = one_step(kind, state, batch, lr, torch.float64)
        rec.append({"state": state, "loss": loss, "delta": delta, "delta64": d64,
                    "grad": grads, "grad64": g64})
        state = nxt
    return rec


def compare(delta_ours, delta_ref):
    """Per tensor: relative L2 distance ||ours - ref|| / ||ref|| and the cosine of the two
    updates (float64 numpy)."""
    out = {}
    for n, r in delta_ref.items():
        a = np.asarray(delta_ours[n], np.float64).reshape(-1)
        b = r.numpy().reshape(-1) if torch.is_tensor(r) else np.asarray(r, np.float64).reshape(-1)
        nb = np.linalg.norm(b)
        na = np.linalg.norm(a)
        if nb == 0.0:
            out[n] = (0.0 if na == 0.0 else np.inf, 1.0 if na == 0.0 else 0.0)
            continue
        out[n] = (float(np.linalg.norm(a - b) / nb), float(a @ b / (na * nb + 1e-300)))
    return out


def batch_rays(kind):
    """The teacher-forced tests' rays (CPU): a 48 x 64 view of create_spheric_poses(4)[2],
    every 12th pixel (vanilla, 256 rays) or every 24th (articulated, 128 rays)."""
    H, Wd = 48, 64
    c2w = torch.as_tensor(O.create_spheric_poses(4.0)[2])[:3, :4]
    ro, rv, rd = O.get_rays(O.get_ray_directions(H, Wd, O.focal_from_fovy(H)), c2w, True)
    sel = torch.arange(0, H * Wd, 12 if kind == "vanilla" else 24)
    return {"rays_o": ro[sel].contiguous(), "rays_d": rd[sel].contiguous(),
            "viewdirs": rv[sel].contiguous()}


def make_batch(kind, rays):
    """Rays (CPU fp32, e.g. the GPU's own rays copied back: identical inputs) -> the batch with
    its target: vanilla -- another NeRF's render (oracle, PCG64 seed 3 weights); articulated -- a
    smooth colour ramp the random-init auto-decoder is far from, instance 7, articulation 3."""
    b = {k: v.float().contiguous() for k, v in rays.items()}
    n = b["rays_o"].shape[0]
    if kind == "vanilla":
        with torch.no_grad():
            b["target"] = O.nerf_forward(O.split_state_dict(W.nerf_state_dict(3)), b, False, True,
                                         2.0, 6.0)[1][0].contiguous()
    else:
        g = torch.linspace(0.0, 1.0, n)
        b["target"] = torch.stack([g, 1.0 - g, 0.5 + 0.4 * torch.sin(12.0 * g)], -1).contiguous()
        b["instance_id"] = 7
        b["articulation_id"] = 3
    return b
