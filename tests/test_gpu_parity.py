"""GPU parity: the HIP kernels (through the C ABI) against the reference's golden vectors and the
CPU oracle.  Everything here needs an MI355X (marker `gpu`).

Tolerances (north star: <= 1e-4 abs on RGB/depth/weights vs the reference on identical rays and
weights; PSNR within 0.05 dB):
  * stage-isolated (each kernel fed the reference's own inputs): 1e-6 for ray generation,
    pos_enc and compositing, 1e-5 for the MLP raw outputs (fp32 MFMA re-association only);
  * end-to-end two-level render, decomposed so that every link is gated at 1e-4 on EVERY ray:
      (1) coarse level vs the reference: rgb/acc/depth/weights within 1e-4;
      (2) fine sample positions == the reference's sample_pdf applied to OUR coarse weights,
          bit for bit (the oracle's pdf is pinned bit-exactly to the reference);
      (3) fine level vs the reference evaluated on OUR fine sample positions: within 1e-4;
    and against the reference's own end-to-end outputs: >= 99.5% of rays within 1e-4, PSNR
    delta <= 0.05 dB, and EVERY ray outside 1e-4 attributed automatically (`Attribution`) to the
    reference's own ill-conditioning in the coarse weights: our coarse weights of that ray are
    within 1e-4 of the reference's, and EITHER the reference's own sample_pdf places some
    fine-sample u in a different CDF bin under our coarse weights than under its own (a plateau
    flip: where coarse weights are exactly 0 -- ReLU'd density -- the CDF has plateaus and a
    ~1e-7 weight change can move a u across a plateau edge, shifting a fine sample by a whole
    bin; observed: one ray in 480 moves 0.0625 in t and 6e-4 in rgb from a 1.8e-7 coarse-weight
    difference), OR the reference's own pipeline, fed our coarse weights, moves its fine output
    by >= AMPLIFICATION x the coarse-weight difference (a near-plateau bin: a sample sits at
    lo + (u - cdf_lo) / (cdf_hi - cdf_lo) * width with a tiny cdf step, where a 1e-7 weight
    change moves it continuously by far more).  The reference's fine output on our coarse
    weights is link (3)'s oracle evaluation, so the attribution reuses the gated chain.  Any
    fp32 implementation with a different summation order shows the same (the reference with an
    fp64 or split-K GEMM moves 2.6e-2 on depth on a 64x64 frame: `env_*` arrays).  An outlier
    attributed neither way fails the test.
"""
import hashlib

import numpy as np
import pytest
import torch

from oracle import nerf_oracle as O
from oracle import weights as W
from oracle import attribution as A
from oracle.attribution import AMPLIFICATION, Attribution, fine_envelope, plateau_flips  # noqa: F401

pytestmark = pytest.mark.gpu

E2E_ATOL = 1e-4
# The end-to-end fraction gate is the reference's self-consistency ON THE SAME RAYS (verdict r05
# #1, oracle/attribution.py): the oracle re-run as another valid fp32 implementation of the
# reference (its GEMMs split-K, SELF_VARIANT) against the reference's own fp32 output gives the
# fraction of rays the reference keeps within 1e-4 of itself; ours must keep at least that
# fraction less max(0.1 pp, 3 binomial standard errors) -- e2e_floor.  At the headline scale
# (61,440 rays of the 640x480 bench frame, tools/diag/self_frac.py ->
# profiles/r06/self_frac/) the reference keeps rgb 99.984% / acc 99.982% / depth 99.857%; bench.py
# measures it on every run beside ours.  (Rounds 2-5 gated depth at a fixed 98.5% taken from the
# C1 frame's fp64 / split-K re-runs.)


def self_floors(params, rays_cpu, ref, **kw):
    """{quantity: floor} of our fraction within 1e-4 from the reference's self-consistency on
    ``rays_cpu`` (ref: the reference's fp32 fine (rgb, acc, depth) there; kw: fine_outputs'
    randomized / u_coarse / u_fine / latents ...)."""
    sc = A.self_consistency(params, rays_cpu, ref, **kw)
    print("  reference self-consistency (" + A.SELF_VARIANT + "): " + ", ".join(
        f"{k} {v['frac'] * 100:.3f}% ({v['outliers']} of {v['n']} out)" for k, v in sc.items()))
    return {k: A.e2e_floor(v["frac"], v["n"]) for k, v in sc.items()}


def assert_e2e(name, err, env=None, attrib=None, floor=None):
    """Direct comparison with the reference's end-to-end output: the fraction of rays within
    1e-4 at least ``floor`` (self_floors: the reference's own self-consistency on these rays),
    and every ray outside it attributed (`attrib`: Attribution.rays; module docstring).  `env`
    (the reference's own re-association envelope) is reported for context."""
    err = np.asarray(err)
    bad = (err > E2E_ATOL).reshape(len(err), -1).any(-1)
    frac = 1.0 - bad.mean() if len(bad) else 1.0
    if bad.any():
        msg = f"  {name}: {bad.sum()} of {len(bad)} rays > 1e-4 (max {err.max():.2e})"
        if env is not None:
            msg += f"; reference re-association envelope there: max {np.asarray(env)[bad].max():.2e}"
        if attrib is not None:
            msg += f"; attributed: {(bad & attrib).sum()}"
        print(msg)
    assert attrib is not None or not bad.any(), f"{name}: outliers and no attribution given"
    if attrib is not None:
        unexplained = np.nonzero(bad & ~attrib)[0]
        assert len(unexplained) == 0, f"{name}: rays {unexplained[:10]} off by > 1e-4, not attributed"
    assert floor is not None, f"{name}: no self-consistency floor given"
    print(f"  {name}: {frac * 100:.3f}% within 1e-4, floor {floor * 100:.3f}%")
    assert frac >= floor, f"{name}: only {frac * 100:.3f}% of rays within {E2E_ATOL} (floor {floor * 100:.3f}%)"


def check_chain(net, rays, params, randomized=False, white=True, u_coarse=None, u_fine=None,
                coarse_ref=None, return_ref=False):
    """Links (1)-(3) of the module docstring on one batch; returns the GPU outputs (and, with
    return_ref, the reference's fine level on our fine samples: dict rgb/acc/depth/weights)."""
    ret = net(rays, randomized, white, 2.0, 6.0, u_coarse=u_coarse, u_fine=u_fine,
              return_weights=True, return_intermediates=True)
    rc = {k: v.cpu() for k, v in rays.items()}
    # (1) coarse level
    if coarse_ref is None:
        t_c = ret[0][4]["t_vals"].cpu()
        coarse_ref = O.render_level(params, rc, t_c, 0, white)
        coarse_ref = (coarse_ref[0], coarse_ref[1], coarse_ref[3], coarse_ref[2])
    for j, k in enumerate(("rgb", "acc", "depth", "weights")):
        err = report(f"chain coarse {k}", npy(ret[0][j]), np.asarray(coarse_ref[j]), E2E_ATOL)
        assert err.max() <= E2E_ATOL, f"coarse {k}: {err.max():.3e}"
    # (2) fine sample positions = reference sampling on our coarse weights
    t_c, w_c = ret[0][4]["t_vals"].cpu(), ret[0][3].cpu()
    t_f, _ = O.sample_pdf(0.5 * (t_c[..., 1:] + t_c[..., :-1]), w_c[..., 1:-1], rc["rays_o"],
                          rc["rays_d"], t_c, net.num_fine_samples, randomized,
                          u=None if u_fine is None else u_fine.cpu())
    np.testing.assert_array_equal(npy(ret[1][4]["t_vals"]), t_f.numpy())
    # (3) fine level vs the reference on those positions
    fine = O.render_level(params, rc, t_f, 1, white)
    for j, k in ((0, "rgb"), (1, "acc"), (3, "depth"), (2, "weights")):
        jj = {"rgb": 0, "acc": 1, "depth": 2, "weights": 3}[k]
        err = report(f"chain fine {k}", npy(ret[1][jj]), fine[j].numpy(), E2E_ATOL)
        assert err.max() <= E2E_ATOL, f"fine {k}: {err.max():.3e}"
    if return_ref:
        return ret, {"rgb": fine[0].numpy(), "acc": fine[1].numpy(), "weights": fine[2].numpy(),
                     "depth": fine[3].numpy()}
    return ret


def cuda(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def npy(t):
    return t.detach().float().cpu().numpy()


PRECISIONS = ["fp32", "f16x3"]


def make_nerf(precision, **kw):
    from aonerf.model import NeRF

    net = NeRF(precision=precision, **kw).cuda()
    net.load_state_dict({k: torch.from_numpy(v) for k, v in W.nerf_state_dict(0).items()})
    return net.requires_grad_(False)  # inference: the fused MLP path (no autograd graph)


@pytest.fixture(scope="module", params=PRECISIONS)
def nerf(request):
    return make_nerf(request.param)


def rays_of(g):
    return {k: cuda(g[k]) for k in ("rays_o", "rays_d", "viewdirs")}


def report(name, got, want, atol):
    err = np.abs(np.asarray(got, np.float64) - np.asarray(want, np.float64))
    frac = float((err <= atol).mean()) if err.size else 1.0
    print(f"{name}: max|err|={err.max() if err.size else 0:.3e}  within {atol:g}: {frac * 100:.3f}%")
    return err


# ----------------------------------------------------------------------------- stages
def test_ray_generation(golden):
    from aonerf import ray_utils

    g = golden("rays.npz")
    for k in (0, 1):
        H, Wd, f = g[f"hwf{k}"]
        H, Wd = int(H), int(Wd)
        dirs = ray_utils.get_ray_directions(H, Wd, float(f))
        np.testing.assert_array_equal(npy(dirs), g[f"dirs{k}"])
        o, v, d, radii = ray_utils.get_rays(dirs, torch.from_numpy(g[f"c2w{k}"]), True, True)
        np.testing.assert_array_equal(npy(o), g[f"rays_o{k}"])
        # a1/a2 reproduce the reference's op order (forward fma chains of (n,3)@(3,3) and the
        # row norm): bit-exact
        report("radii", npy(radii), g[f"radii{k}"], 0)
        np.testing.assert_array_equal(npy(d), g[f"rays_d{k}"])
        np.testing.assert_array_equal(npy(v), g[f"viewdirs{k}"])
        np.testing.assert_array_equal(npy(radii), g[f"radii{k}"])
        fr = ray_utils.frame_rays(torch.from_numpy(g[f"c2w{k}"]), H, Wd, float(f))
        np.testing.assert_array_equal(npy(fr["rays_d"]), npy(d))
        # a band of the frame equals the same rows of the full frame
        band = ray_utils.frame_rays(torch.from_numpy(g[f"c2w{k}"]), H, Wd, float(f), p0=3 * Wd, n=5 * Wd)
        np.testing.assert_array_equal(npy(band["rays_d"]), npy(d)[3 * Wd:8 * Wd])


def test_pos_enc(golden):
    from aonerf import helper

    g = golden("pos_enc.npz")
    report("pos_enc x", npy(helper.pos_enc(cuda(g["x"]), 0, 10)), g["enc_x"], 1e-7)
    np.testing.assert_allclose(npy(helper.pos_enc(cuda(g["x"]), 0, 10)), g["enc_x"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(npy(helper.pos_enc(cuda(g["v"]), 0, 4)), g["enc_v"], rtol=0, atol=1e-6)


def test_sample_along_rays(golden):
    from aonerf import helper

    g = golden("forward_random.npz")
    t, xyz = helper.sample_along_rays(cuda(g["rays_o"]), cuda(g["rays_d"]), 64, 2.0, 6.0, True, False,
                                      u=cuda(g["u_coarse"]))
    np.testing.assert_array_equal(npy(t), g["coarse_t"])
    want = O.cast_rays(torch.from_numpy(g["coarse_t"]), torch.from_numpy(g["rays_o"]),
                       torch.from_numpy(g["rays_d"])).numpy()
    np.testing.assert_array_equal(npy(xyz), want)
    g = golden("forward_eval.npz")
    t, _ = helper.sample_along_rays(cuda(g["rays_o"]), cuda(g["rays_d"]), 64, 2.0, 6.0, False, False)
    np.testing.assert_array_equal(npy(t), g["coarse_t"])


def test_composite_edges(golden):
    from aonerf import helper

    g = golden("composite_edges.npz")
    for wb in (0, 1):
        out = helper.volumetric_rendering(cuda(g["rgb"]), cuda(g["sigma"]), cuda(g["t"]), cuda(g["dirs"]),
                                          bool(wb))
        for k, v in zip(("comp_rgb", "acc", "weights", "depth"), out):
            report(f"composite wb{wb} {k}", npy(v), g[f"wb{wb}_{k}"], 1e-7)
            np.testing.assert_allclose(npy(v), g[f"wb{wb}_{k}"], rtol=1e-6, atol=1e-6, err_msg=k)


def test_composite_levels_from_reference_raw(golden):
    """Fused compositor (raw (B*S,4) + sigmoid/relu) fed the reference's raw MLP outputs."""
    from aonerf import _lib as L

    g = golden("forward_eval.npz")
    d = cuda(g["rays_d"])
    for name in ("coarse", "fine"):
        B, S = g[f"{name}_t"].shape
        raw = torch.cat([cuda(g[f"{name}_raw_rgb"]).reshape(-1, 3), cuda(g[f"{name}_raw_sigma"]).reshape(-1, 1)], 1)
        raw = raw.contiguous()
        comp, acc = torch.empty((B, 3), device="cuda"), torch.empty((B,), device="cuda")
        w, depth = torch.empty((B, S), device="cuda"), torch.empty((B,), device="cuda")
        t_d = cuda(g[f"{name}_t"])  # keep device operands alive until the kernel has run
        L.call("aon_composite_fwd", L.ptr(raw), 4, L.ptr(raw[:, 3:]), 4, L.ptr(t_d),
               L.ptr(d), B, S, 1, L.ACT_VANILLA, L.ptr(comp), L.ptr(acc), L.ptr(w), L.ptr(depth),
               L.stream())
        torch.cuda.synchronize()
        for k, v in (("rgb", comp), ("acc", acc), ("weights", w), ("depth", depth)):
            report(f"{name} composite {k}", npy(v), g[f"{name}_{k}"], 1e-7)
            tol = 1e-5 if k == "depth" else 1e-6  # depth ~ 2..6: a few fp32 ulps
            np.testing.assert_allclose(npy(v), g[f"{name}_{k}"], rtol=0, atol=tol, err_msg=f"{name} {k}")


COMP_S = [1, 2, 3, 5, 7, 8, 9, 17, 33, 63, 64, 65, 100, 128, 129, 193, 255, 256, 257, 385, 448, 512]


@pytest.mark.parametrize("layout", ["raw4", "split"])
def test_composite_sample_counts(layout):
    """Every block count (S = 1..512) and both operand layouts: the weights against the oracle,
    and the per-ray sums bit-for-bit equal to torch CPU's sums of the GPU's own weights (the
    reduction order is the reference's, so given equal weights the sums round identically)."""
    from aonerf import _lib as L

    g = torch.Generator().manual_seed(7)
    B = 96
    for S in COMP_S:
        t = torch.sort(2.0 + 4.0 * torch.rand((B, S), generator=g), -1).values
        rgb = torch.rand((B, S, 3), generator=g)
        sigma = 3.0 * torch.rand((B, S, 1), generator=g)
        dirs = torch.randn((B, 3), generator=g)
        dirs[:4] = 0.0  # zero-length directions: dists * 0
        dirs = dirs.contiguous()
        if layout == "raw4":
            raw = cuda(torch.cat([rgb, sigma], -1).reshape(-1, 4))
            prgb, srgb, psig, ssig = L.ptr(raw), 4, L.ptr(raw[:, 3:]), 4
        else:
            rgb_d, sig_d = cuda(rgb), cuda(sigma)
            prgb, srgb, psig, ssig = L.ptr(rgb_d), 3, L.ptr(sig_d), 1
        comp, acc = torch.empty((B, 3), device="cuda"), torch.empty((B,), device="cuda")
        w, depth = torch.empty((B, S), device="cuda"), torch.empty((B,), device="cuda")
        t_d, dirs_d = cuda(t), cuda(dirs)  # keep device operands alive until the kernel has run
        L.call("aon_composite_fwd", prgb, srgb, psig, ssig, L.ptr(t_d), L.ptr(dirs_d), B, S,
               0, L.ACT_NONE, L.ptr(comp), L.ptr(acc), L.ptr(w), L.ptr(depth), L.stream())
        torch.cuda.synchronize()
        _, _, w_ref, _ = O.volumetric_rendering(rgb, sigma, t, dirs, False)
        np.testing.assert_allclose(npy(w), w_ref.numpy(), rtol=0, atol=1e-6, err_msg=f"S={S} weights")
        wc = w.cpu()
        np.testing.assert_array_equal(npy(acc), wc.sum(-1).numpy(), err_msg=f"S={S} acc")
        np.testing.assert_array_equal(npy(depth), (wc * t).sum(-1).numpy(), err_msg=f"S={S} depth")
        np.testing.assert_array_equal(npy(comp), (wc[..., None] * rgb).sum(-2).numpy(),
                                      err_msg=f"S={S} rgb")


def test_ray_loop_equals_one_ray_per_wave():
    """The compositor and the pdf sampler cap their grids at 65,536 workgroups (262,144 waves)
    and loop: a 270,000-ray launch, where some waves take two rays, must equal launches of 900
    rays (one ray per wave) bit for bit, and a slice of it the oracle."""
    from aonerf import _lib as L
    from aonerf import helper

    g = torch.Generator().manual_seed(11)
    B, S, Sc = 270000, 65, 65
    t = torch.sort(2.0 + 4.0 * torch.rand((B, S), generator=g), -1).values
    raw = torch.cat([torch.rand((B, S, 3), generator=g), 3.0 * torch.rand((B, S, 1), generator=g)],
                    -1).reshape(-1, 4)
    dirs = torch.nn.functional.normalize(torch.randn((B, 3), generator=g), dim=-1)
    raw_d, t_d, dirs_d = cuda(raw), cuda(t), cuda(dirs)

    def composite(lo, hi):
        n = hi - lo
        outs = [torch.empty(s, device="cuda") for s in ((n, 3), (n,), (n, S), (n,))]
        L.call("aon_composite_fwd", L.ptr(raw_d[lo * S:]), 4, L.ptr(raw_d[lo * S:, 3:]), 4,
               L.ptr(t_d[lo:]), L.ptr(dirs_d[lo:]), n, S, 1, L.ACT_VANILLA,
               *[L.ptr(o) for o in outs], L.stream())
        return outs

    whole = composite(0, B)
    parts = [composite(lo, min(lo + 900, B)) for lo in range(0, B, 900)]
    torch.cuda.synchronize()
    for k, name in enumerate(("rgb", "acc", "weights", "depth")):
        assert torch.equal(whole[k], torch.cat([p[k] for p in parts])), f"composite {name}"
    rgb_c = torch.sigmoid(raw[:512 * S, :3].reshape(512, S, 3))
    sig_c = torch.relu(raw[:512 * S, 3:].reshape(512, S, 1))
    _, _, w_ref, _ = O.volumetric_rendering(rgb_c, sig_c, t[:512], dirs[:512], True)
    np.testing.assert_allclose(npy(whole[2][:512]), w_ref.numpy(), rtol=0, atol=1e-6)

    tc = cuda(torch.sort(2.0 + 4.0 * torch.rand((B, Sc), generator=g), -1).values)
    wc = cuda(torch.rand((B, Sc), generator=g) * (torch.rand((B, Sc), generator=g) > 0.3))
    u = cuda(torch.rand((B, 128), generator=g))
    o, d = cuda(torch.randn((B, 3), generator=g)), dirs_d
    mids = 0.5 * (tc[..., 1:] + tc[..., :-1])
    for rnd in (False, True):
        uu = u if rnd else None
        t_all, x_all = helper.sample_pdf(mids, wc[..., 1:-1], o, d, tc, 128, rnd, u=uu)
        chunks = [helper.sample_pdf(mids[lo:lo + 900], wc[lo:lo + 900, 1:-1], o[lo:lo + 900],
                                    d[lo:lo + 900], tc[lo:lo + 900], 128, rnd,
                                    u=None if uu is None else uu[lo:lo + 900])
                  for lo in range(0, B, 900)]
        torch.cuda.synchronize()
        assert torch.equal(t_all, torch.cat([c[0] for c in chunks])), f"pdf t (randomized={rnd})"
        assert torch.equal(x_all, torch.cat([c[1] for c in chunks])), f"pdf xyz (randomized={rnd})"
        t_ref, _ = O.sample_pdf(mids[:256].cpu(), wc[:256, 1:-1].cpu(), o[:256].cpu(),
                                d[:256].cpu(), tc[:256].cpu(), 128, rnd,
                                **({"u": u[:256].cpu()} if rnd else {}))
        np.testing.assert_array_equal(npy(t_all[:256]), t_ref.numpy())


def test_render_replays_from_a_graph():
    """The C ABI neither allocates nor synchronises (include/aonerf.h), so a whole two-level
    render -- ray generation, both MLP levels, compositing, pdf resampling -- captures into one
    HIP graph; its replay equals the eager launches bit for bit."""
    from aonerf.ray_utils import frame_rays
    from aonerf.render import create_spheric_poses, sapien_focal

    net = make_nerf("f16x3")
    H, Wd = 24, 40
    c2w = create_spheric_poses(4.0)[3]

    def render():
        rays = frame_rays(c2w, H, Wd, sapien_focal(H))
        out = net(rays, False, True, 2.0, 6.0)
        return torch.cat([out[1][0], out[1][1][:, None], out[1][2][:, None]], -1)

    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):  # warm-up: schedules cached, workspace sizes and grids known
        eager = render()
        render()
    torch.cuda.current_stream().wait_stream(st)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        captured = render()
    for _ in range(2):
        captured.zero_()
        graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(captured, eager)


def test_pdf_edges(golden):
    from aonerf import helper

    g = golden("pdf_edges.npz")
    bins, w = cuda(g["bins"]), cuda(g["weights"])
    for ns in (128, 16):
        s = helper.sorted_piecewise_constant_pdf(bins, w, ns, False)
        report(f"pdf eval{ns}", npy(s), g[f"eval{ns}_samples"], 0)
        np.testing.assert_allclose(npy(s), g[f"eval{ns}_samples"], rtol=0, atol=1e-5)
        s = helper.sorted_piecewise_constant_pdf(bins, w, ns, True, u=cuda(g[f"rand{ns}_u"]))
        report(f"pdf rand{ns}", npy(s), g[f"rand{ns}_samples"], 0)
        np.testing.assert_allclose(npy(s), g[f"rand{ns}_samples"], rtol=0, atol=1e-5)
    t, xyz = helper.sample_pdf(bins, w, cuda(g["sp_o"]), cuda(g["sp_d"]), cuda(g["sp_tc"]), 128, True,
                               u=cuda(g["sp_u"]))
    np.testing.assert_allclose(npy(t), g["sp_t"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(npy(xyz), g["sp_xyz"], rtol=0, atol=1e-5)
    assert np.all(np.diff(npy(t), axis=-1) >= 0)
    t, _ = helper.sample_pdf(bins, w, cuda(g["sp_o"]), cuda(g["sp_d"]), cuda(g["sp_tc"]), 128, False)
    np.testing.assert_allclose(npy(t), g["spe_t"], rtol=0, atol=1e-5)


def test_fine_t_from_reference_weights(golden):
    """Stage-isolated hierarchical sampling: reference coarse t + weights -> fine t."""
    from aonerf import helper

    g = golden("forward_eval.npz")
    tc = cuda(g["coarse_t"])
    mids = 0.5 * (tc[..., 1:] + tc[..., :-1])
    t, _ = helper.sample_pdf(mids, cuda(g["coarse_weights"])[..., 1:-1], cuda(g["rays_o"]),
                             cuda(g["rays_d"]), tc, 128, False)
    err = report("fine t (eval)", npy(t), g["fine_t"], 0)
    np.testing.assert_allclose(npy(t), g["fine_t"], rtol=0, atol=1e-5)
    assert (err == 0).mean() > 0.99


def test_mlp_from_reference_inputs(golden, nerf):
    """Stage-isolated MLP: reference t per level -> raw rgb / sigma (fp32 MFMA)."""
    g = golden("forward_eval.npz")
    rays = rays_of(g)
    for name, mlp in (("coarse", nerf.coarse_mlp), ("fine", nerf.fine_mlp)):
        t = cuda(g[f"{name}_t"])
        raw = npy(mlp.forward_rays(rays["rays_o"], rays["rays_d"], rays["viewdirs"], t))
        B, S = t.shape
        report(f"{name} raw_rgb", raw[:, :3], g[f"{name}_raw_rgb"].reshape(-1, 3), 1e-6)
        report(f"{name} raw_sigma", raw[:, 3], g[f"{name}_raw_sigma"].reshape(-1), 1e-6)
        np.testing.assert_allclose(raw[:, :3], g[f"{name}_raw_rgb"].reshape(-1, 3), rtol=0, atol=1e-5)
        np.testing.assert_allclose(raw[:, 3], g[f"{name}_raw_sigma"].reshape(-1), rtol=0, atol=1e-5)
        # fused epilogue activations (model.py:186-187) == torch's sigmoid / relu of the raw
        from aonerf import _lib as L

        act = npy(mlp.forward_rays(rays["rays_o"], rays["rays_d"], rays["viewdirs"], t, act=L.ACT_VANILLA))
        raw_t = torch.from_numpy(raw)
        np.testing.assert_allclose(act[:, :3], torch.sigmoid(raw_t[:, :3]).numpy(), rtol=0, atol=1.2e-7)
        np.testing.assert_array_equal(act[:, 3], torch.relu(raw_t[:, 3]).numpy())


def test_mlp_encoded_api(golden, nerf):
    """NeRFMLP.forward(x, condition) on pre-encoded inputs (model.py:95-120)."""
    g = golden("forward_eval.npz")
    t = torch.from_numpy(g["coarse_t"])
    xyz = O.cast_rays(t, torch.from_numpy(g["rays_o"]), torch.from_numpy(g["rays_d"]))
    enc = O.pos_enc(xyz, 0, 10)
    venc = O.pos_enc(torch.from_numpy(g["viewdirs"]), 0, 4)
    raw_rgb, raw_sigma = nerf.coarse_mlp(enc.cuda(), venc.cuda())
    np.testing.assert_allclose(npy(raw_rgb), g["coarse_raw_rgb"], rtol=0, atol=1e-5)
    np.testing.assert_allclose(npy(raw_sigma), g["coarse_raw_sigma"], rtol=0, atol=1e-5)


# ----------------------------------------------------------------------------- end to end
def check_levels(ret, g, fine_ref, randomized=False, white=True):
    att = Attribution(npy(ret[0][3]), g["coarse_weights"], 128, randomized,
                      g["u_fine"] if randomized else None)
    rc = {k: torch.from_numpy(g[k]) for k in ("rays_o", "rays_d", "viewdirs")}
    uk = dict(randomized=True, u_coarse=g["u_coarse"], u_fine=g["u_fine"]) if randomized else {}
    floors = self_floors(O.split_state_dict(W.nerf_state_dict(0)), rc,
                         [g["fine_rgb"], g["fine_acc"], g["fine_depth"]], white_bkgd=white, **uk)
    for lv, name in enumerate(("coarse", "fine")):
        for j, k in enumerate(("rgb", "acc", "depth", "weights")):
            err = report(f"e2e {name} {k}", npy(ret[lv][j]), g[f"{name}_{k}"], E2E_ATOL)
            if name == "coarse":  # no resampling upstream: every ray within 1e-4
                assert err.max() <= E2E_ATOL, f"coarse {k}: {err.max():.3e}"
            else:
                attrib = att.rays(fine_ref[k], g[f"fine_{k}"], err, g[f"env_fine_{k}"])
                att.explain(f"fine {k}", err, attrib)
                assert_e2e(f"fine {k}", err, g[f"env_fine_{k}"], attrib,
                           floors.get(k, floors["depth"]))


def golden_coarse(g):
    return tuple(g[f"coarse_{k}"] for k in ("rgb", "acc", "depth", "weights"))


def test_forward_eval_end_to_end(golden, nerf):
    g = golden("forward_eval.npz")
    params = O.split_state_dict(W.nerf_state_dict(0))
    ret, fine_ref = check_chain(nerf, rays_of(g), params, coarse_ref=golden_coarse(g), return_ref=True)
    check_levels(ret, g, fine_ref)


def test_forward_randomized_end_to_end(golden, nerf):
    g = golden("forward_random.npz")
    params = O.split_state_dict(W.nerf_state_dict(0))
    ret, fine_ref = check_chain(nerf, rays_of(g), params, randomized=True, white=False,
                                u_coarse=cuda(g["u_coarse"]), u_fine=cuda(g["u_fine"]),
                                coarse_ref=golden_coarse(g), return_ref=True)
    check_levels(ret, g, fine_ref, randomized=True, white=False)


_FLOORS = {}


def _frame_floors(g, tag, params, rc, nc):
    """self_floors of a golden frame (cached: both precisions gate against the same floors)."""
    if tag not in _FLOORS:
        _FLOORS[tag] = self_floors(params, rc, [g[f"{tag}_comp_rgb"], g[f"{tag}_acc"],
                                                g[f"{tag}_depth"]], num_coarse_samples=nc)
    return _FLOORS[tag]


@pytest.mark.parametrize("precision", PRECISIONS)
def test_render_frame_chunks(golden, precision):
    """render_rays chunk loop and config C1 (64x64, 32 coarse samples) from c2w alone."""
    from aonerf.render import render_frame, render_rays
    from aonerf.ray_utils import frame_rays

    g = golden("render_frame.npz")
    params = O.split_state_dict(W.nerf_state_dict(0))
    for tag in ("a", "c1"):
        H, Wd, nc, chunk = (int(x) for x in g[f"{tag}_hw"])
        net = make_nerf(precision, num_coarse_samples=nc)
        c2w = torch.from_numpy(g[f"{tag}_c2w"])
        rays = frame_rays(c2w, H, Wd, float(g[f"{tag}_focal"]))
        ret, fine_ref = check_chain(net, rays, params, return_ref=True)
        # the reference's coarse weights on these rays: the oracle's coarse level (pinned to the
        # reference by test_oracle_golden.py) on the same coarse samples (bit-exact, a3)
        rc = {k: v.cpu() for k, v in rays.items()}
        w_ref = O.render_level(params, rc, ret[0][4]["t_vals"].cpu(), 0, True)[2]
        att = Attribution(npy(ret[0][3]), w_ref.numpy(), net.num_fine_samples)
        floors = _frame_floors(g, tag, params, rc, nc)
        out = render_rays(net, rays, chunk, True, 2.0, 6.0)
        for k in ("comp_rgb", "acc", "depth"):
            err = report(f"frame {tag} {k}", npy(out[k]), g[f"{tag}_{k}"], E2E_ATOL)
            attrib = att.rays(fine_ref["rgb" if k == "comp_rgb" else k], g[f"{tag}_{k}"], err,
                              g[f"{tag}_env_{k}"])
            att.explain(f"frame {tag} {k}", err, attrib)
            assert_e2e(f"frame {tag} {k}", err, g[f"{tag}_env_{k}"], attrib,
                       floors["rgb" if k == "comp_rgb" else k])
        full = render_frame(net, c2w, H, Wd, float(g[f"{tag}_focal"]))
        np.testing.assert_array_equal(npy(full[:, :3]), npy(out["comp_rgb"]))


@pytest.mark.parametrize("precision", PRECISIONS)
def test_psnr_delta(golden, precision):
    """PSNR of the GPU render vs the reference render, both against one synthetic target."""
    g = golden("render_frame.npz")
    from aonerf.render import render_frame

    H, Wd = (int(x) for x in g["c1_hw"][:2])
    net = make_nerf(precision, num_coarse_samples=32)
    out = render_frame(net, torch.from_numpy(g["c1_c2w"]), H, Wd, float(g["c1_focal"]))
    target = torch.from_numpy(np.random.Generator(np.random.PCG64(3)).uniform(0, 1, (H * Wd, 3)).astype(np.float32))
    p_gpu = O.psnr_each([out[:, :3].cpu()], [target]).item()
    p_ref = O.psnr_each([torch.from_numpy(g["c1_comp_rgb"])], [target]).item()
    print(f"PSNR gpu {p_gpu:.4f} ref {p_ref:.4f} delta {p_gpu - p_ref:+.2e} dB")
    assert abs(p_gpu - p_ref) <= 0.05


# ----------------------------------------------------------------------------- option paths
@pytest.mark.parametrize("precision", PRECISIONS)
def test_lindisp(golden, precision):
    """NeRF(lindisp=True) (helper.py:117-118): the coarse schedule linear in disparity equals the
    reference's bit for bit, and the two-level chain holds every link at 1e-4."""
    g = golden("forward_eval.npz")
    params = O.split_state_dict(W.nerf_state_dict(0))
    rays = rays_of(g)
    net = make_nerf(precision, lindisp=True)
    ret = check_chain(net, rays, params)
    t_ref, _ = O.sample_along_rays(torch.from_numpy(g["rays_o"]), torch.from_numpy(g["rays_d"]),
                                   64, 2.0, 6.0, False, True)
    np.testing.assert_array_equal(npy(ret[0][4]["t_vals"]), t_ref.numpy())
    assert not np.array_equal(t_ref.numpy(), g["coarse_t"])  # the option changed the schedule


@pytest.mark.parametrize("nf", [300, 447])
def test_large_num_fine_samples(golden, nf):
    """N_importance beyond the fused march kernel's 256 (up to 447: the fine level's 65 + N samples within aon_composite_fwd's 512): the render
    takes aon_composite_fwd + aon_sample_pdf (model.march_ok) for both NeRF and NeRF_AE_Art,
    and the vanilla two-level chain holds every link at 1e-4 (fine t bit-exact)."""
    from aonerf import model as M

    assert not M.march_ok(65, nf) and M.march_ok(65, 256)
    g = golden("forward_eval.npz")
    params = O.split_state_dict(W.nerf_state_dict(0))
    rays = rays_of(g)
    ret = check_chain(make_nerf("f16x3", num_fine_samples=nf), rays, params)
    assert ret[1][4]["t_vals"].shape[1] == 65 + nf
    from aonerf.model_autodecoder import NeRF_AE_Art
    from aonerf.synthetic import art_latents, init_like_reference

    art = init_like_reference(NeRF_AE_Art(num_fine_samples=nf)).cuda().requires_grad_(False)
    out = art(rays, False, True, 2.0, 6.0, art_latents(0, device="cuda"), return_intermediates=True)
    assert out[1][3]["t_vals"].shape[1] == 65 + nf and torch.isfinite(out[1][0]).all()


@pytest.mark.parametrize("path", ["render", "train"])
@pytest.mark.parametrize("precision", PRECISIONS)
def test_density_noise(golden, precision, path):
    """noise_std > 0 in randomized mode (model.py:183-184): raw_sigma += U[0,1) * noise_std
    before the ReLU, drawn from torch's CUDA generator in the reference's order (level 0's B*S
    draws, then level 1's).  Both the fused inference path (noise added to the raw output, the
    activations moved to the compositor) and the training path (noise added in the training
    kernel's epilogue) against the oracle fed the same draws, every level within 1e-4."""
    if path == "train" and precision == "fp32":
        pytest.skip("the training kernels are f16x3")
    g = golden("forward_random.npz")
    params = O.split_state_dict(W.nerf_state_dict(0))
    rays = rays_of(g)
    B = rays["rays_o"].shape[0]
    net = make_nerf(precision, noise_std=1.0)
    kw = dict(u_coarse=cuda(g["u_coarse"]), u_fine=cuda(g["u_fine"]), return_weights=True,
              return_intermediates=True)
    if path == "train":
        net.requires_grad_(True)
    torch.manual_seed(1234)
    with torch.set_grad_enabled(path == "train"):
        ret = net(rays, True, False, 2.0, 6.0, **kw)
    torch.manual_seed(1234)
    draws = [torch.rand((B * 65,), device="cuda"), torch.rand((B * 193,), device="cuda")]
    rc = {k: v.cpu() for k, v in rays.items()}
    for level in range(2):
        t = ret[level][4]["t_vals"].cpu()
        S = t.shape[1]
        samples = O.cast_rays(t, rc["rays_o"], rc["rays_d"])
        raw_rgb, raw_sigma = O.mlp_forward(params[level], O.pos_enc(samples, 0, 10),
                                           O.pos_enc(rc["viewdirs"], 0, 4))
        raw_sigma = raw_sigma + draws[level].cpu().view(B, S, 1) * 1.0
        comp, acc, w, depth = O.volumetric_rendering(torch.sigmoid(raw_rgb), torch.relu(raw_sigma),
                                                     t, rc["rays_d"], False)
        for j, (k, want) in enumerate((("rgb", comp), ("acc", acc), ("depth", depth), ("weights", w))):
            err = report(f"noise {path} level {level} {k}", npy(ret[level][j]), want.numpy(), E2E_ATOL)
            assert err.max() <= E2E_ATOL, (level, k)
    quiet = make_nerf(precision)
    with torch.no_grad():
        ret0 = quiet(rays, True, False, 2.0, 6.0, u_coarse=cuda(g["u_coarse"]), u_fine=cuda(g["u_fine"]))
    assert not torch.equal(ret0[0][0], ret[0][0].detach())  # the noise was applied


# ----------------------------------------------------------------------------- full size
FULL_FRAME_CHUNK = 3840  # one reference chunk (opt.py:103)
FULL_FRAME_CHUNKS = 4    # the central 15,360 rays of the frame (the object region)


_FULL_FRAME_REF = {}


def test_full_frame_properties(nerf):
    """640x480x(64c+128f), the bench frame: invariants at full size, then the reference on the
    central 4 x 3,840 rays of it (verdict r04 #1, r05 #1) -- on IDENTICAL rays: the oracle gets
    the GPU's own rays (a1/a2 are bit-exact against the reference's golden rays,
    test_ray_generation; the oracle re-run on this box's CPU may round a direction 1 ulp
    differently through its BLAS, a different input).  Every link of the chain gated at 1e-4 on
    every ray of one chunk; then the direct end-to-end comparison on all four: the fraction
    within 1e-4 at least the reference's own self-consistency on these rays (self_floors), every
    outlier attributed -- plateau flip, amplification, or within the reference's own
    implementation envelope on that ray (oracle/attribution.py)."""
    from aonerf.ray_utils import frame_rays
    from aonerf.render import create_spheric_poses, render_frame, sapien_focal

    H, Wd = 480, 640
    c2w = create_spheric_poses(4.0)[7]
    f = sapien_focal(H)
    out = render_frame(nerf, c2w, H, Wd, f)
    out2 = render_frame(nerf, c2w, H, Wd, f)
    torch.cuda.synchronize()
    assert torch.equal(out, out2), "render is not deterministic"
    o = npy(out)
    assert np.isfinite(o).all()
    acc = o[:, 4]
    assert (acc >= -1e-6).all() and (acc <= 1 + 1e-5).all()
    # bands rendered separately == full frame, bit for bit (per-ray independence)
    half = render_frame(nerf, c2w, H, Wd, f, p0=123 * Wd, n=7 * Wd)
    np.testing.assert_array_equal(npy(half), o[123 * Wd:130 * Wd])
    n = FULL_FRAME_CHUNK * FULL_FRAME_CHUNKS
    p0 = (H * Wd) // 2 - n // 2
    sel = np.arange(p0, p0 + n)
    gr = frame_rays(c2w, H, Wd, f, p0=int(p0), n=n)
    rc = {k: v.cpu() for k, v in gr.items()}
    dirs = O.get_ray_directions(H, Wd, f)
    _, _, rd_cpu = O.get_rays(dirs, c2w[:3, :4], True)
    dd = np.abs(npy(gr["rays_d"]).astype(np.float64) - rd_cpu[sel].numpy())
    print(f"640x480 rays_d: {int((dd > 0).any(-1).sum())} of {n} rays differ from this CPU's "
          f"torch by <= {dd.max():.2e} (the oracle below takes the GPU's rays)")
    assert dd.max() <= 1.2e-7
    params = O.split_state_dict(W.nerf_state_dict(0))
    # every link at 1e-4 on the first chunk
    c0 = {k: v[:FULL_FRAME_CHUNK] for k, v in gr.items()}
    got_c0 = check_chain(nerf, c0, params)
    np.testing.assert_array_equal(npy(got_c0[1][0]), o[sel[:FULL_FRAME_CHUNK]][:, :3])
    # the reference end to end on the four chunks, its coarse weights and its self-consistency
    # (the same rays for both MLP precisions: computed once per session)
    key = (int(p0), n, hashlib.sha256(npy(gr["rays_d"]).tobytes()).hexdigest())
    if key not in _FULL_FRAME_REF:
        ref_rgb, ref_acc, ref_depth, w_ref = [], [], [], []
        with torch.no_grad():
            for i in range(0, n, FULL_FRAME_CHUNK):
                r, inter = O.nerf_forward(params, {k: v[i:i + FULL_FRAME_CHUNK] for k, v in rc.items()},
                                          False, True, 2.0, 6.0, return_intermediates=True)
                ref_rgb.append(r[1][0])
                ref_acc.append(r[1][1])
                ref_depth.append(r[1][2])
                w_ref.append(inter[0]["weights"])
        ref = [torch.cat(x).numpy() for x in (ref_rgb, ref_acc, ref_depth)]
        _FULL_FRAME_REF[key] = (ref, torch.cat(w_ref).numpy(), self_floors(params, rc, ref))
    ref, w_ref, floors = _FULL_FRAME_REF[key]
    with torch.no_grad():
        mine = nerf(gr, False, True, 2.0, 6.0, return_weights=True, return_intermediates=True)
    for j in range(3):
        np.testing.assert_array_equal(npy(mine[1][j]), o[sel][:, (slice(0, 3), 4, 3)[j]])
    att = Attribution(npy(mine[0][3]), w_ref, nerf.num_fine_samples)
    cols = {0: slice(0, 3), 1: 4, 2: 3}
    errs = {j: report(f"640x480 {k}", o[sel][:, cols[j]], ref[j], E2E_ATOL)
            for j, k in ((0, "rgb"), (1, "acc"), (2, "depth"))}
    bad = np.zeros(n, bool)
    for e in errs.values():
        bad |= (e > E2E_ATOL).reshape(len(e), -1).any(-1)
    rows = np.nonzero(bad)[0]
    env = [None] * 3
    on_ours = [np.zeros((n, 3)), np.zeros(n), np.zeros(n)]
    if len(rows):  # the reference at our fine samples and its envelope, on the outliers only
        sub = {k: v[rows] for k, v in rc.items()}
        t_f = mine[1][4]["t_vals"].cpu()[rows]
        fr = O.render_level(params, sub, t_f, 1, True)
        for j, jj in ((0, 0), (1, 1), (2, 3)):
            on_ours[j][rows] = fr[jj].numpy()
        part, worst = fine_envelope(params, sub)
        env = [np.zeros((n,) + x.shape[1:]) for x in part]
        for full, x in zip(env, part):
            full[rows] = x
        print(f"  reference implementation envelope on the {len(rows)} outlier rays (max): " +
              ", ".join(f"{nm}/{q}: {v:.1e}" for (nm, q), v in sorted(worst.items())))
    for j, k in ((0, "rgb"), (2, "depth"), (1, "acc")):
        err = errs[j]
        attrib = att.rays(on_ours[j], ref[j], err, env[j])
        att.explain(f"640x480 {k}", err, attrib)
        assert_e2e(f"640x480 {k}", err, env[j], attrib, floors[k])


# ----------------------------------------------------------------------------- fused march
MARCH_CASES = [(65, 128), (33, 128), (65, 16), (100, 64), (129, 128), (200, 50), (3, 1)]


@pytest.mark.parametrize("S,Ns", MARCH_CASES)
def test_composite_march_equals_two_kernels(S, Ns):
    """aon_composite_march (coarse compositing + sample_pdf on mids / weights[1:-1] + merge, one
    kernel: helper.py:157-252, model.py:163-172) equals aon_composite_fwd followed by
    aon_sample_pdf bit for bit -- every output, eval (one shared u row) and randomized (per-ray u,
    unsorted), with and without the weights output, every activation mode, white on and off;
    plus the fine t against the oracle's sample_pdf on the GPU's own weights."""
    from aonerf import _lib as L
    from aonerf import helper

    g = torch.Generator().manual_seed(S * 1000 + Ns)
    B = 701  # ragged for the four-rays-per-wave kernel (S = 65, Ns = 128)
    t = torch.sort(2.0 + 4.0 * torch.rand((B, S), generator=g), -1).values
    raw = torch.cat([torch.randn((B, S, 3), generator=g),
                     3.0 * torch.randn((B, S, 1), generator=g)], -1).reshape(-1, 4)
    raw[: 5 * S, 3] = -1.0  # rays of zero density: all-zero weights, the eps padding
    dirs = torch.randn((B, 3), generator=g)
    raw_d, t_d, dirs_d = cuda(raw), cuda(t), cuda(dirs)
    for rnd in (False, True):
        if rnd:
            # per-ray u; every third row sorted, so waves mix rays that need the sort and rays
            # that do not
            ur = torch.rand((B, Ns), generator=g)
            ur[::3] = ur[::3].sort(-1).values
            u, us = cuda(ur), Ns
        else:
            u, us = helper.eval_u(Ns, "cuda"), 0
        for act, white, keep_w in ((L.ACT_VANILLA, 1, True), (L.ACT_ARTIC, 0, False),
                                   (L.ACT_VANILLA, 0, False)):
            two = [torch.empty(s, device="cuda") for s in ((B, 3), (B,), (B, S), (B,))]
            L.call("aon_composite_fwd", L.ptr(raw_d), 4, L.ptr(raw_d[:, 3:]), 4, L.ptr(t_d),
                   L.ptr(dirs_d), B, S, white, act, *[L.ptr(o) for o in two], L.stream())
            t2 = torch.empty((B, S + Ns), device="cuda")
            L.call("aon_sample_pdf", None, 0, L.ptr(two[2][:, 1:]), S, B, S - 1, Ns, L.ptr(u), us,
                   L.ptr(t_d), S, None, None, L.ptr(t2), None, L.stream())
            one = [torch.empty(s, device="cuda") for s in ((B, 3), (B,), (B, S), (B,))]
            t1 = torch.empty((B, S + Ns), device="cuda")
            L.call("aon_composite_march", L.ptr(raw_d), L.ptr(t_d), L.ptr(dirs_d), B, S, white,
                   act, L.ptr(u), us, Ns, L.ptr(one[0]), L.ptr(one[1]),
                   L.ptr(one[2]) if keep_w else None, L.ptr(one[3]), L.ptr(t1), L.stream())
            torch.cuda.synchronize()
            for k, (a, b) in enumerate(zip(one, two)):
                if k == 2 and not keep_w:
                    continue
                assert torch.equal(a, b), f"S={S} Ns={Ns} rnd={rnd} act={act} output {k}"
            assert torch.equal(t1, t2), f"S={S} Ns={Ns} rnd={rnd} act={act} fine t"
        w = two[2].cpu()
        mids = 0.5 * (t[..., 1:] + t[..., :-1])
        t_ref, _ = O.sample_pdf(mids[:64], w[:64, 1:-1], torch.zeros(64, 3), dirs[:64], t[:64], Ns,
                                rnd, **({"u": u[:64].cpu()} if rnd else {}))
        np.testing.assert_array_equal(npy(t1[:64]), t_ref.numpy())


@pytest.mark.parametrize("B,S,Ns", [(600000, 65, 128), (270000, 65, 96)])
def test_composite_march_ray_loop(B, S, Ns):
    """The fused kernels' grids cap at 65,536 workgroups and loop: k_march_rows
    (S = 65, Ns = 128: 8 rays per workgroup) loops only past 524,288 rays -- an 800x800 frame --
    so it runs at 600,000 rays; the one-ray-per-wave k_composite_march (any other shape) at
    270,000.  Each whole launch equals 900-ray launches bit for bit."""
    from aonerf import _lib as L
    from aonerf import helper

    g = torch.Generator().manual_seed(5)
    t = cuda(torch.sort(2.0 + 4.0 * torch.rand((B, S), generator=g), -1).values)
    raw = cuda(torch.cat([torch.rand((B, S, 3), generator=g), 3.0 * torch.rand((B, S, 1), generator=g)],
                         -1).reshape(-1, 4))
    dirs = cuda(torch.nn.functional.normalize(torch.randn((B, 3), generator=g), dim=-1))
    u = helper.eval_u(Ns, "cuda")

    def run(lo, hi):
        n = hi - lo
        outs = [torch.empty(s, device="cuda") for s in ((n, 3), (n,), (n,), (n, S + Ns))]
        L.call("aon_composite_march", L.ptr(raw[lo * S:]), L.ptr(t[lo:]), L.ptr(dirs[lo:]), n, S, 1,
               L.ACT_VANILLA, L.ptr(u), 0, Ns, L.ptr(outs[0]), L.ptr(outs[1]), None, L.ptr(outs[2]),
               L.ptr(outs[3]), L.stream())
        return outs

    whole = run(0, B)
    parts = [run(lo, min(lo + 900, B)) for lo in range(0, B, 900)]
    torch.cuda.synchronize()
    for k in range(4):
        assert torch.equal(whole[k], torch.cat([p[k] for p in parts])), k


@pytest.mark.parametrize("precision", PRECISIONS)
def test_render_fused_march_equals_unfused(golden, precision):
    """NeRF.forward with the fused coarse composite + resample (the model's fused_march) equals
    the two-kernel path bit for bit, eval and randomized."""
    g = golden("forward_random.npz")
    net = make_nerf(precision)
    rays = rays_of(g)
    outs = {}
    for fused in (True, False):
        net.fused_march = fused
        outs[fused] = [net(rays, False, True, 2.0, 6.0),
                       net(rays, True, False, 2.0, 6.0, u_coarse=cuda(g["u_coarse"]),
                           u_fine=cuda(g["u_fine"]))]
    for a, b in zip(outs[True], outs[False]):
        for la, lb in zip(a, b):
            for x, y in zip(la, lb):
                assert torch.equal(x, y)
