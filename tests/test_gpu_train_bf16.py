"""The bf16 training mode (BASELINE config C5: "training step fwd+bwd through volume renderer,
bf16"; NeRF(train_precision="bf16")): one bf16 MFMA per product in the fused training forward
(aon_mlp_fwd_train_bf16), the fused backward chain (aon_mlp_bwd_bf16) and the weight-gradient
GEMMs (aon_gemm mma_bf16), activations and gradients kept as bf16; compositing, the loss, their
backward and Adam stay fp32 on fp32 master weights.

bf16 carries 8 significant bits, so the gates are bf16-sized; the mode is judged step by step
against the fp32 reference, teacher-forced, in tests/test_gpu_teacher_forced.py.
"""
import numpy as np
import pytest
import torch

from oracle import nerf_oracle as O
from oracle import weights as W
from test_gpu_train import _make_trainable, c5_batch, cuda, rel_err

pytestmark = pytest.mark.gpu


@pytest.fixture
def bf16_mode():
    """TrainNumerics fields of the bf16 mode (a per-model setting)."""
    return dict(precision="bf16")


def bf16_round(x):
    return x.to(torch.bfloat16).to(torch.float64)


@pytest.mark.parametrize("K,M,N,rdiv,a_bf,b_bf", [
    (70000, 256, 256, 1, True, True),     # a fine-level dW (split-K; the 256 x 256-tile kernel)
    (250003, 256, 256, 1, True, True),    # 256 K chunks with a ragged last k-tile
    (70000, 128, 256, 1, True, True),     # the 128 x 128-tile kernel
    (1000, 3, 128, 1, False, True),       # rgb_layer: dY = fp32 d raw (strided, 3 of 4 columns)
    (2000, 128, 27, 33, True, False),     # views_linear.0's enc_dir columns: B row k // S
    (517, 256, 63, 1, True, False),       # pts_linears.0: fp32 encodings (ld 63, scalar loads)
])
def test_bf16_weight_gradient_gemm(K, M, N, rdiv, a_bf, b_bf):
    """aon_gemm mma_bf16: C = A^T B (+ C) and rowsum(A) against fp64 products of the operands
    rounded to bf16 (bf16 x bf16 products are exact in fp32: only the fp32 accumulation
    differs), for bf16 and fp32 operands in the reduction-major layouts of the backward."""
    from aonerf.linalg import gemm

    g = torch.Generator(device="cuda").manual_seed(K + M)
    lda = 4 if M == 3 else M
    A_full = torch.randn((K, lda), device="cuda", generator=g) * 1e-3
    A = A_full[:, :M] if M == 3 else A_full
    Bst = torch.randn(((K + rdiv - 1) // rdiv, N), device="cuda", generator=g)
    Aop = A_full.to(torch.bfloat16) if a_bf else A_full
    Bop = Bst.to(torch.bfloat16) if b_bf else Bst
    C0 = torch.randn((M, N), device="cuda", generator=g)
    C = C0.clone()
    rs = torch.empty((M,), device="cuda")
    gemm(C, Aop, Bop, M, N, K, lda=lda, a_kc=False, ldb=N, b_kc=False, b_rdiv=rdiv, ldc=N,
         accumulate=True, rowsum=rs, mma_bf16=True)
    torch.cuda.synchronize()
    a64 = bf16_round(A.cpu())
    b64 = bf16_round(Bst.cpu())[torch.arange(K) // rdiv]
    want = C0.cpu().double() + a64.T @ b64
    err = rel_err(C.cpu().numpy(), want.numpy())
    print(f"bf16 dW K={K} M={M} N={N}: max-rel err {err:.2e}")
    assert err < 2e-5
    np.testing.assert_allclose(rs.cpu().numpy(), a64.sum(0).numpy(), rtol=0,
                               atol=2e-5 * float(a64.abs().sum(0).max()))


def test_bf16_train_step_c5(bf16_mode):
    """One C5 step (4,096 rays, randomized, injected uniforms) in the bf16 mode: the loss against
    the fp32 oracle at our sample positions within 3e-3 relative (measured 5e-4), every
    parameter's gradient teacher-forced against the fp32 oracle within 0.03 of its max
    (measured <= 1e-2) with cosine >= 0.999 (bf16 has 2^-8 resolution; the f16x3 mode meets
    1e-3 here, test_gpu_train.py)."""
    from aonerf import train

    net = _make_trainable(0, **bf16_mode)
    batch, u_c, u_f = c5_batch()
    ret = net(batch, True, True, 2.0, 6.0, u_coarse=u_c, u_fine=u_f, return_intermediates=True)
    loss = train.img2mse(ret[1][0], batch["target"]) + train.img2mse(ret[0][0], batch["target"])
    loss.backward()
    torch.cuda.synchronize()
    rays = {k: batch[k].cpu() for k in ("rays_o", "rays_d", "viewdirs")}
    params = [{k: v.requires_grad_(True) for k, v in p.items()}
              for p in O.split_state_dict(W.nerf_state_dict(0))]
    tgt = batch["target"].cpu()
    ref_loss = 0.0
    for level in range(2):
        t = ret[level][3]["t_vals"].cpu()
        comp, acc, w, depth = O.render_level(params, rays, t, level, True)
        ref_loss = ref_loss + O.img2mse(comp, tgt)
    ref_loss.backward()
    print(f"C5 bf16 loss gpu {loss.item():.6f}  fp32 oracle on our t {ref_loss.item():.6f}")
    np.testing.assert_allclose(loss.item(), ref_loss.item(), rtol=3e-3)
    named = dict(net.named_parameters())
    worst_e, worst_c = 0.0, 1.0
    for lv, pre in ((0, "coarse_mlp."), (1, "fine_mlp.")):
        for n, v in params[lv].items():
            want = v.grad.double().numpy()
            got = named[pre + n].grad.double().cpu().numpy()
            e = rel_err(got, want)
            cos = float((got * want).sum() / (np.linalg.norm(got) * np.linalg.norm(want) + 1e-300))
            worst_e, worst_c = max(worst_e, e), min(worst_c, cos)
            assert e < 0.03 and cos > 0.999, (pre + n, e, cos)
    print(f"C5 bf16 grads vs fp32 oracle: worst max-rel {worst_e:.2e}, worst cosine {worst_c:.5f}")


@pytest.mark.parametrize("mma_bf16,dtype", [(False, torch.float32), (True, torch.float32),
                                            (True, torch.bfloat16)])
@pytest.mark.parametrize("M", [128, 256])
def test_weight_gradient_gemm_tiled_operands(mma_bf16, dtype, M):
    """aon_gemm a_tiled / b_tiled: dW = dZ^T X read in place from the fused training kernels'
    16-row tiled layout (aonerf/tiles.py; 70,003 rows: a partial last block, split-K) is
    bit-identical to the same product on row-major copies -- the staged values and their
    order are the same.  M = 256 with bf16 operands: the 256 x 256-tile kernel
    (k_gemm_bf16_dma256)."""
    from aonerf import tiles
    from aonerf.linalg import gemm

    g = torch.Generator(device="cuda").manual_seed(11)
    K, N = 70003, 256
    A = (torch.randn((K, M), device="cuda", generator=g) * 1e-3).to(dtype)
    B = torch.randn((K, N), device="cuda", generator=g).to(dtype)
    At, Bt = tiles.tile(A), tiles.tile(B)
    out = []
    for a, b, tiled in ((A, B, False), (At, Bt, True)):
        C = torch.zeros((M, N), device="cuda")
        rs = torch.empty((M,), device="cuda")
        gemm(C, a, b, M, N, K, lda=M, a_kc=False, ldb=N, b_kc=False, ldc=N, rowsum=rs,
             a_scale=1.0 if mma_bf16 else 2.0 ** 10, b_scale=1.0 if mma_bf16 else 8.0,
             mma_bf16=mma_bf16, a_tiled=tiled, b_tiled=tiled)
        out.append((C, rs))
    torch.cuda.synchronize()
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])


@pytest.mark.parametrize("K,M,N,a_off,b_tiled", [
    (790528, 1, 256, 3, True),    # density: d raw_sigma (column 3 of d raw, ld 4) x h7
    (790528, 3, 128, 0, True),    # rgb: d raw_rgb x hv3
    (70001, 4, 64, 0, False),     # row-major B, ragged last 16-row block
    (5, 2, 16, 1, True),          # fewer rows than one block
])
def test_bf16_skinny_weight_gradient(K, M, N, a_off, b_tiled):
    """aon_gemm mma_bf16 with M <= 4 (k_gemm_skinny_bf16: the rgb / density heads' dW = d raw^T X)
    against fp64 products of the bf16-rounded operands, C accumulated and the bias row sums, on
    the fused kernels' tiled or row-major bf16 B."""
    from aonerf import tiles
    from aonerf.linalg import gemm

    g = torch.Generator(device="cuda").manual_seed(K + 7 * M)
    draw = torch.randn((K, 4), device="cuda", generator=g) * 1e-3
    A = draw[:, a_off:]
    Bst = torch.randn((K, N), device="cuda", generator=g).to(torch.bfloat16)
    Bop = tiles.tile(Bst) if b_tiled else Bst
    C0 = torch.randn((M, N), device="cuda", generator=g)
    C = C0.clone()
    rs = torch.empty((M,), device="cuda")
    gemm(C, A, Bop, M, N, K, lda=4, a_kc=False, ldb=N, b_kc=False, ldc=N, accumulate=True,
         rowsum=rs, mma_bf16=True, b_tiled=b_tiled)
    torch.cuda.synchronize()
    a64 = bf16_round(A[:, :M].cpu())
    want = C0.cpu().double() + a64.T @ Bst.cpu().double()
    err = rel_err(C.cpu().numpy(), want.numpy())
    print(f"bf16 skinny dW K={K} M={M} N={N}: max-rel err {err:.2e}")
    assert err < 2e-5
    np.testing.assert_allclose(rs.cpu().numpy(), a64.sum(0).numpy(), rtol=0,
                               atol=2e-5 * float(a64.abs().sum(0).max()))


@pytest.mark.parametrize("K", [790528, 266240, 70001, 5])
def test_bf16_skinny_transposed_weight_gradient(K):
    """aon_gemm c_trans (the articulated bf16 step's deformations_linear.0 xyz columns): dW[:, 0:3]
    = (xyz^T dZ)^T written transposed into the wider dW, and the bias = dZ's column sums, on the
    tiled bf16 dZ -- against fp64 of the bf16-rounded operands; the other columns of dW untouched."""
    from aonerf import tiles
    from aonerf.linalg import gemm

    g = torch.Generator(device="cuda").manual_seed(K)
    xyz = torch.randn((K, 3), device="cuda", generator=g) * 2
    dz = (torch.randn((K, 128), device="cuda", generator=g) * 1e-3).to(torch.bfloat16)
    dW = torch.full((128, 40), 7.0, device="cuda")
    db = torch.empty((128,), device="cuda")
    gemm(dW, xyz, tiles.tile(dz), 3, 128, K, lda=3, a_kc=False, ldb=128, b_kc=False,
         ldc=dW.stride(0), rowsum=db, mma_bf16=True, b_tiled=True, c_trans=True)
    torch.cuda.synchronize()
    a64 = bf16_round(xyz.cpu())
    want = (a64.T @ dz.cpu().double()).T  # (128, 3)
    err = rel_err(dW[:, :3].cpu().numpy(), want.numpy())
    print(f"bf16 transposed skinny dW K={K}: max-rel err {err:.2e}")
    assert err < 2e-5
    assert bool((dW[:, 3:] == 7.0).all())
    cs = dz.cpu().double().sum(0)
    np.testing.assert_allclose(db.cpu().numpy(), cs.numpy(), rtol=0,
                               atol=2e-5 * float(dz.cpu().double().abs().sum(0).max()))


@pytest.mark.parametrize("K,rdiv,a_tiled,a_bf", [(4096 * 193, 193, True, True),
                                                  (2000, 33, False, True),
                                                  (29 * 65, 65, True, False)])
def test_bf16_per_ray_weight_gradient(K, rdiv, a_tiled, a_bf):
    """aon_gemm mma_bf16 against a per-ray B (row k of B = k / rdiv: views_linear.0's enc_dir
    columns, k_gemm_segsum_bf16: per-ray sums of A, then their outer products) against fp64
    products of the bf16-rounded operands, accumulated, with the row sums."""
    from aonerf import tiles
    from aonerf.linalg import gemm

    M, N = 128, 27
    g = torch.Generator(device="cuda").manual_seed(K)
    A = torch.randn((K, M), device="cuda", generator=g) * 1e-3
    if a_bf:
        A = A.to(torch.bfloat16)
    Bst = torch.randn(((K + rdiv - 1) // rdiv, N), device="cuda", generator=g)
    C0 = torch.randn((M, 300), device="cuda", generator=g)
    C = C0.clone()
    rs = torch.empty((M,), device="cuda")
    gemm(C[:, 256:], tiles.tile(A) if a_tiled else A, Bst, M, N, K, lda=M, a_kc=False, ldb=N,
         b_kc=False, b_rdiv=rdiv, ldc=300, accumulate=True, rowsum=rs, mma_bf16=True,
         a_tiled=a_tiled)
    torch.cuda.synchronize()
    a64 = bf16_round(A.float().cpu())
    b64 = bf16_round(Bst.cpu())[torch.arange(K) // rdiv]
    want = C0.cpu().double().clone()
    want[:, 256:256 + N] += a64.T @ b64
    err = rel_err(C.cpu().numpy(), want.numpy())
    print(f"bf16 per-ray dW K={K} rdiv={rdiv}: max-rel err {err:.2e}")
    assert err < 2e-5
    assert torch.equal(C[:, :256], C0[:, :256]) and torch.equal(C[:, 256 + N:], C0[:, 256 + N:])
    np.testing.assert_allclose(rs.cpu().numpy(), a64.sum(0).numpy(), rtol=0,
                               atol=2e-5 * float(a64.abs().sum(0).max()))


def test_bf16_n_store_padded_operand():
    """aon_gemm n_store: a bf16 B zero-padded to 128 columns (the bf16 forward's pos_enc copy)
    on the LDS-DMA kernel updates only the first 63 columns of a dW slice (the skip layer's enc
    columns at 256..318 of a 319-wide weight) -- against fp64 products of the bf16 operands --
    and leaves the rest of C untouched."""
    from aonerf import tiles
    from aonerf.linalg import gemm

    K, M = 193 * 300, 256
    g = torch.Generator(device="cuda").manual_seed(5)
    A = tiles.tile((torch.randn((K, M), device="cuda", generator=g) * 1e-3).to(torch.bfloat16))
    X = torch.randn((K, 63), device="cuda", generator=g).to(torch.bfloat16)
    Xp = torch.zeros((K, 128), device="cuda", dtype=torch.bfloat16)
    Xp[:, :63] = X
    C0 = torch.randn((M, 319), device="cuda", generator=g)
    C = C0.clone()
    gemm(C[:, 256:], A, tiles.tile(Xp), M, 128, K, lda=M, a_kc=False, ldb=128, b_kc=False,
         ldc=319, accumulate=True, mma_bf16=True, a_tiled=True, b_tiled=True, n_store=63)
    torch.cuda.synchronize()
    a64 = bf16_round(tiles.untile(A, K).float().cpu())
    want = C0.cpu().double().clone()
    want[:, 256:] += a64.T @ X.cpu().double()
    err = rel_err(C.cpu().numpy(), want.numpy())
    print(f"bf16 n_store dW: max-rel err {err:.2e}")
    assert err < 2e-5
    assert torch.equal(C[:, :256], C0[:, :256])


def test_bf16_forward_keeps_encodings(bf16_mode):
    """aon_mlp_fwd_train_bf16's enc output: pos_enc(o + t d) (aon_cast_rays, fp32) rounded to
    bf16 exactly, in the tiled layout, columns 63..127 zero; rows past N untouched."""
    from aonerf import _lib as L
    from aonerf import tiles, train

    net = _make_trainable(0)
    batch, u_c, u_f = c5_batch(n=300)
    B, S = 300, 65
    t = torch.sort(torch.rand((B, S), device="cuda") * 4 + 2, -1)[0].contiguous()
    R = B * S
    P = [(w.detach(), b.detach()) for w, b in train._mlp_params(net.coarse_mlp)]
    enc_ref = torch.empty((R, 63), device="cuda")
    L.call("aon_cast_rays", L.ptr(batch["rays_o"]), L.ptr(batch["rays_d"]), L.ptr(t), B, S, None,
           0, None, 0, 10, L.ptr(enc_ref), L.stream())
    NR = tiles.rows(R)
    enc = torch.full((NR, 128), 7.0, device="cuda", dtype=torch.bfloat16)
    raw = torch.empty((R, 4), device="cuda")
    train._forward_level_fused(P, batch["rays_o"], batch["rays_d"], batch["viewdirs"], t, raw,
                               None, None, bf16=True, enc=enc)
    torch.cuda.synchronize()
    got = tiles.untile(enc, R)
    assert torch.equal(got[:, :63], enc_ref.to(torch.bfloat16))
    assert not got[:, 63:].float().any()


@pytest.mark.parametrize("count,K", [(8, 70003), (3, 266240), (8, 790528)])
def test_bf16_weight_gradient_batch(count, K):
    """aon_gemm_batch (linalg.batched): one level's 256 x 256 bf16 weight gradients in ONE launch
    (k_gemm_bf16_dma256_batch: count products x 256 / count K chunks, one split-K reduce) --
    every product against fp64 products of its bf16 operands (tiled, as the fused kernels keep
    them; one C a 256-column slice of a 319-wide weight), with its bias row sums, deterministic
    (two runs bit-equal); a lone deferred product of each class (here a 256 x 256 and a
    128 x 256 one) runs as aon_gemm, bit-identical to separate calls."""
    from aonerf import tiles
    from aonerf.linalg import batched, gemm

    g = torch.Generator(device="cuda").manual_seed(count + K)
    As = [tiles.tile((torch.randn((K, 256), device="cuda", generator=g) * 1e-3).to(torch.bfloat16))
          for _ in range(count)]
    Bs = [tiles.tile(torch.randn((K, 256), device="cuda", generator=g).to(torch.bfloat16))
          for _ in range(count)]

    def run():
        Cs = [torch.zeros((256, 319 if i == 1 else 256), device="cuda") for i in range(count)]
        rss = [torch.empty((256,), device="cuda") for _ in range(count)]
        with batched():
            for i in range(count):
                gemm(Cs[i], As[i], Bs[i], 256, 256, K, lda=256, a_kc=False, ldb=256, b_kc=False,
                     ldc=Cs[i].shape[1], rowsum=rss[i], mma_bf16=True, a_tiled=True, b_tiled=True)
        torch.cuda.synchronize()
        return Cs, rss

    Cs, rss = run()
    Cs2, rss2 = run()
    worst = 0.0
    for i in range(count):
        assert torch.equal(Cs[i], Cs2[i]) and torch.equal(rss[i], rss2[i])
        a64 = bf16_round(tiles.untile(As[i], K).float().cpu())
        b64 = bf16_round(tiles.untile(Bs[i], K).float().cpu())
        err = rel_err(Cs[i][:, :256].cpu().numpy(), (a64.T @ b64).numpy())
        worst = max(worst, err)
        assert err < 2e-5
        np.testing.assert_allclose(rss[i].cpu().numpy(), a64.sum(0).numpy(), rtol=0,
                                   atol=2e-5 * float(a64.abs().sum(0).max()))
        if i == 1:
            assert not Cs[i][:, 256:].any()
    print(f"bf16 dW batch of {count}, K={K}: max-rel err {worst:.2e}")

    # a 128-row product in the set: every product on aon_gemm, bit-identical to separate calls
    A128 = tiles.tile((torch.randn((K, 128), device="cuda", generator=g) * 1e-3).to(torch.bfloat16))
    out = []
    for use_batch in (True, False):
        C1, C2 = torch.zeros((256, 256), device="cuda"), torch.zeros((128, 256), device="cuda")
        with batched() if use_batch else torch.no_grad():
            gemm(C1, As[0], Bs[0], 256, 256, K, lda=256, a_kc=False, ldb=256, b_kc=False,
                 ldc=256, mma_bf16=True, a_tiled=True, b_tiled=True)
            gemm(C2, A128, Bs[0], 128, 256, K, lda=128, a_kc=False, ldb=256, b_kc=False,
                 ldc=256, mma_bf16=True, a_tiled=True, b_tiled=True)
        out.append((C1, C2))
    torch.cuda.synchronize()
    assert torch.equal(out[0][1], out[1][1]) and torch.equal(out[0][0], out[1][0])


@pytest.mark.parametrize("K", [70003, 790528])
def test_bf16_weight_gradient_batch_128_tiles(K):
    """aon_gemm_batch's 128 x 128-tile class (k_gemm_bf16_dma_batch): one level's views_linear.0
    (dZv 128 wide x bottleneck 256), skip-layer enc columns (dZ5 x the 128-column zero-padded
    bf16 pos_enc copy, n_store 63 into columns 256.. of a 319-wide weight) and pts_linears.0
    (likewise, with its bias row sums) in ONE launch -- each against fp64 products of its bf16
    operands; the columns past n_store untouched."""
    from aonerf import tiles
    from aonerf.linalg import batched, gemm

    g = torch.Generator(device="cuda").manual_seed(K + 1)

    def rnd(w, s=1.0):
        return (torch.randn((K, w), device="cuda", generator=g) * s).to(torch.bfloat16)

    dzv, bot, dz5, dz0 = rnd(128, 1e-3), rnd(256), rnd(256, 1e-3), rnd(256, 1e-3)
    enc = torch.zeros((K, 128), device="cuda", dtype=torch.bfloat16)
    enc[:, :63] = rnd(63)
    Cv = torch.zeros((128, 283), device="cuda")
    C5 = torch.full((256, 319), 7.0, device="cuda")
    C0 = torch.zeros((256, 63), device="cuda")
    rs_v, rs_0 = torch.empty((128,), device="cuda"), torch.empty((256,), device="cuda")
    with batched():
        gemm(Cv, tiles.tile(dzv), tiles.tile(bot), 128, 256, K, lda=128, a_kc=False, ldb=256,
             b_kc=False, ldc=283, rowsum=rs_v, mma_bf16=True, a_tiled=True, b_tiled=True)
        gemm(C5[:, 256:], tiles.tile(dz5), tiles.tile(enc), 256, 128, K, lda=256, a_kc=False,
             ldb=128, b_kc=False, ldc=319, mma_bf16=True, a_tiled=True, b_tiled=True, n_store=63)
        gemm(C0, tiles.tile(dz0), tiles.tile(enc), 256, 128, K, lda=256, a_kc=False, ldb=128,
             b_kc=False, ldc=63, rowsum=rs_0, mma_bf16=True, a_tiled=True, b_tiled=True,
             n_store=63)
    torch.cuda.synchronize()
    d = lambda t: t.float().cpu().double()  # noqa: E731
    checks = [(Cv[:, :256], d(dzv).T @ d(bot)), (C5[:, 256:], d(dz5).T @ d(enc)[:, :63]),
              (C0, d(dz0).T @ d(enc)[:, :63])]
    for got, want in checks:
        err = rel_err(got.cpu().numpy(), want.numpy())
        print(f"bf16 dW 128-tile batch K={K}: max-rel err {err:.2e}")
        assert err < 2e-5
    assert not Cv[:, 256:].any() and torch.equal(C5[:, :256], torch.full((256, 256), 7.0, device="cuda"))
    for rs, a in ((rs_v, dzv), (rs_0, dz0)):
        np.testing.assert_allclose(rs.cpu().numpy(), d(a).sum(0).numpy(), rtol=0,
                                   atol=2e-5 * float(d(a).abs().sum(0).max()))


def test_f16x3_weight_gradient_batch():
    """aon_gemm_batch's fp16x3 class (k_gemm_f16x3_batch): the parity mode's weight gradients
    (fp32 tiled operands, the activation prescale 2^-8 and a per-call gradient scale word, one
    product accumulating) in ONE launch -- each product against fp64 and within 1e-6 of its own
    aon_gemm launch (the same fp16x3 numerics, other K chunks); deterministic."""
    from aonerf import tiles
    from aonerf.linalg import ACT_SCALE, batched, gemm

    K = 70003
    g = torch.Generator(device="cuda").manual_seed(3)
    shapes = [(256, 256), (128, 256), (256, 256)]
    As = [torch.randn((K, m), device="cuda", generator=g) * 1e-3 for m, _ in shapes]
    Bs = [torch.relu(torch.randn((K, n), device="cuda", generator=g)) for _, n in shapes]
    C_init = torch.randn((256, 256), device="cuda", generator=g)
    word = torch.zeros((1,), dtype=torch.int32, device="cuda")
    from aonerf import _lib as L
    L.call("aon_absmax", L.ptr(As[0]), As[0].numel(), L.ptr(word), L.stream())

    def run(use_batch):
        Cs = [torch.zeros((m, n), device="cuda") for m, n in shapes]
        Cs[2].copy_(C_init)
        rss = [torch.empty((m,), device="cuda") for m, _ in shapes]
        with batched() if use_batch else torch.no_grad():
            for i, (m, n) in enumerate(shapes):
                gemm(Cs[i], tiles.tile(As[i]), tiles.tile(Bs[i]), m, n, K, lda=m, a_kc=False,
                     ldb=n, b_kc=False, ldc=n, rowsum=rss[i], accumulate=i == 2, a_scale=1.0,
                     b_scale=ACT_SCALE, a_amax=word if i == 0 else None, a_tiled=True,
                     b_tiled=True)
        torch.cuda.synchronize()
        return Cs, rss

    (Cb, rb), (Cb2, rb2), (Cs, rs) = run(True), run(True), run(False)
    for i in range(3):
        assert torch.equal(Cb[i], Cb2[i]) and torch.equal(rb[i], rb2[i])
        want = As[i].cpu().double().T @ Bs[i].cpu().double()
        if i == 2:
            want += C_init.cpu().double()
        err = rel_err(Cb[i].cpu().numpy(), want.numpy())
        err_own = rel_err(Cb[i].cpu().numpy(), Cs[i].cpu().numpy())
        print(f"f16x3 dW batch product {i}: max-rel err {err:.2e} (vs its own launch {err_own:.2e})")
        assert err < 2e-6 and err_own < 1e-6
        np.testing.assert_allclose(rb[i].cpu().numpy(), rs[i].cpu().numpy(), rtol=0,
                                   atol=1e-6 * float(As[i].abs().sum(0).max()))


def test_gemm_small_batch_equals_sequential_launches():
    """aon_gemm_small_batch (the articulated bf16 step's latent terms and folded biases in one
    launch) gives exactly what the same exact_fp32 products give launched one by one in argument
    order: outer products (K = 1, one lane per output), row products (K > 16, one wave per
    output), a three-product accumulate chain on one C, a bias, column slices of one dW."""
    from aonerf import _lib as L
    from aonerf.linalg import gemm, small_batched

    g = torch.Generator(device="cuda").manual_seed(5)
    r = lambda *s: torch.randn(*s, device="cuda", generator=g)  # noqa: E731
    db = [r(1, 256), r(1, 256), r(1, 128)]
    lat = [r(1, 128), r(1, 32)]
    Ws = [r(256, 447), r(256, 191), r(128, 163)]
    bias = r(256)

    def run():
        dW = torch.full((128, 163), 7.0, device="cuda")
        dW2 = torch.full((256, 447), 3.0, device="cuda")
        dl = torch.full((1, 128), 2.0, device="cuda")
        fold = torch.empty((1, 256), device="cuda")
        # outer products into column slices of dW (K = 1)
        gemm(dW[:, 3:], db[2], lat[0], 128, 128, 1, lda=1, a_kc=True, ldb=128, b_kc=False, ldc=163,
             exact_fp32=True)
        gemm(dW[:, 131:], db[2], lat[1], 128, 32, 1, lda=1, a_kc=True, ldb=32, b_kc=False, ldc=163,
             exact_fp32=True)
        gemm(dW2[:, 319:], db[0], lat[0], 256, 128, 1, lda=1, a_kc=True, ldb=128, b_kc=False,
             ldc=447, exact_fp32=True)
        # the shape code's gradient: three row products chained on one C
        gemm(dl, db[0], Ws[0][:, 319:], 1, 128, 256, lda=256, a_kc=True, ldb=447, b_kc=False,
             ldc=128, exact_fp32=True)
        gemm(dl, db[1], Ws[1][:, 63:], 1, 128, 256, lda=256, a_kc=True, ldb=191, b_kc=False,
             ldc=128, accumulate=True, exact_fp32=True)
        gemm(dl, db[2], Ws[2][:, 3:131], 1, 128, 128, lda=128, a_kc=True, ldb=163, b_kc=False,
             ldc=128, accumulate=True, exact_fp32=True)
        # a folded bias: b + W[:, c0:] . lat (b_kc, bias)
        gemm(fold, lat[0], Ws[0][:, 319:], 1, 256, 128, lda=128, a_kc=True, ldb=447, b_kc=True,
             ldc=256, bias=bias, exact_fp32=True)
        return dW, dW2, dl, fold

    seq = run()
    with small_batched():
        bat = run()
    torch.cuda.synchronize()
    for a, b in zip(seq, bat):
        assert torch.equal(a, b)
    assert bool((seq[0][:, :3] == 7.0).all())  # columns no product writes are untouched
    # a product reading another group's output is refused
    x = torch.zeros((1, 128), device="cuda")
    y = torch.zeros((1, 128), device="cuda")
    with pytest.raises(ValueError, match="reads a batch output"):
        with small_batched():
            gemm(x, lat[0], Ws[0][:, 319:], 1, 128, 128, lda=128, a_kc=True, ldb=447, b_kc=True,
                 ldc=128, exact_fp32=True)
            gemm(y, x, Ws[0][:128, 319:], 1, 128, 128, lda=128, a_kc=True, ldb=447, b_kc=True,
                 ldc=128, exact_fp32=True)
    assert L.GEMM_SMALL_BATCH_MAX == 16
