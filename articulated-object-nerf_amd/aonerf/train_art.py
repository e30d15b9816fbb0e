"""Training step of the articulated auto-decoder (reference LitNeRF_AutoDecoder.training_step,
models/vanilla_nerf/model_autodecoder.py:395-477; configure_optimizers / optimizer_step :599-633)
on the HIP kernels.

One NeRF_AE_Art level under autograd is ``ArtRenderLevel`` (a torch.autograd.Function) with
gradients for the level's 40 MLP parameters AND the three latent codes:

  forward   one fused kernel per level (aon_mlp_art_fwd_train, the inference kernel with
            activation stores): cast_rays -> deformation MLP on cat[xyz, shape, articulation] ->
            x' = delta + xyz, pos_enc(x') -> trunk on cat[pos_enc(x'), shape] with the skip
            concat -> density, bottleneck -> view branch on cat[bottleneck, enc_dir tiled over
            samples, appearance] -> rgb, every activation, pos_enc(x') and the points kept
            (model_autodecoder.py:168-239); or the same layer by layer on aon_gemm
            (TrainNumerics.fused_forward False) -> compositing with the padded sigmoid / softplus
            (aon_composite_fwd, AON_ACT_ARTIC; :321-333)
  backward  aon_composite_bwd -> every input gradient dX = (dZ W) * relu'(X) in one fused
            kernel (aon_mlp_art_bwd): view branch, heads, trunk, the gradient w.r.t.
            pos_enc(x') (skip + first layer) through pos_enc's backward into the deformation
            head and MLP -> per layer dW = dZ^T X with db = sum_rows dZ from the same pass
            (aon_gemm); or the whole chain as GEMMs + aon_pos_enc_bwd (fused_backward False).

The latent codes are the same row for every sample (repeated over B*S rows,
model_autodecoder.py:186-194), so their columns are folded into per-call biases in the
forward, and in the backward a layer z = W [x; l] + b gives dL/dl = W_l^T db and
dL/dW_l = db l^T from the bias gradient db alone (aon_gemm with K = 1 / M = 1); the shape code
collects three such terms (deformation input, trunk input, skip), appearance one, articulation
one, both levels add through autograd.  The regulariser 1e-4 * sum of mean code norms
(:456-466) is aon_latent_reg.  All arithmetic is in HIP kernels; torch allocates, routes
autograd and looks up / scatters the code-library rows (nn.Embedding).
"""
import torch

from . import _lib as L
from . import tiles
from . import train as _train
from .linalg import ACT_SCALE, GRAD_SCALE, W_SCALE, batched, gemm, small_batched
from .numerics import ART_FORWARD, DEFAULT
from .train import Adam, _amax_word, img2mse, learning_rate, loss_pair, mse2psnr, relu_masks  # noqa: F401 (shared)

# parameter layout of one articulated NeRFMLP in ArtRenderLevel: 20 layers x (weight, bias)
DEF0, DL, PTS0, DENS, BOT, VIEW0, RGB = 0, 4, 5, 13, 14, 15, 19


def art_layers(mlp):
    """The 20 nn.Linear layers of an articulated NeRFMLP in ArtRenderLevel order."""
    return (list(mlp.deformations_linear) + [mlp.deformation_layer] + list(mlp.pts_linears)
            + [mlp.density_layer, mlp.bottleneck_layer] + list(mlp.views_linear) + [mlp.rgb_layer])


def _check_geometry(mlp):
    ok = (mlp.netdepth == 8 and mlp.skip_layer == 4 and mlp.netdepth_deformation == 4
          and mlp.netdepth_condition == 4 and mlp.input_ch == 3 and mlp.input_ch_view == 3
          and mlp.num_rgb_channels == 3 and mlp.num_density_channels == 1)
    if not ok:
        raise ValueError("the articulated training path implements the reference's default layer "
                         "counts (netdepth 8, skip 4, 4 deformation / 4 condition layers)")


class _Geo:
    """Widths of one articulated NeRFMLP (model_autodecoder.py:60-166)."""

    def __init__(self, mlp):
        _check_geometry(mlp)
        self.wd, self.nw, self.wc = mlp.netwidth_deformation, mlp.netwidth, mlp.netwidth_condition
        self.ne = mlp.pos_size_enc  # 3 + 6 (max_deg - min_deg)
        self.min_deg, self.max_deg, self.deg_view = mlp.min_deg_point, mlp.max_deg_point, mlp.deg_view
        self.nv = (mlp.deg_view * 2 + 1) * mlp.input_ch_view
        self.n_shape, self.n_app = mlp.shape_latent_dim, mlp.appearance_latent_dim
        self.n_art = mlp.articulation_latent_dim


def _fold(W, b, c0, lat, exact=False):
    """b + W[:, c0:c0+n] . lat (the latent columns of a layer as a per-call bias); exact (the
    bf16 mode): on aon_gemm's exact-fp32 tiny-product path."""
    N, n = W.shape[0], lat.shape[1]
    out = torch.empty((1, N), device=W.device)
    gemm(out, lat, W[:, c0:], 1, N, n, lda=n, a_kc=True, ldb=W.stride(0), b_kc=True, ldc=N,
         bias=b, a_scale=1.0, b_scale=W_SCALE, exact_fp32=exact)
    return out.reshape(-1)


def _linear(out, X, ldx, W, bias, K, *, relu=False, X2=None, K2=0, ld2=0, rdiv2=1, ldo=None,
            accumulate=False):
    """out (R x N) (+)= [X | X2] W[:, :K+K2]^T + bias (+ReLU)."""
    R, N = out.shape[0], W.shape[0]
    gemm(out, X, W, R, N, K + K2, lda=ldx, a_kc=True, ldb=W.stride(0), b_kc=True,
         ldc=ldo or out.stride(0), A2=X2, lda2=ld2, K1=K if X2 is not None else 0, a2_rdiv=rdiv2,
         bias=bias, relu=relu, accumulate=accumulate, a_scale=ACT_SCALE, b_scale=W_SCALE)


def _forward_level(geo, P, lat, xyz, venc, S, raw, noise=None, exact_folds=False):
    """NeRFMLP.forward (model_autodecoder.py:168-239) layer by layer, keeping activations
    (exact_folds: the latent folds on the exact-fp32 path, as the bf16 mode computes them)."""
    R, dev = xyz.shape[0], xyz.device
    shape, app, art = lat
    wd, nw, wc, ne, nv = geo.wd, geo.nw, geo.wc, geo.ne, geo.nv
    # deformation MLP on cat[xyz, shape, art] (:196-203), the latent columns folded
    hd = torch.empty((4, R, wd), device=dev)
    _linear(hd[0], xyz, 3, P[DEF0][0],
            _fold(*P[DEF0], 3, torch.cat([shape, art], -1), exact_folds), 3, relu=True)
    for i in range(1, 4):
        _linear(hd[i], hd[i - 1], wd, *P[DEF0 + i], wd, relu=True)
    delta = torch.empty((R, 3), device=dev)
    _linear(delta, hd[3], wd, *P[DL], wd)  # deformation_layer (:205)
    # x' = delta + xyz -> pos_enc (enc_after, :205-212); enc[:, :3] is x' itself
    enc = torch.empty((R, ne), device=dev)
    L.call("aon_cast_rays", L.ptr(xyz), None, None, R, 1, L.ptr(delta), 3, None, geo.min_deg,
           geo.max_deg, L.ptr(enc), L.stream(dev))
    # trunk on cat[enc, shape] with the skip concat cat[h4, enc, shape] (:214-220)
    h = torch.empty((8, R, nw), device=dev)
    W0 = P[PTS0][0]
    _linear(h[0], enc, ne, W0, _fold(W0, P[PTS0][1], ne, shape, exact_folds), ne, relu=True)
    for i in range(1, 8):
        W_, b_ = P[PTS0 + i]
        if i == 5:
            _linear(h[5], h[4], nw, W_, _fold(W_, b_, nw + ne, shape, exact_folds), nw,
                    relu=True, X2=enc, K2=ne, ld2=ne)
        else:
            _linear(h[i], h[i - 1], nw, W_, b_, nw, relu=True)
    if noise is not None:  # raw_sigma + noise (:318-319), added in the GEMM epilogue
        raw[:, 3].copy_(noise)
    _linear(raw[:, 3:], h[7], nw, *P[DENS], nw, ldo=4, accumulate=noise is not None)
    bot = torch.empty((R, nw), device=dev)
    _linear(bot, h[7], nw, *P[BOT], nw)  # bottleneck, no activation (:225)
    # view branch on cat[bottleneck, enc_dir tiled over samples, appearance] (:226-235)
    hv = torch.empty((4, R, wc), device=dev)
    Wv = P[VIEW0][0]
    _linear(hv[0], bot, nw, Wv, _fold(Wv, P[VIEW0][1], nw + nv, app, exact_folds), nw,
            relu=True, X2=venc, K2=nv, ld2=nv, rdiv2=S)
    for i in range(1, 4):
        _linear(hv[i], hv[i - 1], wc, *P[VIEW0 + i], wc, relu=True)
    _linear(raw, hv[3], wc, *P[RGB], wc, ldo=4)  # rgb_layer (:237)
    return hd, enc, h, bot, hv


# Which kernels, precision and (bf16 mode) forward numerics a level trains with is the MODEL's
# TrainNumerics (aonerf/numerics.py; NeRF_AE_Art(train_precision=...)), passed into
# ArtRenderLevel per call -- no module-level switch.  The bf16 mode: the whole backward chain and
# the weight-gradient GEMMs bf16 (aon_mlp_art_bwd_bf16, aon_gemm mma_bf16), kept activations and
# gradients bf16 (aon_mlp_art_fwd_train_bf16); compositing, the loss, their backward, the latent
# terms and Adam fp32 on fp32 master weights (tests/test_gpu_art_train_bf16.py).  Its forward
# past the deformation MLP (TrainNumerics.art_forward): "f16_acts" (default) two fp16 MFMAs per
# product, the weights' exact hi / lo split kept, the activations rounded once to fp16 per sample
# (the backward already reads bf16 copies, 8x coarser; C5 gradients cosine 0.99919 / max-rel
# 0.049 against the fp32 oracle at the 0.999 / 0.05 gates); "f16x3" fp16x3 throughout, only the
# stores bf16; held off by their measured gates: "f16_weights" (weights rounded to fp16: 0.99886
# / 0.074), "bf16_view" (view branch bf16: deformation gradients cosine 0.9968 for 2% of the
# step) and "bf16_trunk" (trunk, heads and view branch bf16: 0.987 -- the articulated gradients
# are ill-conditioned in the forward values).

_packed = {}


def _params_struct(P, fb=None):
    """AonMlpArtParams of one level's parameters (``fb``: folded biases by layer index)."""
    fb = fb or {}
    order = [DEF0 + i for i in range(4)] + [DL] + [PTS0 + i for i in range(8)] + [DENS, BOT] + \
        [VIEW0 + i for i in range(4)] + [RGB]
    # shape / dtype / device checked against the layer table (ValueError) before any pointer
    # reaches a pack kernel; the C side checks the shapes again (aon_mlp_art_params, ABI 9)
    return L.mlp_art_params([(P[i][0], fb.get(i, P[i][1])) for i in order])


def _buffer(key, nbytes, dev, guard=False, params=()):
    # one buffer per kind and device: a pack and the kernel reading it are stream-ordered.
    # guard: a packed weight stream whose range-status word the next optimizer step over
    # ``params`` (the packed parameters) checks
    buf = _packed.get((key, str(dev)))
    if buf is None:
        buf = torch.empty(max(nbytes // 4, 1), dtype=torch.float32, device=dev)
        _packed[(key, str(dev))] = buf
    if guard:
        L.register_pack(("train_art", key), buf, params)
    return buf


def _pack(geo, P, lat, tag="", mixed=0, exact_folds=False):
    """The fused kernel's fp16x3 weight stream (aon_mlp_art_pack) of one level's parameters with
    this call's latent codes folded into the biases; re-packed on every call (the optimizer
    updates the parameters in place).  mixed: the bf16 mode's mixed streams
    (aon_mlp_art_pack_mixed: 1 trunk bf16, 2 view branch bf16, 3 fp16 weights; range-guarded,
    their deformation part is fp16x3).  exact_folds (the bf16 mode): the folds on the exact-fp32
    path."""
    shape, app, art = lat
    dev = shape.device
    with small_batched():  # bf16: the four folds as one launch (exact-fp32 path, same bits)
        fb = {DEF0: _fold(*P[DEF0], 3, torch.cat([shape, art], -1), exact_folds),
              PTS0: _fold(*P[PTS0], geo.ne, shape, exact_folds),
              PTS0 + 5: _fold(*P[PTS0 + 5], geo.nw + geo.ne, shape, exact_folds),
              VIEW0: _fold(*P[VIEW0], geo.nw + geo.nv, app, exact_folds)}
    buf = _buffer(f"fwd{'bf' if mixed else ''}{tag}", L.lib().aon_mlp_art_packed_bytes(), dev,
                  guard=True, params=[t for wb in P for t in wb])
    if mixed:
        L.call("aon_mlp_art_pack_mixed", L.ctypes.byref(_params_struct(P, fb)), mixed, L.ptr(buf),
               L.stream(dev))
    else:
        L.call("aon_mlp_art_pack", L.ctypes.byref(_params_struct(P, fb)), L.ptr(buf), L.stream(dev))
    return buf


def _pack_bwd(P, dev, tag="", bf16=False):
    """The transposed weight stream of the fused backward chain (aon_mlp_art_bwd_pack[_bf16])."""
    buf = _buffer(f"bwd{'bf' if bf16 else ''}{tag}", L.lib().aon_mlp_art_bwd_packed_bytes(), dev,
                  guard=not bf16, params=[t for wb in P for t in wb])
    L.call("aon_mlp_art_bwd_pack_bf16" if bf16 else "aon_mlp_art_bwd_pack",
           L.ctypes.byref(_params_struct(P)), L.ptr(buf), L.stream(dev))
    return buf


def _forward_level_fused(geo, P, lat, rays_o, rays_d, viewdirs, t_vals, raw, noise=None,
                         masks=None, bf16=False, enc_bf=None, return_enc_bf=False,
                         art_forward="f16_acts", timers=None, exact_folds=None):
    """_forward_level on the fused kernel (aon_mlp_art_fwd_train): raw (R x 4) and the kept
    activations (tiled, tiles.rows(R) rows each), the sample points (row-major) and pos_enc(x')
    (tiled, (tiles.rows(R), 64), column 63 zero); ``masks`` ((16, tiles.rows(R), 8) int32)
    receives the ReLU' bits of hd0..3, h0..7, hv0..3 for the backward chain.  bf16: the bf16
    mode (aon_mlp_art_fwd_train_bf16; hd / h / bot / hv kept as torch.bfloat16; enc keeps
    columns 0..15 only, (tiles.rows(R), 16) -- the chain reads x' = columns 0..2 -- and
    ``enc_bf`` ((tiles.rows(R), 128) bfloat16, allocated when None) receives pos_enc(x') tiled,
    columns 63.. zero: the enc-column weight gradients' operand; ``art_forward``: its forward numerics past
    the deformation MLP, TrainNumerics.art_forward).  enc_rows() converts enc for the all-GEMM
    backward.  ``timers``: hip events (bench.py); ``exact_folds``: the latent folds on the
    exact-fp32 path (None: as the mode computes them -- exact in bf16, fp16x3 otherwise)."""
    B, S = t_vals.shape
    R, dev = B * S, t_vals.device
    NR = tiles.rows(R)
    if masks is None:
        masks = torch.empty((16, NR, 8), dtype=torch.int32, device=dev)
    dt = torch.bfloat16 if bf16 else torch.float32
    hd = torch.empty((4, NR, geo.wd), device=dev, dtype=dt)
    h = torch.empty((8, NR, geo.nw), device=dev, dtype=dt)
    bot = torch.empty((NR, geo.nw), device=dev, dtype=dt)
    hv = torch.empty((4, NR, geo.wc), device=dev, dtype=dt)
    enc = torch.empty((NR, 16 if bf16 else 64), device=dev)
    if bf16 and enc_bf is None:
        enc_bf = torch.empty((NR, 128), device=dev, dtype=torch.bfloat16)
    xyz = torch.empty((R, 3), device=dev)
    mixed, mixed_stream = ART_FORWARD[art_forward] if bf16 else (0, False)
    # (f16_acts, 4, and f16x3, 0, read the plain fp16x3 stream)
    packed = _pack(geo, P, lat, S, mixed if mixed_stream else 0,
                   exact_folds=bf16 if exact_folds is None else exact_folds)
    e0 = _train._ev(timers)
    args = (L.ptr(packed), L.ptr(rays_o), L.ptr(rays_d), L.ptr(viewdirs), L.ptr(t_vals), B, S,
            L.ptr(noise) if noise is not None else None, L.ptr(hd), L.ptr(h), L.ptr(bot),
            L.ptr(hv), L.ptr(enc), L.ptr(xyz), L.ptr(raw), L.ptr(masks))
    if bf16:
        L.call("aon_mlp_art_fwd_train_bf16", *args, L.ptr(enc_bf), mixed, L.stream(dev))
    else:
        L.call("aon_mlp_art_fwd_train", *args, L.stream(dev))
    L.snapshot_pack(packed)  # the forward was the pack's last reader (range guard, _lib)
    _train._rec(timers, f"art_fwd_train{S}", e0, R)
    return (xyz, hd, enc, h, bot, hv) + ((enc_bf,) if return_enc_bf else ())


def enc_rows(geo, enc, R):
    """pos_enc(x') row-major (R, 63) fp32 from what a level's forward kept: as is (the
    layer-by-layer forward), untiled (the fused fp16x3 forward's (NR, 64)), or recomputed from
    x' (the fused bf16 forward keeps columns 0..15 only) by aon_pos_enc -- the kernel's own
    pos_enc_feature, bit-identical."""
    if enc.shape[1] == geo.ne:
        return enc
    if enc.shape[1] == 64:
        return tiles.untile(enc, R)[:, :geo.ne].contiguous()
    xp = tiles.untile(enc, R)[:, :3].contiguous()
    out = torch.empty((R, geo.ne), device=enc.device)
    L.call("aon_pos_enc", L.ptr(xp), R, geo.min_deg, geo.max_deg, L.ptr(out), L.stream(enc.device))
    return out


def _enc_tiled(enc, width):
    """The chain's enc operand (tiled, ``width`` columns) from a row-major (R, 63) pos_enc(x')."""
    if enc.shape[1] == width:
        return enc
    pad = torch.zeros((enc.shape[0], width), device=enc.device)
    n = min(width, enc.shape[1])
    pad[:, :n] = enc[:, :n]
    return tiles.tile(pad)


def _fused_ok(geo):
    # the fused kernel is compiled for the default widths (mlp_layout.hpp kLayersArt)
    return (geo.wd == 128 and geo.nw == 256 and geo.wc == 128 and geo.ne == 63 and geo.nv == 27
            and geo.min_deg == 0)


def _backward_level(geo, P, G, lat, dlat, xyz, enc, venc, S, hd, h, bot, hv, draw):
    """Autograd of _forward_level from dL/draw (R x 4): G[i] = (dW, db) of layer i; dlat =
    (dshape, dapp, dart) (1 x n each) receive the latent-code gradients.  Every dY enters the
    f16x3 split at a per-call power-of-two scale from max |dY| (aon_absmax -> a_amax; for the
    density column of d raw, from all of d raw), as the fused chain scales its gradients."""
    R, dev = xyz.shape[0], xyz.device
    wd, nw, wc, ne, nv = geo.wd, geo.nw, geo.wc, geo.ne, geo.nv
    enc = enc_rows(geo, enc, R)
    shape, app, art = lat
    dshape, dapp, dart = dlat
    gs, acts = GRAD_SCALE, ACT_SCALE
    word = torch.zeros((1,), dtype=torch.int32, device=dev)  # stream-ordered: reused per call

    def amax(dY):
        return _amax_word(draw if dY.data_ptr() == draw.data_ptr() + 12 else dY, word)

    def dweight(i, dY, ldy, X, ldx, n_in, col0=0, rdiv=1, bias=True):
        # dW_i[:, col0:col0+n_in] = dY^T X (K = rows, split-K); db_i = sum_rows dY, same pass
        dW = G[i][0]
        n_out = dW.shape[0]
        gemm(dW[:, col0:] if col0 else dW, dY, X, n_out, n_in, R, lda=ldy, a_kc=False, ldb=ldx,
             b_kc=False, b_rdiv=rdiv, ldc=dW.stride(0), a_scale=1.0, b_scale=acts,
             rowsum=G[i][1] if bias else None, a_amax=amax(dY))

    def dinput(dX, dY, ldy, i, col0, n_in, mask=None, accumulate=False):
        # dX (R x n_in) (+)= dY W_i[:, col0:col0+n_in] (* relu'(mask))
        W = P[i][0]
        gemm(dX, dY, W[:, col0:] if col0 else W, R, n_in, W.shape[0], lda=ldy, a_kc=True,
             ldb=W.stride(0), b_kc=False, ldc=dX.stride(0), mask=mask,
             ldm=mask.stride(0) if mask is not None else 0, accumulate=accumulate, a_scale=1.0,
             b_scale=W_SCALE, a_amax=amax(dY))

    def dlatent(i, col0, l, dl, accumulate):
        # z = W [x; l] + b with l on every row: dW[:, col0:col0+n] = db l^T, dl (+)= db^T W_l
        dW, db = G[i]
        W = P[i][0]
        n_out, n = W.shape[0], l.shape[1]
        gemm(dW[:, col0:], db, l, n_out, n, 1, lda=1, a_kc=True, ldb=n, b_kc=False,
             ldc=dW.stride(0), a_scale=gs, b_scale=1.0)
        gemm(dl, db, W[:, col0:], 1, n, n_out, lda=n_out, a_kc=True, ldb=W.stride(0), b_kc=False,
             ldc=n, accumulate=accumulate, a_scale=gs, b_scale=W_SCALE)

    # rgb head and the view branch
    dweight(RGB, draw, 4, hv[3], wc, wc)
    dz = torch.empty((R, wc), device=dev)
    dz2 = torch.empty((R, wc), device=dev)
    dinput(dz, draw, 4, RGB, 0, wc, mask=hv[3])
    for i in range(3, 0, -1):
        dweight(VIEW0 + i, dz, wc, hv[i - 1], wc, wc)
        dinput(dz2, dz, wc, VIEW0 + i, 0, wc, mask=hv[i - 1])
        dz, dz2 = dz2, dz
    dweight(VIEW0, dz, wc, bot, nw, nw)
    dweight(VIEW0, dz, wc, venc, nv, nv, col0=nw, rdiv=S, bias=False)
    dlatent(VIEW0, nw + nv, app, dapp, False)
    dbot = torch.empty((R, nw), device=dev)
    dinput(dbot, dz, wc, VIEW0, 0, nw)  # the bottleneck has no activation
    del dz, dz2
    # bottleneck + density heads on h7
    dweight(BOT, dbot, nw, h[7], nw, nw)
    dweight(DENS, draw[:, 3:], 4, h[7], nw, nw)
    dy = torch.empty((R, nw), device=dev)
    dinput(dy, dbot, nw, BOT, 0, nw)
    dinput(dy, draw[:, 3:], 4, DENS, 0, nw, mask=h[7], accumulate=True)
    del dbot
    # trunk; the gradient w.r.t. enc = pos_enc(x') collects the skip and the first layer
    denc = torch.empty((R, ne), device=dev)
    dx = torch.empty((R, nw), device=dev)
    for i in range(7, -1, -1):  # dy = dL/d(pre-activation of pts_linears.i)
        if i == 5:
            dweight(PTS0 + 5, dy, nw, h[4], nw, nw)
            dweight(PTS0 + 5, dy, nw, enc, ne, ne, col0=nw, bias=False)
            dlatent(PTS0 + 5, nw + ne, shape, dshape, False)
            dinput(denc, dy, nw, PTS0 + 5, nw, ne)
        elif i == 0:
            dweight(PTS0, dy, nw, enc, ne, ne)
            dlatent(PTS0, ne, shape, dshape, True)
            dinput(denc, dy, nw, PTS0, 0, ne, accumulate=True)
        else:
            dweight(PTS0 + i, dy, nw, h[i - 1], nw, nw)
        if i > 0:
            dinput(dx, dy, nw, PTS0 + i, 0, nw, mask=h[i - 1])
            dx, dy = dy, dx
    del dx, dy
    # x' = deformation_layer(hd3) + xyz, enc = pos_enc(x') (:205-212)
    dxp = torch.empty((R, 3), device=dev)
    L.call("aon_pos_enc_bwd", L.ptr(enc), ne, L.ptr(denc), ne, R, geo.min_deg, geo.max_deg, 0,
           L.ptr(dxp), 3, L.stream(dev))
    del denc
    dweight(DL, dxp, 3, hd[3], wd, wd)
    dz = torch.empty((R, wd), device=dev)
    dz2 = torch.empty((R, wd), device=dev)
    dinput(dz, dxp, 3, DL, 0, wd, mask=hd[3])
    for i in range(3, 0, -1):
        dweight(DEF0 + i, dz, wd, hd[i - 1], wd, wd)
        dinput(dz2, dz, wd, DEF0 + i, 0, wd, mask=hd[i - 1])
        dz, dz2 = dz2, dz
    # deformations_linear.0 on cat[xyz, shape, art]
    dweight(DEF0, dz, wd, xyz, 3, 3)
    dlatent(DEF0, 3, shape, dshape, True)
    dlatent(DEF0, 3 + geo.n_shape, art, dart, False)


def _backward_level_fused(geo, P, G, lat, dlat, xyz, enc, venc, S, hd, h, bot, hv, draw,
                          masks=None, h_tiled=True, enc_bf=None, timers=None, cfg=DEFAULT):
    """_backward_level with every input-gradient product (and pos_enc's backward) in one fused
    kernel (aon_mlp_art_bwd); the weight gradients dW = dZ^T X, db = sum_rows dZ and the latent
    terms stay GEMMs.  ``masks``: the fused forward's ReLU' bits (built from the activations
    when None); h_tiled: hd / h / bot / hv in the fused forward's tiled layout (else
    row-major); the chain's dzv / dbot / dz / dzd are tiled.  enc: the fused forward's tiled
    pos_enc(x') ((NR, 64) fp16x3, (NR, 16) bf16) or the layer-by-layer forward's row-major
    (R, 63).  enc_bf: the bf16 forward's tiled 128-column pos_enc(x') (the enc-column weight
    gradients then run on the LDS-DMA kernel).  ``timers``: hip events (bench.py); ``cfg``: the
    model's TrainNumerics (the weight-gradient batching)."""
    R, dev = xyz.shape[0], xyz.device
    bf16 = h[0].dtype == torch.bfloat16  # activations kept by the bf16 training forward
    if masks is None:
        acts = list(hd) + list(h) + list(hv)
        masks = relu_masks([tiles.untile(a, R).float() for a in acts] if h_tiled else acts, R)
    wd, nw, wc, ne, nv = geo.wd, geo.nw, geo.wc, geo.ne, geo.nv
    shape, app, art = lat
    dshape, dapp, dart = dlat
    NR = tiles.rows(R)
    dt = torch.bfloat16 if bf16 else torch.float32
    dzv = torch.empty((4, NR, wc), device=dev, dtype=dt)
    dbot = torch.empty((NR, nw), device=dev, dtype=dt)
    dz = torch.empty((8, NR, nw), device=dev, dtype=dt)
    dxp = torch.empty((R, 3), device=dev)
    dzd = torch.empty((4, NR, wd), device=dev, dtype=dt)
    work = _buffer("work", 4, dev)
    packed = _pack_bwd(P, dev, S, bf16)
    enc_t = enc.shape[1] != ne  # the fused forward's tiled copy
    enc_chain = enc if enc_t else _enc_tiled(enc, 16 if bf16 else 64)
    e0 = _train._ev(timers)
    L.call("aon_mlp_art_bwd_bf16" if bf16 else "aon_mlp_art_bwd", L.ptr(packed), L.ptr(draw), L.ptr(masks), L.ptr(enc_chain), R,
           L.ptr(dzv), L.ptr(dbot), L.ptr(dz), L.ptr(dxp), L.ptr(dzd), L.ptr(work), L.stream(dev))
    L.snapshot_pack(packed)  # the chain was the pack's last reader
    _train._rec(timers, f"art_bwd_chain{S}", e0, R)
    e0 = _train._ev(timers)
    gs, acts = GRAD_SCALE, ACT_SCALE

    def dweight(i, dY, ldy, X, ldx, n_in, col0=0, rdiv=1, bias=True, chain_scale=True, a_t=True):
        n_store = 0
        if X is enc and bf16 and enc_bf is not None:  # the tiled bf16 copy, 63 of 128 columns
            X, ldx, n_store, n_in = enc_bf, 128, n_in, 128
        elif X is enc and enc_t:  # the fused fp16x3 forward's tiled fp32 copy, 63 of 64 columns
            if enc.shape[1] != 64:
                raise ValueError("the bf16 forward keeps 16 enc columns: pass its enc_bf")
            ldx, n_store, n_in = 64, n_in, 64
        # chain_scale: dY is in the chain's d raw domain (draw, view/trunk outputs): A rides at
        # the chain's own per-call scale from max |d raw| (the word it left in `work`); the
        # deformation branch (dL/dx' carries pos_enc's 2^9, rescaled per sample) keeps 2^10.
        # a_t: dY is one of the chain's tiled gradients; X is tiled when it is a kept activation.
        # bf16: one bf16 MFMA per product, no scales (bf16 has fp32's exponent range)
        dW = G[i][0]
        b_t = ((h_tiled and X is not enc and X is not venc and X is not xyz) or X is enc_bf
               or (X is enc and enc_t))
        # f16x3, the 256 x 256 / 128 x 256 / 256 x 64 products of the fused kernels' tiled
        # tensors: one accumulator (aon_gemm f16_single), dY at the chain's scale, X at the
        # forward's 2^3 (train.py; pos_enc(x') and x' far inside the range)
        single = (not bf16 and chain_scale and a_t and b_t and ldx == n_in
                  and (dW.shape[0], n_in) in ((256, 256), (128, 256), (256, 64)))
        gemm(dW[:, col0:] if col0 else dW, dY, X, dW.shape[0], n_in, R, lda=ldy, a_kc=False,
             ldb=ldx, b_kc=False, b_rdiv=rdiv, ldc=dW.stride(0),
             a_scale=1.0 if (chain_scale or bf16) else gs,
             b_scale=1.0 if bf16 else (8.0 if single else acts),
             rowsum=G[i][1] if bias else None,
             a_amax=work if (chain_scale and not bf16) else None, mma_bf16=bf16, a_tiled=a_t,
             b_tiled=b_t, n_store=n_store, f16_single=single)

    def dlatent(i, col0, l, dl, accumulate):
        # (bf16 mode: the exact-fp32 tiny-product path)
        dW, db = G[i]
        W = P[i][0]
        n_out, n = W.shape[0], l.shape[1]
        gemm(dW[:, col0:], db, l, n_out, n, 1, lda=1, a_kc=True, ldb=n, b_kc=False,
             ldc=dW.stride(0), a_scale=gs, b_scale=1.0, exact_fp32=bf16)
        gemm(dl, db, W[:, col0:], 1, n, n_out, lda=n_out, a_kc=True, ldb=W.stride(0), b_kc=False,
             ldc=n, accumulate=accumulate, a_scale=gs, b_scale=W_SCALE, exact_fp32=bf16)

    # every whole-tile product of the level deferred to aon_gemm_batch launches (bf16: the eight
    # 256 x 256 ones -- bottleneck, pts_linears.1-7 -- and the 128-wide view / deformation / enc
    # column ones; fp16x3: all as the fp16x3 class), flushed before the latent terms read the
    # bias gradients; the latent terms then run in the same order as before (bit-identical)
    with batched(cfg.batch_dweights, cfg.batch_128):
        dweight(RGB, draw, 4, hv[3], wc, wc, a_t=False)                   # rgb_layer
        for i in range(3, 0, -1):                                         # views_linear.i
            dweight(VIEW0 + i, dzv[i], wc, hv[i - 1], wc, wc)
        dweight(VIEW0, dzv[0], wc, bot, nw, nw)                           # views_linear.0
        dweight(VIEW0, dzv[0], wc, venc, nv, nv, col0=nw, rdiv=S, bias=False)
        dweight(BOT, dbot, nw, h[7], nw, nw)                              # bottleneck
        dweight(DENS, draw[:, 3:], 4, h[7], nw, nw, a_t=False)            # density
        for i in range(7, 0, -1):                                         # pts_linears.i
            dweight(PTS0 + i, dz[i], nw, h[i - 1], nw, nw)
        dweight(PTS0 + 5, dz[5], nw, enc, ne, ne, col0=nw, bias=False)
        dweight(PTS0, dz[0], nw, enc, ne, ne)                             # pts_linears.0
        dweight(DL, dxp, 3, hd[3], wd, wd, chain_scale=False, a_t=False)  # deformation_layer
        for i in range(3, 0, -1):                                         # deformations_linear.i
            dweight(DEF0 + i, dzd[i], wd, hd[i - 1], wd, wd, chain_scale=False)
        if bf16:  # deformations_linear.0's xyz columns: (xyz^T dZ)^T on the skinny kernel, the
            # bias gradient as dZ's column sums (a 128-wide tile for 3 columns took 0.12 ms)
            gemm(G[DEF0][0], xyz, dzd[0], 3, wd, R, lda=3, a_kc=False, ldb=wd, b_kc=False,
                 ldc=G[DEF0][0].stride(0), rowsum=G[DEF0][1], mma_bf16=True, b_tiled=True,
                 c_trans=True)
        else:
            dweight(DEF0, dzd[0], wd, xyz, 3, 3, chain_scale=False)       # deformations_linear.0
    # the latent terms read the bias gradients just flushed; bf16 (exact-fp32 tiny products): all
    # ten as ONE aon_gemm_small_batch launch, bit-identical to ten launches in this order
    with small_batched():
        dlatent(VIEW0, nw + nv, app, dapp, False)
        dlatent(PTS0 + 5, nw + ne, shape, dshape, False)
        dlatent(PTS0, ne, shape, dshape, True)
        dlatent(DEF0, 3, shape, dshape, True)
        dlatent(DEF0, 3 + geo.n_shape, art, dart, False)
    _train._rec(timers, f"art_dweight{S}", e0, R)


class ArtRenderLevel(torch.autograd.Function):
    """cast_rays + articulated NeRFMLP + activations + volumetric_rendering of one level
    (model_autodecoder.py:296-333) with gradients for the level's 40 MLP parameters and the
    three latent codes (density = shape, color = appearance, articulation)."""

    @staticmethod
    def forward(ctx, geo, cfg, timers, rays_o, rays_d, viewdirs, t_vals, white_bkgd, noise,
                shape, app, art, *params):
        # cfg: the model's TrainNumerics; timers: a dict of hip events (bench.py) or None
        B, S = t_vals.shape
        R, dev = B * S, t_vals.device
        lat = tuple(L.contig(x.detach().reshape(1, -1)) for x in (shape, app, art))
        L.require_gpu(rays_o, rays_d, viewdirs, t_vals, *lat)
        if lat[0].shape[1] != geo.n_shape or lat[1].shape[1] != geo.n_app or lat[2].shape[1] != geo.n_art:
            raise ValueError("latent code sizes do not match the MLP")
        for p in params:
            if not p.is_contiguous():
                raise ValueError("MLP parameters must be contiguous")
        venc = torch.empty((B, geo.nv), device=dev)
        L.call("aon_pos_enc", L.ptr(viewdirs), B, 0, geo.deg_view, L.ptr(venc), L.stream(dev))
        P = [(params[2 * i], params[2 * i + 1]) for i in range(20)]
        # the kernels' layer order, shapes, dtype and device (ValueError, before any launch)
        L.check_mlp_art_layers(P)
        raw = torch.empty((R, 4), device=dev)
        noise = L.contig(noise) if noise is not None else None
        masks = None  # ReLU' bits for the fused backward chain (built there when None)
        enc_bf = None  # the bf16 forward's tiled pos_enc(x') copy
        if cfg.fused_forward and _fused_ok(geo):
            masks = torch.empty((16, tiles.rows(R), 8), dtype=torch.int32, device=dev)
            xyz, hd, enc, h, bot, hv, enc_bf = _forward_level_fused(
                geo, P, lat, L.contig(rays_o), L.contig(rays_d), L.contig(viewdirs),
                L.contig(t_vals), raw, noise, masks, bf16=cfg.bf16, return_enc_bf=True,
                art_forward=cfg.art_forward, timers=timers)
        else:
            xyz = torch.empty((R, 3), device=dev)
            L.call("aon_cast_rays", L.ptr(rays_o), L.ptr(rays_d), L.ptr(t_vals), B, S, None, 0,
                   L.ptr(xyz), 0, 0, None, L.stream(dev))
            hd, enc, h, bot, hv = _forward_level(geo, P, lat, xyz, venc, S, raw, noise,
                                                 exact_folds=cfg.bf16)
        comp = torch.empty((B, 3), device=dev)
        acc = torch.empty((B,), device=dev)
        weights = torch.empty((B, S), device=dev)
        depth = torch.empty((B,), device=dev)
        L.call("aon_composite_fwd", L.ptr(raw), 4, L.ptr(raw[:, 3:]), 4, L.ptr(t_vals),
               L.ptr(rays_d), B, S, int(bool(white_bkgd)), L.ACT_ARTIC, L.ptr(comp), L.ptr(acc),
               L.ptr(weights), L.ptr(depth), L.stream(dev))
        ctx.save_for_backward(rays_d, t_vals, xyz, enc, venc, raw, hd, h, bot, hv, *lat, *params)
        ctx.masks = masks
        ctx.enc_bf = enc_bf if masks is not None else None
        ctx.h_tiled = masks is not None  # the fused forward keeps its tensors tiled
        ctx.meta = (geo, B, S, bool(white_bkgd), tuple(x.shape for x in (shape, app, art)))
        ctx.cfg, ctx.timers = cfg, timers
        ctx.mark_non_differentiable(weights)
        # unused outputs (acc, depth, weights in training_step) get no zero-filled gradients
        ctx.set_materialize_grads(False)
        return comp, acc, depth, weights

    @staticmethod
    def backward(ctx, g_rgb, g_acc, g_depth, _g_w):
        geo, B, S, white, lat_shapes = ctx.meta
        saved = ctx.saved_tensors
        rays_d, t_vals, xyz, enc, venc, raw, hd, h, bot, hv = saved[:10]
        lat = saved[10:13]
        params = saved[13:]
        dev = raw.device
        R = B * S
        draw = torch.empty((R, 4), device=dev)
        if g_rgb is None:
            g_rgb = torch.zeros((B, 3), device=dev)
        L.call("aon_composite_bwd", L.ptr(raw), 4, L.ptr(raw[:, 3:]), 4, L.ptr(t_vals),
               L.ptr(rays_d), B, S, int(white), L.ACT_ARTIC, L.ptr(L.contig(g_rgb)),
               L.ptr(L.contig(g_acc)) if g_acc is not None else None,
               L.ptr(L.contig(g_depth)) if g_depth is not None else None,
               L.ptr(draw), L.ptr(draw[:, 3:]), 4, L.stream(dev))
        P = [(params[2 * i], params[2 * i + 1]) for i in range(20)]
        G = [(torch.empty_like(w), torch.empty_like(b)) for w, b in P]
        dlat = tuple(torch.empty_like(x) for x in lat)
        if ctx.cfg.fused_backward and _fused_ok(geo):
            _backward_level_fused(geo, P, G, lat, dlat, xyz, enc, venc, S, hd, h, bot, hv, draw,
                                  ctx.masks, ctx.h_tiled, ctx.enc_bf, timers=ctx.timers,
                                  cfg=ctx.cfg)
        else:
            if ctx.h_tiled:  # the all-GEMM backward reads row-major fp32 activations
                hd, h, hv = (torch.stack([tiles.untile(x, R).float() for x in t]) for t in (hd, h, hv))
                bot = tiles.untile(bot, R).float()
            _backward_level(geo, P, G, lat, dlat, xyz, enc, venc, S, hd, h, bot, hv, draw)
        grads = [g for pair in G for g in pair]
        dlat = [d.reshape(s) for d, s in zip(dlat, lat_shapes)]
        return (None, None, None, None, None, None, None, None, None, *dlat, *grads)


def render_level(mlp, rays_o, rays_d, viewdirs, t_vals, white_bkgd, latents, noise=None,
                 cfg=DEFAULT, timers=None):
    """One NeRF_AE_Art level under autograd -> (comp_rgb, acc, depth, weights); ``cfg``: the
    model's TrainNumerics."""
    params = [p for m in art_layers(mlp) for p in (m.weight, m.bias)]
    geo = getattr(mlp, "_geo", None)
    if geo is None:
        geo = mlp._geo = _Geo(mlp)
    return ArtRenderLevel.apply(geo, cfg, timers, rays_o, rays_d, viewdirs, t_vals,
                                bool(white_bkgd), noise,
                                latents["density"], latents["color"], latents["articulation"],
                                *params)


class LatentReg(torch.autograd.Function):
    """The latent regulariser of training_step (model_autodecoder.py:456-466):
    1e-4 * (mean ||shape||_0 + mean ||appearance||_0 + mean ||articulation||_0), norms over
    dim 0 (aon_latent_reg)."""

    @staticmethod
    def forward(ctx, shape, app, art):
        codes = [L.contig(x.detach()) for x in (shape, app, art)]
        L.require_gpu(*codes)
        loss = torch.empty((), device=shape.device)
        grads = []
        for i, c in enumerate(codes):
            c2 = c.reshape(c.shape[0], -1)  # norm over dim 0: (1, C) -> |x|, (C,) -> ||x||
            g = torch.empty_like(c)
            L.call("aon_latent_reg", L.ptr(c2), c2.shape[0], c2.shape[1], 1e-4, int(i > 0),
                   L.ptr(loss), L.ptr(g), L.stream(shape.device))
            grads.append(g)
        ctx.save_for_backward(*grads)
        return loss

    @staticmethod
    def backward(ctx, g):
        # the regulariser is a leaf term of the loss: g is dL/dreg = 1 (a scalar multiply by
        # a non-unit g would be the only torch arithmetic; training_step always passes 1)
        return tuple(x * g for x in ctx.saved_tensors)


def training_step(model, code_library, batch, randomized, white_bkgd, near, far, *,
                  u_coarse=None, u_fine=None, timers=None):
    """LitNeRF_AutoDecoder.training_step (model_autodecoder.py:395-477) ->
    (loss, logs{loss0, loss1, reg, psnr0, psnr1}).  ``batch`` holds rays_o / rays_d / viewdirs /
    target (B, 3) and instance_id / articulation_id (1,) as the reference's loader gives them
    after its squeeze (model_autodecoder.py:396-399).  The kernels and precision are the model's
    own (model.train_numerics)."""
    latents = code_library(batch)
    ret = model(batch, randomized, white_bkgd, near, far, latents, u_coarse=u_coarse,
                u_fine=u_fine, timers=timers)
    reg = LatentReg.apply(latents["density"], latents["color"], latents["articulation"])
    # loss1 + loss0 + reg and the psnrs in one launch (train.LossPair)
    loss, loss0, loss1, psnr0, psnr1 = loss_pair(ret[0][0], ret[1][0], batch["target"], reg)
    return loss, dict(loss0=loss0, loss1=loss1, reg=reg, psnr0=psnr0, psnr1=psnr1)


def configure_optimizers(model, code_library, lr_init=5.0e-4):
    """configure_optimizers (model_autodecoder.py:599-601): Adam over the MLPs and the code
    library (the fused aon_adam_step, betas (0.9, 0.999))."""
    return Adam(list(model.parameters()) + list(code_library.parameters()), lr=lr_init,
                betas=(0.9, 0.999))
