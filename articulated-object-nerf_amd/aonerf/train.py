"""Training step of the reference (LitNeRF.training_step, model.py:256-282; configure_optimizers /
optimizer_step, model.py:386-419) on the HIP kernels.

One render level under autograd is ``RenderLevel`` (a torch.autograd.Function):

  forward   ONE fused kernel (aon_mlp_fwd_train: cast_rays, pos_enc, the whole NeRFMLP and the
            sigmoid/relu of model.py:186-187 in registers) that also stores every hidden
            activation and their ReLU' bits for the backward -> compositing (aon_composite_fwd)
  backward  aon_composite_bwd (dL/draw) -> ONE fused kernel for the whole input-gradient chain
            dX = (dY W) * relu'(X) (aon_mlp_bwd, masks from the stored bits) -> per layer
            dW = dY^T X and db = sum_rows dY from the same pass (aon_gemm, split-K,
            deterministic)

(The model's TrainNumerics -- aonerf/numerics.py, per model -- with fused_forward /
fused_backward False selects the layer-by-layer aon_gemm forward and backward that the fused
kernels replaced; both are gated identically in tests/test_gpu_train.py.)

Gradients land in each parameter's ``.grad`` through autograd, so the reference's own
optimizer code runs unchanged (the fp16x3 range guard reaches it through a global
torch.optim step pre-hook); ``Adam`` below is the fused replacement (aon_adam_step) with the
reference's learning-rate schedule.  All arithmetic is in the HIP kernels; torch only
allocates buffers and routes autograd.
"""
import contextlib

import numpy as np
import torch
import torch.optim.optimizer as _torch_optim

from . import _lib as L
from . import tiles

from .linalg import ACT_SCALE, GRAD_SCALE, W_SCALE, batched, colsum, gemm, linear_fwd  # noqa: F401
from .numerics import DEFAULT, TrainNumerics  # noqa: F401

# ---------------------------------------------------------------------------- one render level
def _mlp_params(mlp):
    """(weight, bias) of pts_linears[0..7], density, bottleneck, views[0], rgb."""
    return [(m.weight, m.bias) for m in mlp._layers()]


def _forward_level(P, enc, venc, S, raw, noise=None):
    """NeRFMLP.forward (model.py:95-120) layer by layer; returns the kept activations."""
    R, dev = enc.shape[0], enc.device
    h = [torch.empty((R, 256), device=dev) for _ in range(8)]
    linear_fwd(h[0], enc, 63, *P[0], relu=True)
    for i in range(1, 8):
        if i == 5:  # cat[h4, enc] (model.py:102-103)
            linear_fwd(h[5], h[4], 256, *P[5], relu=True, X2=enc, K2=63, ld2=63)
        else:
            linear_fwd(h[i], h[i - 1], 256, *P[i], relu=True)
    if noise is not None:  # raw_sigma + noise (model.py:183-184), added in the GEMM epilogue
        raw[:, 3].copy_(noise)
    linear_fwd(raw[:, 3:], h[7], 256, *P[8], ldo=4, accumulate=noise is not None)  # (:105-107)
    bot = torch.empty((R, 256), device=dev)
    linear_fwd(bot, h[7], 256, *P[9])                                    # bottleneck, no act
    hv = torch.empty((R, 128), device=dev)
    linear_fwd(hv, bot, 256, *P[10], relu=True, X2=venc, K2=27, ld2=27, rdiv2=S)  # (:110-116)
    linear_fwd(raw, hv, 128, *P[11], ldo=4)                              # rgb (model.py:118)
    return h, bot, hv


def _amax_word(x, word):
    """word (one int32 of a device tensor) = the bits of max |x| (aon_absmax): the per-call
    scale of a gradient operand's fp16 hi/lo split (include/aonerf.h a_amax)."""
    L.call("aon_absmax", L.ptr(x), x.numel(), L.ptr(word), L.stream(x.device))
    return word


def _backward_level(P, G, enc, venc, S, h, bot, hv, draw):
    """Autograd of _forward_level: G[i] = (dW, db) of layer i, from dL/draw (R x 4).  Every
    gradient operand dY enters the f16x3 split at its own per-call power-of-two scale from
    max |dY| (aon_absmax -> aon_gemm a_amax), as the fused chain scales its d raw: a fixed
    prescale would push the small dL/dz of a late-training step into fp16's subnormals."""
    R, dev = enc.shape[0], enc.device
    acts = ACT_SCALE
    words = torch.zeros((8,), dtype=torch.int32, device=dev)

    def dweight(dW, dY, ldy, n_out, X, ldx, n_in, rdiv=1, col0=0, ldw=None, db=None, amax=None):
        # dW[:, col0:col0+n_in] = dY^T X (K = rows, split over workgroups); db = sum_rows dY
        # from the same pass over dY
        gemm(dW[:, col0:] if col0 else dW, dY, X, n_out, n_in, R, lda=ldy, a_kc=False, ldb=ldx,
             b_kc=False, b_rdiv=rdiv, ldc=ldw or dW.shape[1], a_scale=1.0, b_scale=acts,
             rowsum=db, a_amax=amax)

    def dinput(dX, dY, ldy, n_out, W, n_in, mask=None, accumulate=False, amax=None):
        # dX (R x n_in) = dY W[:, :n_in] (* relu mask)
        gemm(dX, dY, W, R, n_in, n_out, lda=ldy, a_kc=True, ldb=W.shape[1], b_kc=False,
             ldc=dX.shape[1], mask=mask, ldm=mask.shape[1] if mask is not None else 0,
             accumulate=accumulate, a_scale=1.0, b_scale=W_SCALE, a_amax=amax)

    # rgb head (N=3) and view layer
    wd = _amax_word(draw, words[0:1])  # d raw (its sigma column too: a max over both is safe)
    dweight(G[11][0], draw, 4, 3, hv, 128, 128, db=G[11][1], amax=wd)
    dhv = torch.empty((R, 128), device=dev)
    dinput(dhv, draw, 4, 3, P[11][0], 128, mask=hv, amax=wd)
    wv = _amax_word(dhv, words[1:2])
    dweight(G[10][0], dhv, 128, 128, bot, 256, 256, db=G[10][1], amax=wv)
    dweight(G[10][0], dhv, 128, 128, venc, 27, 27, rdiv=S, col0=256, amax=wv)
    dbot = torch.empty((R, 256), device=dev)
    dinput(dbot, dhv, 128, 128, P[10][0], 256, amax=wv)
    del dhv
    # bottleneck + density heads on h7
    wb = _amax_word(dbot, words[2:3])
    dweight(G[9][0], dbot, 256, 256, h[7], 256, 256, db=G[9][1], amax=wb)
    dweight(G[8][0], draw[:, 3:], 4, 1, h[7], 256, 256, db=G[8][1], amax=wd)
    dy = torch.empty((R, 256), device=dev)
    dinput(dy, dbot, 256, 256, P[9][0], 256, amax=wb)
    dinput(dy, draw[:, 3:], 4, 1, P[8][0], 256, mask=h[7], accumulate=True, amax=wd)
    del dbot
    dx = torch.empty((R, 256), device=dev)
    for i in range(7, -1, -1):  # dy = dL/d(pre-activation of layer i)
        wy = _amax_word(dy, words[3 + (i & 1):4 + (i & 1)])
        if i == 5:
            dweight(G[5][0], dy, 256, 256, h[4], 256, 256, db=G[5][1], amax=wy)
            dweight(G[5][0], dy, 256, 256, enc, 63, 63, col0=256, amax=wy)
        elif i == 0:
            dweight(G[0][0], dy, 256, 256, enc, 63, 63, db=G[0][1], amax=wy)
        else:
            dweight(G[i][0], dy, 256, 256, h[i - 1], 256, 256, db=G[i][1], amax=wy)
        if i > 0:
            dinput(dx, dy, 256, 256, P[i][0], 256, mask=h[i - 1], amax=wy)
            dx, dy = dy, dx


# Which kernels and precision a level trains with is the MODEL's TrainNumerics
# (aonerf/numerics.py; NeRF(train_precision=...)), passed into RenderLevel per call -- no
# module-level switch.  ``timers`` (a dict, optional, per call) -> hip events around each level's
# training kernels (bench.py's train_step roofline): "fwd_train<S>", "bwd_chain<S>", "dweight<S>".


def _ev(timers):
    if timers is None:
        return None
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return e


def _rec(timers, key, e0, rows):
    if e0 is not None:
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        timers.setdefault(key, []).append((e0, e1, rows))


class JoinToken:
    """The side-stream work of one forward's render levels, joined by Join.backward."""

    def __init__(self):
        self.pending = []  # (stream the caller waits on, event on the side stream)


class Join(torch.autograd.Function):
    """Identity on the render levels' parameters (views), whose backward runs after every
    level's: it joins the side stream (TrainNumerics.overlap_dweight) before the gradients reach the
    parameters."""

    @staticmethod
    def forward(ctx, token, *params):
        ctx.token = token
        ctx.set_materialize_grads(False)
        return tuple(p.view_as(p) for p in params)

    @staticmethod
    def backward(ctx, *grads):
        for stream, ev in ctx.token.pending:
            stream.wait_event(ev)
        ctx.token.pending.clear()
        return (None, *grads)


_side = {}


def _side_stream(dev):
    s = _side.get(str(dev))
    if s is None:
        s = _side[str(dev)] = torch.cuda.Stream(device=dev)
    return s


@contextlib.contextmanager
def _on_side(token, dev, tensors):
    """Run the enclosed launches on the device's side stream after the current stream's work so
    far; ``tensors`` (every tensor they touch) are kept from the caching allocator until the
    side stream is done with them, and ``token`` records the join.  token None: in place."""
    if token is None:
        yield
        return
    main = torch.cuda.current_stream(dev)
    side = _side_stream(dev)
    side.wait_stream(main)
    with torch.cuda.stream(side):
        yield
    for t in tensors:
        if t is not None:
            t.record_stream(side)
    ev = torch.cuda.Event()
    ev.record(side)
    token.pending.append((main, ev))


_packed = {}


def _params_struct(P):
    """AonMlpParams of one level's (weight, bias) pairs in the kernels' layer order (pts_linears.0
    ..7, density, bottleneck, views_linear.0, rgb): shapes, dtype, device and contiguity are
    checked against the layer table (ValueError) before any pointer reaches a pack kernel, and
    the C side checks the shapes again (aon_mlp_params, ABI 9)."""
    return L.mlp_params(P)


def _buffer(key, nbytes, dev, guard=False, params=()):
    # one buffer per kind and device: a pack and the kernel reading it are stream-ordered.
    # guard: a packed weight stream whose range-status word the next optimizer step over
    # ``params`` (the packed parameters) checks
    buf = _packed.get((key, str(dev)))
    if buf is None:
        buf = torch.empty(max(nbytes // 4, 1), dtype=torch.float32, device=dev)
        _packed[(key, str(dev))] = buf
    if guard:
        L.register_pack(("train", key), buf, params)
    return buf


# an optimizer step refuses gradients whose kernels met a fp16x3 range overflow (one sync per
# step): aonerf's Adam.step, and every other torch.optim optimizer through a global step pre-hook
_RANGE_MSG = ("a fp16x3 training kernel met a value beyond its fp16 hi/lo range (|activation| > "
              "8188 or an overflowing gradient): the gradients of this step are invalid and were "
              "not applied.  Train this model on the layer-by-layer GEMM path "
              "(train_numerics=TrainNumerics(fused_forward=False, fused_backward=False)), whose "
              "operands carry a 2^-8 scale (range 1.6e7), or with train_precision='bf16'.")


def check_range(devices=None, params=None):
    """Raise FloatingPointError if a fused fp16x3 training kernel on ``devices`` that packed any
    of ``params`` (None: any) overflowed since the last check (consumes those pending packs)."""
    ids = None if params is None else {p.data_ptr() for p in params}
    if L.check_pending(devices, ids):
        raise FloatingPointError(_RANGE_MSG)


def _optimizer_step_pre_hook(optimizer, args, kwargs):
    # the reference trains through Lightning with torch.optim.Adam (configure_optimizers,
    # model.py:386-389): the guard must hold for any optimizer, not only aonerf's Adam -- but only
    # for the packs of the parameters it steps: an unrelated optimizer neither pays
    # the sync nor consumes this model's overflow
    if not L.PENDING_PACKS and not L._STICKY:
        return
    params = [p for g in optimizer.param_groups for p in g["params"]]
    devs = {str(p.device) for p in params}
    if L.has_pending(devs, {p.data_ptr() for p in params}):
        check_range(devs, params)


_HOOK = _torch_optim.register_optimizer_step_pre_hook(_optimizer_step_pre_hook)


def _pack(P, dev, tag="", bf16=False):
    """The f16x3 (or bf16) weight stream of one level's parameters, re-packed on every call (the
    optimizer updates the parameters in place behind torch's version counters).  ``tag``: one
    buffer per level (its range-status word must survive until the optimizer step)."""
    prec = L.PREC_BF16 if bf16 else L.PREC_F16X3_TRAIN
    buf = _buffer(f"fwd{'bf' if bf16 else ''}{tag}", L.lib().aon_mlp_packed_bytes(prec), dev,
                  guard=not bf16, params=[t for wb in P for t in wb])
    L.call("aon_mlp_pack", L.ctypes.byref(_params_struct(P)), prec, L.ptr(buf), L.stream(dev))
    return buf


def _pack_bwd(P, dev, tag="", bf16=False):
    """The transposed weight stream of the fused backward chain (aon_mlp_bwd_pack[_bf16])."""
    buf = _buffer(f"bwd{'bf' if bf16 else ''}{tag}", L.lib().aon_mlp_bwd_packed_bytes(), dev,
                  guard=not bf16, params=[t for wb in P for t in wb])
    L.call("aon_mlp_bwd_pack_bf16" if bf16 else "aon_mlp_bwd_pack",
           L.ctypes.byref(_params_struct(P)), L.ptr(buf), L.stream(dev))
    return buf


def relu_masks(acts, R):
    """ReLU' bits (len(acts), tiles.rows(R), 4) x 64-bit words (aon_relu_masks) of row-major
    stored activations, in the (tiled) layout the fused training forwards write: the masks of
    the fused backward chains after a layer-by-layer forward."""
    dev = acts[0].device
    masks = torch.empty((len(acts), tiles.rows(R), 8), dtype=torch.int32, device=dev)
    for i, a in enumerate(acts):
        L.call("aon_relu_masks", L.ptr(L.contig(a)), R, a.shape[-1], L.ptr(masks[i]), L.stream(dev))
    return masks


def _backward_level_fused(P, G, enc, venc, S, h, bot, hv, draw, masks=None, h_tiled=True,
                          token=None, timers=None, cfg=DEFAULT):
    """_backward_level with every input-gradient product in one fused kernel (aon_mlp_bwd);
    the weight gradients dW = dZ^T X and db = sum_rows dZ stay split-K GEMMs.  ``masks``: the
    ReLU' bits of h0..h7, hv from the fused forward (built from the activations when None).
    h_tiled: h / bot / hv in the fused forward's tiled layout (tiles.py), else row-major (the
    layer-by-layer forward).  The chain's dz / dzb / dzv are always tiled.  ``token`` (a
    JoinToken): the weight gradients run on the side stream (TrainNumerics.overlap_dweight);
    ``timers``: hip events per kernel class (bench.py); ``cfg``: the model's TrainNumerics (the
    weight-gradient batching)."""
    R, dev = draw.shape[0], draw.device
    bf16 = h[0].dtype == torch.bfloat16  # activations kept by the bf16 training forward
    if masks is None:
        acts = list(h) + [hv]
        masks = relu_masks([tiles.untile(a, R) for a in acts] if h_tiled else acts, R)
    dt = torch.bfloat16 if bf16 else torch.float32
    NR = tiles.rows(R)
    dzv = torch.empty((NR, 128), device=dev, dtype=dt)
    dzb = torch.empty((NR, 256), device=dev, dtype=dt)
    dz = torch.empty((8, NR, 256), device=dev, dtype=dt)
    # the chain's d raw scale word: the weight gradients read it, on the side stream while the
    # next level's chain may already run -- its own word then
    work = _buffer("work", 4, dev) if token is None else torch.empty((1,), device=dev)
    packed = _pack_bwd(P, dev, S, bf16)
    e0 = _ev(timers)
    L.call("aon_mlp_bwd_bf16" if bf16 else "aon_mlp_bwd", L.ptr(packed), L.ptr(draw), L.ptr(masks),
           R, L.ptr(dzv), L.ptr(dzb), L.ptr(dz), L.ptr(work), L.stream(dev))
    L.snapshot_pack(packed)  # the chain was the pack's last reader (range guard, _lib)
    _rec(timers, f"bwd_chain{S}", e0, R)
    e0 = _ev(timers)
    acts = ACT_SCALE

    # the tiled copy of pos_enc(x): the bf16 forward's (NR, 128) bf16 or the f16x3 mode's
    # (NR, 64) fp32 (aon_cast_rays_tiled); else row-major (R, 63)
    enc_t = enc.shape[1] != 63

    def dweight(dW, dY, ldy, n_out, X, ldx, n_in, rdiv=1, col0=0, db=None, a_t=True):
        # f16x3: dY rides at the chain's own per-call scale from max |d raw| (the word in
        # `work`); bf16: one bf16 MFMA per product, no scales needed.  dY: the chain's tiled
        # gradients (a_t) or row-major d raw; X: a kept activation (tiled when h_tiled), the
        # encodings (row-major (R, 63), or the bf16 forward's tiled (NR, 128): n_store 63) or
        # the per-ray view encodings
        b_t = (h_tiled and X is not enc and X is not venc) or (X is enc and enc_t)
        n_store = 0
        if X is enc and enc_t:
            ldx, n_store, n_in = enc.shape[1], n_in, enc.shape[1]
        # f16x3, the 256 x 256 / 128 x 256 / 256 x 64 products of the fused kernels' tiled
        # tensors: one accumulator (aon_gemm f16_single) with dY at the chain's scale and X at
        # the forward's 2^3, the scales both kernels range-guard their own splits at (pos_enc(x)
        # and x itself: far inside the range)
        single = (not bf16 and a_t and b_t
                  and (n_out, n_in) in ((256, 256), (128, 256), (256, 64)))
        gemm(dW[:, col0:] if col0 else dW, dY, X, n_out, n_in, R, lda=ldy, a_kc=False, ldb=ldx,
             b_kc=False, b_rdiv=rdiv, ldc=dW.shape[1], a_scale=1.0,
             b_scale=1.0 if bf16 else (8.0 if single else acts), rowsum=db,
             a_amax=None if bf16 else work, mma_bf16=bf16, a_tiled=a_t, b_tiled=b_t,
             n_store=n_store, f16_single=single)

    # bf16: the eight 256 x 256 products (bottleneck, pts_linears.1-7) run as one aon_gemm_batch
    touched = [dzv, dzb, dz, draw, work, enc, venc, bot, hv, *h, *(t for wb in G for t in wb)]
    with _on_side(token, dev, touched), batched(cfg.batch_dweights, cfg.batch_128):
        dweight(G[11][0], draw, 4, 3, hv, 128, 128, db=G[11][1], a_t=False)    # rgb_layer
        dweight(G[10][0], dzv, 128, 128, bot, 256, 256, db=G[10][1])           # views_linear.0
        dweight(G[10][0], dzv, 128, 128, venc, 27, 27, rdiv=S, col0=256)
        dweight(G[9][0], dzb, 256, 256, h[7], 256, 256, db=G[9][1])            # bottleneck
        dweight(G[8][0], draw[:, 3:], 4, 1, h[7], 256, 256, db=G[8][1], a_t=False)  # density
        for i in range(7, -1, -1):                                             # pts_linears.i
            if i == 5:
                dweight(G[5][0], dz[5], 256, 256, h[4], 256, 256, db=G[5][1])
                dweight(G[5][0], dz[5], 256, 256, enc, 63, 63, col0=256)
            elif i == 0:
                dweight(G[0][0], dz[0], 256, 256, enc, 63, 63, db=G[0][1])
            else:
                dweight(G[i][0], dz[i], 256, 256, h[i - 1], 256, 256, db=G[i][1])
    _rec(timers, f"dweight{S}", e0, R)


def _forward_level_fused(P, rays_o, rays_d, viewdirs, t_vals, raw, noise=None, masks=None,
                         bf16=False, enc=None):
    """_forward_level on the fused kernel: raw (R x 4) and the kept activations (tiled,
    tiles.rows(R) rows each); ``masks`` ((9, tiles.rows(R), 8) int32) receives their ReLU' bits
    for the backward chain.  bf16: the bf16 training mode (activations kept as torch.bfloat16;
    ``enc``, optional, (tiles.rows(R), 128) bfloat16, receives pos_enc(x) tiled, columns 63..
    zero)."""
    B, S = t_vals.shape
    R, dev = B * S, t_vals.device
    NR = tiles.rows(R)  # kept tensors: the tiled layout (tiles.py)
    if masks is None:
        masks = torch.empty((9, NR, 8), dtype=torch.int32, device=dev)
    dt = torch.bfloat16 if bf16 else torch.float32
    hbuf = torch.empty((8, NR, 256), device=dev, dtype=dt)
    bot = torch.empty((NR, 256), device=dev, dtype=dt)
    hv = torch.empty((NR, 128), device=dev, dtype=dt)
    for w, b in P:
        if not (w.is_contiguous() and b.is_contiguous()):
            raise ValueError("MLP parameters must be contiguous")
    packed = _pack(P, dev, S, bf16)
    args = (L.ptr(packed), L.ptr(rays_o), L.ptr(rays_d), L.ptr(viewdirs), L.ptr(t_vals), B, S,
            L.ptr(noise) if noise is not None else None, L.ptr(hbuf), L.ptr(bot), L.ptr(hv),
            L.ptr(raw), L.ptr(masks))
    if bf16:
        L.call("aon_mlp_fwd_train_bf16", *args, L.ptr(enc) if enc is not None else None,
               L.stream(dev))
    else:
        L.call("aon_mlp_fwd_train", *args, L.stream(dev))
    L.snapshot_pack(packed)  # the forward was the pack's last reader (range guard, _lib)
    return list(hbuf.unbind(0)), bot, hv


class RenderLevel(torch.autograd.Function):
    """cast_rays + pos_enc + NeRFMLP + activations + volumetric_rendering of one level
    (model.py:175-197) with gradients for the level's 24 MLP parameters."""

    @staticmethod
    def forward(ctx, rays_o, rays_d, viewdirs, t_vals, white_bkgd, noise, token, cfg, timers,
                *params):
        # cfg: the model's TrainNumerics; timers: a dict of hip events (bench.py) or None
        B, S = t_vals.shape
        ctx.token = token  # a JoinToken: the weight gradients may run on the side stream
        ctx.cfg, ctx.timers = cfg, timers
        R, dev = B * S, t_vals.device
        bf16 = cfg.fused_forward and cfg.bf16
        if bf16:  # the bf16 training forward keeps pos_enc(x) itself (bf16, tiled, 128 columns)
            enc = torch.empty((tiles.rows(R), 128), device=dev, dtype=torch.bfloat16)
        elif cfg.fused_forward and cfg.fused_backward:
            # xyz = o + t d straight into the encodings, tiled with 64 columns (column 63 zero):
            # the fused backward's enc-column weight gradients read whole 16-column tiles
            enc = torch.empty((tiles.rows(R), 64), device=dev)
            L.call("aon_cast_rays_tiled", L.ptr(L.contig(rays_o)), L.ptr(L.contig(rays_d)),
                   L.ptr(L.contig(t_vals)), B, S, 0, 10, 64, L.ptr(enc), L.stream(dev))
        else:
            # xyz = o + t d (helper.py:25-26) straight into the encodings (helper.py:136-140)
            enc = torch.empty((R, 63), device=dev)
            L.call("aon_cast_rays", L.ptr(rays_o), L.ptr(rays_d), L.ptr(t_vals), B, S, None, 0,
                   None, 0, 10, L.ptr(enc), L.stream(dev))
        venc = torch.empty((B, 27), device=dev)
        L.call("aon_pos_enc", L.ptr(viewdirs), B, 0, 4, L.ptr(venc), L.stream(dev))
        P = [(params[2 * i], params[2 * i + 1]) for i in range(12)]
        # the kernels' layer order, shapes, dtype and device (ValueError, before any launch)
        L.check_mlp_layers(P)
        raw = torch.empty((R, 4), device=dev)
        masks = None  # ReLU' bits for the fused backward chain (built there when None)
        if cfg.fused_forward:
            noise = L.contig(noise) if noise is not None else None
            masks = torch.empty((9, tiles.rows(R), 8), dtype=torch.int32, device=dev)
            e0 = _ev(timers)
            h, bot, hv = _forward_level_fused(P, L.contig(rays_o), L.contig(rays_d),
                                              L.contig(viewdirs), L.contig(t_vals), raw, noise,
                                              masks, bf16=bf16, enc=enc if bf16 else None)
            _rec(timers, f"fwd_train{S}", e0, R)
        else:
            h, bot, hv = _forward_level(P, enc, venc, S, raw, noise)
        comp = torch.empty((B, 3), device=dev)
        acc = torch.empty((B,), device=dev)
        weights = torch.empty((B, S), device=dev)
        depth = torch.empty((B,), device=dev)
        L.call("aon_composite_fwd", L.ptr(raw), 4, L.ptr(raw[:, 3:]), 4, L.ptr(t_vals),
               L.ptr(rays_d), B, S, int(bool(white_bkgd)), L.ACT_VANILLA, L.ptr(comp), L.ptr(acc),
               L.ptr(weights), L.ptr(depth), L.stream(dev))
        ctx.save_for_backward(rays_d, t_vals, enc, venc, raw, bot, hv, *h, *params)
        ctx.masks = masks
        ctx.h_tiled = cfg.fused_forward  # the fused forward keeps its tensors tiled
        ctx.meta = (B, S, bool(white_bkgd))
        ctx.mark_non_differentiable(weights)
        # unused outputs (acc, depth, weights in training_step) get no zero-filled gradients
        ctx.set_materialize_grads(False)
        return comp, acc, depth, weights

    @staticmethod
    def backward(ctx, g_rgb, g_acc, g_depth, _g_w):
        B, S, white = ctx.meta
        saved = ctx.saved_tensors
        rays_d, t_vals, enc, venc, raw, bot, hv = saved[:7]
        h = list(saved[7:15])
        params = saved[15:]
        dev = raw.device
        R = B * S
        draw = torch.empty((R, 4), device=dev)
        g_rgb = L.contig(g_rgb) if g_rgb is not None else torch.zeros((B, 3), device=dev)
        L.call("aon_composite_bwd", L.ptr(raw), 4, L.ptr(raw[:, 3:]), 4, L.ptr(t_vals),
               L.ptr(rays_d), B, S, int(white), L.ACT_VANILLA, L.ptr(g_rgb),
               L.ptr(L.contig(g_acc)) if g_acc is not None else None,
               L.ptr(L.contig(g_depth)) if g_depth is not None else None,
               L.ptr(draw), L.ptr(draw[:, 3:]), 4, L.stream(dev))
        P = [(params[2 * i], params[2 * i + 1]) for i in range(12)]
        G = [(torch.empty_like(w), torch.empty_like(b)) for w, b in P]
        cfg, timers = ctx.cfg, ctx.timers
        if cfg.fused_backward:
            # (not while timers time each level's kernels on the current stream)
            token = ctx.token if cfg.overlap_dweight and timers is None else None
            _backward_level_fused(P, G, enc, venc, S, h, bot, hv, draw, ctx.masks, ctx.h_tiled,
                                  token=token, timers=timers, cfg=cfg)
        else:
            if ctx.h_tiled:  # the all-GEMM backward reads row-major fp32 activations
                h = [tiles.untile(x, R).float() for x in h]
                bot, hv = tiles.untile(bot, R).float(), tiles.untile(hv, R).float()
            if enc.shape[1] != 63:  # a tiled copy (the bf16 forward's, or aon_cast_rays_tiled's)
                enc = tiles.untile(enc, R)[:, :63].float().contiguous()
            _backward_level(P, G, enc, venc, S, h, bot, hv, draw)
        grads = [g for pair in G for g in pair]
        return (None, None, None, None, None, None, None, None, None, *grads)


class Mse(torch.autograd.Function):
    """img2mse (helper.py:17-18) on aon_mse."""

    @staticmethod
    def forward(ctx, pred, target):
        L.require_gpu(pred, target)
        pred, target = L.contig(pred), L.contig(target)
        loss = torch.empty((), device=pred.device)
        grad = torch.empty_like(pred)
        L.call("aon_mse", L.ptr(pred), L.ptr(target), pred.numel(), 1.0, L.ptr(loss), L.ptr(grad),
               L.stream(pred.device))
        ctx.save_for_backward(grad)
        return loss

    @staticmethod
    def backward(ctx, g):
        (grad,) = ctx.saved_tensors
        return grad * g, None


def img2mse(x, y):
    return Mse.apply(x, y)


def mse2psnr(x):
    """helper.py:21-22 (host-side scalar formula)."""
    return -10.0 * torch.log(x) / np.log(10.0)


class LossPair(torch.autograd.Function):
    """The training step's loss terms (model.py:265-270; model_autodecoder.py:455-470):
    loss = (img2mse(fine) + img2mse(coarse)) [+ reg] and both mses in one aon_loss_pair launch,
    mse2psnr of both in one pass of torch's own log / mul / div (torch's device log is not
    correctly rounded: tools/diag/psnr_ulp.py) -- the same values as img2mse / `+` / mse2psnr,
    bit for bit, in 4 launches where those took 9.  Backward: one aon_loss_pair_bwd launch for
    both levels' rgb gradients."""

    @staticmethod
    def forward(ctx, pred0, pred1, target, reg):
        L.require_gpu(pred0, pred1, target)
        pred0, pred1, target = L.contig(pred0), L.contig(pred1), L.contig(target)
        if pred0.shape != target.shape or pred1.shape != target.shape:
            raise ValueError("LossPair: predictions and target must have one shape")
        out = torch.empty((3,), device=pred0.device)
        g0, g1 = torch.empty_like(pred0), torch.empty_like(pred1)
        L.call("aon_loss_pair", L.ptr(pred0), L.ptr(pred1), L.ptr(target), pred0.numel(),
               L.ptr(L.contig(reg)) if reg is not None else None, L.ptr(out), L.ptr(g0), L.ptr(g1),
               L.stream(pred0.device))
        ctx.save_for_backward(g0, g1)
        ctx.has_reg = reg is not None
        ctx.set_materialize_grads(False)
        psnr0, psnr1 = mse2psnr(out[1:]).unbind(0)
        loss, loss0, loss1 = out.unbind(0)
        ctx.mark_non_differentiable(psnr0, psnr1)
        return loss, loss0, loss1, psnr0, psnr1

    @staticmethod
    def backward(ctx, g, g0, g1, _p0, _p1):
        grad0, grad1 = ctx.saved_tensors
        if g is None and g0 is None and g1 is None:
            return None, None, None, None
        d0, d1 = torch.empty_like(grad0), torch.empty_like(grad1)
        L.call("aon_loss_pair_bwd", L.ptr(grad0), L.ptr(grad1), grad0.numel(),
               *(L.ptr(L.contig(x)) if x is not None else None for x in (g, g0, g1)),
               L.ptr(d0), L.ptr(d1), L.stream(grad0.device))
        return d0, d1, None, (g if ctx.has_reg else None)


def loss_pair(pred0, pred1, target, reg=None):
    """(loss, loss0, loss1, psnr0, psnr1) of a training step (LossPair)."""
    return LossPair.apply(pred0, pred1, target, reg)


def training_step(model, batch, randomized, white_bkgd, near, far, *, u_coarse=None, u_fine=None,
                  timers=None):
    """LitNeRF.training_step (model.py:256-282): loss = mse(fine) + mse(coarse) and the psnrs.
    The kernels and precision are the model's own (model.train_numerics)."""
    ret = model(batch, randomized, white_bkgd, near, far, u_coarse=u_coarse, u_fine=u_fine,
                timers=timers)
    loss, loss0, loss1, psnr0, psnr1 = loss_pair(ret[0][0], ret[1][0], batch["target"])
    return loss, dict(loss0=loss0, loss1=loss1, psnr0=psnr0, psnr1=psnr1)


# ---------------------------------------------------------------------------- optimizer
def learning_rate(step, max_steps, lr_init=5.0e-4, lr_final=5.0e-6, lr_delay_steps=2500,
                  lr_delay_mult=0.01):
    """LitNeRF.optimizer_step's schedule (model.py:399-416), host-side like the reference."""
    if lr_delay_steps > 0:
        delay_rate = lr_delay_mult + (1 - lr_delay_mult) * np.sin(
            0.5 * np.pi * np.clip(step / lr_delay_steps, 0, 1))
    else:
        delay_rate = 1.0
    t = np.clip(step / max_steps, 0, 1)
    scaled_lr = np.exp(np.log(lr_init) * (1 - t) + np.log(lr_final) * t)
    return float(delay_rate * scaled_lr)


class Adam:
    """torch.optim.Adam(params, lr, betas=(0.9, 0.999)) (model.py:386-389) as one fused
    aon_adam_step launch over every parameter tensor."""

    def __init__(self, params, lr=5.0e-4, betas=(0.9, 0.999), eps=1e-8):
        self.params = [p for p in params if p.requires_grad]
        L.require_gpu(*self.params)
        self.lr, self.betas, self.eps = lr, betas, eps
        self.state = [(torch.zeros_like(p), torch.zeros_like(p)) for p in self.params]
        self.step_count = 0

    def zero_grad(self, set_to_none=True):
        for p in self.params:
            p.grad = None

    @torch.no_grad()
    def step(self, lr=None):
        check_range({str(p.device) for p in self.params}, self.params)
        self.step_count += 1
        for p in self.params:
            if p.grad is None:
                raise RuntimeError("Adam.step: a parameter has no gradient")
            if not p.is_contiguous() or not p.grad.is_contiguous():
                raise ValueError("Adam.step: parameters and grads must be contiguous")
        # one launch per AON_ADAM_MAX_TENSORS tensors (the articulated model + code library
        # has 83)
        n = L.ADAM_MAX_TENSORS
        for c0 in range(0, len(self.params), n):
            chunk = list(zip(self.params, self.state))[c0:c0 + n]
            table = (L.AonAdamTensor * len(chunk))()
            for i, (p, (m, v)) in enumerate(chunk):
                table[i] = L.AonAdamTensor(p.data_ptr(), p.grad.data_ptr(), m.data_ptr(),
                                           v.data_ptr(), p.numel())
            L.call("aon_adam_step", table, len(chunk), float(self.lr if lr is None else lr),
                   float(self.betas[0]), float(self.betas[1]), float(self.eps), self.step_count,
                   L.stream(self.params[0].device))
        # the update is in place through raw pointers: bump each parameter's version counter so
        # version-keyed caches (NeRFMLP.packed_weights) and autograd's saved-tensor checks see it
        for p in self.params:
            torch.autograd.graph.increment_version(p)
