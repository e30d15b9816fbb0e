"""ctypes binding of the C ABI in include/aonerf.h (libaonerf.so, built for gfx950).

This is the reference-side binding a maintainer adds: plain pointers, sizes
and the current torch stream go through; tensors stay owned by PyTorch.  There is NO CPU
fallback: a missing library or a non-CUDA tensor raises.
"""
import ctypes
import os

import torch  # load torch's HIP runtime first: libaonerf.so binds to the same libamdhip64.so.7

_HERE = os.path.dirname(os.path.abspath(__file__))
# the release library; an A/B driver under tools/ may name another build with use_library()
# before the first call (the product path reads no environment variable)
LIB_PATH = os.path.join(os.path.dirname(_HERE), "lib", "libaonerf.so")

c_i64, c_int, c_float, c_size, vp = ctypes.c_int64, ctypes.c_int, ctypes.c_float, ctypes.c_size_t, ctypes.c_void_p

# render precisions (aon_mlp_fwd): exact fp32 MFMA, the fp16x3 split on 16x16x32 MFMAs
PREC = {"fp32": 0, "f16x3": 1}
PREC_F16X3_TRAIN = 1  # the training forwards' fp16x3 stream (aon_mlp_fwd_train)
PREC_BF16 = 2  # the training step's bf16 mode (aon_mlp_fwd_train_bf16, aon_mlp_bwd_bf16)
ACT_NONE, ACT_VANILLA, ACT_ARTIC = 0, 1, 2


class AonMlpParams(ctypes.Structure):
    _fields_ = [("pts_w", vp * 8), ("pts_b", vp * 8), ("density_w", vp), ("density_b", vp),
                ("bottleneck_w", vp), ("bottleneck_b", vp), ("views_w", vp), ("views_b", vp),
                ("rgb_w", vp), ("rgb_b", vp), ("w_rows", c_i64 * 12), ("w_cols", c_i64 * 12),
                ("b_len", c_i64 * 12)]


class AonMlpArtParams(ctypes.Structure):
    _fields_ = [("def_w", vp * 4), ("def_b", vp * 4), ("deformation_w", vp), ("deformation_b", vp),
                ("pts_w", vp * 8), ("pts_b", vp * 8), ("density_w", vp), ("density_b", vp),
                ("bottleneck_w", vp), ("bottleneck_b", vp), ("views_w", vp * 4),
                ("views_b", vp * 4), ("rgb_w", vp), ("rgb_b", vp), ("w_rows", c_i64 * 20),
                ("w_cols", c_i64 * 20), ("b_len", c_i64 * 20)]


# [out][in] of each layer in the kernels' layer order (= the order of the struct fields):
# reference model.py:39-93 (vanilla) and model_autodecoder.py:60-166 (articulated, whose four
# latent-carrying layers may be wider: their latent columns are folded into the bias)
MLP_LAYERS = (["pts_linears.%d" % i for i in range(8)] +
              ["density_layer", "bottleneck_layer", "views_linear.0", "rgb_layer"])
MLP_SHAPES = [(256, 63)] + [(256, 256)] * 4 + [(256, 319)] + [(256, 256)] * 2 + \
    [(1, 256), (256, 256), (128, 283), (3, 128)]
ART_LAYERS = (["deformations_linear.%d" % i for i in range(4)] + ["deformation_layer"] +
              ["pts_linears.%d" % i for i in range(8)] + ["density_layer", "bottleneck_layer"] +
              ["views_linear.%d" % i for i in range(4)] + ["rgb_layer"])
ART_SHAPES = [(128, 3)] + [(128, 128)] * 3 + [(3, 128), (256, 63)] + [(256, 256)] * 4 + \
    [(256, 319)] + [(256, 256)] * 2 + [(1, 256), (256, 256), (128, 283)] + [(128, 128)] * 3 + \
    [(3, 128)]
ART_LATENT = {0, 5, 10, 15}  # deformations_linear.0, pts_linears.0 / .5, views_linear.0


def _check_layers(pairs, names, shapes, latent=()):
    """Raise ValueError unless ``pairs`` = [(weight, bias)] matches the layer table: count,
    order (by shape), dtype, device and contiguity -- BEFORE any pointer reaches a kernel."""
    if len(pairs) != len(names):
        raise ValueError(f"expected {len(names)} (weight, bias) pairs in the kernels' layer order "
                         f"({', '.join(names)}), got {len(pairs)}")
    for i, ((w, b), name, (out, inp)) in enumerate(zip(pairs, names, shapes)):
        if not (isinstance(w, torch.Tensor) and isinstance(b, torch.Tensor)):
            raise ValueError(f"{name}: (weight, bias) must be tensors")
        ok_w = (w.dim() == 2 and w.shape[0] == out and
                (w.shape[1] >= inp if i in latent else w.shape[1] == inp))
        if not ok_w or tuple(b.shape) != (out,):
            raise ValueError(f"{name}: weight {tuple(w.shape)}, bias {tuple(b.shape)}; expected "
                             f"weight ({out}, {'>=' if i in latent else ''}{inp}), bias ({out},) "
                             "-- parameters must come in the kernels' layer order "
                             f"({', '.join(names)}), not nn.Module registration order")
    dev = pairs[0][0].device
    for (w, b), name in zip(pairs, names):
        for t, what in ((w, "weight"), (b, "bias")):
            if not t.is_cuda or t.dtype != torch.float32 or not t.is_contiguous():
                raise ValueError(f"{name}.{what}: needs a contiguous float32 GPU tensor, got "
                                 f"{t.dtype} on {t.device}{'' if t.is_contiguous() else ' (strided)'}")
            if t.device != dev:
                raise ValueError(f"{name}.{what}: on {t.device}, the others on {dev}")


def check_mlp_layers(pairs):
    """ValueError unless ``pairs`` are one vanilla NeRFMLP's 12 (weight, bias) GPU tensors in the
    kernels' layer order (as mlp_params checks them)."""
    _check_layers([tuple(p) for p in pairs], MLP_LAYERS, MLP_SHAPES)


def check_mlp_art_layers(pairs):
    """The same for one articulated NeRFMLP's 20 pairs (mlp_art_params' order)."""
    _check_layers([tuple(p) for p in pairs], ART_LAYERS, ART_SHAPES, ART_LATENT)


def _fill_shapes(prm, pairs):
    for i, (w, b) in enumerate(pairs):
        prm.w_rows[i], prm.w_cols[i], prm.b_len[i] = w.shape[0], w.shape[1], b.numel()


def mlp_params(pairs):
    """AonMlpParams of one vanilla NeRFMLP: ``pairs`` = 12 (weight, bias) tensors in the order
    pts_linears.0..7, density_layer, bottleneck_layer, views_linear.0, rgb_layer; validated
    (ValueError) against the layer table before the struct exists."""
    pairs = [tuple(p) for p in pairs]
    _check_layers(pairs, MLP_LAYERS, MLP_SHAPES)
    prm = AonMlpParams()
    for i in range(8):
        prm.pts_w[i], prm.pts_b[i] = pairs[i][0].data_ptr(), pairs[i][1].data_ptr()
    for name, idx in (("density", 8), ("bottleneck", 9), ("views", 10), ("rgb", 11)):
        setattr(prm, f"{name}_w", pairs[idx][0].data_ptr())
        setattr(prm, f"{name}_b", pairs[idx][1].data_ptr())
    _fill_shapes(prm, pairs)
    return prm


def mlp_art_params(pairs):
    """AonMlpArtParams of one articulated NeRFMLP: ``pairs`` = 20 (weight, bias) tensors in the
    order deformations_linear.0..3, deformation_layer, pts_linears.0..7, density_layer,
    bottleneck_layer, views_linear.0..3, rgb_layer (the latent-carrying layers' biases folded by
    the caller); validated (ValueError) against the layer table."""
    pairs = [tuple(p) for p in pairs]
    _check_layers(pairs, ART_LAYERS, ART_SHAPES, ART_LATENT)
    prm = AonMlpArtParams()
    for i in range(4):
        prm.def_w[i], prm.def_b[i] = pairs[i][0].data_ptr(), pairs[i][1].data_ptr()
        prm.views_w[i], prm.views_b[i] = pairs[15 + i][0].data_ptr(), pairs[15 + i][1].data_ptr()
    for i in range(8):
        prm.pts_w[i], prm.pts_b[i] = pairs[5 + i][0].data_ptr(), pairs[5 + i][1].data_ptr()
    prm.deformation_w, prm.deformation_b = pairs[4][0].data_ptr(), pairs[4][1].data_ptr()
    prm.density_w, prm.density_b = pairs[13][0].data_ptr(), pairs[13][1].data_ptr()
    prm.bottleneck_w, prm.bottleneck_b = pairs[14][0].data_ptr(), pairs[14][1].data_ptr()
    prm.rgb_w, prm.rgb_b = pairs[19][0].data_ptr(), pairs[19][1].data_ptr()
    _fill_shapes(prm, pairs)
    return prm


class AonGemmArgs(ctypes.Structure):
    _fields_ = [("M", c_i64), ("N", c_i64), ("K", c_i64), ("A", vp), ("lda", c_i64), ("a_kc", c_int),
                ("A2", vp), ("lda2", c_i64), ("K1", c_i64), ("a2_rdiv", c_i64),
                ("B", vp), ("ldb", c_i64), ("b_kc", c_int), ("b_rdiv", c_i64),
                ("C", vp), ("ldc", c_i64), ("bias", vp), ("mask", vp), ("ldm", c_i64),
                ("relu", c_int), ("accumulate", c_int), ("a_scale", c_float), ("b_scale", c_float),
                ("k_splits", c_i64), ("rowsum", vp), ("a_amax", vp), ("mma_bf16", c_int),
                ("a_bf16", c_int), ("b_bf16", c_int), ("a_tiled", c_int), ("b_tiled", c_int),
                ("n_store", c_i64), ("exact_fp32", c_int), ("c_trans", c_int),
                ("f16_single", c_int)]


class AonAdamTensor(ctypes.Structure):
    _fields_ = [("param", vp), ("grad", vp), ("exp_avg", vp), ("exp_avg_sq", vp), ("numel", c_i64)]


ADAM_MAX_TENSORS = 64
GEMM_BATCH_MAX = 12  # AON_GEMM_BATCH_MAX
GEMM_SMALL_BATCH_MAX = 16  # AON_GEMM_SMALL_BATCH_MAX

_SIGNATURES = {
    "aon_abi_version": (c_int, []),
    "aon_last_error": (ctypes.c_char_p, []),
    "aon_ray_directions": (c_int, [c_int, c_int, c_float, vp, vp]),
    "aon_get_rays": (c_int, [vp, c_i64, vp, vp, vp, vp, c_int, c_int, vp, vp]),
    "aon_frame_rays": (c_int, [c_int, c_int, c_float, vp, c_i64, c_i64, vp, vp, vp, vp]),
    "aon_sample_along_rays": (c_int, [vp, vp, c_i64, c_int, vp, vp, vp, vp, vp, vp]),
    "aon_pos_enc": (c_int, [vp, c_i64, c_int, c_int, vp, vp]),
    "aon_sample_rays": (c_int, [vp, vp, c_int, c_i64, c_int, c_int, c_float, vp, c_i64, c_int,
                                c_float, vp, vp, vp, vp, vp]),
    "aon_cast_rays": (c_int, [vp, vp, vp, c_i64, c_int, vp, c_i64, vp, c_int, c_int, vp, vp]),
    "aon_cast_rays_tiled": (c_int, [vp, vp, vp, c_i64, c_int, c_int, c_int, c_int, vp, vp]),
    "aon_sample_pdf": (c_int, [vp, c_i64, vp, c_i64, c_i64, c_int, c_int, vp, c_i64, vp, c_int,
                               vp, vp, vp, vp, vp]),
    "aon_composite_march": (c_int, [vp, vp, vp, c_i64, c_int, c_int, c_int, vp, c_i64, c_int, vp,
                                    vp, vp, vp, vp, vp]),
    "aon_mlp_packed_bytes": (c_size, [c_int]),
    "aon_mlp_read_status": (c_int, [vp, c_size, ctypes.POINTER(ctypes.c_uint32), vp]),
    "aon_mlp_pack": (c_int, [ctypes.POINTER(AonMlpParams), c_int, vp, vp]),
    "aon_mlp_fwd": (c_int, [vp, c_int, vp, vp, vp, vp, c_i64, c_int, c_int, vp, vp]),
    "aon_mlp_fwd_encoded": (c_int, [vp, c_int, vp, vp, c_i64, c_int, c_int, vp, vp]),
    "aon_mlp_fwd_train": (c_int, [vp, vp, vp, vp, vp, c_i64, c_int, vp, vp, vp, vp, vp, vp, vp]),
    "aon_mlp_fwd_train_bf16": (c_int, [vp, vp, vp, vp, vp, c_i64, c_int, vp, vp, vp, vp, vp, vp,
                                       vp, vp]),
    "aon_mlp_bwd_pack_bf16": (c_int, [ctypes.POINTER(AonMlpParams), vp, vp]),
    "aon_mlp_bwd_bf16": (c_int, [vp, vp, vp, c_i64, vp, vp, vp, vp, vp]),
    "aon_relu_masks": (c_int, [vp, c_i64, c_int, vp, vp]),
    "aon_absmax": (c_int, [vp, c_i64, vp, vp]),
    "aon_mlp_bwd_packed_bytes": (c_size, []),
    "aon_mlp_bwd_pack": (c_int, [ctypes.POINTER(AonMlpParams), vp, vp]),
    "aon_mlp_bwd": (c_int, [vp, vp, vp, c_i64, vp, vp, vp, vp, vp]),
    "aon_mlp_art_packed_bytes": (c_size, []),
    "aon_mlp_art_pack": (c_int, [ctypes.POINTER(AonMlpArtParams), vp, vp]),
    "aon_mlp_art_fwd": (c_int, [vp, vp, vp, vp, vp, c_i64, c_int, c_int, vp, vp]),
    "aon_mlp_art_fwd_points": (c_int, [vp, vp, vp, c_i64, c_int, c_int, vp, vp]),
    "aon_mlp_art_bwd_packed_bytes": (c_size, []),
    "aon_mlp_art_bwd_pack": (c_int, [ctypes.POINTER(AonMlpArtParams), vp, vp]),
    "aon_mlp_art_bwd": (c_int, [vp, vp, vp, vp, c_i64, vp, vp, vp, vp, vp, vp, vp]),
    "aon_mlp_art_pack_bf16": (c_int, [ctypes.POINTER(AonMlpArtParams), vp, vp]),
    "aon_mlp_art_pack_mixed": (c_int, [ctypes.POINTER(AonMlpArtParams), c_int, vp, vp]),
    "aon_mlp_art_bwd_pack_bf16": (c_int, [ctypes.POINTER(AonMlpArtParams), vp, vp]),
    "aon_mlp_art_bwd_bf16": (c_int, [vp, vp, vp, vp, c_i64, vp, vp, vp, vp, vp, vp, vp]),
    "aon_mlp_art_fwd_train": (c_int, [vp, vp, vp, vp, vp, c_i64, c_int, vp, vp, vp, vp, vp, vp, vp,
                                      vp, vp, vp]),
    "aon_mlp_art_fwd_train_bf16": (c_int, [vp, vp, vp, vp, vp, c_i64, c_int, vp, vp, vp, vp, vp,
                                           vp, vp, vp, vp, vp, c_int, vp]),
    "aon_composite_fwd": (c_int, [vp, c_i64, vp, c_i64, vp, vp, c_i64, c_int, c_int, c_int, vp,
                                  vp, vp, vp, vp]),
    "aon_image_mse": (c_int, [vp, vp, c_i64, c_i64, vp, c_int, vp, vp, vp]),
    "aon_to8b": (c_int, [vp, c_i64, vp, vp]),
    "aon_gemm_workspace_bytes": (c_size, [ctypes.POINTER(AonGemmArgs)]),
    "aon_gemm": (c_int, [ctypes.POINTER(AonGemmArgs), vp, c_size, vp]),
    "aon_gemm_batch_workspace_bytes": (c_size, [ctypes.POINTER(AonGemmArgs), c_int]),
    "aon_gemm_batch": (c_int, [ctypes.POINTER(AonGemmArgs), c_int, vp, c_size, vp]),
    "aon_gemm_small_batch": (c_int, [ctypes.POINTER(AonGemmArgs), c_int, vp]),
    "aon_composite_bwd": (c_int, [vp, c_i64, vp, c_i64, vp, vp, c_i64, c_int, c_int, c_int, vp, vp,
                                  vp, vp, vp, c_i64, vp]),
    "aon_mse": (c_int, [vp, vp, c_i64, c_float, vp, vp, vp]),
    "aon_loss_pair": (c_int, [vp, vp, vp, c_i64, vp, vp, vp, vp, vp]),
    "aon_loss_pair_bwd": (c_int, [vp, vp, c_i64, vp, vp, vp, vp, vp, vp]),
    "aon_colsum_workspace_bytes": (c_size, [c_i64, c_i64]),
    "aon_colsum": (c_int, [vp, c_i64, c_i64, c_i64, c_int, vp, vp, c_size, vp]),
    "aon_adam_step": (c_int, [ctypes.POINTER(AonAdamTensor), c_int, ctypes.c_double,
                              ctypes.c_double, ctypes.c_double, ctypes.c_double, c_i64, vp]),
    "aon_pos_enc_bwd": (c_int, [vp, c_i64, vp, c_i64, c_i64, c_int, c_int, c_int, vp, c_i64, vp]),
    "aon_latent_reg": (c_int, [vp, c_i64, c_i64, c_float, c_int, vp, vp, vp]),
}

_lib = None


ABI_VERSION = 13


def _load(path):
    if not os.path.exists(path):
        raise ImportError(f"aonerf: HIP library not built: {path} "
                          "(run `make -C articulated-object-nerf_amd/csrc` or __graft_entry__.build())")
    handle = ctypes.CDLL(path)
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(handle, name)
        fn.restype = res
        fn.argtypes = args
    if handle.aon_abi_version() != ABI_VERSION:
        raise ImportError(f"aonerf: ABI version mismatch ({path})")
    return handle


def lib():
    """Load libaonerf.so once; raise loudly if it is missing (no silent fallback)."""
    global _lib
    if _lib is None:
        _lib = _load(LIB_PATH)
    return _lib


def use_library(path):
    """Bind ``path`` (an A/B build of the library, same ABI) instead of the release library --
    before anything has loaded one (tools/ A/B drivers; never the product path)."""
    global LIB_PATH
    if _lib is not None and os.path.abspath(path) != os.path.abspath(LIB_PATH):
        raise RuntimeError(f"aonerf: {LIB_PATH} is already loaded")
    LIB_PATH = path


_variants = {}


def variant(name):
    """An A/B build of the library beside the release one (lib/variants/libaonerf_<name>.so,
    e.g. ``make -C csrc variant-ws``): same ABI and packed formats, a different kernel behind
    some entry points.  Test infrastructure only; the product path always uses lib()."""
    if name not in _variants:
        _variants[name] = _load(os.path.join(os.path.dirname(LIB_PATH), "variants",
                                             f"libaonerf_{name}.so"))
    return _variants[name]


def call(name, *args):
    """Invoke an aon_* entry point and turn a non-zero status into an exception."""
    st = getattr(lib(), name)(*args)
    if st != 0:
        msg = lib().aon_last_error().decode(errors="replace")
        if st < 0:
            raise ValueError(f"{name}: {msg}")
        raise RuntimeError(f"{name}: HIP error {st}: {msg}")


def stream(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def require_gpu(*tensors):
    """Every hot-path tensor must be a CUDA (HIP) fp32 tensor; the product path never runs on CPU."""
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise ValueError("aonerf runs on the MI355X only: got a CPU tensor "
                             "(the CPU restatement lives in oracle/, test infrastructure only)")
        if t.dtype != torch.float32:
            raise ValueError(f"aonerf expects float32 tensors, got {t.dtype}")


def contig(t):
    return t if t.is_contiguous() else t.contiguous()


# ---------------------------------------------------------------------------- fp16x3 range guard
# Every packed weight buffer ends in a 16-B status block (include/aonerf.h aon_mlp_read_status):
# word 0 is set by a fp16x3 kernel that met a value its fp16 hi/lo split cannot hold.  Each
# training pack registers here when it is (re)packed (register_pack), so the next optimizer step
# -- aonerf's Adam, or ANY torch optimizer through the global step pre-hook aonerf.train
# installs -- can refuse gradients computed from such values (check_pending).  A buffer re-packed
# before a step looked at it (gradient accumulation, two forwards of one level) first ORs its
# status word into its device's sticky word, so the re-pack cannot erase an overflow.
PENDING_PACKS = {}
_STICKY = {}
# data pointers of the parameters each pending pack was packed from (the tensor objects an
# autograd Function sees are not always the optimizer's, their storage is): an optimizer step
# checks only the packs of ITS parameters, so an unrelated model's optimizer neither pays the
# sync nor consumes (hides) this model's overflow.  The sticky words are kept per (device,
# parameter set) for the same reason: two models that both re-pack before either
# steps keep separate words, and each optimizer consumes only its own.
PACK_PARAMS = {}
# pending pack -> (pinned host copy of its status word, event after the copy): taken after the
# last kernel that can set the word (snapshot_pack), so check_pending reads host memory once that
# point has passed instead of draining the device queue with a sync on the device word -- the
# step's later kernels (weight gradients) keep the GPU busy while the optimizer waits
SNAPSHOTS = {}
_PINNED = {}


def status_word(buf):
    """Device int32 0-dim view of a packed buffer's range-status word."""
    return buf.view(torch.int32)[-4]


def register_pack(key, buf, params=()):
    """Call BEFORE (re)packing ``buf`` on the current stream: keep the status a pending pack
    still holds (stream-ordered device OR, no sync), then mark ``buf`` pending.  ``params``: the
    parameter tensors packed into ``buf`` (empty: the pack concerns every optimizer)."""
    dev = str(buf.device)
    k = (key[0], key[1], dev)
    SNAPSHOTS.pop(k, None)  # a snapshot of the previous pack no longer covers the buffer
    if k in PENDING_PACKS:
        sk = (dev, PACK_PARAMS.get(k) or frozenset({None}))
        w = _STICKY.get(sk)
        if w is None:
            w = _STICKY[sk] = torch.zeros((), dtype=torch.int32, device=buf.device)
        w.bitwise_or_(status_word(PENDING_PACKS[k]))
    PENDING_PACKS[k] = buf
    PACK_PARAMS[k] = frozenset(p.data_ptr() for p in params)


def snapshot_pack(buf):
    """Call after the LAST kernel that reads the pending pack ``buf`` (the only writers of its
    status word) on the current stream: an asynchronous copy of the word to pinned host memory
    and an event after it (no sync).  No-op for a buffer that is not pending."""
    k = next((k for k, b in PENDING_PACKS.items() if b is buf), None)
    if k is None:
        return
    h = _PINNED.get(k)
    if h is None:
        h = _PINNED[k] = torch.empty((1,), dtype=torch.int32, pin_memory=True)
    # the copy and its event on the current stream of the BUFFER's device (the
    # current device may be another one; an event there would not order after the copy)
    with torch.cuda.device(buf.device):
        h.copy_(status_word(buf).view(1), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(buf.device))
    SNAPSHOTS[k] = (h, ev)


def _concerns(ids, param_ids):
    # a pack registered without parameters (or a sticky word holding one) concerns everyone
    return param_ids is None or not ids or None in ids or bool(ids & param_ids)


def has_pending(devices=None, param_ids=None):
    """Whether check_pending(devices, param_ids) would look at anything (no sync)."""
    return (any((devices is None or k[2] in devices) and _concerns(PACK_PARAMS.get(k), param_ids)
                for k in PENDING_PACKS) or
            any((devices is None or d in devices) and _concerns(ps, param_ids)
                for d, ps in _STICKY))


def range_overflow(bufs):
    """True if any of these packed buffers' kernels saw a fp16x3 range overflow (one sync)."""
    bufs = [b for b in bufs if b is not None]
    if not bufs:
        return False
    return bool(torch.stack([status_word(b) for b in bufs]).any().item())


def check_pending(devices=None, param_ids=None):
    """Consume the pending training packs (and sticky words) of ``devices`` (str, None = all)
    that concern ``param_ids`` (data pointers of an optimizer's parameters; None = all):
    True if any saw an overflow since the last check.  A pack with a snapshot (snapshot_pack)
    is read from host memory once its event has passed; the others (and sticky words) with one
    device sync; none pending: no sync at all."""
    keys = [k for k in PENDING_PACKS if (devices is None or k[2] in devices)
            and _concerns(PACK_PARAMS.get(k), param_ids)]
    words, bad = [], False
    for k in keys:
        buf = PENDING_PACKS.pop(k)
        PACK_PARAMS.pop(k, None)
        snap = SNAPSHOTS.pop(k, None)
        if snap is None:
            words.append(status_word(buf))
        else:
            snap[1].synchronize()
            bad |= int(snap[0][0]) != 0
    for sk in [sk for sk in _STICKY if (devices is None or sk[0] in devices)
               and _concerns(sk[1], param_ids)]:
        words.append(_STICKY.pop(sk))
    if not words:
        return bad
    return bool(torch.stack(words).any().item()) or bad
