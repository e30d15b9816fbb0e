"""Drop-in for ``NeRFMLP`` / ``NeRF`` of the reference (models/vanilla_nerf/model.py:39-199).

Identical constructor keywords, forward signatures, return tuples and parameter (state_dict)
names, so a reference Lightning checkpoint (``model.coarse_mlp.pts_linears.0.weight`` ...)
loads unchanged.  The forward pass runs on the fused HIP kernels:

    level 0: aon_sample_along_rays (t only) -> aon_mlp_fwd (xyz + pos_enc + MLP + sigmoid/relu
             fused) -> aon_composite_march (alpha compositing fused with the fine level's
             sample_pdf: the coarse weights stay on chip; NeRF.fused_march / march_ok)
    level 1: aon_mlp_fwd on the merged t -> aon_composite_fwd
    (fused_march False, or N_importance > 256: aon_composite_fwd + aon_sample_pdf, bit-identical)

Per-model configuration only (no mutable globals): the render precision
(``precision``), the training numerics (``train_precision`` / ``train_numerics``,
aonerf/numerics.py), ``fused_march`` and ``range_check`` are attributes of each NeRF.

Intermediates live in HBM (a 640x480 frame needs ~1.6 GB), so a whole frame is one launch
per stage instead of the reference's 80 chunk iterations.
"""
import warnings

import torch
import torch.nn as nn
import torch.nn.init as init

from . import _lib as L
from . import helper
from .numerics import resolve as _resolve_numerics

_DEFAULT_GEOMETRY = dict(min_deg_point=0, max_deg_point=10, deg_view=4, netdepth=8, netwidth=256,
                         netdepth_condition=1, netwidth_condition=128, skip_layer=4, input_ch=3,
                         input_ch_view=3, num_rgb_channels=3, num_density_channels=1)


class NeRFMLP(nn.Module):
    """reference model.py:39-120 (same nn.Linear layout and init)."""

    def __init__(self, min_deg_point, max_deg_point, deg_view, netdepth: int = 8,
                 netwidth: int = 256, netdepth_condition: int = 1, netwidth_condition: int = 128,
                 skip_layer: int = 4, input_ch: int = 3, input_ch_view: int = 3,
                 num_rgb_channels: int = 3, num_density_channels: int = 1,
                 precision: str = "f16x3"):
        super().__init__()
        self.min_deg_point, self.max_deg_point, self.deg_view = min_deg_point, max_deg_point, deg_view
        self.netdepth, self.netwidth, self.skip_layer = netdepth, netwidth, skip_layer
        self.netdepth_condition, self.netwidth_condition = netdepth_condition, netwidth_condition
        self.input_ch, self.input_ch_view = input_ch, input_ch_view
        self.num_rgb_channels, self.num_density_channels = num_rgb_channels, num_density_channels
        geometry = dict(min_deg_point=min_deg_point, max_deg_point=max_deg_point, deg_view=deg_view,
                        netdepth=netdepth, netwidth=netwidth, netdepth_condition=netdepth_condition,
                        netwidth_condition=netwidth_condition, skip_layer=skip_layer,
                        input_ch=input_ch, input_ch_view=input_ch_view,
                        num_rgb_channels=num_rgb_channels, num_density_channels=num_density_channels)
        if geometry != _DEFAULT_GEOMETRY:
            raise ValueError("aonerf's fused MLP kernel implements the reference's default NeRFMLP "
                             f"geometry {_DEFAULT_GEOMETRY}; got {geometry}")
        if precision not in L.PREC:
            raise ValueError(f"precision must be one of {sorted(L.PREC)}")
        self.precision = precision

        pos_size = ((max_deg_point - min_deg_point) * 2 + 1) * input_ch
        view_pos_size = (deg_view * 2 + 1) * input_ch_view
        init_layer = nn.Linear(pos_size, netwidth)
        init.xavier_uniform_(init_layer.weight)
        pts = [init_layer]
        for idx in range(netdepth - 1):
            k = netwidth + pos_size if (idx % skip_layer == 0 and idx > 0) else netwidth
            layer = nn.Linear(k, netwidth)
            init.xavier_uniform_(layer.weight)
            pts.append(layer)
        self.pts_linears = nn.ModuleList(pts)
        views = [nn.Linear(netwidth + view_pos_size, netwidth_condition)]  # default init (model.py:79)
        for idx in range(netdepth_condition - 1):
            layer = nn.Linear(netwidth_condition, netwidth_condition)
            init.xavier_uniform_(layer.weight)
            views.append(layer)
        self.views_linear = nn.ModuleList(views)
        self.bottleneck_layer = nn.Linear(netwidth, netwidth)
        self.density_layer = nn.Linear(netwidth, num_density_channels)
        self.rgb_layer = nn.Linear(netwidth_condition, num_rgb_channels)
        for m in (self.bottleneck_layer, self.density_layer, self.rgb_layer):
            init.xavier_uniform_(m.weight)
        self._packed = None
        self._packed_key = None

    # -- weight packing (cached; repacked whenever a parameter is replaced or updated in place)
    def _layers(self):
        return list(self.pts_linears) + [self.density_layer, self.bottleneck_layer,
                                         self.views_linear[0], self.rgb_layer]

    def packed_weights(self):
        params = [p for m in self._layers() for p in (m.weight, m.bias)]
        L.require_gpu(*params)
        key = (self.precision,) + tuple((p.data_ptr(), p._version) for p in params)
        if key != self._packed_key:
            params = [L.contig(p.detach()) for p in params]
            prm = L.mlp_params(zip(params[0::2], params[1::2]))  # shape-checked (ValueError)
            prec = L.PREC[self.precision]
            nbytes = L.lib().aon_mlp_packed_bytes(prec)
            if nbytes == 0:
                raise NotImplementedError(f"precision {self.precision!r} is not built yet")
            buf = torch.empty(nbytes // 4, dtype=torch.float32, device=params[0].device)
            L.call("aon_mlp_pack", L.ctypes.byref(prm), prec, L.ptr(buf), L.stream(buf.device))
            self._packed, self._packed_key = buf, key
        return self._packed

    def forward_rays(self, rays_o, rays_d, viewdirs, t_vals, act=L.ACT_NONE):
        """Fused cast_rays + pos_enc + forward: (B*S, 4) = [raw_rgb, raw_sigma]; with
        ``act=L.ACT_VANILLA`` the rgb/sigma activations of model.py:186-187 are applied too."""
        L.require_gpu(rays_o, rays_d, viewdirs, t_vals)
        B, S = t_vals.shape
        raw = torch.empty((B * S, 4), device=t_vals.device)
        L.call("aon_mlp_fwd", L.ptr(self.packed_weights()), L.PREC[self.precision],
               L.ptr(L.contig(rays_o)), L.ptr(L.contig(rays_d)), L.ptr(L.contig(viewdirs)),
               L.ptr(L.contig(t_vals)), B, S, act, L.ptr(raw), L.stream(t_vals.device))
        return raw

    def forward(self, x, condition):
        """reference model.py:95-120: x (B, S, 63) encoded points, condition (B, 27)."""
        L.require_gpu(x, condition)
        B, S, C = x.shape
        if C != 63 or tuple(condition.shape) != (B, 27):
            raise ValueError("NeRFMLP.forward expects x (B, S, 63) and condition (B, 27)")
        raw = torch.empty((B * S, 4), device=x.device)
        L.call("aon_mlp_fwd_encoded", L.ptr(self.packed_weights()), L.PREC[self.precision],
               L.ptr(L.contig(x)), L.ptr(L.contig(condition)), B, S, L.ACT_NONE, L.ptr(raw),
               L.stream(x.device))
        raw = raw.view(B, S, 4)
        return raw[..., :3], raw[..., 3:]


def _events(timers):
    """HIP events bracketing one launch on the current stream (the stream the C ABI uses)."""
    if timers is None:
        return None
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    ev[0].record()
    return ev


def _record(timers, ev, key, rows):
    if ev is not None:
        ev[1].record()
        timers.setdefault(key, []).append((ev[0], ev[1], rows))


def fine_uniforms(B, num_fine_samples, randomized, dev, u_fine=None):
    """The u of the fine level's inverse-CDF sampling (helper.py:227-231) and its row stride:
    per-ray draws in randomized mode (or the injected ``u_fine``), else one shared linspace."""
    if randomized:
        u = torch.rand((B, num_fine_samples), device=dev) if u_fine is None else L.contig(u_fine)
        return u, num_fine_samples
    return helper.eval_u(num_fine_samples, dev), 0


def composite_march(raw, t_vals, d, white_bkgd, act, u, u_stride, num_fine_samples,
                    keep_weights):
    """Coarse compositing + the fine level's resampling in one kernel (aon_composite_march):
    (comp, acc, depth, weights or None), t_fine (B, S + Nf) -- helper.py:157-252 and
    model.py:163-172, the coarse weights kept on chip unless asked for."""
    B, S = t_vals.shape
    dev = t_vals.device
    comp = torch.empty((B, 3), device=dev)
    acc = torch.empty((B,), device=dev)
    depth = torch.empty((B,), device=dev)
    weights = torch.empty((B, S), device=dev) if keep_weights else None
    t_fine = torch.empty((B, S + num_fine_samples), device=dev)
    L.call("aon_composite_march", L.ptr(raw), L.ptr(t_vals), L.ptr(d), B, S, int(bool(white_bkgd)),
           act, L.ptr(u), u_stride, num_fine_samples, L.ptr(comp), L.ptr(acc), L.ptr(weights),
           L.ptr(depth), L.ptr(t_fine), L.stream(dev))
    return (comp, acc, depth, weights), t_fine


def march_ok(S, num_fine_samples, fused=True):
    """The fused march kernel's limits (include/aonerf.h: 3 <= S <= 256, 1 <= Ns <= 256); larger
    N_importance (up to aon_sample_pdf's 512) takes the two-kernel path, as does a model whose
    ``fused_march`` is False (aon_composite_fwd + aon_sample_pdf, bit-identical outputs)."""
    return fused and 3 <= S <= 256 and 1 <= num_fine_samples <= 256


def level_t_vals(level, o, d, t_prev, w_prev, randomized, near, far, num_coarse_samples,
                 num_fine_samples, lindisp, u_coarse=None, u_fine=None):
    """Sample positions of a level: stratified (helper.py:106-133) or inverse-CDF resampling
    of the previous level's weights merged with its samples (model.py:163-172)."""
    dev = o.device
    B = o.shape[0]
    if level == 0:
        t_vals, _ = helper.sample_along_rays(o, d, num_coarse_samples, near, far, randomized,
                                             lindisp, u=u_coarse, want_coords=False)
        return t_vals
    Sc = t_prev.shape[1]
    u, u_stride = fine_uniforms(B, num_fine_samples, randomized, dev, u_fine)
    w_prev = L.contig(w_prev.detach())
    t_new = torch.empty((B, Sc + num_fine_samples), device=dev)
    # bins = mids of t (model.py:163), weights[..., 1:-1] as a strided view
    L.call("aon_sample_pdf", None, 0, L.ptr(w_prev[:, 1:]), Sc, B, Sc - 1, num_fine_samples,
           L.ptr(u), u_stride, L.ptr(t_prev), Sc, None, None, L.ptr(t_new), None, L.stream(dev))
    return t_new


class NeRF(nn.Module):
    """reference model.py:123-199 (two-level coarse/fine render)."""

    def __init__(self, num_levels: int = 2, min_deg_point: int = 0, max_deg_point: int = 10,
                 deg_view: int = 4, num_coarse_samples: int = 64, num_fine_samples: int = 128,
                 use_viewdirs: bool = True, noise_std: float = 0.0, lindisp: bool = False,
                 precision: str = "f16x3", train_precision: str = "f16x3", train_numerics=None,
                 fused_march: bool = True, range_check: bool = True):
        """The reference's kwargs (model.py:124-145) plus, per model: ``precision`` (render MLP:
        "f16x3" or exact "fp32"), ``train_precision`` / ``train_numerics`` (the training step's
        kernels, aonerf/numerics.py), ``fused_march`` (the coarse compositor fused with the fine
        level's resampling) and ``range_check`` (after a f16x3 render, read the packs'
        range-status words -- one sync per forward, skipped under HIP-graph capture -- and
        re-render on the fp32 kernels on overflow)."""
        super().__init__()
        if num_levels != 2:
            raise ValueError("the reference NeRF is two-level (coarse + fine)")
        self.train_numerics = _resolve_numerics(train_precision, train_numerics)
        self.fused_march, self.range_check = bool(fused_march), bool(range_check)
        self.num_levels, self.min_deg_point, self.max_deg_point = num_levels, min_deg_point, max_deg_point
        self.deg_view, self.num_coarse_samples, self.num_fine_samples = deg_view, num_coarse_samples, num_fine_samples
        self.use_viewdirs, self.noise_std, self.lindisp = use_viewdirs, noise_std, lindisp
        self.coarse_mlp = NeRFMLP(min_deg_point, max_deg_point, deg_view, precision=precision)
        self.fine_mlp = NeRFMLP(min_deg_point, max_deg_point, deg_view, precision=precision)

    def set_precision(self, precision):
        for m in (self.coarse_mlp, self.fine_mlp):
            if precision not in L.PREC:
                raise ValueError(precision)
            m.precision = precision
        return self

    def forward(self, rays, randomized, white_bkgd, near, far, *, u_coarse=None, u_fine=None,
                return_weights=False, return_intermediates=False, timers=None):
        """reference model.py:147-199 -> [(comp_rgb, acc, depth)_coarse, (...)_fine].

        ``u_coarse`` (B, Sc+1) / ``u_fine`` (B, Nf) inject the uniforms of randomized mode;
        ``return_weights`` adds each level's weights (B, S) as a 4th element;
        ``return_intermediates`` adds a dict(t_vals, weights[, rgb_sigma]) as the last element
        (rgb_sigma (B*S, 4), inference path only: the activated MLP outputs the compositor
        consumed);
        ``timers`` (dict) records hip events around each level's MLP / composite launches (the
        training path: around its fused training kernels).

        With autograd enabled and trainable parameters, each level runs the training path
        (train.RenderLevel: the fused training forward aon_mlp_fwd_train, which also stores the
        activations and their ReLU' bits, then the HIP backward); otherwise the fused inference
        kernels.
        """
        o, d, v = rays["rays_o"], rays["rays_d"], rays["viewdirs"]
        L.require_gpu(o, d, v)
        o, d, v = L.contig(o), L.contig(d), L.contig(v)
        training = torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())
        B = o.shape[0]
        dev = o.device
        # the fp16x3 overflow fallback below re-renders with the same random draws (density
        # noise, stratified t, fine u) and leaves the generator where one forward leaves it
        rng = torch.cuda.get_rng_state(dev) if randomized and not training else None
        ret = []
        t_vals = weights = t_next = None
        token, joined = None, {}
        cfg = self.train_numerics
        if training:
            from . import train
            if cfg.overlap_dweight and cfg.fused_backward and timers is None:
                # both levels' parameters through one Join: its backward, after both levels',
                # joins the fine level's weight-gradient stream (overlap_dweight)
                token = train.JoinToken()
                ps = [p for m in (self.coarse_mlp, self.fine_mlp) for l in m._layers()
                      for p in (l.weight, l.bias)]
                joined = dict(zip(map(id, ps), train.Join.apply(token, *ps)))
        for level in range(2):
            with torch.no_grad():
                t_vals = t_next if t_next is not None else self._level_t(
                    level, o, d, t_vals, weights, randomized, near, far, u_coarse, u_fine)
            mlp = self.coarse_mlp if level == 0 else self.fine_mlp
            S = t_vals.shape[1]
            if training:
                from .train import RenderLevel
                noise = None
                if self.noise_std > 0 and randomized:  # model.py:183-184
                    noise = torch.rand((B * S,), device=dev) * self.noise_std
                params = [p for m in mlp._layers() for p in (m.weight, m.bias)]
                params = [joined.get(id(p), p) for p in params]
                comp, acc, depth, weights = RenderLevel.apply(o, d, v, t_vals, bool(white_bkgd),
                                                              noise, token, cfg, timers, *params)
                out = (comp, acc, depth, weights) if return_weights else (comp, acc, depth)
                if return_intermediates:
                    out = out + (dict(t_vals=t_vals, weights=weights),)
                ret.append(out)
                continue
            # the last level's weights are an output only when asked for: otherwise the
            # compositor skips writing them (4 B of its 24 B per sample)
            keep_w = level == 0 or return_weights or return_intermediates
            march = level == 0 and march_ok(S, self.num_fine_samples, self.fused_march)
            if march:  # the coarse weights are needed on chip only
                keep_w = return_weights or return_intermediates
            with torch.no_grad():
                out, weights, t_next = self._render_level_fused(
                    mlp, o, d, v, t_vals, randomized, white_bkgd, level, timers, keep_w,
                    # drawn inside, after the level's density noise (the reference's RNG order)
                    march_u=(lambda: fine_uniforms(B, self.num_fine_samples, randomized, dev,
                                                   u_fine)) if march else None)
            if not return_weights:
                out = out[:3] + out[4:]
            if not return_intermediates:
                out = out[:4] if return_weights else out[:3]
            ret.append(out)
        if (not training and self.range_check and self.coarse_mlp.precision.startswith("f16x3")
                and not torch.cuda.is_current_stream_capturing()
                and L.range_overflow([self.coarse_mlp._packed, self.fine_mlp._packed])):
            # an activation left the fp16x3 split's range (|x| > 8188): these outputs are
            # invalid -- render again on the exact-fp32 MFMA kernels (no range limit)
            warnings.warn("NeRF: an MLP activation exceeded the fp16x3 range; re-rendered with "
                          "precision='fp32'", RuntimeWarning)
            prec = self.coarse_mlp.precision
            self.set_precision("fp32")
            if rng is not None:
                torch.cuda.set_rng_state(rng, dev)
            try:
                return self.forward(rays, randomized, white_bkgd, near, far, u_coarse=u_coarse,
                                    u_fine=u_fine, return_weights=return_weights,
                                    return_intermediates=return_intermediates, timers=timers)
            finally:
                self.set_precision(prec)
        return ret

    def _level_t(self, level, o, d, t_prev, w_prev, randomized, near, far, u_coarse, u_fine):
        return level_t_vals(level, o, d, t_prev, w_prev, randomized, near, far,
                            self.num_coarse_samples, self.num_fine_samples, self.lindisp,
                            u_coarse, u_fine)

    def _render_level_fused(self, mlp, o, d, v, t_vals, randomized, white_bkgd, level, timers,
                            keep_weights=True, march_u=None):
        """One inference level: fused MLP, then compositing -- with ``march_u`` (a callable
        returning the fine level's (u, u_stride)) also the next level's resampling in the same
        kernel (returned t_next, else None)."""
        B, S = t_vals.shape
        dev = o.device
        # the activations (model.py:186-187) run in the MLP epilogue, unless density noise
        # must be added to the raw sigma first (model.py:183-184)
        noisy = self.noise_std > 0 and randomized
        ev = _events(timers)
        raw = mlp.forward_rays(o, d, v, t_vals, act=L.ACT_NONE if noisy else L.ACT_VANILLA)
        _record(timers, ev, f"mlp{level}", B * S)
        if noisy:
            raw[:, 3] += torch.rand_like(raw[:, 3]) * self.noise_std
        act = L.ACT_VANILLA if noisy else L.ACT_NONE
        t_next = None
        ev = _events(timers)
        if march_u is not None:
            u, u_stride = march_u()
            (comp, acc, depth, weights), t_next = composite_march(
                raw, t_vals, d, white_bkgd, act, u, u_stride, self.num_fine_samples, keep_weights)
            _record(timers, ev, f"march{level}", B * S)
        else:
            comp = torch.empty((B, 3), device=dev)
            acc = torch.empty((B,), device=dev)
            weights = torch.empty((B, S), device=dev) if keep_weights else None
            depth = torch.empty((B,), device=dev)
            L.call("aon_composite_fwd", L.ptr(raw), 4, L.ptr(raw[:, 3:]), 4, L.ptr(t_vals), L.ptr(d),
                   B, S, int(bool(white_bkgd)), act, L.ptr(comp), L.ptr(acc), L.ptr(weights),
                   L.ptr(depth), L.stream(dev))
            _record(timers, ev, f"comp{level}", B * S)
        return (comp, acc, depth, weights, dict(t_vals=t_vals, weights=weights, rgb_sigma=raw)), weights, t_next
