"""Drop-in for the articulated ``NeRFMLP`` / ``NeRF_AE_Art`` of the reference
(models/vanilla_nerf/model_autodecoder.py:60-337; config C3).

Identical constructor keywords, forward signatures and parameter (state_dict) names.  One
inference level runs ONE fused kernel (aon_mlp_art_fwd, k_mlp_art_f16x3; NeRFMLP.fused, the
default):

    cast_rays                                                              helper.py:25-26
    deformation MLP on cat[xyz, shape, articulation]: 4 x (MFMA + ReLU),   model_autodecoder.py:
      deformation_layer                                                    196-205
    x' = deformation + xyz, pos_enc(x') in registers                       :205-212
    trunk on cat[pos_enc(x'), shape] with the skip concat, density,        :214-223
      bottleneck
    view branch on cat[bottleneck, enc_dir, appearance]: 4 x (MFMA + ReLU) :224-235
    rgb head; padded sigmoid / softplus(raw - 1) in the epilogue           :321-323

then the coarse compositor fused with the fine level's resampling (aon_composite_march) or, for
the fine level, aon_composite_fwd (AON_ACT_ARTIC; :324-333).  The latent codes are the same for
every sample (the reference repeats (1, C) rows over all B*S rows, :186-194), so their products
with the weight columns they meet are folded into per-call biases (b' = b + W[:, latent cols] .
latent, one tiny GEMM each).  ``NeRFMLP.fused = False`` selects the layer-by-layer path, every
product on the f16x3 MFMA GEMM (aon_gemm), which is also the fallback when an activation leaves
the fused kernel's fp16x3 range.  No torch arithmetic on the path.
"""
import warnings

import torch
import torch.nn as nn
import torch.nn.init as init

from . import _lib as L
from .linalg import ACT_SCALE, W_SCALE, gemm, linear_fwd
from .model import _events, _record, composite_march, fine_uniforms, level_t_vals, march_ok
from .numerics import resolve as _resolve_numerics


class NeRFMLP(nn.Module):
    """reference model_autodecoder.py:60-166 (same nn.Linear layout and init)."""

    def __init__(self, min_deg_point, max_deg_point, deg_view, netdepth: int = 8,
                 netwidth: int = 256, netdepth_deformation=4, netwidth_deformation: int = 128,
                 netdepth_condition: int = 4, netwidth_condition: int = 128,
                 shape_latent_dim=128, appearance_latent_dim=128, articulation_latent_dim=32,
                 skip_layer: int = 4, input_ch: int = 3, input_ch_view: int = 3,
                 num_rgb_channels: int = 3, num_density_channels: int = 1,
                 deformation_mlp: bool = True, enc_after: bool = True, embed_deg: bool = False,
                 fused: bool = True):
        super().__init__()
        self.fused = fused  # one fused kernel per level (aon_mlp_art_fwd) vs GEMM per layer
        cfg = dict(netdepth=netdepth, netwidth=netwidth, netdepth_deformation=netdepth_deformation,
                   netwidth_deformation=netwidth_deformation, netdepth_condition=netdepth_condition,
                   netwidth_condition=netwidth_condition, shape_latent_dim=shape_latent_dim,
                   appearance_latent_dim=appearance_latent_dim,
                   articulation_latent_dim=articulation_latent_dim, skip_layer=skip_layer,
                   input_ch=input_ch, input_ch_view=input_ch_view,
                   num_rgb_channels=num_rgb_channels, num_density_channels=num_density_channels,
                   deformation_mlp=deformation_mlp, enc_after=enc_after, embed_deg=embed_deg)
        for k, v in cfg.items():
            setattr(self, k, v)
        self.min_deg_point, self.max_deg_point, self.deg_view = min_deg_point, max_deg_point, deg_view
        if not (deformation_mlp and enc_after and not embed_deg):
            raise ValueError("aonerf implements the reference's default articulated MLP "
                             "(deformation_mlp=True, enc_after=True, embed_deg=False)")
        view_pos_size = (deg_view * 2 + 1) * input_ch_view
        pos_size_deformation = input_ch + shape_latent_dim + articulation_latent_dim
        deformations = [nn.Linear(pos_size_deformation, netwidth_deformation)]
        for _ in range(netdepth_deformation - 1):
            deformations.append(nn.Linear(netwidth_deformation, netwidth_deformation))
        for m in deformations:
            init.xavier_uniform_(m.weight)
        self.deformations_linear = nn.ModuleList(deformations)
        self.deformation_layer = nn.Linear(netwidth_deformation, 3)
        init.xavier_uniform_(self.deformation_layer.weight)
        pos_size = ((max_deg_point - min_deg_point) * 2 + 1) * input_ch + shape_latent_dim
        pts = [nn.Linear(pos_size, netwidth)]
        for idx in range(netdepth - 1):
            k = netwidth + pos_size if (idx % skip_layer == 0 and idx > 0) else netwidth
            pts.append(nn.Linear(k, netwidth))
        for m in pts:
            init.xavier_uniform_(m.weight)
        self.pts_linears = nn.ModuleList(pts)
        views = [nn.Linear(netwidth + view_pos_size + appearance_latent_dim, netwidth_condition)]
        for _ in range(netdepth_condition - 1):
            layer = nn.Linear(netwidth_condition, netwidth_condition)
            init.xavier_uniform_(layer.weight)
            views.append(layer)
        self.views_linear = nn.ModuleList(views)
        self.bottleneck_layer = nn.Linear(netwidth, netwidth)
        self.density_layer = nn.Linear(netwidth, num_density_channels)
        self.rgb_layer = nn.Linear(netwidth_condition, num_rgb_channels)
        for m in (self.bottleneck_layer, self.density_layer, self.rgb_layer):
            init.xavier_uniform_(m.weight)
        self.pos_size_enc = pos_size - shape_latent_dim  # 63

    # -- latent folding: b' = b + W[:, c0:c0+n] . latent (one M=1 GEMM with bias epilogue)
    @staticmethod
    def _fold(layer, c0, latent):
        W = layer.weight.detach()
        out = torch.empty((1, W.shape[0]), device=W.device)
        n = latent.shape[-1]
        gemm(out, latent, W[:, c0:], 1, W.shape[0], n, lda=n, a_kc=True, ldb=W.shape[1], b_kc=True,
             ldc=W.shape[0], bias=layer.bias.detach(), a_scale=1.0, b_scale=W_SCALE)
        return out.reshape(-1)

    def folded_biases(self, latents):
        shape = L.contig(latents["density"].detach().reshape(1, -1))
        app = L.contig(latents["color"].detach().reshape(1, -1))
        art = L.contig(latents["articulation"].detach().reshape(1, -1))
        L.require_gpu(shape, app, art)
        if shape.shape[1] != self.shape_latent_dim or art.shape[1] != self.articulation_latent_dim:
            raise ValueError("latent code sizes do not match the MLP")
        lat_def = torch.cat([shape, art], -1)  # the 160 latent columns of cat[pos, shape, art]
        return {
            "def0": self._fold(self.deformations_linear[0], self.input_ch, lat_def),
            "pts0": self._fold(self.pts_linears[0], self.pos_size_enc, shape),
            "pts_skip": self._fold(self.pts_linears[self.skip_layer + 1],
                                   self.netwidth + self.pos_size_enc, shape),
            "view0": self._fold(self.views_linear[0],
                                self.netwidth + (self.deg_view * 2 + 1) * self.input_ch_view, app),
        }

    @torch.no_grad()
    def packed_weights(self, latents):
        """The fused kernel's fp16x3 weight stream with this call's folded biases
        (aon_mlp_art_pack; re-packed per call: the folded biases follow the latent codes)."""
        fb = self.folded_biases(latents)
        W = lambda m: L.contig(m.weight.detach())  # noqa: E731
        b = lambda m: L.contig(m.bias.detach())  # noqa: E731
        # (weight, bias) in the kernels' layer order; contiguous copies (if any) live in `pairs`
        # until the pack is enqueued
        pairs = [(W(m), fb["def0"] if i == 0 else b(m)) for i, m in enumerate(self.deformations_linear)]
        pairs.append((W(self.deformation_layer), b(self.deformation_layer)))
        pairs += [(W(m), fb["pts0"] if i == 0 else fb["pts_skip"] if i == self.skip_layer + 1
                   else b(m)) for i, m in enumerate(self.pts_linears)]
        pairs += [(W(self.density_layer), b(self.density_layer)),
                  (W(self.bottleneck_layer), b(self.bottleneck_layer))]
        pairs += [(W(m), fb["view0"] if i == 0 else b(m)) for i, m in enumerate(self.views_linear)]
        pairs.append((W(self.rgb_layer), b(self.rgb_layer)))
        prm = L.mlp_art_params(pairs)  # shape-checked (ValueError) before the pack
        dev = self.rgb_layer.weight.device
        nbytes = L.lib().aon_mlp_art_packed_bytes()
        buf = getattr(self, "_art_packed", None)
        if buf is None or buf.device != dev:
            buf = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
            self._art_packed = buf
        L.call("aon_mlp_art_pack", L.ctypes.byref(prm), L.ptr(buf), L.stream(dev))
        return buf

    def _fused_ok(self):
        # the fused kernel is compiled for the default geometry (mlp_layout.hpp kLayersArt)
        return (self.fused and self.netdepth == 8 and self.netwidth == 256 and self.skip_layer == 4
                and self.netdepth_deformation == 4 and self.netwidth_deformation == 128
                and self.netdepth_condition == 4 and self.netwidth_condition == 128
                and self.input_ch == 3 and self.input_ch_view == 3 and self.min_deg_point == 0
                and self.max_deg_point == 10 and self.deg_view == 4
                and self.num_rgb_channels == 3 and self.num_density_channels == 1)

    @torch.no_grad()
    def forward_rays(self, rays_o, rays_d, viewdirs, t_vals, latents, act=L.ACT_NONE):
        """One level's MLP on samples o + t d -> raw (B*S, 4) = [raw_rgb, raw_sigma]: one fused
        kernel (aon_mlp_art_fwd: cast_rays, deformation, both pos_encs, trunk, view branch;
        ``act=L.ACT_ARTIC`` also applies model_autodecoder.py:321-323), or the layer-by-layer
        GEMM path when ``fused`` is off."""
        L.require_gpu(rays_o, rays_d, viewdirs, t_vals)
        B, S = t_vals.shape
        if self._fused_ok():
            raw = torch.empty((B * S, 4), device=t_vals.device)
            L.call("aon_mlp_art_fwd", L.ptr(self.packed_weights(latents)), L.ptr(L.contig(rays_o)),
                   L.ptr(L.contig(rays_d)), L.ptr(L.contig(viewdirs)), L.ptr(L.contig(t_vals)), B,
                   S, act, L.ptr(raw), L.stream(t_vals.device))
            return raw
        if act != L.ACT_NONE:
            raise ValueError("the layer-by-layer path returns raw outputs only")
        R, dev = B * S, t_vals.device
        xyz = torch.empty((R, 3), device=dev)
        L.call("aon_cast_rays", L.ptr(rays_o), L.ptr(rays_d), L.ptr(t_vals), B, S, None, 0,
               L.ptr(xyz), 0, 0, None, L.stream(dev))
        venc = torch.empty((B, (self.deg_view * 2 + 1) * self.input_ch_view), device=dev)
        L.call("aon_pos_enc", L.ptr(viewdirs), B, 0, self.deg_view, L.ptr(venc), L.stream(dev))
        return self._mlp(xyz, venc, S, latents)

    @torch.no_grad()
    def _mlp(self, xyz, venc, S, latents):
        """The MLP on sample positions xyz (R, 3), view encodings venc (R / S, 27) -> (R, 4)."""
        R, dev = xyz.shape[0], xyz.device
        fb = self.folded_biases(latents)
        W = lambda m: m.weight.detach()  # noqa: E731
        b = lambda m: m.bias.detach()  # noqa: E731
        # deformation MLP (model_autodecoder.py:196-205); layer 0 sees only xyz per sample
        wd = self.netwidth_deformation
        h = torch.empty((R, wd), device=dev)
        h2 = torch.empty((R, wd), device=dev)
        d0 = self.deformations_linear[0]
        gemm(h, xyz, W(d0), R, wd, 3, lda=3, a_kc=True, ldb=W(d0).shape[1], b_kc=True, ldc=wd,
             bias=fb["def0"], relu=True, a_scale=ACT_SCALE, b_scale=W_SCALE)
        for m in list(self.deformations_linear)[1:]:
            linear_fwd(h2, h, wd, W(m), b(m), relu=True)
            h, h2 = h2, h
        delta = torch.empty((R, 3), device=dev)
        linear_fwd(delta, h, wd, W(self.deformation_layer), b(self.deformation_layer))
        del h, h2
        # x' = deformation + xyz, then pos_enc (enc_after, :205-212), points given directly
        enc = torch.empty((R, self.pos_size_enc), device=dev)
        L.call("aon_cast_rays", L.ptr(xyz), None, None, R, 1, L.ptr(delta), 3, None,
               self.min_deg_point, self.max_deg_point, L.ptr(enc), L.stream(dev))
        # trunk on inputs = cat[enc, shape] (:214-220), shape folded into the biases
        nw, ne = self.netwidth, self.pos_size_enc
        x = torch.empty((R, nw), device=dev)
        y = torch.empty((R, nw), device=dev)
        p0 = self.pts_linears[0]
        gemm(x, enc, W(p0), R, nw, ne, lda=ne, a_kc=True, ldb=W(p0).shape[1], b_kc=True, ldc=nw,
             bias=fb["pts0"], relu=True, a_scale=ACT_SCALE, b_scale=W_SCALE)
        for idx in range(1, self.netdepth):
            m = self.pts_linears[idx]
            if idx == self.skip_layer + 1:  # cat[h, enc, shape]
                gemm(y, x, W(m), R, nw, nw + ne, lda=nw, a_kc=True, ldb=W(m).shape[1], b_kc=True,
                     ldc=nw, A2=enc, lda2=ne, K1=nw, bias=fb["pts_skip"], relu=True,
                     a_scale=ACT_SCALE, b_scale=W_SCALE)
            else:
                linear_fwd(y, x, nw, W(m), b(m), relu=True)
            x, y = y, x
        raw = torch.empty((R, 4), device=dev)
        linear_fwd(raw[:, 3:], x, nw, W(self.density_layer), b(self.density_layer), ldo=4)
        bot = y
        linear_fwd(bot, x, nw, W(self.bottleneck_layer), b(self.bottleneck_layer))
        # view branch on cat[bottleneck, enc_dir tiled over samples, appearance] (:224-235)
        wc, nv = self.netwidth_condition, venc.shape[1]
        v0 = self.views_linear[0]
        hv = torch.empty((R, wc), device=dev)
        hv2 = torch.empty((R, wc), device=dev)
        gemm(hv, bot, W(v0), R, wc, nw + nv, lda=nw, a_kc=True, ldb=W(v0).shape[1], b_kc=True,
             ldc=wc, A2=venc, lda2=nv, K1=nw, a2_rdiv=S, bias=fb["view0"], relu=True,
             a_scale=ACT_SCALE, b_scale=W_SCALE)
        for m in list(self.views_linear)[1:]:
            linear_fwd(hv2, hv, wc, W(m), b(m), relu=True)
            hv, hv2 = hv2, hv
        linear_fwd(raw, hv, wc, W(self.rgb_layer), b(self.rgb_layer), ldo=4)
        return raw

    def forward(self, pos, condition, latents):
        """reference model_autodecoder.py:168-239: pos (B, S, 3) sample positions (enc_after),
        condition (B, 27) encoded view directions -> (raw_rgb (B, S, 3), raw_density (B, S, 1))."""
        L.require_gpu(pos, condition)
        B, S, _ = pos.shape
        if self._fused_ok():
            raw = torch.empty((B * S, 4), device=pos.device)
            L.call("aon_mlp_art_fwd_points", L.ptr(self.packed_weights(latents)),
                   L.ptr(L.contig(pos.reshape(-1, 3))), L.ptr(L.contig(condition)), B, S,
                   L.ACT_NONE, L.ptr(raw), L.stream(pos.device))
            raw = raw.view(B, S, 4)
            return raw[..., :3], raw[..., 3:]
        raw = self._mlp(L.contig(pos.reshape(-1, 3)), L.contig(condition), S, latents).view(B, S, 4)
        return raw[..., :3], raw[..., 3:]


class NeRF_AE_Art(nn.Module):  # noqa: N801 (reference name)
    """reference model_autodecoder.py:242-337 (two-level render with latent codes)."""

    def __init__(self, num_levels: int = 2, min_deg_point: int = 0, max_deg_point: int = 10,
                 deg_view: int = 4, num_coarse_samples: int = 64, num_fine_samples: int = 128,
                 use_viewdirs: bool = True, noise_std: float = 0.0, lindisp: bool = False,
                 rgb_padding: float = 0.001, density_bias: float = -1.0, enc_after=True,
                 embed_deg=False, train_precision: str = "f16x3", train_numerics=None,
                 fused_march: bool = True, range_check: bool = True):
        """The reference's kwargs (model_autodecoder.py:243-276) plus the per-model settings of
        aonerf.model.NeRF: ``train_precision`` / ``train_numerics`` (aonerf/numerics.py),
        ``fused_march`` and ``range_check``."""
        super().__init__()
        self.train_numerics = _resolve_numerics(train_precision, train_numerics)
        self.fused_march, self.range_check = bool(fused_march), bool(range_check)
        if num_levels != 2:
            raise ValueError("the reference NeRF_AE_Art is two-level (coarse + fine)")
        if rgb_padding != 0.001 or density_bias != -1.0:
            raise ValueError("the fused epilogue implements rgb_padding=0.001, density_bias=-1")
        self.num_levels, self.min_deg_point, self.max_deg_point = num_levels, min_deg_point, max_deg_point
        self.deg_view, self.num_coarse_samples, self.num_fine_samples = deg_view, num_coarse_samples, num_fine_samples
        self.use_viewdirs, self.noise_std, self.lindisp = use_viewdirs, noise_std, lindisp
        self.rgb_padding, self.density_bias = rgb_padding, density_bias
        self.enc_after, self.embed_deg = enc_after, embed_deg
        self.coarse_mlp = NeRFMLP(min_deg_point, max_deg_point, deg_view, enc_after=enc_after,
                                  embed_deg=embed_deg)
        self.fine_mlp = NeRFMLP(min_deg_point, max_deg_point, deg_view, enc_after=enc_after,
                                embed_deg=embed_deg)

    def forward(self, rays, randomized, white_bkgd, near, far, latents, train=True, *,
                u_coarse=None, u_fine=None, return_weights=False, return_intermediates=False,
                timers=None):
        """reference model_autodecoder.py:278-337 -> [(comp_rgb, acc, depth)_coarse, (...)_fine]
        (``u_coarse`` / ``u_fine`` inject randomized-mode uniforms; the extras as NeRF.forward;
        ``timers`` (dict) records hip events around each level's MLP / composite launches).

        With autograd enabled and trainable parameters or latent codes, each level runs the
        training path (train_art.ArtRenderLevel: the fused training forward
        aon_mlp_art_fwd_train, which also stores the activations, then the HIP backward into the
        MLP parameters and the latent codes); otherwise the fused inference kernel."""
        o, d, v = rays["rays_o"], rays["rays_d"], rays["viewdirs"]
        L.require_gpu(o, d, v)
        o, d, v = L.contig(o), L.contig(d), L.contig(v)
        training = torch.is_grad_enabled() and (
            any(p.requires_grad for p in self.parameters())
            or any(x.requires_grad for x in latents.values()))
        if training:
            return self._forward_train(o, d, v, randomized, white_bkgd, near, far, latents,
                                       u_coarse, u_fine, return_weights, return_intermediates,
                                       timers)
        with torch.no_grad():
            return self._forward_render(o, d, v, randomized, white_bkgd, near, far, latents,
                                        u_coarse, u_fine, return_weights, return_intermediates,
                                        timers)

    def _forward_train(self, o, d, v, randomized, white_bkgd, near, far, latents, u_coarse,
                       u_fine, return_weights, return_intermediates, timers=None):
        from .train_art import render_level

        B, dev = o.shape[0], o.device
        ret = []
        t_vals = weights = None
        for level in range(2):
            with torch.no_grad():  # no gradient reaches the sampling (helper.py:246-252)
                t_vals = level_t_vals(level, o, d, t_vals, weights, randomized, near, far,
                                      self.num_coarse_samples, self.num_fine_samples,
                                      self.lindisp, u_coarse, u_fine)
            mlp = self.coarse_mlp if level == 0 else self.fine_mlp
            noise = None
            if self.noise_std > 0 and randomized:  # model_autodecoder.py:318-319
                noise = torch.rand((B * t_vals.shape[1],), device=dev) * self.noise_std
            comp, acc, depth, weights = render_level(mlp, o, d, v, t_vals, white_bkgd, latents,
                                                     noise, self.train_numerics, timers)
            out = (comp, acc, depth, weights) if return_weights else (comp, acc, depth)
            if return_intermediates:
                out = out + (dict(t_vals=t_vals, weights=weights),)
            ret.append(out)
        return ret

    def _forward_render(self, o, d, v, randomized, white_bkgd, near, far, latents, u_coarse,
                        u_fine, return_weights, return_intermediates, timers=None):
        B, dev = o.shape[0], o.device
        # the overflow fallback below re-renders with the same random draws
        rng = torch.cuda.get_rng_state(dev) if randomized else None
        ret = []
        t_vals = weights = t_next = None
        for level in range(2):
            t_vals = t_next if t_next is not None else level_t_vals(
                level, o, d, t_vals, weights, randomized, near, far, self.num_coarse_samples,
                self.num_fine_samples, self.lindisp, u_coarse, u_fine)
            mlp = self.coarse_mlp if level == 0 else self.fine_mlp
            S = t_vals.shape[1]
            ev = _events(timers)
            raw = mlp.forward_rays(o, d, v, t_vals, latents)
            _record(timers, ev, f"mlp{level}", B * S)
            if self.noise_std > 0 and randomized:  # model_autodecoder.py:318-319
                raw[:, 3].copy_(raw[:, 3] + torch.rand_like(raw[:, 3]) * self.noise_std)
            ev = _events(timers)
            if level == 0 and march_ok(S, self.num_fine_samples, self.fused_march):
                # coarse compositing + the fine level's resampling in one kernel; the coarse
                # weights reach HBM only when asked for
                u, u_stride = fine_uniforms(B, self.num_fine_samples, randomized, dev, u_fine)
                (comp, acc, depth, weights), t_next = composite_march(
                    raw, t_vals, d, white_bkgd, L.ACT_ARTIC, u, u_stride, self.num_fine_samples,
                    return_weights or return_intermediates)
                _record(timers, ev, f"march{level}", B * S)
            else:
                comp = torch.empty((B, 3), device=dev)
                acc = torch.empty((B,), device=dev)
                weights = torch.empty((B, S), device=dev)
                depth = torch.empty((B,), device=dev)
                L.call("aon_composite_fwd", L.ptr(raw), 4, L.ptr(raw[:, 3:]), 4, L.ptr(t_vals),
                       L.ptr(d), B, S, int(bool(white_bkgd)), L.ACT_ARTIC, L.ptr(comp), L.ptr(acc),
                       L.ptr(weights), L.ptr(depth), L.stream(dev))
                _record(timers, ev, f"comp{level}", B * S)
            out = (comp, acc, depth, weights) if return_weights else (comp, acc, depth)
            if return_intermediates:
                out = out + (dict(t_vals=t_vals, weights=weights, raw=raw),)
            ret.append(out)
        mlps = (self.coarse_mlp, self.fine_mlp)
        if (self.range_check and all(m._fused_ok() for m in mlps)
                and not torch.cuda.is_current_stream_capturing()
                and L.range_overflow([getattr(m, "_art_packed", None) for m in mlps])):
            # an activation left the fp16x3 split's range (|x| > 8188) in the fused kernel:
            # render again layer by layer (aon_gemm operands carry 2^-8: range 1.6e7)
            warnings.warn("NeRF_AE_Art: an MLP activation exceeded the fused fp16x3 range; "
                          "re-rendered on the layer-by-layer path", RuntimeWarning)
            fused = [m.fused for m in mlps]
            for m in mlps:
                m.fused = False
            if rng is not None:
                torch.cuda.set_rng_state(rng, dev)
            try:
                return self._forward_render(o, d, v, randomized, white_bkgd, near, far, latents,
                                            u_coarse, u_fine, return_weights,
                                            return_intermediates, timers)
            finally:
                for m, f in zip(mlps, fused):
                    m.fused = f
        return ret
