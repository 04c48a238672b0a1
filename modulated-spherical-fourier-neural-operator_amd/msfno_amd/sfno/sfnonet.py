"""SFNO-Block and network — mirror of MSFNO/Models/sfno/sfnonet.py
(SpectralFilterLayer :56-133, FourierNeuralOperatorBlock :136-251,
FourierNeuralOperatorBlock_Filmed :254-393, FourierNeuralOperatorNet :406-686,
FiLM :689-697, FourierNeuralOperatorNet_Filmed :699-860).

Same constructor signatures, submodule names and state-dict keys as the
reference.  ``forward`` executes the whole block — norm0, SHT, spectral filter,
inverse SHT, inner skip (+GELU for the linear filter), norm1, FiLM, MLP and the
outer skip — as ONE native call (``msfno_block_forward``) on the current HIP
stream: the FFT kernel emits the norm0 statistics, norm0 is folded into the
spectrum transpose, norm1+FiLM are folded into fc1's weights, and GELU / bias /
residual adds live in GEMM epilogues.  Autograd (SFNO weights frozen, as MSFNO's FiLM
fine-tuning): gradients to the FiLM modulation and to the block input through native
backward calls (msfno_block_film_backward, msfno_block_backward).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import _native as N
from ..harmonics import RealSHT, adopt
from .layers import MLP, DropPath, SpectralAttentionS2, SpectralConvS2, WeightCache


def _is_real_sht(t):
    """A RealSHT of this package or of torch-harmonics (harmonics.adopt wraps the latter)."""
    try:
        adopt(t, False)
        return True
    except NotImplementedError:
        return False


class SpectralFilterLayer(nn.Module):
    def __init__(self, forward_transform, inverse_transform, embed_dim_sfno, filter_type="linear",
                 sparsity_threshold=0.0, use_complex_kernels=True, hidden_size_factor=2,
                 compression=None, rank=128, complex_network=True, complex_activation="real",
                 spectral_layers=1, drop_rate=0.0):
        super().__init__()
        if filter_type == "non-linear" and _is_real_sht(forward_transform):
            self.filter = SpectralAttentionS2(
                forward_transform, inverse_transform, embed_dim_sfno, sparsity_threshold,
                use_complex_network=complex_network, use_complex_kernels=use_complex_kernels,
                hidden_size_factor=hidden_size_factor, complex_activation=complex_activation,
                spectral_layers=spectral_layers, drop_rate=drop_rate, bias=False)
        elif filter_type == "linear" and _is_real_sht(forward_transform):
            self.filter = SpectralConvS2(
                forward_transform, inverse_transform, embed_dim_sfno, sparsity_threshold,
                use_complex_kernels=use_complex_kernels, compression=compression, rank=rank,
                bias=False)
        else:
            # RealFFT2 ("fft" spectral transform) is out of scope
            raise NotImplementedError

    def forward(self, x):
        return self.filter(x)


class FiLM(nn.Module):
    """(1 + γ·scale)·x + β·scale with γ, β of shape (B, C).  Inside the block it is
    folded into the per-channel norm1 affine; standalone calls broadcast."""

    def forward(self, x, gammas, betas, scale=1):
        g = gammas[:, :, None, None]
        b = betas[:, :, None, None]
        return ((1 + g * scale) * x) + b * scale


def _is_exact_gelu(m):
    return isinstance(m, nn.GELU) and getattr(m, "approximate", "none") == "none"


class FourierNeuralOperatorBlock(WeightCache, nn.Module):
    _filmed = False

    def __init__(self, forward_transform, inverse_transform, embed_dim_sfno, filter_type="linear",
                 mlp_ratio=2.0, drop_rate=0.0, drop_path=0.0, act_layer=nn.GELU,
                 norm_layer=(nn.LayerNorm, nn.LayerNorm), sparsity_threshold=0.0,
                 use_complex_kernels=True, compression=None, rank=128, inner_skip="linear",
                 outer_skip=None, concat_skip=False, mlp_mode="none", complex_network=True,
                 complex_activation="real", spectral_layers=1, checkpointing_mlp=False):
        super().__init__()
        self.norm0 = norm_layer[0]()
        if self._filmed:
            self.film = FiLM()
        self.filter_layer = SpectralFilterLayer(
            forward_transform, inverse_transform, embed_dim_sfno, filter_type, sparsity_threshold,
            use_complex_kernels=use_complex_kernels, hidden_size_factor=mlp_ratio,
            compression=compression, rank=rank, complex_network=complex_network,
            complex_activation=complex_activation, spectral_layers=spectral_layers,
            drop_rate=drop_rate)
        if inner_skip == "linear":
            self.inner_skip = nn.Conv2d(embed_dim_sfno, embed_dim_sfno, 1, 1)
        elif inner_skip == "identity":
            self.inner_skip = nn.Identity()
        self.concat_skip = concat_skip
        if concat_skip and inner_skip is not None:
            self.inner_skip_conv = nn.Conv2d(2 * embed_dim_sfno, embed_dim_sfno, 1, bias=False)
        if filter_type == "linear":
            self.act_layer = act_layer()
        self.drop_path = DropPath(drop_path) if drop_path > 0.0 else nn.Identity()
        self.norm1 = norm_layer[1]()
        if mlp_mode != "none":
            mlp_hidden_dim = int(embed_dim_sfno * mlp_ratio)
            self.mlp = MLP(in_features=embed_dim_sfno, hidden_features=mlp_hidden_dim,
                           act_layer=act_layer, drop_rate=drop_rate,
                           checkpointing_mlp=checkpointing_mlp)
        if outer_skip == "linear":
            self.outer_skip = nn.Conv2d(embed_dim_sfno, embed_dim_sfno, 1, 1)
        elif outer_skip == "identity":
            self.outer_skip = nn.Identity()
        if concat_skip and outer_skip is not None:
            self.outer_skip_conv = nn.Conv2d(2 * embed_dim_sfno, embed_dim_sfno, 1, bias=False)
        self.embed_dim_sfno = embed_dim_sfno

    # -- native descriptor -------------------------------------------------------
    def _norm_params(self, norm, keep):
        if not isinstance(norm, nn.InstanceNorm2d) or norm.track_running_stats:
            raise NotImplementedError("the fused block needs InstanceNorm2d(track_running_stats=False)")
        w = b = None
        if norm.affine:
            w = norm.weight.detach().float().contiguous()
            b = norm.bias.detach().float().contiguous()
            keep += [w, b]
        return N.ptr(w), N.ptr(b), float(norm.eps)

    def native_desc(self):
        keep = []
        flt = self.filter_layer.filter
        d, fkeep = flt.native_desc(self.embed_dim_sfno)
        keep += fkeep
        C = self.embed_dim_sfno
        if self.concat_skip:
            raise NotImplementedError("concat_skip=True is not on the MI355X path")
        if self.training and not isinstance(self.drop_path, nn.Identity):
            raise NotImplementedError("drop_path in training mode is not fused")
        d.norm0_w, d.norm0_b, eps0 = self._norm_params(self.norm0, keep)
        d.norm1_w, d.norm1_b, eps1 = self._norm_params(self.norm1, keep)
        if eps0 != eps1:
            raise NotImplementedError("norm0/norm1 with different eps")
        d.norm_eps = eps0
        if hasattr(self, "act_layer") and not _is_exact_gelu(self.act_layer):
            raise NotImplementedError("only nn.GELU() (erf) is fused after the inner skip")
        if hasattr(self, "inner_skip"):
            if isinstance(self.inner_skip, nn.Conv2d):
                w = self.inner_skip.weight.detach().float().contiguous()
                b = self.inner_skip.bias
                b = b.detach().float().contiguous() if b is not None else None
                keep += [w, b]
                d.inner_skip, d.skip_w, d.skip_b = N.SKIP_LINEAR, w.data_ptr(), N.ptr(b)
            else:
                d.inner_skip = N.SKIP_IDENTITY
        else:
            d.inner_skip = N.SKIP_NONE
        if hasattr(self, "outer_skip"):
            if isinstance(self.outer_skip, nn.Conv2d):
                raise NotImplementedError("outer_skip='linear' is not on the MI355X path")
            d.outer_skip = N.SKIP_IDENTITY
        else:
            d.outer_skip = N.SKIP_NONE
        if hasattr(self, "mlp"):
            seq = self.mlp.fwd
            # the fused MLP applies GELU(erf) whatever the module says: refuse anything else
            # (layers.py:161-178 builds fc1, act, [drop], fc2, [drop])
            if len(seq) not in (3, 5) or not _is_exact_gelu(seq[1]):
                raise NotImplementedError("the block MLP fuses fc1 -> nn.GELU() (erf) -> fc2 only")
            if len(seq) == 5 and self.training:
                raise NotImplementedError("MLP dropout in training mode is not fused")
            fc1, fc2 = seq[0], seq[-2] if len(seq) == 5 else seq[2]
            w1 = fc1.weight.detach().float().contiguous()
            b1 = fc1.bias.detach().float().contiguous() if fc1.bias is not None else None
            w2 = fc2.weight.detach().float().contiguous()
            b2 = fc2.bias.detach().float().contiguous() if fc2.bias is not None else None
            keep += [w1, b1, w2, b2]
            d.has_mlp = 1
            d.mlp_hidden = w1.shape[0]
            d.fc1_w, d.fc1_b, d.fc2_w, d.fc2_b = w1.data_ptr(), N.ptr(b1), w2.data_ptr(), N.ptr(b2)
        else:
            d.has_mlp = 0
        return d, keep

    def _transforms(self):
        return self.filter_layer.filter._transforms()

    def _wcache_bytes(self, d):
        return N.lib().msfno_block_wcache_size(d)

    @N.on_input_device
    def _native_forward(self, x, gamma=None, beta=None, scale=1.0):
        dtype = x.dtype
        x = N.require_device_f32(x, "block input")
        B, C, H, W = x.shape
        fwd, inv = self._transforms()
        assert H == fwd.nlat and W == fwd.nlon and C == self.embed_dim_sfno
        pf = fwd._plan(x.device)
        pi = inv._plan(x.device)
        d, keep = self.native_desc()
        if gamma is not None:
            gamma = gamma.detach().float().reshape(B, C).contiguous()
            beta = beta.detach().float().reshape(B, C).contiguous()
        L = N.lib()
        wkey = self.wcache_attach(d, keep, x.device)
        nbytes = L.msfno_block_workspace_size(d, pf.handle, pi.handle, B)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=x.device)
        out = torch.empty(B, C, inv.nlat, inv.nlon, dtype=torch.float32, device=x.device)
        N.check(L.msfno_block_forward(d, pf.handle, pi.handle, x.data_ptr(), N.ptr(gamma),
                                      N.ptr(beta), float(scale), out.data_ptr(), B, ws.data_ptr(),
                                      nbytes, N.stream_of(x.device)),
                type(self).__name__ + ".forward")
        self.wcache_commit(wkey)
        del keep
        return out.to(dtype)

    def trainable(self):
        """The parameters that require grad (passed to autograd, whose backward computes
        their gradients natively: msfno_block_backward_params)."""
        return tuple(p for p in self.parameters() if p.requires_grad)

    def param_grad_fields(self):
        """(parameter, msfno_block_param_grads field, index) of every parameter the native
        backward differentiates -- all of the block's parameters."""
        out = []

        def add(p, field, idx=None):
            if p is not None:
                out.append((p, field, idx))
        for norm, tag in ((self.norm0, "norm0"), (self.norm1, "norm1")):
            if norm.affine:
                add(norm.weight, tag + "_w")
                add(norm.bias, tag + "_b")
        flt = self.filter_layer.filter
        if isinstance(flt.w, nn.ParameterList):
            for l, w in enumerate(flt.w):
                add(w, "spec_w", l)
            add(flt.wout, "spec_wout")
        else:
            add(flt.w, "lin_w")
        if isinstance(getattr(self, "inner_skip", None), nn.Conv2d):
            add(self.inner_skip.weight, "skip_w")
            add(self.inner_skip.bias, "skip_b")
        if hasattr(self, "mlp"):
            seq = self.mlp.fwd
            fc1, fc2 = seq[0], seq[-2] if len(seq) == 5 else seq[2]
            add(fc1.weight, "fc1_w")
            add(fc1.bias, "fc1_b")
            add(fc2.weight, "fc2_w")
            add(fc2.bias, "fc2_b")
        return out

    def forward(self, x, *overflow):
        if torch.is_grad_enabled():
            params = self.trainable()
            if x.requires_grad or params:
                return _BlockFn.apply(x, self, *params)
        return self._native_forward(x)

    def _adjoint_plans(self, device):
        """The two adjoint transform plans of msfno_block_backward (include/msfno.h): a
        forward plan on the output grid with table pct c_m nlon_out / 2pi (the adjoint of
        the inverse SHT: irfft(norm="forward") weighs bin m by c_m = 2 but the DC and
        Nyquist bins) and an inverse plan on the input grid with table weights d_m 2pi /
        nlon_in (the adjoint of 2pi rfft(norm="forward"): d_m = 1/2 but DC and Nyquist).
        Rebuilt only when a transform table tensor changes."""
        import math
        fwd, inv = self._transforms()
        idx = device.index if device.index is not None else torch.cuda.current_device()
        key = (idx,) + tuple((t.data_ptr(), t._version, t.dtype, str(t.device))
                             for t in (fwd.weights, inv.pct))
        cache = getattr(self, "_adj", None)
        if cache is not None and cache[0] == key:
            return cache[1], cache[2]
        mmax = fwd.mmax
        m = torch.arange(mmax, dtype=torch.float64)

        def weights(n, inner, edge):
            w = torch.full((mmax,), inner, dtype=torch.float64)
            w[(m == 0) | (2 * m == n)] = edge
            return w[:, None, None]
        t1 = (inv.pct.detach().double().cpu() * weights(inv.nlon, 2.0, 1.0)
              * (inv.nlon / (2 * math.pi))).float().to(device).contiguous()
        t2 = (fwd.weights.detach().double().cpu() * weights(fwd.nlon, 0.5, 1.0)
              * (2 * math.pi / fwd.nlon)).float().to(device).contiguous()
        fa = N.SHTPlan(inv.nlat, inv.nlon, inv.lmax, inv.mmax, False, idx)
        fa.load(t1, key)
        ga = N.SHTPlan(fwd.nlat, fwd.nlon, fwd.lmax, fwd.mmax, True, idx)
        ga.load(t2, key)
        self._adj = (key, fa, ga)
        return fa, ga

    @N.on_input_device
    def native_backward(self, x, dout, gamma=None, beta=None, scale=1.0, need_dx=True,
                        hidden_tap=None, params=()):
        """(dL/dx, dL/dgamma, dL/dbeta) for dout = dL/d(out) (msfno_block_backward_params;
        the forward is recomputed), plus a list of dL/dp for the parameters ``params``
        (--retrain-film).  dgamma / dbeta are None for an unfilmed call; dx is None unless
        need_dx.  ``hidden_tap`` (tests) receives the non-linear filter's recomputed hidden
        activations, (B, hidden, lmax, mmax) complex per layer, whose ReLU(real) masks this
        backward applied."""
        x = N.require_device_f32(x, "block input")
        dout = N.require_device_f32(dout, "block output gradient")
        B, C, H, W = x.shape
        fwd, inv = self._transforms()
        assert H == fwd.nlat and W == fwd.nlon and C == self.embed_dim_sfno
        assert dout.shape == (B, C, inv.nlat, inv.nlon)
        pf = fwd._plan(x.device)
        pi = inv._plan(x.device)
        fa, ga = self._adjoint_plans(x.device)
        d, keep = self.native_desc()
        g = b = dg = db = None
        if gamma is not None:
            g = gamma.detach().float().reshape(B, C).contiguous()
            b = beta.detach().float().reshape(B, C).contiguous()
            dg = torch.empty(B, C, dtype=torch.float32, device=x.device)
            db = torch.empty(B, C, dtype=torch.float32, device=x.device)
        dx = torch.empty_like(x) if need_dx else None
        L = N.lib()
        pgs, pg = [], None
        if params:
            fields = {id(p): (f, i) for p, f, i in self.param_grad_fields()}
            pg = N.BlockParamGrads()
            for p in params:
                if id(p) not in fields:
                    raise NotImplementedError(f"no native gradient for parameter {tuple(p.shape)}")
                f, i = fields[id(p)]
                t = torch.empty(p.shape, dtype=torch.float32, device=x.device)
                pgs.append(t)
                if i is None:
                    setattr(pg, f, t.data_ptr())
                else:
                    getattr(pg, f)[i] = t.data_ptr()
            nbytes = L.msfno_block_backward_params_workspace_size(d, pf.handle, pi.handle,
                                                                  fa.handle, ga.handle, B)
        else:
            nbytes = L.msfno_block_backward_workspace_size(d, pf.handle, pi.handle, fa.handle,
                                                            ga.handle, B)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=x.device)
        N.check(L.msfno_block_backward_params(d, pf.handle, pi.handle, fa.handle, ga.handle,
                                              x.data_ptr(), N.ptr(g), N.ptr(b), float(scale),
                                              dout.data_ptr(), N.ptr(dx), N.ptr(dg), N.ptr(db),
                                              pg, B, ws.data_ptr(), nbytes,
                                              N.stream_of(x.device)),
                type(self).__name__ + ".backward")
        if hidden_tap is not None:
            import ctypes
            offs = (ctypes.c_size_t * 8)()
            nl = ctypes.c_int(0)
            N.check(L.msfno_block_backward_hidden_offsets(d, pf.handle, pi.handle, fa.handle,
                                                          ga.handle, B, offs, 8, ctypes.byref(nl)),
                    "hidden offsets")
            n = B * d.spec_hidden * fwd.lmax * fwd.mmax * 2
            hs = [ws[offs[l]:offs[l] + 4 * n].view(torch.float32)
                  .view(B, d.spec_hidden, fwd.lmax, fwd.mmax, 2) for l in range(nl.value)]
            hidden_tap([torch.view_as_complex(h.clone()) for h in hs])
        del keep
        if params:
            return dx, dg, db, pgs
        return dx, dg, db

    def defers_output_affine(self):
        """True for blocks whose output is one per-channel affine of x1 (no MLP, no outer
        skip: the network's last block), which msfno_block_forward_deferred can leave
        to the consumer."""
        d, _ = self.native_desc()
        return d.has_mlp == 0 and d.outer_skip == N.SKIP_NONE

    @N.on_input_device
    def native_forward_deferred(self, x, gamma=None, beta=None, scale=1.0):
        """(x1, affine) with out = affine[0] * x1 + affine[1] per (b, c): the block without
        its output affine pass (msfno_block_forward_deferred)."""
        x = N.require_device_f32(x, "block input")
        B, C, H, W = x.shape
        fwd, inv = self._transforms()
        assert H == fwd.nlat and W == fwd.nlon and C == self.embed_dim_sfno
        pf = fwd._plan(x.device)
        pi = inv._plan(x.device)
        d, keep = self.native_desc()
        if gamma is not None:
            gamma = gamma.detach().float().reshape(B, C).contiguous()
            beta = beta.detach().float().reshape(B, C).contiguous()
        L = N.lib()
        wkey = self.wcache_attach(d, keep, x.device)
        nbytes = L.msfno_block_workspace_size(d, pf.handle, pi.handle, B)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=x.device)
        x1 = torch.empty(B, C, inv.nlat, inv.nlon, dtype=torch.float32, device=x.device)
        aff = torch.empty(2, B, C, dtype=torch.float32, device=x.device)
        N.check(L.msfno_block_forward_deferred(d, pf.handle, pi.handle, x.data_ptr(),
                                               N.ptr(gamma), N.ptr(beta), float(scale),
                                               x1.data_ptr(), aff.data_ptr(), B, ws.data_ptr(),
                                               nbytes, N.stream_of(x.device)),
                type(self).__name__ + ".forward_deferred")
        self.wcache_commit(wkey)
        del keep
        return x1, aff


class FourierNeuralOperatorBlock_Filmed(FourierNeuralOperatorBlock):
    _filmed = True

    def forward(self, x, gamma, beta, scale=1):
        if torch.is_grad_enabled():
            params = self.trainable()
            if gamma.requires_grad or beta.requires_grad or x.requires_grad or params:
                return _FilmedBlockFn.apply(x, gamma, beta, float(scale), self, *params)
        return self._native_forward(x, gamma, beta, scale)

    @N.on_input_device
    def global_conv(self, x, residual):
        """sfnonet.py:341-356: norm0(x) -> filter -> + inner_skip(residual) (+ GELU for
        the linear filter) -> norm1, without FiLM, MLP or outer skip
        (msfno_block_global_conv; inference only)."""
        dtype = x.dtype
        x = N.require_device_f32(x, "global_conv input")
        residual = N.require_device_f32(residual, "global_conv residual")
        B, C, H, W = x.shape
        fwd, inv = self._transforms()
        assert H == fwd.nlat and W == fwd.nlon and C == self.embed_dim_sfno
        if hasattr(self, "inner_skip"):
            assert residual.shape == x.shape
        pf = fwd._plan(x.device)
        pi = inv._plan(x.device)
        d, keep = self.native_desc()
        L = N.lib()
        wkey = self.wcache_attach(d, keep, x.device)
        nbytes = L.msfno_block_workspace_size(d, pf.handle, pi.handle, B)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=x.device)
        out = torch.empty(B, C, inv.nlat, inv.nlon, dtype=torch.float32, device=x.device)
        N.check(L.msfno_block_global_conv(d, pf.handle, pi.handle, x.data_ptr(),
                                          residual.data_ptr(), out.data_ptr(), B, ws.data_ptr(),
                                          nbytes, N.stream_of(x.device)),
                "FourierNeuralOperatorBlock_Filmed.global_conv")
        self.wcache_commit(wkey)
        del keep
        return out.to(dtype)

    @N.on_input_device
    def native_film_backward(self, x, gamma, beta, scale, dout):
        """(dL/dgamma, dL/dbeta) of this block for dout = dL/d(out), SFNO weights frozen
        (msfno_block_film_backward; the forward up to x1 is recomputed)."""
        x = N.require_device_f32(x, "block input")
        dout = N.require_device_f32(dout, "block output gradient")
        B, C, H, W = x.shape
        fwd, inv = self._transforms()
        pf = fwd._plan(x.device)
        pi = inv._plan(x.device)
        d, keep = self.native_desc()
        g = gamma.detach().float().reshape(B, C).contiguous()
        b = beta.detach().float().reshape(B, C).contiguous()
        L = N.lib()
        nbytes = L.msfno_block_film_backward_workspace_size(d, pf.handle, pi.handle, B)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=x.device)
        dg = torch.empty(B, C, dtype=torch.float32, device=x.device)
        db = torch.empty(B, C, dtype=torch.float32, device=x.device)
        N.check(L.msfno_block_film_backward(d, pf.handle, pi.handle, x.data_ptr(), g.data_ptr(),
                                            b.data_ptr(), float(scale), dout.data_ptr(),
                                            dg.data_ptr(), db.data_ptr(), B, ws.data_ptr(),
                                            nbytes, N.stream_of(x.device)),
                "FourierNeuralOperatorBlock_Filmed.backward")
        del keep
        return dg, db


def _wanted(ctx, first, params):
    """The trailing parameter inputs (from ``first``) whose gradient autograd asks for."""
    return [p for p, need in zip(params, ctx.needs_input_grad[first:]) if need]


def _scatter(params, wanted, grads):
    """Gradients in the order of ``params`` (None where not wanted), cast to each dtype."""
    by_id = {id(p): g for p, g in zip(wanted, grads)}
    return tuple(by_id[id(p)].to(p.dtype) if id(p) in by_id else None for p in params)


class _FilmedBlockFn(torch.autograd.Function):
    """Native filmed-block forward; backward to (x, gamma, beta) and, for parameters that
    require grad (--retrain-film: the last film_layers blocks train, MSFNO/Models/sfno/
    model.py:922-923, 1016-1019), to the block's own weights (msfno_block_backward_params).
    sfnonet.py:787-860 runs the filmed blocks with autograd and every earlier block under
    no_grad; the trainable parameters ride along as trailing inputs."""

    @staticmethod
    def forward(ctx, x, gamma, beta, scale, blk, *params):
        ctx.blk, ctx.scale, ctx.params = blk, scale, params
        ctx.save_for_backward(x, gamma, beta)
        return blk._native_forward(x, gamma, beta, scale)

    @staticmethod
    def backward(ctx, dout):
        x, gamma, beta = ctx.saved_tensors
        wanted = _wanted(ctx, 5, ctx.params)
        dx, pgs = None, []
        if ctx.needs_input_grad[0] or wanted:
            # dL/dx too (film_layers > 1, repeat_film: filmed blocks back to back)
            res = ctx.blk.native_backward(x, dout, gamma, beta, ctx.scale,
                                          need_dx=ctx.needs_input_grad[0], params=wanted)
            dx, dg, db = res[:3]
            pgs = res[3] if wanted else []
            dx = dx.to(x.dtype) if dx is not None else None
        else:
            dg, db = ctx.blk.native_film_backward(x, gamma, beta, ctx.scale, dout)
        return (dx, dg.reshape(gamma.shape).to(gamma.dtype),
                db.reshape(beta.shape).to(beta.dtype), None, None) + \
            _scatter(ctx.params, wanted, pgs)


class _BlockFn(torch.autograd.Function):
    """Native unfilmed block forward with dL/dx and the gradients of its trainable
    parameters (msfno_block_backward_params)."""

    @staticmethod
    def forward(ctx, x, blk, *params):
        ctx.blk, ctx.params = blk, params
        ctx.save_for_backward(x)
        return blk._native_forward(x)

    @staticmethod
    def backward(ctx, dout):
        (x,) = ctx.saved_tensors
        wanted = _wanted(ctx, 2, ctx.params)
        res = ctx.blk.native_backward(x, dout, need_dx=ctx.needs_input_grad[0], params=wanted)
        dx = res[0].to(x.dtype) if res[0] is not None else None
        return (dx, None) + _scatter(ctx.params, wanted, res[3] if wanted else [])


def _trunc_normal_init(m):
    """FourierNeuralOperatorNet._init_weights (sfnonet.py:632-640)."""
    from .layers import trunc_normal_
    if isinstance(m, (nn.Linear, nn.Conv2d)):
        trunc_normal_(m.weight, std=0.02)
        if m.bias is not None:
            nn.init.constant_(m.bias, 0)
    elif isinstance(m, nn.LayerNorm):
        nn.init.constant_(m.bias, 0)
        nn.init.constant_(m.weight, 1.0)


class FourierNeuralOperatorNet(nn.Module):
    """Mirror of MSFNO/Models/sfno/sfnonet.py:406-686 (the network around the
    block): encoder MLP → + pos_embed → num_layers blocks (block 0 maps the
    img_size equiangular grid to the (h, w) Legendre-Gauss grid, the last one
    maps back) → big-skip concat → decoder MLP.  Same constructor arguments,
    submodule names and state-dict keys; every stage runs natively (the encoder
    adds pos_embed in its fc2 epilogue, the decoder consumes the concatenation
    in place).  ``spectral_transform="fft"`` is out of scope."""

    def __init__(self, device, cfg, spectral_transform="sht", filter_type="non-linear",
                 img_size=(721, 1440), scale_factor=6, in_chans=73, out_chans=73,
                 embed_dim_sfno=256, num_layers=12, mlp_mode="distributed", mlp_ratio=2.0,
                 drop_rate=0.0, drop_path_rate=0.0, num_blocks=8, sparsity_threshold=0.0,
                 normalization_layer="instance_norm", hard_thresholding_fraction=1.0,
                 use_complex_kernels=True, big_skip=True, compression=None, rank=128,
                 complex_network=True, complex_activation="real", spectral_layers=3,
                 laplace_weighting=False, checkpointing_mlp=False, checkpointing_block=False,
                 checkpointing_encoder=False, checkpointing_decoder=False, batch_size=1,
                 **overflow):
        super().__init__()
        from functools import partial

        from ..harmonics import InverseRealSHT
        from .layers import trunc_normal_
        self.cfg, self.device = cfg, device
        self.spectral_transform = spectral_transform
        self.filter_type = filter_type
        self.img_size = img_size
        self.scale_factor = scale_factor
        self.in_chans, self.out_chans = in_chans, out_chans
        self.embed_dim_sfno = self.num_features = embed_dim_sfno
        self.num_layers, self.num_blocks = num_layers, num_blocks
        self.hard_thresholding_fraction = hard_thresholding_fraction
        self.normalization_layer = normalization_layer
        self.mlp_mode = mlp_mode
        self.big_skip = big_skip
        self.compression, self.rank = compression, rank
        self.complex_network, self.complex_activation = complex_network, complex_activation
        self.spectral_layers = spectral_layers
        self.laplace_weighting = laplace_weighting
        self.checkpointing_mlp = checkpointing_mlp
        self.checkpointing_block = checkpointing_block
        self.checkpointing_encoder = checkpointing_encoder
        self.checkpointing_decoder = checkpointing_decoder
        self.batch_size = batch_size
        self.h = self.img_size[0] // self.scale_factor
        self.w = self.img_size[1] // self.scale_factor
        self.pos_drop = nn.Dropout(p=drop_rate) if drop_rate > 0.0 else nn.Identity()
        self.dpr = [x.item() for x in torch.linspace(0, drop_path_rate, self.num_layers)]
        if self.normalization_layer == "layer_norm":
            # sfnonet.py:482-490 builds nn.LayerNorm over (H, W) with a per-pixel affine;
            # the fused block folds its norms into per-(batch, channel) affines (norm0 into
            # the spectral transpose, norm1 into the MLP's input loads), which a per-pixel
            # affine does not fit.  Refused here, at construction, not at the first forward.
            raise NotImplementedError(
                "normalization_layer='layer_norm' is not on the MI355X path (the fused block "
                "implements the reference default 'instance_norm')")
        if self.normalization_layer == "instance_norm":
            self.norm_layer0 = partial(nn.InstanceNorm2d, num_features=embed_dim_sfno, eps=1e-6,
                                       affine=True, track_running_stats=False)
            self.norm_layer1 = self.norm_layer0
        else:
            raise NotImplementedError(
                f"Error, normalization {self.normalization_layer} not implemented.")
        self.encoder = MLP(in_features=in_chans, hidden_features=embed_dim_sfno,
                           out_features=embed_dim_sfno, output_bias=False, act_layer=nn.GELU,
                           drop_rate=0.0, checkpointing_mlp=checkpointing_mlp)
        self.pos_embed = nn.Parameter(torch.zeros(1, embed_dim_sfno, img_size[0], img_size[1]))
        modes_lat = int(self.h * self.hard_thresholding_fraction)
        modes_lon = int((self.w // 2 + 1) * self.hard_thresholding_fraction)
        if self.spectral_transform == "sht":
            self.trans_down = RealSHT(*self.img_size, lmax=modes_lat, mmax=modes_lon,
                                      grid="equiangular").float()
            self.itrans_up = InverseRealSHT(*self.img_size, lmax=modes_lat, mmax=modes_lon,
                                            grid="equiangular").float()
            self.trans = RealSHT(self.h, self.w, lmax=modes_lat, mmax=modes_lon,
                                 grid="legendre-gauss").float()
            self.itrans = InverseRealSHT(self.h, self.w, lmax=modes_lat, mmax=modes_lon,
                                         grid="legendre-gauss").float()
            sht_rescaling_factor = 1e5  # sfnonet.py:550-555
            self.trans_down.weights = self.trans_down.weights * sht_rescaling_factor
            self.itrans_up.pct = self.itrans_up.pct / sht_rescaling_factor
            self.trans.weights = self.trans.weights * sht_rescaling_factor
            self.itrans.pct = self.itrans.pct / sht_rescaling_factor
        elif self.spectral_transform == "fft":
            raise NotImplementedError("spectral_transform='fft' (RealFFT2) is not on the MI355X path")
        else:
            raise ValueError("Unknown spectral transform")
        self.blocks = nn.ModuleList([self._make_block(i, drop_rate, sparsity_threshold,
                                                      use_complex_kernels, mlp_ratio)
                                     for i in range(self.num_layers)])
        self.decoder = MLP(in_features=embed_dim_sfno + self.big_skip * in_chans,
                           hidden_features=embed_dim_sfno, out_features=out_chans,
                           output_bias=False, act_layer=nn.GELU, drop_rate=0.0,
                           checkpointing_mlp=checkpointing_mlp)
        trunc_normal_(self.pos_embed, std=0.02)
        self.apply(_trunc_normal_init)

    def _block_class(self, i):
        return FourierNeuralOperatorBlock

    def _make_block(self, i, drop_rate, sparsity_threshold, use_complex_kernels, mlp_ratio):
        first_layer, last_layer = i == 0, i == self.num_layers - 1
        forward_transform = self.trans_down if first_layer else self.trans
        inverse_transform = self.itrans_up if last_layer else self.itrans
        inner_skip = "linear" if 0 < i < self.num_layers - 1 else None
        outer_skip = "identity" if 0 < i < self.num_layers - 1 else None
        mlp_mode = self.mlp_mode if not last_layer else "none"
        if first_layer:
            norm_layer = (self.norm_layer0, self.norm_layer1)
        elif last_layer:
            norm_layer = (self.norm_layer1, self.norm_layer0)
        else:
            norm_layer = (self.norm_layer1, self.norm_layer1)
        return self._block_class(i)(
            forward_transform, inverse_transform, self.embed_dim_sfno,
            filter_type=self.filter_type, mlp_ratio=mlp_ratio, drop_rate=drop_rate,
            drop_path=self.dpr[i], norm_layer=norm_layer, sparsity_threshold=sparsity_threshold,
            use_complex_kernels=use_complex_kernels, inner_skip=inner_skip,
            outer_skip=outer_skip, mlp_mode=mlp_mode, compression=self.compression,
            rank=self.rank, complex_network=self.complex_network,
            complex_activation=self.complex_activation, spectral_layers=self.spectral_layers,
            checkpointing_mlp=self.checkpointing_mlp)

    @torch.jit.ignore
    def no_weight_decay(self):
        return {"pos_embed", "cls_token"}

    def encode(self, x):
        """encoder(x) + pos_embed (sfnonet.py:667-674), pos_embed added in fc2's epilogue;
        with autograd (a plain network in training) the gradients reach x, the encoder
        weights and pos_embed natively (_MLPFn)."""
        if torch.is_grad_enabled():
            params = tuple(p for p in self.encoder.parameters() if p.requires_grad)
            if x.requires_grad or self.pos_embed.requires_grad or params:
                from .layers import _MLPFn
                return _MLPFn.apply(x, None, self.pos_embed, self.encoder, *params)
        return self.encoder.native_forward(x, addend=self.pos_embed)

    def decode(self, x, residual):
        """decoder(cat(x, residual)) (sfnonet.py:679-686) without materialising the concat;
        with autograd (FiLM fine-tuning) the gradient reaches x through the frozen decoder."""
        x2 = residual if self.big_skip else None
        if torch.is_grad_enabled():
            params = tuple(p for p in self.decoder.parameters() if p.requires_grad)
            if x.requires_grad or (x2 is not None and x2.requires_grad) or params:
                from .layers import _MLPFn
                return _MLPFn.apply(x, x2, None, self.decoder, *params)
        return self.decoder.native_forward(x, x2=x2)

    def _fuse_last_affine(self, x):
        """Whether the last block's output affine can ride in the decoder's input loads
        (inference, a last block without MLP / outer skip, a fused decoder); x is the
        network input (the decoder's second input, the big skip)."""
        if torch.is_grad_enabled() or not self.big_skip:
            return False
        blk = self.blocks[-1]
        if not blk.defers_output_affine():
            return False
        d, _ = self.decoder.native_desc(cin2=x.shape[1])
        return bool(N.lib().msfno_mlp_fused_supported(d))

    def decode_deferred(self, x1, aff, residual):
        """decoder(cat(aff[0] * x1 + aff[1], residual)) with the affine applied as the
        decoder loads x1 (msfno_mlp_forward_affine)."""
        return self.decoder.native_forward_affine(x1, aff[0], aff[1], x2=residual)

    def forward_features(self, x):
        x = self.pos_drop(x)
        for blk in self.blocks:
            x = blk(x)
        return x

    def forward(self, x):
        residual = x
        x = self.encode(x)
        if self._fuse_last_affine(residual):
            x = self.pos_drop(x)
            for blk in self.blocks[:-1]:
                x = blk(x)
            x1, aff = self.blocks[-1].native_forward_deferred(x)
            return self.decode_deferred(x1, aff, residual)
        x = self.forward_features(x)
        return self.decode(x, residual)


class FourierNeuralOperatorNet_Filmed(FourierNeuralOperatorNet):
    """Mirror of sfnonet.py:699-860: the last ``film_layers`` blocks (every block
    with cfg.repeat_film) are FourierNeuralOperatorBlock_Filmed.  The FiLM
    generator (Film_wrapper: GCN / ViT / MAE over SST fields, :862-) is outside
    the MI355X hot path: pass ``film_gen`` (any module mapping sst to
    (B, 2, film_layers, C)) or call forward with the modulation tensor itself as
    ``sst`` (film_mod[:, 0] = gamma, film_mod[:, 1] = beta, :812)."""

    def __init__(self, device, cfg, mlp_ratio=2.0, drop_rate=0.0, sparsity_threshold=0.0,
                 use_complex_kernels=True, film_gen=None, **kwargs):
        self.advanced_logging = kwargs.get("advanced_logging", False)
        self.film_layers = kwargs["film_layers"]
        self.depth = kwargs.get("model_depth")
        self._repeat_film = bool(getattr(cfg, "repeat_film", False))
        super().__init__(device, cfg, mlp_ratio=mlp_ratio, drop_rate=drop_rate,
                         sparsity_threshold=sparsity_threshold,
                         use_complex_kernels=use_complex_kernels, **kwargs)
        self.film_gen = film_gen

    def _filmed(self, i):
        return self._repeat_film or i >= self.num_layers - self.film_layers

    def _block_class(self, i):
        return FourierNeuralOperatorBlock_Filmed if self._filmed(i) else FourierNeuralOperatorBlock

    def forward(self, x, sst, scale=1):
        film_mod = self.film_gen(sst) if self.film_gen is not None else sst
        gamma, beta = film_mod[:, 0], film_mod[:, 1]
        if self.advanced_logging:
            self.gamma, self.beta = gamma, beta
        residual = x
        with torch.no_grad():  # sfnonet.py:816-827: encoder and pos_embed without autograd
            x = self.pos_drop(self.encode(x))
        fuse = self._fuse_last_affine(residual)
        nb = len(self.blocks)
        for i, blk in enumerate(self.blocks):
            film = ()
            if self._filmed(i):
                film_idx = i - (self.num_layers - self.film_layers)
                film = (gamma[:, film_idx], beta[:, film_idx], scale)
            if fuse and i == nb - 1:
                x1, aff = blk.native_forward_deferred(x, *film)
                return self.decode_deferred(x1, aff, residual)
            if film:
                x = blk(x, *film)
            else:  # sfnonet.py:838-844: unfilmed blocks under no_grad
                with torch.no_grad():
                    x = blk(x)
        return self.decode(x, residual)
