"""Spherical spectral filters and the channel MLP — mirror of
MSFNO/Models/sfno/layers.py (SpectralConvS2 :336-427, SpectralAttentionS2
:536-639, MLP :145-178, trunc_normal_ :29-84, DropPath :88-118).

Constructor signatures, parameter/buffer names and shapes follow the reference
so state dicts load unchanged.  ``forward`` runs SHT → filter → inverse SHT as
one native call (``msfno_filter_forward``): HIP longitude FFTs, MFMA Legendre
contractions and either the MFMA spectral MLP (non-linear) or the per-mode
weight-streaming contraction (linear)."""
from __future__ import annotations

import math
import os
import warnings

import torch
import torch.nn as nn

from .. import _native as N
from ..harmonics import adopt
from .activations import ComplexReLU


def _no_grad_trunc_normal_(tensor, mean, std, a, b):
    def norm_cdf(x):
        return (1.0 + math.erf(x / math.sqrt(2.0))) / 2.0

    if (mean < a - 2 * std) or (mean > b + 2 * std):
        warnings.warn("mean is more than 2 std from [a, b] in nn.init.trunc_normal_.", stacklevel=2)
    with torch.no_grad():
        lo = norm_cdf((a - mean) / std)
        hi = norm_cdf((b - mean) / std)
        tensor.uniform_(2 * lo - 1, 2 * hi - 1)
        tensor.erfinv_()
        tensor.mul_(std * math.sqrt(2.0))
        tensor.add_(mean)
        tensor.clamp_(min=a, max=b)
        return tensor


def trunc_normal_(tensor, mean=0.0, std=1.0, a=-2.0, b=2.0):
    return _no_grad_trunc_normal_(tensor, mean, std, a, b)


# MSFNO_WCACHE=0: rebuild the weight images on every call (A/B of the prepared-weight cache)
_WCACHE = not os.environ.get("MSFNO_WCACHE", "").startswith("0")


class WeightCache:
    """Prepared-weight cache of a module whose native call consumes its weights as
    x3h / bf16x3 images (msfno_block_desc.wcache, msfno_mlp_desc.wcache): a device
    buffer per module, rebuilt by the native call only when a weight changed.
    Subclasses give the buffer size of a descriptor (``_wcache_bytes``)."""

    def _wcache_bytes(self, d):
        raise NotImplementedError

    def _wcache_key_of(self, device, nbytes):
        """The prepared images depend only on the module's own weights: key on the
        Parameters themselves (data_ptr, _version, dtype), not on the fp32 copies the
        descriptor points at (those are fresh tensors, version 0, often at a reused
        address)."""
        return (str(device), nbytes) + tuple(
            (p.data_ptr(), p._version, p.dtype) for p in self.parameters())

    def wcache_attach(self, d, keep, device):
        """Point the descriptor at this module's prepared-weight cache (bf16x3 weight
        images, the descriptor's wcache) and mark it valid when the weights are
        unchanged since it was filled.  Returns the key to pass to wcache_commit once
        the native call has been issued.  In-place weight updates bump _version, so
        the next call rebuilds the images; a HIP graph captured with a valid cache
        replays without the preparation (weights frozen, as in Rollout).

        Stream safety: the images were written (and last read) on the stream of the
        previous committed call; a call on another stream first waits for that call's
        completion event, so it neither reads unwritten images nor rebuilds them under
        a reader."""
        nbytes = self._wcache_bytes(d)
        if nbytes == 0 or not _WCACHE:
            return None
        buf = getattr(self, "_wcache_buf", None)
        if buf is None or buf.device != device or buf.numel() < nbytes:
            old_ev = getattr(self, "_wcache_event", None)
            if buf is not None and old_ev is not None:
                # the old buffer's last user may be another stream: the allocator must
                # not hand its memory out before that stream's work is done
                buf.record_stream(torch.cuda.ExternalStream(old_ev[0], device=buf.device))
            buf = self._wcache_buf = torch.empty(nbytes, dtype=torch.uint8, device=device)
            self._wcache_key = None
            self._wcache_event = None
        cur = torch.cuda.current_stream(device)
        ev = getattr(self, "_wcache_event", None)
        if ev is not None and ev[0] != cur.cuda_stream \
                and not torch.cuda.is_current_stream_capturing():
            cur.wait_event(ev[1])
        key = self._wcache_key_of(device, nbytes)
        d.wcache = buf.data_ptr()
        d.wcache_valid = int(key == getattr(self, "_wcache_key", None))
        return key

    def wcache_commit(self, key):
        """Mark the images valid after the native call that (re)built them.  Never
        while the stream is being captured: the preparation then lives only in the
        graph, and the buffer has not been written yet (a capture that found the
        images valid leaves the key as it was)."""
        if key is None or torch.cuda.is_current_stream_capturing():
            return
        dev = self._wcache_buf.device
        cur = torch.cuda.current_stream(dev)
        e = torch.cuda.Event()
        e.record(cur)
        self._wcache_event = (cur.cuda_stream, e)
        self._wcache_key = key



class DropPath(nn.Module):
    """Stochastic depth; identity at inference (the only mode of the fused path)."""

    def __init__(self, drop_prob=None):
        super().__init__()
        self.drop_prob = drop_prob

    def forward(self, x):
        if not self.drop_prob or not self.training:
            return x
        keep = 1.0 - self.drop_prob
        mask = (keep + torch.rand((x.shape[0],) + (1,) * (x.ndim - 1), dtype=x.dtype,
                                  device=x.device)).floor_()
        return x.div(keep) * mask


class MLP(WeightCache, nn.Module):
    """Conv1x1 → act → Conv1x1 (state-dict keys fwd.0.*, fwd.2.*).  Inside a
    block it is executed by the fused native block (two MFMA GEMMs with the
    norm1/FiLM affine folded into fc1 and GELU / bias / residual in epilogues);
    standalone (the network encoder / decoder) by msfno_mlp_forward."""

    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU,
                 output_bias=True, drop_rate=0.0, checkpointing_mlp=False):
        super().__init__()
        self.checkpointing_mlp = checkpointing_mlp
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        fc1 = nn.Conv2d(in_features, hidden_features, 1, bias=True)
        act = act_layer()
        fc2 = nn.Conv2d(hidden_features, out_features, 1, bias=output_bias)
        if drop_rate > 0.0:
            drop = nn.Dropout(drop_rate)
            self.fwd = nn.Sequential(fc1, act, drop, fc2, drop)
        else:
            self.fwd = nn.Sequential(fc1, act, fc2)

    def native_desc(self, cin2=0):
        fc1, act, fc2 = self.fwd[0], self.fwd[1], self.fwd[-1]
        if not (isinstance(act, nn.GELU) and getattr(act, "approximate", "none") == "none"):
            raise NotImplementedError("the native MLP fuses GELU(approximate='none') only")
        if self.training and len(self.fwd) > 3:
            raise NotImplementedError("MLP dropout in training mode is not fused")
        keep = []

        def f32(t):
            t = t.detach().float().contiguous()
            keep.append(t)
            return t

        w1, w2 = f32(fc1.weight), f32(fc2.weight)
        b1 = f32(fc1.bias)
        b2 = f32(fc2.bias) if fc2.bias is not None else None
        d = N.MlpDesc()
        d.Cin = w1.shape[1] - cin2
        d.Cin2 = cin2
        d.Hid = w1.shape[0]
        d.Cout = w2.shape[0]
        d.fc1_w, d.fc1_b, d.fc2_w, d.fc2_b = w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), N.ptr(b2)
        return d, keep

    def _wcache_bytes(self, d):
        return N.lib().msfno_mlp_wcache_size(d)

    @N.on_input_device
    def native_forward(self, x, x2=None, addend=None):
        """out = fc2(GELU(fc1(cat(x, x2)))) (+ addend, broadcast over the batch when its
        leading dimension is 1) in two MFMA GEMMs (msfno_mlp_forward); the channel
        concatenation is consumed in place (sfnonet.py:680-686)."""
        dtype = x.dtype
        x = N.require_device_f32(x, "MLP input")
        B, Cin, H, W = x.shape
        cin2 = 0
        if x2 is not None:
            x2 = N.require_device_f32(x2, "MLP second input")
            assert x2.shape[0] == B and x2.shape[2:] == x.shape[2:]
            cin2 = x2.shape[1]
        d, keep = self.native_desc(cin2)
        if d.Cin != Cin:
            raise ValueError(f"MLP expects {d.Cin} (+{cin2}) input channels, got {Cin}")
        bstride = 0
        if addend is not None:
            addend = N.require_device_f32(addend, "MLP addend")
            assert addend.shape[1:] == (d.Cout, H, W)
            bstride = 0 if addend.shape[0] == 1 else d.Cout * H * W
        L = N.lib()
        P = H * W
        wkey = self.wcache_attach(d, keep, x.device)
        nbytes = L.msfno_mlp_workspace_size(d, B, P)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=x.device)
        out = torch.empty(B, d.Cout, H, W, dtype=torch.float32, device=x.device)
        N.check(L.msfno_mlp_forward(d, x.data_ptr(), N.ptr(x2), N.ptr(addend), bstride,
                                    out.data_ptr(), B, P, ws.data_ptr(), nbytes,
                                    N.stream_of(x.device)), "MLP.forward")
        self.wcache_commit(wkey)
        del keep
        return out.to(dtype)

    @N.on_input_device
    def native_forward_affine(self, x, x_scale, x_shift, x2=None, addend=None):
        """native_forward of (x_scale * x + x_shift) per (batch, channel) — the deferred
        output affine of the block that produced x (msfno_mlp_forward_affine; fused widths
        only)."""
        dtype = x.dtype
        x = N.require_device_f32(x, "MLP input")
        B, Cin, H, W = x.shape
        xa = x_scale.detach().float().reshape(B, Cin).contiguous()
        xt = x_shift.detach().float().reshape(B, Cin).contiguous()
        cin2 = 0
        if x2 is not None:
            x2 = N.require_device_f32(x2, "MLP second input")
            assert x2.shape[0] == B and x2.shape[2:] == x.shape[2:]
            cin2 = x2.shape[1]
        d, keep = self.native_desc(cin2)
        if d.Cin != Cin:
            raise ValueError(f"MLP expects {d.Cin} (+{cin2}) input channels, got {Cin}")
        bstride = 0
        if addend is not None:
            addend = N.require_device_f32(addend, "MLP addend")
            assert addend.shape[1:] == (d.Cout, H, W)
            bstride = 0 if addend.shape[0] == 1 else d.Cout * H * W
        L = N.lib()
        P = H * W
        wkey = self.wcache_attach(d, keep, x.device)
        nbytes = L.msfno_mlp_workspace_size(d, B, P)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=x.device)
        out = torch.empty(B, d.Cout, H, W, dtype=torch.float32, device=x.device)
        N.check(L.msfno_mlp_forward_affine(d, x.data_ptr(), xa.data_ptr(), xt.data_ptr(),
                                           N.ptr(x2), N.ptr(addend), bstride, out.data_ptr(), B,
                                           P, ws.data_ptr(), nbytes, N.stream_of(x.device)),
                "MLP.forward_affine")
        self.wcache_commit(wkey)
        del keep
        return out.to(dtype)

    @N.on_input_device
    def native_backward_input(self, x, dy, x2=None, need_dx=True, params=(), need_dx2=False):
        """dL/dx of fc2(GELU(fc1(cat(x, x2)))) (msfno_mlp_backward_params): the decoder's
        backward in FiLM fine-tuning, plus the gradients of ``params`` (a subset of fc1 /
        fc2 weight and bias: the decoder trains under --retrain-film, MSFNO/Models/sfno/
        model.py:922-923), and dL/dx2 when need_dx2.  Returns dx, or (dx, [dL/dp ...])
        when params are given, with dx2 appended when asked for."""
        x = N.require_device_f32(x, "MLP input")
        dy = N.require_device_f32(dy, "MLP output gradient")
        B, Cin, H, W = x.shape
        cin2 = 0
        if x2 is not None:
            x2 = N.require_device_f32(x2, "MLP second input")
            cin2 = x2.shape[1]
        d, keep = self.native_desc(cin2)
        L = N.lib()
        P = H * W
        fc1, fc2 = self.fwd[0], self.fwd[-1]
        slots = {id(fc1.weight): 0, id(fc2.weight): 2}
        if fc1.bias is not None:
            slots[id(fc1.bias)] = 1
        if fc2.bias is not None:
            slots[id(fc2.bias)] = 3
        outs, pgs = [None] * 4, []
        for p in params:
            if id(p) not in slots:
                raise NotImplementedError(f"no native gradient for parameter {tuple(p.shape)}")
            t = torch.empty(p.shape, dtype=torch.float32, device=x.device)
            outs[slots[id(p)]] = t
            pgs.append(t)
        nbytes = (L.msfno_mlp_backward_params_workspace_size(d, B, P) if params or need_dx2
                  else L.msfno_mlp_backward_input_workspace_size(d, B, P))
        ws = torch.empty(nbytes, dtype=torch.uint8, device=x.device)
        dx = torch.empty(B, Cin, H, W, dtype=torch.float32, device=x.device) if need_dx else None
        dx2 = torch.empty_like(x2) if need_dx2 else None
        N.check(L.msfno_mlp_backward_params(d, x.data_ptr(), N.ptr(x2), dy.data_ptr(), N.ptr(dx),
                                            N.ptr(dx2), *[N.ptr(t) for t in outs], B, P,
                                            ws.data_ptr(), nbytes, N.stream_of(x.device)),
                "MLP.backward")
        del keep
        if need_dx2:
            return dx, pgs, dx2
        return (dx, pgs) if params else dx

    def forward(self, x):
        if torch.is_grad_enabled():
            params = tuple(p for p in self.parameters() if p.requires_grad)
            if x.requires_grad or params:
                return _MLPFn.apply(x, None, None, self, *params)
        return self.native_forward(x)


class _MLPFn(torch.autograd.Function):
    """Native MLP forward; backward to the first input (MSFNO's FiLM fine-tuning,
    sfnonet.py:787-860) and to the MLP's trainable weights (the decoder under
    --retrain-film), which ride along as trailing inputs."""

    @staticmethod
    def forward(ctx, x, x2, addend, mlp, *params):
        ctx.mlp, ctx.params = mlp, params
        if addend is not None:
            ctx.addend_shape, ctx.addend_dtype = addend.shape, addend.dtype
        ctx.save_for_backward(x, x2)
        return mlp.native_forward(x, x2=x2, addend=addend)

    @staticmethod
    def backward(ctx, dy):
        from .sfnonet import _scatter, _wanted
        x, x2 = ctx.saved_tensors
        wanted = _wanted(ctx, 4, ctx.params)
        need2 = bool(ctx.needs_input_grad[1])  # the decoder's big skip (the network input)
        dx, dx2, pgs = None, None, []
        if ctx.needs_input_grad[0] or wanted or need2:
            res = ctx.mlp.native_backward_input(x, dy, x2=x2, need_dx=ctx.needs_input_grad[0],
                                                params=wanted, need_dx2=need2)
            if need2:
                dx, pgs, dx2 = res
                dx2 = dx2.to(x2.dtype)
            else:
                dx, pgs = res if wanted else (res, [])
            dx = dx.to(x.dtype) if dx is not None else None
        dadd = None
        if ctx.needs_input_grad[2]:  # the encoder's pos_embed, broadcast over the batch
            dadd = dy.sum(0, keepdim=True) if ctx.addend_shape[0] == 1 else dy
            dadd = dadd.reshape(ctx.addend_shape).to(ctx.addend_dtype)
        return (dx, dx2, dadd, None) + _scatter(ctx.params, wanted, pgs)


def _check_transforms(fwd, inv):
    """The native transforms for the filter's (fwd, inv): msfno_amd.harmonics objects as
    they are, torch-harmonics-style ones wrapped around their own tables (harmonics.adopt)."""
    fwd, inv = adopt(fwd, False), adopt(inv, True)
    assert inv.lmax == fwd.lmax
    assert inv.mmax == fwd.mmax
    return fwd, inv


class _S2FilterBase(nn.Module):
    """Shared native dispatch for the two S2 filters."""

    def _fill_desc(self, d: N.BlockDesc, keep: list):  # pragma: no cover - overridden
        raise NotImplementedError

    def native_desc(self, C):
        d = N.BlockDesc()
        keep = []
        d.C = C
        d.norm_eps = 1e-6
        self._fill_desc(d, keep)
        return d, keep

    @N.on_input_device
    def forward(self, x):
        dtype = x.dtype
        x = N.require_device_f32(x, "filter input")
        B, C, H, W = x.shape
        fwd, inv = self._transforms()
        assert H == fwd.nlat and W == fwd.nlon
        pf = fwd._plan(x.device)
        pi = inv._plan(x.device)
        d, keep = self.native_desc(C)
        L = N.lib()
        nbytes = L.msfno_block_workspace_size(d, pf.handle, pi.handle, B)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=x.device)
        y = torch.empty(B, C, inv.nlat, inv.nlon, dtype=torch.float32, device=x.device)
        N.check(L.msfno_filter_forward(d, pf.handle, pi.handle, x.data_ptr(), y.data_ptr(), B,
                                       ws.data_ptr(), nbytes, N.stream_of(x.device)),
                type(self).__name__ + ".forward")
        del keep
        return y.to(dtype)


class SpectralConvS2(_S2FilterBase):
    """Linear spectral filter: per-(l,m) complex C×C weights on the tril modes."""

    def __init__(self, forward_transform, inverse_transform, hidden_size, sparsity_threshold=0.0,
                 use_complex_kernels=False, compression=None, rank=128, bias=False):
        super().__init__()
        self.hidden_size = hidden_size
        self.sparsity_threshold = sparsity_threshold
        self.scale = 0.02
        self.forward_transform = forward_transform
        self.inverse_transform = inverse_transform
        self.modes_lat = self.forward_transform.lmax
        self.modes_lon = self.forward_transform.mmax
        assert self.inverse_transform.lmax == self.modes_lat
        assert self.inverse_transform.mmax == self.modes_lon
        ii, jj = torch.tril_indices(self.modes_lat, self.modes_lon)
        self.register_buffer("ii", ii)
        self.register_buffer("jj", jj)
        if compression == "tt":
            raise NotImplementedError("compression='tt' is not on the MI355X path (SURVEY §2 row 3)")
        self.w = nn.Parameter(self.scale * torch.randn(self.hidden_size, self.hidden_size,
                                                       len(ii), 2))
        if bias:
            raise NotImplementedError("SpectralConvS2(bias=True) is not on the MI355X path")

    def _transforms(self):
        return _check_transforms(self.forward_transform, self.inverse_transform)

    def _fill_desc(self, d, keep):
        if self.sparsity_threshold != 0.0:
            raise NotImplementedError("softshrink with a non-zero threshold is not fused")
        key = (self.ii.data_ptr(), self.ii._version, self.jj.data_ptr(), self.jj._version)
        if getattr(self, "_tril_checked", None) != key:  # validated once (avoids a D2H sync per call)
            ref_ii, ref_jj = torch.tril_indices(self.modes_lat, self.modes_lon)
            if not (torch.equal(self.ii.cpu(), ref_ii) and torch.equal(self.jj.cpu(), ref_jj)):
                raise NotImplementedError("ii/jj must be torch.tril_indices(lmax, mmax)")
            self._tril_checked = key
        w = self.w.detach()
        if w.dtype != torch.float32 or not w.is_contiguous():
            w = w.float().contiguous()
        keep.append(w)
        d.filter_type = N.FILTER_LINEAR
        d.lin_w = w.data_ptr()


class SpectralAttentionS2(_S2FilterBase):
    """Non-linear spectral filter: complex MLP shared over all (l,m) modes."""

    def __init__(self, forward_transform, inverse_transform, embed_dim, sparsity_threshold=0.0,
                 hidden_size_factor=2, use_complex_network=True, use_complex_kernels=False,
                 complex_activation="real", bias=False, spectral_layers=1, drop_rate=0.0):
        super().__init__()
        self.embed_dim = embed_dim
        self.sparsity_threshold = sparsity_threshold
        self.hidden_size = int(hidden_size_factor * self.embed_dim)
        self.scale = 0.02
        self.spectral_layers = spectral_layers
        self.modes_lat = forward_transform.lmax
        self.modes_lon = forward_transform.mmax
        # the reference stores only the bound forward methods (layers.py:573-574)
        self.forward_transform = forward_transform.forward
        self.inverse_transform = inverse_transform.forward
        assert inverse_transform.lmax == self.modes_lat
        assert inverse_transform.mmax == self.modes_lon
        w = [self.scale * torch.randn(self.embed_dim, self.hidden_size, 2)]
        for _ in range(1, self.spectral_layers):
            w.append(self.scale * torch.randn(self.hidden_size, self.hidden_size, 2))
        self.w = nn.ParameterList(w)
        if bias:
            raise NotImplementedError("SpectralAttentionS2(bias=True) is not on the MI355X path")
        self.wout = nn.Parameter(self.scale * torch.randn(self.hidden_size, self.embed_dim, 2))
        self.drop = nn.Dropout(drop_rate) if drop_rate > 0.0 else nn.Identity()
        self.activation = ComplexReLU(mode=complex_activation, bias_shape=(self.hidden_size, 1, 1))

    def _transforms(self):
        return _check_transforms(self.forward_transform.__self__, self.inverse_transform.__self__)

    def _fill_desc(self, d, keep):
        if self.activation.mode != "real":
            raise NotImplementedError("only complex_activation='real' is fused")
        if self.training and not isinstance(self.drop, nn.Identity):
            raise NotImplementedError("spectral dropout in training mode is not fused")
        if self.spectral_layers > 8:
            raise NotImplementedError("spectral_layers > 8")
        d.filter_type = N.FILTER_NONLINEAR
        d.spectral_layers = self.spectral_layers
        d.spec_hidden = self.hidden_size
        for l, p in enumerate(self.w):
            t = p.detach().float().contiguous()
            keep.append(t)
            d.spec_w[l] = t.data_ptr()
        t = self.wout.detach().float().contiguous()
        keep.append(t)
        d.spec_wout = t.data_ptr()
