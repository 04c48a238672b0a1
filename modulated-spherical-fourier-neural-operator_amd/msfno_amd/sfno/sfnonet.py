"""SFNO-Block — mirror of MSFNO/Models/sfno/sfnonet.py (SpectralFilterLayer
:56-133, FourierNeuralOperatorBlock :136-251, FourierNeuralOperatorBlock_Filmed
:254-393, FiLM :689-697).

Same constructor signatures, submodule names and state-dict keys as the
reference.  ``forward`` executes the whole block — norm0, SHT, spectral filter,
inverse SHT, inner skip (+GELU for the linear filter), norm1, FiLM, MLP and the
outer skip — as ONE native call (``msfno_block_forward``) on the current HIP
stream: the FFT kernel emits the norm0 statistics, norm0 is folded into the
spectrum transpose, norm1+FiLM are folded into fc1's weights, and GELU / bias /
residual adds live in GEMM epilogues.  Inference semantics (no autograd graph).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .. import _native as N
from ..harmonics import RealSHT
from .layers import MLP, DropPath, SpectralAttentionS2, SpectralConvS2


class SpectralFilterLayer(nn.Module):
    def __init__(self, forward_transform, inverse_transform, embed_dim_sfno, filter_type="linear",
                 sparsity_threshold=0.0, use_complex_kernels=True, hidden_size_factor=2,
                 compression=None, rank=128, complex_network=True, complex_activation="real",
                 spectral_layers=1, drop_rate=0.0):
        super().__init__()
        if filter_type == "non-linear" and isinstance(forward_transform, RealSHT):
            self.filter = SpectralAttentionS2(
                forward_transform, inverse_transform, embed_dim_sfno, sparsity_threshold,
                use_complex_network=complex_network, use_complex_kernels=use_complex_kernels,
                hidden_size_factor=hidden_size_factor, complex_activation=complex_activation,
                spectral_layers=spectral_layers, drop_rate=drop_rate, bias=False)
        elif filter_type == "linear" and isinstance(forward_transform, RealSHT):
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


class FourierNeuralOperatorBlock(nn.Module):
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
            if len(seq) != 3 or not _is_exact_gelu(seq[1]):
                if self.training:
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
        nbytes = L.msfno_block_workspace_size(d, pf.handle, pi.handle, B)
        ws = torch.empty(nbytes, dtype=torch.uint8, device=x.device)
        out = torch.empty(B, C, inv.nlat, inv.nlon, dtype=torch.float32, device=x.device)
        N.check(L.msfno_block_forward(d, pf.handle, pi.handle, x.data_ptr(), N.ptr(gamma),
                                      N.ptr(beta), float(scale), out.data_ptr(), B, ws.data_ptr(),
                                      nbytes, N.stream_of(x.device)),
                type(self).__name__ + ".forward")
        del keep
        return out.to(dtype)

    def forward(self, x, *overflow):
        return self._native_forward(x)


class FourierNeuralOperatorBlock_Filmed(FourierNeuralOperatorBlock):
    _filmed = True

    def forward(self, x, gamma, beta, scale=1):
        return self._native_forward(x, gamma, beta, scale)
