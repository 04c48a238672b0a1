"""ORACLE — test infrastructure only (never imported by the product path).

Functional torch-CPU restatement of the reference SFNO-Block forward, op for op
(same einsum strings and op order as the reference), driven by a state dict that
uses the reference's own parameter names.  It is the parity checker for the HIP
path and the ``cpu_baseline`` leg of ``bench.py``.

Followed reference code (paths relative to ``/root/reference``):

* ``MSFNO/Models/sfno/sfnonet.py:221-251``  FourierNeuralOperatorBlock.forward
* ``MSFNO/Models/sfno/sfnonet.py:359-393``  FourierNeuralOperatorBlock_Filmed.forward
* ``MSFNO/Models/sfno/sfnonet.py:689-697``  FiLM.forward
* ``MSFNO/Models/sfno/layers.py:398-427``   SpectralConvS2.forward  (linear filter)
* ``MSFNO/Models/sfno/layers.py:604-639``   SpectralAttentionS2.forward_mlp/forward
* ``MSFNO/Models/sfno/layers.py:145-178``   MLP (1x1 conv → GELU → 1x1 conv)
* ``MSFNO/Models/sfno/contractions.py:37-41``   compl_contract_fwd_c
* ``MSFNO/Models/sfno/contractions.py:132-137`` compl_mul2d_fwd_c
* ``MSFNO/Models/sfno/activations.py:42-46``    ComplexReLU mode="real"
* InstanceNorm2d(eps=1e-6, affine=True, track_running_stats=False):
  ``sfnonet.py:491-499``

Pinned against the reference import by ``tests/golden/make_golden.py`` (the
golden fixtures) and ``tests/test_oracle_golden.py``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn.functional as F

from .sht_ref import InverseRealSHT, RealSHT


# --- contractions.py -------------------------------------------------------
def compl_contract_fwd_c(a, b):
    ac = torch.view_as_complex(a)
    bc = torch.view_as_complex(b)
    return torch.view_as_real(torch.einsum("bin,kin->bkn", ac, bc))


def compl_mul2d_fwd_c(a, b):
    ac = torch.view_as_complex(a)
    bc = torch.view_as_complex(b)
    return torch.view_as_real(torch.einsum("bixy,io->boxy", ac, bc))


# --- activations.py --------------------------------------------------------
def complex_relu_real(z):
    zr = torch.view_as_real(z)
    outr = zr.clone()
    outr[..., 0] = F.leaky_relu(zr[..., 0], negative_slope=0.0)
    return torch.view_as_complex(outr)


# --- layers.py filters -----------------------------------------------------
def spectral_attention_s2(x, sht, isht, ws, wout):
    """SpectralAttentionS2.forward with bias=False, drop=Identity."""
    dtype = x.dtype
    x = x.to(sht.weights.dtype)
    xr = torch.view_as_real(sht(x))
    for w in ws:
        xr = compl_mul2d_fwd_c(xr, w.to(xr.dtype))
        xr = torch.view_as_real(complex_relu_real(torch.view_as_complex(xr)))
    xr = compl_mul2d_fwd_c(xr, wout.to(xr.dtype))
    x = isht(torch.view_as_complex(xr))
    return x.to(dtype)


def spectral_conv_s2(x, sht, isht, w, ii, jj, sparsity_threshold=0.0):
    """SpectralConvS2.forward with compression=None, bias=False."""
    dtype = x.dtype
    x = x.to(sht.weights.dtype)
    xr = torch.view_as_real(sht(x))
    modes = torch.zeros(xr.shape, dtype=xr.dtype)
    modes[:, :, ii, jj, :] = compl_contract_fwd_c(xr[:, :, ii, jj, :], w.to(xr.dtype))
    xr = F.softshrink(modes, lambd=sparsity_threshold)
    return isht(torch.view_as_complex(xr)).to(dtype)


def instance_norm(x, weight, bias, eps=1e-6):
    return F.instance_norm(x, weight=weight, bias=bias, eps=eps)


def film(x, gammas, betas, scale=1.0):
    g = gammas[:, :, None, None].expand(-1, -1, x.shape[2], x.shape[3])
    b = betas[:, :, None, None].expand(-1, -1, x.shape[2], x.shape[3])
    return ((1 + g * scale) * x) + b * scale


def conv1x1(x, w, b=None):
    return F.conv2d(x, w, b)


def mlp(x, p, prefix="mlp.fwd."):
    h = conv1x1(x, p[prefix + "0.weight"], p.get(prefix + "0.bias"))
    h = F.gelu(h)
    return conv1x1(h, p[prefix + "2.weight"], p.get(prefix + "2.bias"))


@dataclass
class BlockCfg:
    filter_type: str = "non-linear"     # "linear" | "non-linear"
    inner_skip: str | None = "linear"   # "linear" | "identity" | None
    outer_skip: str | None = "identity"  # "linear" | "identity" | None
    has_mlp: bool = True
    spectral_layers: int = 3
    eps: float = 1e-6


def global_conv(p, x, residual, sht, isht, cfg: BlockCfg):
    """FourierNeuralOperatorBlock_Filmed.global_conv(x, residual) (sfnonet.py:341-356):
    the block up to norm1, the inner skip applied to `residual`."""
    x = instance_norm(x, p["norm0.weight"], p["norm0.bias"], cfg.eps)
    if cfg.filter_type == "non-linear":
        ws = [p[f"filter_layer.filter.w.{i}"] for i in range(cfg.spectral_layers)]
        x = spectral_attention_s2(x, sht, isht, ws, p["filter_layer.filter.wout"])
    else:
        x = spectral_conv_s2(x, sht, isht, p["filter_layer.filter.w"],
                             p["filter_layer.filter.ii"], p["filter_layer.filter.jj"])
    x = x.contiguous()
    if cfg.inner_skip == "linear":
        x = x + conv1x1(residual, p["inner_skip.weight"], p["inner_skip.bias"])
    elif cfg.inner_skip == "identity":
        x = x + residual
    if cfg.filter_type == "linear":
        x = F.gelu(x)
    return instance_norm(x, p["norm1.weight"], p["norm1.bias"], cfg.eps)


def block_forward(p, x, sht, isht, cfg: BlockCfg, gamma=None, beta=None, scale=1.0):
    """SFNO-Block forward (sfnonet.py:221-251, 359-393); FiLM applied iff gamma is not
    None (Filmed block)."""
    residual = x
    x = global_conv(p, x, residual, sht, isht, cfg)
    if gamma is not None:
        x = film(x, gamma, beta, scale)
    if cfg.has_mlp:
        x = mlp(x, p)
    if cfg.outer_skip == "linear":
        x = x + conv1x1(residual, p["outer_skip.weight"], p["outer_skip.bias"])
    elif cfg.outer_skip == "identity":
        x = x + residual
    return x


# --- parameter generation (reference init recipe, layers.py:356,386-387,580-596;
#     sfnonet.py:638-646 trunc_normal_(std=.02) for convs; InstanceNorm affine = 1/0) --
def make_block_params(C, lmax, mmax, cfg: BlockCfg, seed=1, hidden_factor=2.0,
                      randomize_affine=False, dtype=torch.float32):
    g = torch.Generator().manual_seed(seed)

    def randn(*s):
        return torch.randn(*s, generator=g, dtype=dtype)

    def tn(*s, std=0.02):
        t = torch.empty(*s, dtype=dtype)
        t.normal_(0.0, std, generator=g)
        return t.clamp_(-2.0, 2.0)

    p = {}
    for n in ("norm0", "norm1"):
        if randomize_affine:
            p[f"{n}.weight"] = 1.0 + 0.1 * randn(C)
            p[f"{n}.bias"] = 0.1 * randn(C)
        else:
            p[f"{n}.weight"] = torch.ones(C, dtype=dtype)
            p[f"{n}.bias"] = torch.zeros(C, dtype=dtype)
    hidden = int(hidden_factor * C)
    if cfg.filter_type == "non-linear":
        p["filter_layer.filter.w.0"] = 0.02 * randn(C, hidden, 2)
        for i in range(1, cfg.spectral_layers):
            p[f"filter_layer.filter.w.{i}"] = 0.02 * randn(hidden, hidden, 2)
        p["filter_layer.filter.wout"] = 0.02 * randn(hidden, C, 2)
        p["filter_layer.filter.activation.bias"] = torch.zeros(1, dtype=dtype)
    else:
        ii, jj = torch.tril_indices(lmax, mmax)
        p["filter_layer.filter.ii"] = ii
        p["filter_layer.filter.jj"] = jj
        p["filter_layer.filter.w"] = 0.02 * randn(C, C, ii.numel(), 2)
    if cfg.inner_skip == "linear":
        p["inner_skip.weight"] = tn(C, C, 1, 1)
        p["inner_skip.bias"] = 0.02 * randn(C) if randomize_affine else torch.zeros(C, dtype=dtype)
    if cfg.has_mlp:
        p["mlp.fwd.0.weight"] = tn(hidden, C, 1, 1)
        p["mlp.fwd.0.bias"] = 0.02 * randn(hidden) if randomize_affine else torch.zeros(hidden, dtype=dtype)
        p["mlp.fwd.2.weight"] = tn(C, hidden, 1, 1)
        p["mlp.fwd.2.bias"] = 0.02 * randn(C) if randomize_affine else torch.zeros(C, dtype=dtype)
    if cfg.outer_skip == "linear":
        p["outer_skip.weight"] = tn(C, C, 1, 1)
        p["outer_skip.bias"] = torch.zeros(C, dtype=dtype)
    return p


def make_transforms(nlat, nlon, lmax, mmax, grid="equiangular", rescale=1e5, dtype=torch.float32):
    """The reference's transform pair incl. ``.float()`` and the ad-hoc ×1e5/÷1e5
    rescale (``sfnonet.py:537-555``)."""
    sht = RealSHT(nlat, nlon, lmax=lmax, mmax=mmax, grid=grid).to(dtype)
    isht = InverseRealSHT(nlat, nlon, lmax=lmax, mmax=mmax, grid=grid).to(dtype)
    if rescale is not None:
        sht.weights = sht.weights * rescale
        isht.pct = isht.pct / rescale
    return sht, isht


def algorithmic_flops(B, C, nlat, nlon, lmax, mmax, cfg: BlockCfg, hidden_factor=2.0):
    """Algorithmic FLOPs of one block forward (SURVEY §8(d) accounting: FFT as
    2.5·N·log2(N) per real length-N transform, triangular l>=m Legendre/spectral)."""
    T = sum(max(lmax - m, 0) for m in range(mmax))
    hid = int(hidden_factor * C)
    fft = 2 * B * C * nlat * 2.5 * nlon * math.log2(nlon)
    leg = 2 * (2 * B * C * nlat * T * 2)                    # fwd + inv, re+im rows
    if cfg.filter_type == "non-linear":
        spec = 8 * B * T * (C * hid + (cfg.spectral_layers - 1) * hid * hid + hid * C)
    else:
        spec = 8 * B * C * C * T
    P = nlat * nlon
    skip = 2 * B * C * C * P if cfg.inner_skip == "linear" else 0
    mlpf = 2 * B * P * (2 * C * hid) if cfg.has_mlp else 0
    return fft + leg + spec + skip + mlpf


# --- the network around the block (sfnonet.py:406-686) ----------------------------
@dataclass
class NetCfg:
    img_size: tuple = (721, 1440)
    scale_factor: int = 6
    num_layers: int = 12
    filter_type: str = "non-linear"
    big_skip: bool = True
    spectral_layers: int = 3
    hard_thresholding_fraction: float = 1.0


def make_net_transforms(cfg: NetCfg, dtype=torch.float32):
    """trans_down / itrans_up on the image grid, trans / itrans on the (h, w)
    Legendre-Gauss grid, all with the x1e5 rescale (sfnonet.py:532-555)."""
    h, w = cfg.img_size[0] // cfg.scale_factor, cfg.img_size[1] // cfg.scale_factor
    lmax = int(h * cfg.hard_thresholding_fraction)
    mmax = int((w // 2 + 1) * cfg.hard_thresholding_fraction)
    down = RealSHT(*cfg.img_size, lmax=lmax, mmax=mmax, grid="equiangular").to(dtype)
    up = InverseRealSHT(*cfg.img_size, lmax=lmax, mmax=mmax, grid="equiangular").to(dtype)
    tr = RealSHT(h, w, lmax=lmax, mmax=mmax, grid="legendre-gauss").to(dtype)
    itr = InverseRealSHT(h, w, lmax=lmax, mmax=mmax, grid="legendre-gauss").to(dtype)
    for f in (down, tr):
        f.weights = f.weights * 1e5
    for g in (up, itr):
        g.pct = g.pct / 1e5
    return down, up, tr, itr


def net_forward(p, x, cfg: NetCfg, transforms=None, film=None, scale=1.0):
    """FourierNeuralOperatorNet.forward (sfnonet.py:662-686); with ``film`` =
    (gamma, beta) of shape (B, film_layers, C) the last film_layers blocks are
    FiLM-modulated as in FourierNeuralOperatorNet_Filmed.forward (:837-844)."""
    down, up, tr, itr = transforms if transforms is not None else make_net_transforms(cfg)
    residual = x
    x = mlp(x, p, prefix="encoder.fwd.")
    x = x + p["pos_embed"]
    n = cfg.num_layers
    film_layers = film[0].shape[1] if film is not None else 0
    for i in range(n):
        first, last = i == 0, i == n - 1
        bcfg = BlockCfg(filter_type=cfg.filter_type,
                        inner_skip="linear" if 0 < i < n - 1 else None,
                        outer_skip="identity" if 0 < i < n - 1 else None,
                        has_mlp=not last, spectral_layers=cfg.spectral_layers)
        bp = {k[len(f"blocks.{i}."):]: v for k, v in p.items() if k.startswith(f"blocks.{i}.")}
        g = b = None
        if film is not None and i >= n - film_layers:
            g, b = film[0][:, i - (n - film_layers)], film[1][:, i - (n - film_layers)]
        x = block_forward(bp, x, down if first else tr, up if last else itr, bcfg, g, b, scale)
    if cfg.big_skip:
        x = torch.cat((x, residual), dim=1)
    return mlp(x, p, prefix="decoder.fwd.")
