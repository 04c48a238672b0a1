"""ORACLE — test infrastructure only (never imported by the product path).

CPU restatement of the spherical harmonic transform that the reference uses
through the *un-vendored* third-party package ``torch-harmonics`` (pip,
unpinned: ``/root/reference/conda_environment.yml:62``; API evidence fits the
0.6.x–0.7.x line).  torch-harmonics is NOT installed in
this image and cannot be fetched, so this module restates its published
algorithm:

* quadrature   — ``torch_harmonics.quadrature.legendre_gauss_weights`` (numpy
  ``leggauss``) and ``clenshaw_curtiss_weights`` (Waldvogel 2003 FFT formula);
* Legendre     — ``torch_harmonics.legendre.legpoly`` 3-term recurrence for the
  orthonormal associated Legendre functions, Condon–Shortley phase on odd m,
  tables indexed ``[m, l, k]`` and truncated to ``[:mmax, :lmax]``;
* RealSHT      — ``X = 2π·rfft(x, norm="forward")``; ``a = einsum('...km,mlk->...lm')``
  on real and imaginary parts separately, with ``weights = pct·w_k``;
* InverseRealSHT — ``einsum('...lm,mlk->...km')`` then ``irfft(n=nlon,
  norm="forward")``.

Call sites in the reference: ``MSFNO/Models/sfno/sfnonet.py:45,75-77,105,537-555``
(construction + the ×1e5 / ÷1e5 rescale) and ``layers.py:403-422,627-637``
(forward/inverse calls).

Parity status: torch-harmonics itself is absent, so this restatement is pinned
by mathematical known-answer tests (band-limited round trips, closed-form Y_lm,
quadrature exactness, orthonormality) in ``tests/test_oracle_sht.py`` — NOT by
reference-produced golden vectors.  The block code around it IS pinned to the
reference import (``tests/golden/make_golden.py``).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn as nn


# --------------------------------------------------------------------------
# quadrature  ([TH] torch_harmonics/quadrature.py)
# --------------------------------------------------------------------------
def legendre_gauss_weights(n: int, a: float = -1.0, b: float = 1.0):
    """Gauss–Legendre nodes/weights on [a, b] (ascending nodes)."""
    xlg, wlg = np.polynomial.legendre.leggauss(n)
    xlg = (b - a) * 0.5 * xlg + (b + a) * 0.5
    wlg = wlg * (b - a) * 0.5
    return xlg, wlg


def clenshaw_curtiss_weights(n: int, a: float = -1.0, b: float = 1.0):
    """Clenshaw–Curtis nodes ``cos(linspace(π, 0, n))`` and weights (Waldvogel)."""
    assert n > 1
    tcc = np.cos(np.linspace(np.pi, 0, n))
    if n == 2:
        wcc = np.array([1.0, 1.0])
    else:
        n1 = n - 1
        N = np.arange(1, n1, 2)
        l = len(N)
        m = n1 - l
        v = np.concatenate([2 / N / (N - 2), 1 / N[-1:], np.zeros(m)])
        v = 0 - v[:-1] - v[-1:0:-1]
        g0 = -np.ones(n1)
        g0[l] = g0[l] + n1
        g0[m] = g0[m] + n1
        g = g0 / (n1 ** 2 - 1 + (n1 % 2))
        wcc = np.fft.ifft(v + g).real
        wcc = np.concatenate((wcc, wcc[:1]))
    tcc = (b - a) * 0.5 * tcc + (b + a) * 0.5
    wcc = wcc * (b - a) * 0.5
    return tcc, wcc


def quadrature(nlat: int, grid: str):
    if grid == "legendre-gauss":
        return legendre_gauss_weights(nlat, -1, 1)
    if grid == "equiangular":
        return clenshaw_curtiss_weights(nlat, -1, 1)
    raise ValueError(f"Unknown quadrature mode {grid}")


# --------------------------------------------------------------------------
# associated Legendre functions  ([TH] torch_harmonics/legendre.py)
# --------------------------------------------------------------------------
def legpoly(mmax: int, lmax: int, x: np.ndarray, norm: str = "ortho",
            inverse: bool = False, csphase: bool = True) -> np.ndarray:
    """(-1)^m c_l^m P_l^m(x) for m<mmax, l<lmax, shape (mmax, lmax, len(x)), float64."""
    nmax = max(mmax, lmax)
    vdm = np.zeros((nmax, nmax, len(x)), dtype=np.float64)
    norm_factor = 1.0 if norm == "ortho" else np.sqrt(4 * np.pi)
    norm_factor = 1.0 / norm_factor if inverse else norm_factor
    vdm[0, 0, :] = norm_factor / np.sqrt(4 * np.pi)
    for l in range(1, nmax):
        vdm[l - 1, l, :] = np.sqrt(2 * l + 1) * x * vdm[l - 1, l - 1, :]
        vdm[l, l, :] = np.sqrt((2 * l + 1) * (1 + x) * (1 - x) / 2 / l) * vdm[l - 1, l - 1, :]
    for l in range(2, nmax):
        m = np.arange(0, l - 1)
        a = x[None, :] * np.sqrt((2 * l - 1) / (l - m) * (2 * l + 1) / (l + m))[:, None]
        b = np.sqrt((l + m - 1) / (l - m) * (2 * l + 1) / (2 * l - 3) * (l - m - 1) / (l + m))[:, None]
        vdm[m, l, :] = a * vdm[m, l - 1, :] - b * vdm[m, l - 2, :]
    if norm == "schmidt":
        for l in range(0, nmax):
            if inverse:
                vdm[:, l, :] = vdm[:, l, :] * np.sqrt(2 * l + 1)
            else:
                vdm[:, l, :] = vdm[:, l, :] / np.sqrt(2 * l + 1)
    vdm = vdm[:mmax, :lmax]
    if csphase:
        vdm[1::2] *= -1
    return vdm


def precompute_legpoly(mmax, lmax, t, norm="ortho", inverse=False, csphase=True):
    return legpoly(mmax, lmax, np.cos(t), norm=norm, inverse=inverse, csphase=csphase)


def colatitudes(nlat: int, grid: str):
    """θ north→south = flip(arccos(nodes)) and the (unflipped, symmetric) weights."""
    cost, w = quadrature(nlat, grid)
    return np.flip(np.arccos(cost)).copy(), w


# --------------------------------------------------------------------------
# transforms  ([TH] torch_harmonics/sht.py)
# --------------------------------------------------------------------------
class RealSHT(nn.Module):
    """CPU restatement of ``torch_harmonics.RealSHT`` (forward real SHT)."""

    def __init__(self, nlat, nlon, lmax=None, mmax=None, grid="equiangular",
                 norm="ortho", csphase=True):
        super().__init__()
        self.nlat, self.nlon, self.grid = nlat, nlon, grid
        self.norm, self.csphase = norm, csphase
        tq, w = colatitudes(nlat, grid)
        self.lmax = lmax or nlat
        self.mmax = mmax or nlon // 2 + 1
        pct = precompute_legpoly(self.mmax, self.lmax, tq, norm=norm, csphase=csphase)
        weights = torch.einsum("mlk,k->mlk", torch.from_numpy(pct), torch.from_numpy(w))
        self.register_buffer("weights", weights)

    def forward(self, x):
        assert x.shape[-2] == self.nlat and x.shape[-1] == self.nlon
        x = 2.0 * torch.pi * torch.fft.rfft(x, dim=-1, norm="forward")
        x = torch.view_as_real(x)
        out_shape = list(x.size())
        out_shape[-3] = self.lmax
        out_shape[-2] = self.mmax
        xout = torch.zeros(out_shape, dtype=x.dtype, device=x.device)
        w = self.weights.to(x.dtype)
        xout[..., 0] = torch.einsum("...km,mlk->...lm", x[..., : self.mmax, 0], w)
        xout[..., 1] = torch.einsum("...km,mlk->...lm", x[..., : self.mmax, 1], w)
        return torch.view_as_complex(xout)


class InverseRealSHT(nn.Module):
    """CPU restatement of ``torch_harmonics.InverseRealSHT``."""

    def __init__(self, nlat, nlon, lmax=None, mmax=None, grid="equiangular",
                 norm="ortho", csphase=True):
        super().__init__()
        self.nlat, self.nlon, self.grid = nlat, nlon, grid
        self.norm, self.csphase = norm, csphase
        t, _ = colatitudes(nlat, grid)
        self.lmax = lmax or nlat
        self.mmax = mmax or nlon // 2 + 1
        pct = precompute_legpoly(self.mmax, self.lmax, t, norm=norm, inverse=True, csphase=csphase)
        self.register_buffer("pct", torch.from_numpy(pct))

    def forward(self, x):
        assert x.shape[-2] == self.lmax and x.shape[-1] == self.mmax
        x = torch.view_as_real(x)
        p = self.pct.to(x.dtype)
        rl = torch.einsum("...lm,mlk->...km", x[..., 0], p)
        im = torch.einsum("...lm,mlk->...km", x[..., 1], p)
        xs = torch.stack((rl, im), -1)
        x = torch.view_as_complex(xs)
        return torch.fft.irfft(x, n=self.nlon, dim=-1, norm="forward")


def ylm_closed_form(l: int, m: int, theta: np.ndarray) -> np.ndarray:
    """Orthonormal P̄_l^m(cos θ) with Condon–Shortley phase from the explicit formula
    (scipy-free: ratio of factorials via lgamma), used by known-answer tests."""
    x = np.cos(theta)
    # P_l^m via the standard recurrence in (l) at fixed m, fp64, starting at P_m^m.
    pmm = np.ones_like(x)
    somx2 = np.sqrt((1.0 - x) * (1.0 + x))
    fact = 1.0
    for _ in range(m):
        pmm = -pmm * fact * somx2
        fact += 2.0
    if l == m:
        plm = pmm
    else:
        pmmp1 = x * (2 * m + 1) * pmm
        if l == m + 1:
            plm = pmmp1
        else:
            for ll in range(m + 2, l + 1):
                pll = (x * (2 * ll - 1) * pmmp1 - (ll + m - 1) * pmm) / (ll - m)
                pmm, pmmp1 = pmmp1, pll
            plm = pmmp1
    lognorm = 0.5 * (math.log(2 * l + 1) - math.log(4 * math.pi)
                     + math.lgamma(l - m + 1) - math.lgamma(l + m + 1))
    return plm * math.exp(lognorm)
