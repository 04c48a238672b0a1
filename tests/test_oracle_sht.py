"""Known-answer tests that pin the oracle's torch-harmonics restatement
(oracle/sht_ref.py).  torch-harmonics is un-vendored and absent, so these
mathematical identities are what pins the SHT."""
import math

import numpy as np
import pytest
import torch

from oracle import sht_ref as S


@pytest.mark.parametrize("n", [5, 32, 33, 91, 721])
def test_clenshaw_curtis_exactness(n):
    x, w = S.clenshaw_curtiss_weights(n)
    assert np.all(np.diff(x) > 0)
    for k in range(0, n, 2):          # exact for polynomials of degree <= n-1
        ref = 2.0 / (k + 1)
        assert abs((w * x ** k).sum() - ref) < 1e-12 * max(1, n / 32), (k, n)
    assert np.allclose(w, w[::-1])


@pytest.mark.parametrize("n", [4, 24, 120])
def test_legendre_gauss_exactness(n):
    x, w = S.legendre_gauss_weights(n)
    for k in range(0, 2 * n, 2):      # exact up to degree 2n-1
        assert abs((w * x ** k).sum() - 2.0 / (k + 1)) < 1e-12


def test_legpoly_closed_form():
    theta, _ = S.colatitudes(64, "equiangular")
    P = S.precompute_legpoly(41, 60, theta)
    for (l, m) in [(0, 0), (1, 0), (1, 1), (7, 3), (20, 20), (33, 11), (59, 40)]:
        ref = S.ylm_closed_form(l, m, theta)
        assert np.abs(P[m, l] - ref).max() < 1e-12 * max(1.0, np.abs(ref).max())
    # structural zeros l < m are exact zeros
    for m in range(1, 41):
        assert np.all(P[m, :m] == 0.0)


@pytest.mark.parametrize("grid,nlat,nlon,lmax,mmax", [
    ("legendre-gauss", 32, 64, 32, 33),
    ("equiangular", 33, 64, 17, 17),
    ("equiangular", 91, 180, 45, 46),
    ("legendre-gauss", 120, 240, 120, 121),
])
def test_band_limited_round_trip(grid, nlat, nlon, lmax, mmax):
    g = torch.Generator().manual_seed(0)
    sht = S.RealSHT(nlat, nlon, lmax=lmax, mmax=mmax, grid=grid)
    isht = S.InverseRealSHT(nlat, nlon, lmax=lmax, mmax=mmax, grid=grid)
    a = torch.randn(2, lmax, mmax, 2, dtype=torch.float64, generator=g)
    a = torch.view_as_complex(a)
    l = torch.arange(lmax)[:, None]
    m = torch.arange(mmax)[None, :]
    a = torch.where(l >= m, a, torch.zeros_like(a))
    a[..., 0] = a[..., 0].real.to(a.dtype)       # m = 0 real (real field)
    if 2 * (mmax - 1) >= nlon:
        a[..., nlon // 2:] = 0
    x = isht(a)
    back = sht(x)
    assert (back - a).abs().max().item() < 1e-11


def test_full_resolution_equiangular_round_trip_721():
    """721x1440 equiangular, lmax=360: the config-2 transform round-trips exactly
    (Clenshaw–Curtis on 721 points integrates degree <= 720)."""
    sht = S.RealSHT(721, 1440, lmax=360, mmax=361, grid="equiangular")
    isht = S.InverseRealSHT(721, 1440, lmax=360, mmax=361, grid="equiangular")
    g = torch.Generator().manual_seed(1)
    a = torch.view_as_complex(torch.randn(1, 360, 361, 2, dtype=torch.float64, generator=g))
    l = torch.arange(360)[:, None]
    m = torch.arange(361)[None, :]
    a = torch.where(l >= m, a, torch.zeros_like(a))
    a[..., 0] = a[..., 0].real.to(a.dtype)
    back = sht(isht(a))
    assert (back - a).abs().max().item() < 1e-9


def test_single_ylm_synthesis():
    nlat, nlon, lmax, mmax = 33, 64, 32, 33
    isht = S.InverseRealSHT(nlat, nlon, lmax=lmax, mmax=mmax, grid="equiangular")
    theta, _ = S.colatitudes(nlat, "equiangular")
    phi = 2 * np.pi * np.arange(nlon) / nlon
    for (l, m) in [(0, 0), (3, 2), (17, 9), (31, 31)]:
        a = torch.zeros(lmax, mmax, dtype=torch.complex128)
        a[l, m] = 1.0 + 0.5j
        x = isht(a).numpy()
        c = 1.0 if m == 0 else 2.0      # Hermitian half-spectrum synthesis
        ref = c * S.ylm_closed_form(l, m, theta)[:, None] * (
            np.cos(m * phi)[None, :] * (1.0 if True else 0) - (0.5 if m else 0) * np.sin(m * phi)[None, :])
        assert np.abs(x - ref).max() < 1e-12


def test_orthonormality_quadrature():
    theta, w = S.colatitudes(64, "legendre-gauss")
    P = S.precompute_legpoly(20, 40, theta)
    for m in (0, 5, 19):
        G = 2 * np.pi * np.einsum("lk,jk,k->lj", P[m], P[m], w)
        G = G[m:, m:]
        assert np.abs(G - np.eye(G.shape[0])).max() < 1e-12


def test_rescale_is_identity_roundtrip():
    """The reference's ×1e5/÷1e5 rescale (sfnonet.py:551-555) cancels in SHT∘ISHT."""
    sht = S.RealSHT(32, 64, lmax=32, mmax=33, grid="equiangular")
    isht = S.InverseRealSHT(32, 64, lmax=32, mmax=33, grid="equiangular")
    x = torch.randn(3, 32, 64, dtype=torch.float64)
    y0 = isht(sht(x))
    sht.weights = sht.weights * 1e5
    isht.pct = isht.pct / 1e5
    y1 = isht(sht(x))
    assert (y0 - y1).abs().max() < 1e-10
