"""Size-independent properties of the native path that do
not go through the oracle: a one-hot spectrum synthesised and analysed again at
the full 721 x 1440 equiangular resolution (lmax 360) comes back one-hot, and the
linear spectral filter (SpectralConvS2, layers.py:336-427, softshrink(0) = id) is
affine in its input.  Tolerances are stated per test."""
import os

import pytest
import torch

from block_util import make_block, make_transforms
from golden_util import golden_files, load

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("l,m", [(0, 0), (1, 0), (1, 1), (5, 3), (200, 150), (359, 0), (359, 359)])
def test_one_hot_spectrum_round_trip_full_resolution(l, m):
    """ISHT(e_lm) then SHT: the coefficient comes back to 2e-5 and every other one
    stays below 2e-5 (fp32 transforms over 721 latitudes, ortho normalisation)."""
    meta = {"nlat": 721, "nlon": 1440, "lmax": 360, "mmax": 361, "grid": "equiangular"}
    sht, isht = make_transforms(meta, rescale=False)
    sht, isht = sht.to(DEV), isht.to(DEV)
    a = torch.zeros(1, 1, 360, 361, dtype=torch.complex64, device=DEV)
    a[0, 0, l, m] = complex(1.0, 0.5 if m > 0 else 0.0)  # Im of m = 0 is not representable
    with torch.no_grad():
        x = isht(a)
        b = sht(x)
    err = (b - a).abs().max().item()
    assert err < 2e-5, err


@pytest.mark.parametrize("l,m", [(0, 0), (1, 1), (60, 30), (119, 0), (119, 119)])
def test_one_hot_spectrum_round_trip_gauss_120x240(l, m):
    """The config-3 latent grid (120 x 240 Legendre-Gauss, lmax 120, sfnonet.py:573-614):
    a Gauss grid of 120 nodes integrates degree <= 239 exactly, so ISHT then SHT of a
    one-hot spectrum is the identity to fp32 rounding (2e-5)."""
    meta = {"nlat": 120, "nlon": 240, "lmax": 120, "mmax": 120, "grid": "legendre-gauss"}
    sht, isht = make_transforms(meta, rescale=False)
    sht, isht = sht.to(DEV), isht.to(DEV)
    a = torch.zeros(1, 1, 120, 120, dtype=torch.complex64, device=DEV)
    a[0, 0, l, m] = complex(1.0, -0.25 if m > 0 else 0.0)
    with torch.no_grad():
        b = sht(isht(a))
    assert (b - a).abs().max().item() < 2e-5


@pytest.mark.parametrize("meta", [
    {"nlat": 721, "nlon": 1440, "lmax": 360, "mmax": 361, "grid": "equiangular"},
    {"nlat": 120, "nlon": 240, "lmax": 120, "mmax": 120, "grid": "legendre-gauss"},
], ids=["eq721", "lg120"])
def test_random_band_limited_spectra_round_trip(meta):
    """SHT(ISHT(a)) == a for a random triangular spectrum (l >= m, Im a_l0 = 0), 4 channels
    at once: max-abs < 1e-4 x max|a| (fp32 transforms; the batch exercises the channel
    stride of both Legendre GEMMs)."""
    sht, isht = make_transforms(meta, rescale=False)
    sht, isht = sht.to(DEV), isht.to(DEV)
    L, M = meta["lmax"], meta["mmax"]
    g = torch.Generator().manual_seed(11)
    a = torch.complex(torch.randn(1, 4, L, M, generator=g), torch.randn(1, 4, L, M, generator=g))
    a = torch.tril(a)  # [l, m]: keep m <= l
    a[..., 0] = a[..., 0].real.to(a.dtype)
    a = a.to(DEV)
    with torch.no_grad():
        b = sht(isht(a))
    assert (b - a).abs().max().item() < 1e-4 * a.abs().max().item()


@pytest.mark.parametrize("path", [p for p in golden_files() if "_lin_" in p and "middle" in p][:3],
                         ids=lambda p: os.path.basename(p)[:-4])
def test_linear_filter_is_affine(path):
    """f(a x + (1 - a) y) == a f(x) + (1 - a) f(y) for the linear spectral filter;
    max-abs < 1e-5 x max|f|."""
    meta, params, arrays, _ = load(path)
    blk, _, _ = make_block(meta, params)
    f = blk.to(DEV).filter_layer
    g = torch.Generator().manual_seed(3)
    x = torch.randn(arrays["x"].shape, generator=g).to(DEV)
    y = torch.randn(arrays["x"].shape, generator=g).to(DEV)
    a = 0.3
    with torch.no_grad():
        lhs = f(a * x + (1 - a) * y)
        rhs = a * f(x) + (1 - a) * f(y)
    scale = max(lhs.abs().max().item(), 1e-6)
    assert (lhs - rhs).abs().max().item() < 1e-5 * scale
