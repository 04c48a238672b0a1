"""GPU parity: the HIP path (through the C-ABI, via msfno_amd) against the oracle
and the reference-produced golden vectors.  Tolerances are stated per test;
the north-star bar is max-abs error < 1e-4 on the block output."""
import os

import pytest
import torch

from block_util import make_block, make_transforms
from golden_util import golden_files, load
from oracle import sfno_ref
from oracle import sht_ref as S

pytestmark = pytest.mark.gpu
DEV = "cuda"

SHT_CASES = [
    ("equiangular", 32, 64, 32, 33),
    ("equiangular", 33, 64, 16, 17),
    ("legendre-gauss", 24, 48, 24, 25),
    ("equiangular", 91, 180, 45, 46),
    ("legendre-gauss", 20, 45, 20, 21),     # odd nlon (full complex FFT path)
    ("legendre-gauss", 120, 240, 120, 121),
    ("equiangular", 13, 26, 7, 9),           # mmax > lmax + 1 (zero m blocks)
]


def _rel(a, b):
    return (a - b).abs().max().item() / max(b.abs().max().item(), 1e-30)


@pytest.mark.parametrize("grid,nlat,nlon,lmax,mmax", SHT_CASES)
def test_sht_forward_matches_oracle(grid, nlat, nlon, lmax, mmax):
    from msfno_amd.harmonics import RealSHT
    g = torch.Generator().manual_seed(nlat * nlon)
    x = torch.randn(3, 5, nlat, nlon, generator=g)
    ref = S.RealSHT(nlat, nlon, lmax=lmax, mmax=mmax, grid=grid)  # fp64 tables
    want = ref(x.double())
    mine = RealSHT(nlat, nlon, lmax=lmax, mmax=mmax, grid=grid).float().to(DEV)
    got = mine(x.to(DEV)).cpu()
    assert got.shape == want.shape and got.dtype == torch.complex64
    assert _rel(got.to(torch.complex128), want) < 2e-6          # fp32 vs fp64
    # structural zeros l < m are exact
    l = torch.arange(lmax)[:, None]
    m = torch.arange(mmax)[None, :]
    assert (got[..., l < m] == 0).all()


@pytest.mark.parametrize("grid,nlat,nlon,lmax,mmax", SHT_CASES)
def test_sht_inverse_matches_oracle(grid, nlat, nlon, lmax, mmax):
    from msfno_amd.harmonics import InverseRealSHT
    g = torch.Generator().manual_seed(7 + nlat)
    a = torch.view_as_complex(torch.randn(2, 3, lmax, mmax, 2, generator=g))
    ref = S.InverseRealSHT(nlat, nlon, lmax=lmax, mmax=mmax, grid=grid)
    want = ref(a.to(torch.complex128))
    mine = InverseRealSHT(nlat, nlon, lmax=lmax, mmax=mmax, grid=grid).float().to(DEV)
    got = mine(a.to(DEV)).cpu()
    assert got.shape == want.shape
    assert _rel(got.double(), want) < 2e-6


def test_sht_round_trip_full_resolution():
    """Config-2 transform pair (721x1440 equiangular, lmax=360) round-trips a
    band-limited field on the GPU (size-independent property)."""
    from msfno_amd.harmonics import InverseRealSHT, RealSHT
    f = RealSHT(721, 1440, lmax=360, mmax=361, grid="equiangular").float().to(DEV)
    gi = InverseRealSHT(721, 1440, lmax=360, mmax=361, grid="equiangular").float().to(DEV)
    g = torch.Generator().manual_seed(3)
    a = torch.view_as_complex(torch.randn(4, 360, 361, 2, generator=g))
    l = torch.arange(360)[:, None]
    m = torch.arange(361)[None, :]
    a = torch.where(l >= m, a, torch.zeros_like(a))
    a[..., 0] = a[..., 0].real.to(a.dtype)
    back = f(gi(a.to(DEV))).cpu()
    assert (back - a).abs().max().item() < 2e-4 * a.abs().max().item()


@pytest.mark.parametrize("grid,nlat,nlon,lmax,mmax", SHT_CASES[:5])
def test_sht_general_layout_matches_oracle(grid, nlat, nlon, lmax, mmax, monkeypatch):
    """MSFNO_NO_SYM=1 forces the general (non-folded) Legendre layout that
    non-symmetric tables use; it must agree with the oracle as well."""
    from msfno_amd.harmonics import InverseRealSHT, RealSHT
    monkeypatch.setenv("MSFNO_NO_SYM", "1")
    g = torch.Generator().manual_seed(11 + nlat)
    x = torch.randn(2, 3, nlat, nlon, generator=g)
    want = S.RealSHT(nlat, nlon, lmax=lmax, mmax=mmax, grid=grid)(x.double())
    got = RealSHT(nlat, nlon, lmax=lmax, mmax=mmax, grid=grid).float().to(DEV)(x.to(DEV)).cpu()
    assert _rel(got.to(torch.complex128), want) < 2e-6
    a = torch.view_as_complex(torch.randn(2, 3, lmax, mmax, 2, generator=g))
    want = S.InverseRealSHT(nlat, nlon, lmax=lmax, mmax=mmax, grid=grid)(a.to(torch.complex128))
    got = InverseRealSHT(nlat, nlon, lmax=lmax, mmax=mmax, grid=grid).float().to(DEV)(a.to(DEV)).cpu()
    assert _rel(got.double(), want) < 2e-6


def test_asymmetric_table_uses_general_layout():
    """A table without the equatorial symmetry (here: one latitude perturbed)
    must not be folded: the transform follows the table exactly."""
    from msfno_amd.harmonics import InverseRealSHT, RealSHT
    nlat, nlon, lmax, mmax = 33, 64, 16, 17
    f = RealSHT(nlat, nlon, lmax=lmax, mmax=mmax, grid="equiangular").float()
    f.weights = f.weights.clone()
    f.weights[:, :, 3] *= 1.5
    gi = InverseRealSHT(nlat, nlon, lmax=lmax, mmax=mmax, grid="equiangular").float()
    gi.pct = gi.pct.clone()
    gi.pct[:, :, 30] *= 0.5
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, nlat, nlon, generator=g, dtype=torch.float64)
    X = 2.0 * torch.pi * torch.fft.rfft(x, norm="forward")[..., :mmax]
    want = torch.einsum("...km,mlk->...lm", X, f.weights.double().to(torch.complex128))
    got = f.to(DEV)(x.float().to(DEV)).cpu()
    assert _rel(got.to(torch.complex128), want) < 2e-6
    a = torch.view_as_complex(torch.randn(2, lmax, mmax, 2, generator=g, dtype=torch.float64))
    Y = torch.einsum("...lm,mlk->...km", a, gi.pct.double().to(torch.complex128))
    want = torch.fft.irfft(Y, n=nlon, norm="forward")
    got = gi.to(DEV)(a.to(torch.complex64).to(DEV)).cpu()
    assert _rel(got.double(), want) < 2e-6


def test_compl_contract_matches_einsum():
    from msfno_amd.sfno import compl_contract_fwd_c
    for (B, Ci, Co, T) in [(1, 8, 8, 528), (2, 16, 12, 1035), (3, 4, 20, 7), (8, 8, 8, 100)]:
        g = torch.Generator().manual_seed(T)
        a = torch.randn(B, Ci, T, 2, generator=g)
        w = torch.randn(Co, Ci, T, 2, generator=g)
        want = sfno_ref.compl_contract_fwd_c(a.double(), w.double())
        got = compl_contract_fwd_c(a.to(DEV), w.to(DEV)).cpu()
        assert _rel(got.double(), want) < 1e-5


def test_compl_mul2d_matches_einsum():
    from msfno_amd.sfno import compl_mul2d_fwd_c
    g = torch.Generator().manual_seed(0)
    a = torch.randn(2, 8, 5, 6, 2, generator=g)
    w = torch.randn(8, 16, 2, generator=g)
    want = sfno_ref.compl_mul2d_fwd_c(a.double(), w.double())
    got = compl_mul2d_fwd_c(a.to(DEV), w.to(DEV)).cpu()
    assert _rel(got.double(), want) < 1e-5


@pytest.mark.parametrize("path", golden_files(), ids=lambda p: os.path.basename(p)[:-4])
def test_block_matches_reference_golden(path):
    """Reference-produced golden vectors (tests/golden/make_golden.py).
    Tolerance: max-abs < 1e-4 (north-star bar)."""
    meta, params, arrays, _ = load(path)
    blk, _, _ = make_block(meta, params)
    blk = blk.to(DEV)
    x = arrays["x"].to(DEV)
    with torch.no_grad():
        if meta["filmed"]:
            y = blk(x, arrays["gamma"].to(DEV), arrays["beta"].to(DEV), meta["scale"])
        else:
            y = blk(x)
    y = y.cpu()
    err = (y - arrays["y"]).abs().max().item()
    assert y.shape == arrays["y"].shape
    assert err < 1e-4, f"max-abs {err:.3e} (|y|max {arrays['y'].abs().max().item():.3f})"


@pytest.mark.parametrize("path", [p for p in golden_files() if "_film_" in p][:6],
                         ids=lambda p: os.path.basename(p)[:-4])
def test_filter_only_matches_oracle(path):
    """SpectralFilterLayer.forward alone (no norms) vs the oracle filter."""
    meta, params, arrays, _ = load(path)
    blk, sht, isht = make_block(meta, params)
    x = arrays["x"]
    o_sht, o_isht = sfno_ref.make_transforms(meta["nlat"], meta["nlon"], meta["lmax"], meta["mmax"],
                                             meta["grid"])
    if "out_nlat" in meta:
        o_isht = S.InverseRealSHT(meta["out_nlat"], meta["out_nlon"], lmax=meta["lmax"],
                                  mmax=meta["mmax"], grid=meta["out_grid"]).float()
        o_isht.pct = o_isht.pct / 1e5
    with torch.no_grad():
        if meta["filter"] == "non-linear":
            ws = [params[f"filter_layer.filter.w.{i}"] for i in range(3)]
            want = sfno_ref.spectral_attention_s2(x, o_sht, o_isht, ws,
                                                  params["filter_layer.filter.wout"])
        else:
            want = sfno_ref.spectral_conv_s2(x, o_sht, o_isht, params["filter_layer.filter.w"],
                                             params["filter_layer.filter.ii"],
                                             params["filter_layer.filter.jj"])
        got = blk.to(DEV).filter_layer(x.to(DEV)).cpu()
    assert (got - want).abs().max().item() < 1e-4 * max(1.0, want.abs().max().item())


def test_film_scale_zero_equals_unfilmed():
    """FiLM with scale=0 equals the plain block (the reference's 'sfno' baseline,
    model.py:1347-1353)."""
    path = [p for p in golden_files() if os.path.basename(p) == "c1_nl_film_middle.npz"][0]
    meta, params, arrays, _ = load(path)
    blk, _, _ = make_block(meta, params)
    blk = blk.to(DEV)
    x = arrays["x"].to(DEV)
    y0 = blk(x, arrays["gamma"].to(DEV), arrays["beta"].to(DEV), 0.0)
    meta2 = dict(meta, filmed=0)
    plain, _, _ = make_block(meta2, params)
    y1 = plain.to(DEV)(x)
    assert (y0 - y1).abs().max().item() < 1e-6


def test_batch_consistency():
    """Each batch entry is independent: block(x)[b] == block(x[b:b+1])."""
    path = [p for p in golden_files() if os.path.basename(p) == "c1b2_lin_film_middle.npz"][0]
    meta, params, arrays, _ = load(path)
    blk, _, _ = make_block(meta, params)
    blk = blk.to(DEV)
    x = torch.cat([arrays["x"], 0.5 * arrays["x"].flip(0), arrays["x"][:1]], 0).to(DEV)
    g = torch.randn(x.shape[0], meta["C"]).to(DEV) * 0.1
    b = torch.randn(x.shape[0], meta["C"]).to(DEV) * 0.1
    y = blk(x, g, b, 1.0)
    for i in range(x.shape[0]):
        yi = blk(x[i:i + 1], g[i:i + 1], b[i:i + 1], 1.0)
        assert (y[i:i + 1] - yi).abs().max().item() < 1e-5


def test_rescale_invariance_nonlinear_filter():
    """The ×1e5/÷1e5 table rescale (sfnonet.py:551-555) is invariant for the
    positively homogeneous non-linear filter."""
    path = [p for p in golden_files() if os.path.basename(p) == "mid_nl_film_middle.npz"][0]
    meta, params, arrays, _ = load(path)
    blk, sht, isht = make_block(meta, params)
    blk = blk.to(DEV)
    x = arrays["x"].to(DEV)
    y1 = blk.filter_layer(x)
    sht.weights = sht.weights / 1e5
    isht.pct = isht.pct * 1e5
    y2 = blk.filter_layer(x)
    assert (y1 - y2).abs().max().item() < 1e-5 * max(1.0, y1.abs().max().item())


def test_block_over_torch_harmonics_style_transforms():
    """The block built around torch-harmonics-style transform objects (the oracle's
    restatement of torch_harmonics.RealSHT / InverseRealSHT, rescaled x1e5 / /1e5 as
    sfnonet.py:551-555 does) equals the block built around msfno_amd.harmonics ones."""
    from functools import partial

    from msfno_amd.harmonics import InverseRealSHT, RealSHT
    from msfno_amd.sfno import FourierNeuralOperatorBlock_Filmed
    from oracle import sht_ref as S
    C, nlat, nlon, lmax = 32, 33, 64, 32

    def build(Fwd, Inv):
        sht = Fwd(nlat, nlon, lmax=lmax, mmax=lmax + 1, grid="equiangular").float()
        isht = Inv(nlat, nlon, lmax=lmax, mmax=lmax + 1, grid="equiangular").float()
        sht.weights = sht.weights * 1e5
        isht.pct = isht.pct / 1e5
        norm = partial(torch.nn.InstanceNorm2d, num_features=C, eps=1e-6, affine=True,
                       track_running_stats=False)
        torch.manual_seed(3)
        return FourierNeuralOperatorBlock_Filmed(sht, isht, C, filter_type="non-linear",
                                                 mlp_ratio=2.0, norm_layer=(norm, norm),
                                                 inner_skip="linear", outer_skip="identity",
                                                 mlp_mode="distributed",
                                                 spectral_layers=3).eval().to(DEV)

    a = build(RealSHT, InverseRealSHT)
    b = build(S.RealSHT, S.InverseRealSHT)
    b.load_state_dict(a.state_dict(), strict=False)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(2, C, nlat, nlon, generator=g).to(DEV)
    gm, bt = (0.2 * torch.randn(2, C, generator=g)).to(DEV), (0.2 * torch.randn(2, C, generator=g)).to(DEV)
    with torch.no_grad():
        ya, yb = a(x, gm, bt, 0.7), b(x, gm, bt, 0.7)
    assert (ya - yb).abs().max().item() < 1e-5 * max(1.0, ya.abs().max().item())


@pytest.mark.parametrize("ft", ["nl", "lin"])
def test_global_conv_matches_reference_golden(ft):
    """FourierNeuralOperatorBlock_Filmed.global_conv(x, residual) (sfnonet.py:341-356) on
    the native block (msfno_block_global_conv), residual != x (its x3h scales from its
    own max) and residual == x, against the reference's own output."""
    from golden_util import GOLDEN
    meta, params, arrays, _ = load(os.path.join(GOLDEN, "gconv", f"gconv_{ft}.npz"))
    meta = dict(meta, filmed=1, wiring="middle")
    blk, _, _ = make_block(meta, params)
    blk = blk.to(DEV)
    x, r = arrays["x"].to(DEV), arrays["residual"].to(DEV)
    with torch.no_grad():
        y = blk.global_conv(x, r).cpu()
        y_self = blk.global_conv(x, x).cpu()
    for got, want in ((y, arrays["y"]), (y_self, arrays["y_self"])):
        err = (got - want).abs().max().item()
        assert got.shape == want.shape
        assert err < 1e-4, f"max-abs {err:.3e}"


@pytest.mark.parametrize("env", ["MSFNO_SKIP_X3H=0", "MSFNO_ENGINE=x6", "MSFNO_SKIP_PLANES=1"])
@pytest.mark.parametrize("ft", ["nl", "lin"])
def test_global_conv_skip_engines(ft, env):
    """global_conv's inner skip multiplies the residual on every skip engine (the x3h
    default, the x6 fp32 split, the x6 planes path and the dense fallback), not the filter
    input x.  The engines are chosen once per process from the environment, so each
    runs in a child process (this file as a script)."""
    import subprocess
    import sys
    from conftest import PKG_DIR, REPO
    k, v = env.split("=")
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "gconv", ft],
                       env=dict(os.environ, PYTHONPATH=os.pathsep.join([REPO, PKG_DIR]), **{k: v}),
                       cwd=os.path.dirname(__file__),
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    print(r.stdout.strip())


if __name__ == "__main__":
    import sys
    if sys.argv[1] == "gconv":
        test_global_conv_matches_reference_golden(sys.argv[2])
        print(f"global_conv {sys.argv[2]} ok under "
              f"{[k + '=' + v for k, v in os.environ.items() if k.startswith('MSFNO_')]}")
