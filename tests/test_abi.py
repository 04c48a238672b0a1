"""CPU-side checks of the C-ABI library: it loads, exports every symbol that
include/msfno.h declares, and its host-side plan math (fp64 quadrature and
Legendre tables) matches the oracle's torch-harmonics restatement."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "msfno.h")


def _declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(msfno_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_entry_points():
    syms = _declared_symbols()
    for s in ("msfno_sht_forward", "msfno_sht_inverse", "msfno_block_forward",
              "msfno_compl_contract_fwd_c", "msfno_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from msfno_amd import _native as N
    lib = N.lib()
    for s in _declared_symbols():
        assert hasattr(lib, s), s
    # and the ctypes binding covers all of them
    assert {n for n, _, _ in N.SIGNATURES} == set(_declared_symbols())
    assert lib.msfno_abi_version() == 6


def test_block_param_grads_struct_layout():
    from msfno_amd import _native as N
    # 2 norm0, 8 spec_w, wout, lin_w, 2 skip, 2 norm1, 4 MLP pointers
    assert ctypes.sizeof(N.BlockParamGrads) == (2 + 8 + 2 + 2 + 2 + 4) * 8
    assert N.BlockParamGrads.fc2_b.offset == (2 + 8 + 2 + 2 + 2 + 3) * 8


def test_block_desc_struct_layout():
    from msfno_amd import _native as N
    # 8 ints + float, 4 norm ptrs, 8 spec_w, wout, lin_w, 6 more pointers, the weight
    # cache pointer and its valid flag (padded to 8)
    assert ctypes.sizeof(N.BlockDesc) == 9 * 4 + 4 + (4 + 8 + 2 + 6 + 1) * 8 + 8
    assert N.BlockDesc.wcache.offset == 9 * 4 + 4 + (4 + 8 + 2 + 6) * 8


@pytest.mark.parametrize("grid", ["equiangular", "legendre-gauss"])
@pytest.mark.parametrize("n", [2, 5, 32, 91, 721])
def test_native_quadrature_matches_oracle(grid, n):
    from msfno_amd.harmonics import quadrature as q
    from oracle import sht_ref as S
    if grid == "equiangular":
        x, w = q.clenshaw_curtiss_weights(n)
        x2, w2 = S.clenshaw_curtiss_weights(n)
    else:
        x, w = q.legendre_gauss_weights(n)
        x2, w2 = S.legendre_gauss_weights(n)
    assert np.abs(x - x2).max() < 1e-14
    assert np.abs(w - w2).max() < 1e-13


@pytest.mark.parametrize("grid,nlat,lmax,mmax", [("equiangular", 33, 32, 33),
                                                  ("legendre-gauss", 24, 24, 25),
                                                  ("equiangular", 91, 45, 46),
                                                  ("legendre-gauss", 120, 120, 121)])
def test_native_legendre_tables_match_oracle(grid, nlat, lmax, mmax):
    from msfno_amd.harmonics import InverseRealSHT, RealSHT
    from oracle import sht_ref as S
    f = RealSHT(nlat, 2 * (mmax - 1), lmax=lmax, mmax=mmax, grid=grid)
    g = InverseRealSHT(nlat, 2 * (mmax - 1), lmax=lmax, mmax=mmax, grid=grid)
    f2 = S.RealSHT(nlat, 2 * (mmax - 1), lmax=lmax, mmax=mmax, grid=grid)
    g2 = S.InverseRealSHT(nlat, 2 * (mmax - 1), lmax=lmax, mmax=mmax, grid=grid)
    assert f.weights.shape == f2.weights.shape == (mmax, lmax, nlat)
    scale = f2.weights.abs().max().item()
    assert (f.weights - f2.weights).abs().max().item() < 1e-12 * scale
    assert (g.pct - g2.pct).abs().max().item() < 1e-12 * g2.pct.abs().max().item()


def test_unsupported_grid_raises_not_implemented():
    from msfno_amd.harmonics import RealSHT
    with pytest.raises(NotImplementedError):
        RealSHT(10, 20, grid="lobatto")


def test_cpu_tensor_is_rejected_loudly():
    import torch
    from msfno_amd.harmonics import RealSHT
    s = RealSHT(8, 16, lmax=8, mmax=9)
    with pytest.raises(ValueError):
        s(torch.zeros(1, 8, 16))


@pytest.mark.parametrize("cin,cin2,hid,cout,fused", [
    (73, 0, 256, 256, True),     # the encoder (sfnonet.py:513-523)
    (256, 73, 256, 73, True),    # the decoder over cat(x, residual) (:617-629)
    (5, 0, 16, 16, False),       # fixture-sized nets: the x6 GEMM pair
    (256, 73, 512, 73, False),   # hidden wider than the fused kernel's LDS vectors
    (256, 0, 256, 256, False),   # widths without an instantiated kernel
])
def test_mlp_fused_widths_and_workspace(cin, cin2, hid, cout, fused):
    """Host-side dispatch of the standalone MLP (no GPU call): which widths take the
    one-launch x3h kernel, and that its workspace is the weight image only (no hidden
    activation through HBM), far below the two-GEMM path's."""
    from msfno_amd import _native as N
    lib = N.lib()
    d = N.MlpDesc()
    d.Cin, d.Cin2, d.Hid, d.Cout = cin, cin2, hid, cout
    assert bool(lib.msfno_mlp_fused_supported(ctypes.byref(d))) == fused
    P = 721 * 1440
    ws = lib.msfno_mlp_workspace_size(ctypes.byref(d), 1, P)
    if fused:
        assert ws < 4 << 20        # the image and scale vectors
    else:
        assert ws >= hid * P * 4   # the hidden activation
