"""Oracle (oracle/sfno_ref.py) vs golden vectors produced by the reference code.

Pins the CPU restatement of the block (filters, norms, FiLM, MLP, wiring) to the
reference's own implementation (tests/golden/make_golden.py)."""
import os

import pytest
import torch

from golden_util import golden_files, load, wiring_cfg
from oracle import sfno_ref
from oracle.sht_ref import InverseRealSHT, RealSHT


def _transforms(meta):
    sht = RealSHT(meta["nlat"], meta["nlon"], lmax=meta["lmax"], mmax=meta["mmax"],
                  grid=meta["grid"]).float()
    if "out_nlat" in meta:
        isht = InverseRealSHT(meta["out_nlat"], meta["out_nlon"], lmax=meta["lmax"],
                              mmax=meta["mmax"], grid=meta["out_grid"]).float()
    else:
        isht = InverseRealSHT(meta["nlat"], meta["nlon"], lmax=meta["lmax"], mmax=meta["mmax"],
                              grid=meta["grid"]).float()
    sht.weights = sht.weights * 1e5
    isht.pct = isht.pct / 1e5
    return sht, isht


@pytest.mark.parametrize("path", golden_files(), ids=lambda p: os.path.basename(p)[:-4])
def test_oracle_block_matches_reference(path):
    meta, p, a, keys = load(path)
    sht, isht = _transforms(meta)
    inner, outer, has_mlp = wiring_cfg(meta)
    cfg = sfno_ref.BlockCfg(filter_type=meta["filter"], inner_skip=inner, outer_skip=outer,
                            has_mlp=has_mlp)
    g = a["gamma"] if meta["filmed"] else None
    b = a["beta"] if meta["filmed"] else None
    with torch.no_grad():
        y = sfno_ref.block_forward(p, a["x"], sht, isht, cfg, g, b, meta["scale"])
        s = sht(a["x"])
    # same op sequence in fp32 on the same CPU: agreement to rounding
    assert torch.allclose(s, a["sht_x"], rtol=1e-5, atol=1e-3 * float(a["sht_x"].abs().max()) * 1e-3)
    err = (y - a["y"]).abs().max().item()
    assert err < 1e-5, err
    # state-dict names the oracle consumes exist in the reference module
    for k in p:
        assert k in keys


@pytest.mark.parametrize("ft", ["nl", "lin"])
def test_oracle_global_conv_matches_reference(ft):
    """FourierNeuralOperatorBlock_Filmed.global_conv(x, residual) (sfnonet.py:341-356),
    residual != x and residual == x, against the reference (make_golden.py --gconv)."""
    meta, p, a, keys = load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                         "gconv", f"gconv_{ft}.npz"))
    sht, isht = _transforms(meta)
    cfg = sfno_ref.BlockCfg(filter_type=meta["filter"])
    with torch.no_grad():
        y = sfno_ref.global_conv(p, a["x"], a["residual"], sht, isht, cfg)
        y_self = sfno_ref.global_conv(p, a["x"], a["x"], sht, isht, cfg)
    assert (y - a["y"]).abs().max().item() < 1e-5
    assert (y_self - a["y_self"]).abs().max().item() < 1e-5
