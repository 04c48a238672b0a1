"""Oracle (oracle/sfno_ref.py) vs reference-produced fixtures at the sizes that matter
(SURVEY §8(c)): 121x240 Legendre-Gauss C=64 lmax 60 (both filters), the default
network's inner block (120x240 LG, C=256, lmax 120, non-linear) and config 2
(721x1440, C=256, lmax 360, non-linear, filmed).  Inputs and weights come from the
committed recipe (golden_util.load_large); the fixtures hold output rows x channels
and per-channel moments of the reference's own block (make_golden.py --large).
Same op sequence in fp32 on a CPU: agreement to 1e-5 max-abs on the stored rows."""
import glob
import os

import pytest
import torch

from golden_util import GOLDEN, load_large, moments, wiring_cfg
from oracle import sfno_ref

LARGE = sorted(glob.glob(os.path.join(GOLDEN, "large", "*.npz")))


def oracle_output(meta, params, x, gamma, beta):
    sht, isht = sfno_ref.make_transforms(meta["nlat"], meta["nlon"], meta["lmax"], meta["mmax"],
                                         meta["grid"])
    inner, outer, has_mlp = wiring_cfg(meta)
    cfg = sfno_ref.BlockCfg(filter_type=meta["filter"], inner_skip=inner, outer_skip=outer,
                            has_mlp=has_mlp)
    film = (gamma, beta) if meta["filmed"] else (None, None)
    with torch.no_grad():
        return sfno_ref.block_forward(params, x, sht, isht, cfg, *film, meta["scale"])


def check_against(y, exp, tol_rows, tol_mom):
    r, c = exp["rows"], exp["chans"]
    got = y[0][c][:, r]
    err = (got - exp["rows_y"]).abs().max().item()
    mean, std, mx = moments(y)
    em = max((mean - exp["mom_mean"]).abs().max().item(), (std - exp["mom_std"]).abs().max().item(),
             (mx - exp["mom_maxabs"]).abs().max().item())
    assert err < tol_rows, f"rows max-abs {err:.3e}"
    assert em < tol_mom, f"moments max-abs {em:.3e}"
    return err, em


def test_large_fixtures_present():
    assert len(LARGE) == 4, LARGE


@pytest.mark.parametrize("path", LARGE, ids=lambda p: os.path.basename(p)[:-4])
def test_oracle_matches_reference_large(path):
    meta, params, x, gamma, beta, exp = load_large(path)
    y = oracle_output(meta, params, x, gamma, beta)
    err, em = check_against(y, exp, 1e-5, 1e-5)
    print(f"{os.path.basename(path)}: rows max-abs {err:.2e}, moments {em:.2e}")
