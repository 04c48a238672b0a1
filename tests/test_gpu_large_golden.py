"""The HIP block against the REFERENCE's own output at the sizes that matter
(make_golden.py --large): 121x240 Legendre-Gauss C=64 lmax 60 (both
filters, filmed), the default network's inner block (120x240 LG, C=256, lmax 120,
non-linear) and config 2 (721x1440, C=256, lmax 360, non-linear, filmed).  Inputs and
weights are rebuilt from the committed recipe; the fixture holds output rows x
channels and per-(batch, channel) mean / std / max-abs.
Bar (north_star): max-abs < 1e-4 on the stored rows and on the moments."""
import os

import pytest
import torch

from block_util import make_block
from golden_util import load_large
from test_oracle_large import LARGE, check_against

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("path", LARGE, ids=lambda p: os.path.basename(p)[:-4])
def test_block_matches_reference_large(path):
    meta, params, x, gamma, beta, exp = load_large(path)
    blk, _, _ = make_block(meta, None)
    missing, unexpected = blk.load_state_dict(params, strict=False)
    assert not unexpected, unexpected
    assert all(k.endswith((".weights", ".pct", "activation.bias")) for k in missing), missing
    blk = blk.to(DEV)
    with torch.no_grad():
        if meta["filmed"]:
            y = blk(x.to(DEV), gamma.to(DEV), beta.to(DEV), meta["scale"])
        else:
            y = blk(x.to(DEV))
    torch.cuda.synchronize()
    err, em = check_against(y.cpu(), exp, 1e-4, 1e-4)
    print(f"{os.path.basename(path)}: HIP vs reference rows max-abs {err:.2e}, moments {em:.2e}")
