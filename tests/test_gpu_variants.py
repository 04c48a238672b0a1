"""The run-time A/B alternatives of the native block stay correct.

Every switch is read once per process, so each variant runs the reference-produced
golden blocks (tests/golden/make_golden.py) in a child process with its
environment and reports the max-abs error; the bar is the same as the default
path's (max-abs < 1e-4).  The cases cover the non-linear filter with FiLM on a
180-longitude grid, a batch of two fields, and the linear filter on a 121x240
Legendre-Gauss grid (whose 29,040 pixels end in a ragged 112-pixel MLP chunk)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
CASES = ["mid_nl_film_middle.npz", "c1b2_nl_film_middle.npz", "lg_lin_film_middle.npz",
         "lg_nl_plain_middle.npz"]

VARIANTS = [
    {"MSFNO_SKIP_PLANES": "0"},
    {"MSFNO_X1_PLANES": "0", "MSFNO_H_PLANES": "0"},
    {"MSFNO_X6P_STAGES": "3"},
    {"MSFNO_X6P_WAVES": "4"},
    {"MSFNO_X6P_WAVES": "4x128"},
    {"MSFNO_X6P_MFMA": "16"},
    {"MSFNO_MLP_CHUNK": "256"},
    {"MSFNO_R2C_CFG": "8x3", "MSFNO_C2R_WV": "4", "MSFNO_C2R_AREG": "0"},
    {"MSFNO_C2R_AREG": "0"},
    {"MSFNO_R2C_CFG": "16x1"},
    {"MSFNO_SPEC_3M": "0"},
    {"MSFNO_SIDE_STREAM": "0"},
    {"MSFNO_GEMM": "f32"},
    {"MSFNO_CONTRACT_DMA": "0"},
    {"MSFNO_CONTRACT_NS": "3"},
    {"MSFNO_CX16": "0"},
    {"MSFNO_SPEC_L0F32": "0"},
    {"MSFNO_X6C_TILED": "0"},
    {"MSFNO_MF_XS": "1"},
    {"MSFNO_X6C_WAVES": "24", "MSFNO_X6C_TILED": "0"},
    {"MSFNO_X6C_WAVES": "4", "MSFNO_X6C_TILED": "0"},
    {"MSFNO_TR_FWD": "2p", "MSFNO_TR_INV": "2p"},
    {"MSFNO_TR_INV": "16x128"},
    {"MSFNO_SIDE_CUSTRIDE": "3"},
    {"MSFNO_LEG_X3R": "0"},
    {"MSFNO_LEG_X3F": "0"},
    {"MSFNO_X3F_NS": "2"},
    {"MSFNO_SKIP_H": "0"},
    {"MSFNO_X3C_BM64": "0"},
    # round 6
    {"MSFNO_MH_ILV": "0"},
    {"MSFNO_MH_BUF": "1"},
    {"MSFNO_X3C_L0_BM64": "0"},
    {"MSFNO_SKIP_GRID": "2"},
    {"MSFNO_TR_XCD": "00"},
    {"MSFNO_TR_XCD": "11"},
    {"MSFNO_TR_FWD_PRE": "0", "MSFNO_TR_INV_BF": "0"},
    # older switches no test exercised before
    {"MSFNO_FFT_DMA": "0"},
    {"MSFNO_FFT_TILE": "1", "MSFNO_NO_SYM": "1"},
    {"MSFNO_SIDE_PRIO": "normal"},
    {"MSFNO_SPEC_4M": "1"},
    {"MSFNO_SPEC_X6": "0", "MSFNO_C3M_TILE": "0"},
    {"MSFNO_WCACHE": "0"},
    {"MSFNO_ENGINE": "x6", "MSFNO_MF_SCHED": "0"},
    {"MSFNO_ENGINE": "x6", "MSFNO_MF_AHEAD": "3"},
    {"MSFNO_ENGINE": "x6", "MSFNO_X6_TILE": "4"},
    {"MSFNO_C2R_SWZ": "1"},
]


def _errors():
    import torch

    from block_util import make_block
    from golden_util import load
    out = {}
    for name in CASES:
        meta, params, arrays, _ = load(os.path.join(HERE, "golden", name))
        blk, _, _ = make_block(meta, params)
        blk = blk.to("cuda:0")
        x = arrays["x"].to("cuda:0")
        with torch.no_grad():
            if meta["filmed"]:
                y = blk(x, arrays["gamma"].to("cuda:0"), arrays["beta"].to("cuda:0"), meta["scale"])
            else:
                y = blk(x)
        out[name] = (y.cpu() - arrays["y"]).abs().max().item()
    return out


@pytest.mark.parametrize("env", VARIANTS, ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
def test_variant_matches_reference_golden(env):
    r = subprocess.run([sys.executable, os.path.abspath(__file__)], env=dict(os.environ, **env),
                       cwd=HERE, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    errs = json.loads(r.stdout.strip().splitlines()[-1])
    bad = {k: v for k, v in errs.items() if not v < 1e-4}
    assert not bad, bad


if __name__ == "__main__":
    repo = os.path.dirname(HERE)
    for d in (HERE, repo, os.path.join(repo, "modulated-spherical-fourier-neural-operator_amd")):
        sys.path.insert(0, d)
    print(json.dumps(_errors()))
