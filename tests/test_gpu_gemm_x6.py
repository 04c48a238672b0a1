"""Accuracy of the dense 1x1-conv GEMMs (skip, MLP fc1/fc2) on the bf16 matrix
cores with the exact three-term operand split ("x6", csrc/gemm_x6.hip).

The reference computes these as fp32 convolutions (layers.py:145-178 MLP,
sfnonet.py:304-306 inner skip).  The x6 GEMM must be as accurate as an fp32
GEMM: checked against an fp64 evaluation of the same MLP, next to the fp32 MFMA
kernel (MSFNO_GEMM=f32, run in a child process since the switch is read once
per process).  The error measure is |y - y64| / (|W2|·|GELU(W1 x + b1)| + |b2|),
i.e. relative to the magnitude of the summed products, the scale fp32 rounding
works on.
"""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
HERE = os.path.dirname(os.path.abspath(__file__))


def _gelu64(x):
    return 0.5 * x * (1.0 + torch.erf(x / 2 ** 0.5))


def _case(Cin, Hid, Cout, P, B, seed):
    from msfno_amd.sfno import MLP
    torch.manual_seed(seed)
    m = MLP(in_features=Cin, hidden_features=Hid, out_features=Cout, output_bias=True).eval()
    # O(1) weights so every product term matters (the reference init is 0.02-scaled)
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(torch.randn_like(p) / p.shape[1] ** 0.5 if p.dim() > 1 else 0.1 * torch.randn_like(p))
    x = torch.randn(B, Cin, 1, P)
    sd = {k: v.double() for k, v in m.fwd.state_dict().items()}
    W1, b1 = sd["0.weight"][:, :, 0, 0], sd["0.bias"]
    W2, b2 = sd["2.weight"][:, :, 0, 0], sd["2.bias"]
    xd = x.double()[:, :, 0, :]
    h = _gelu64(torch.einsum("oi,bip->bop", W1, xd) + b1[None, :, None])
    y64 = torch.einsum("oi,bip->bop", W2, h) + b2[None, :, None]
    scale = torch.einsum("oi,bip->bop", W2.abs(), h.abs()) + b2.abs()[None, :, None]
    with torch.no_grad():
        got = m.to(DEV)(x.to(DEV)).double().cpu()[:, :, 0, :]
    return ((got - y64).abs() / scale).max().item(), (got - y64).abs().max().item()


CASES = [
    (256, 512, 256, 8192, 1),   # block MLP shape (config 2), a slab of pixels
    (73, 256, 73, 3001, 2),     # ragged: encoder-like K/M, N not a tile multiple
    (329, 256, 73, 1000, 1),    # decoder-like K = 256 + 73
]


def _errors():
    return [_case(*c, seed=i) for i, c in enumerate(CASES)]


def test_x6_matches_fp64_like_fp32():
    x6 = _errors()
    env = dict(os.environ, MSFNO_GEMM="f32")
    out = subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, cwd=HERE,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    f32 = json.loads(out.stdout.strip().splitlines()[-1])
    for c, (rx, ax), (rf, af) in zip(CASES, x6, f32):
        print(f"{c}: x6 rel {rx:.2e} abs {ax:.2e} | f32 MFMA rel {rf:.2e} abs {af:.2e}")
        # fp32-level accuracy: within 2x of the fp32 MFMA kernel and under 4 ulp-scale
        assert rx < max(2.0 * rf, 1e-7), (c, rx, rf)
        assert rx < 5e-7, (c, rx)


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(HERE))
    import conftest  # noqa: F401  (puts the package on sys.path)
    print(json.dumps(_errors()))
