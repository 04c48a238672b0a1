"""x3h range guard of the fused block MLP (mlp_fused_h.hip): the fc1 input
a ⊙ x1 + t and the GELU outputs are scaled by powers of two from their bounds
(chan_affine's abound, the weights' row L1 norms), so large norm1 / FiLM gains or
fc1 weights can neither overflow fp16 (65504) nor lose precision to subnormals.

Reference arithmetic: sfnonet.py:376-382 (norm1, FiLM, MLP, outer skip) and
layers.py:161-168 (fc1 -> GELU -> fc2), evaluated in fp32 by the oracle.  Bar: the
north-star 1e-4 relative to max(1, |y|), with every output finite.
"""
import pytest
import torch

from oracle import sfno_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (norm1 weight factor, fc1 weight factor): the review's case (x100, x50), one that
# drives the hidden pre-activations far past fp16's range (x100, x2000), and one with
# tiny activations (x1e-3) whose fp16 low terms would be subnormal unscaled
CASES = [(100.0, 50.0), (100.0, 2000.0), (1e-3, 1.0)]


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"norm1x{c[0]:g}_fc1x{c[1]:g}")
def test_mlp_range_guard_matches_oracle(case):
    from test_gpu_mlp_fused import _block
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    nf, wf = case
    nlat, nlon, lmax, C = 90, 180, 45, 256
    cfg = sfno_ref.BlockCfg(filter_type="non-linear")
    p = sfno_ref.make_block_params(C, lmax, lmax + 1, cfg, seed=31, randomize_affine=True)
    p["norm1.weight"] = p["norm1.weight"] * nf
    p["norm1.bias"] = p["norm1.bias"] * nf
    p["mlp.fwd.0.weight"] = p["mlp.fwd.0.weight"] * wf
    g = torch.Generator().manual_seed(32)
    x = torch.randn(1, C, nlat, nlon, generator=g)
    gamma = 0.2 * torch.randn(1, C, generator=g)
    beta = 0.2 * torch.randn(1, C, generator=g)
    blk = _block(cfg, p, nlat, nlon, lmax)
    with torch.no_grad():
        y = blk(x.to(DEV), gamma.to(DEV), beta.to(DEV), 0.7).cpu()
    sht, isht = sfno_ref.make_transforms(nlat, nlon, lmax, lmax + 1)
    with torch.no_grad():
        want = sfno_ref.block_forward(p, x, sht, isht, cfg, gamma, beta, 0.7)
    assert torch.isfinite(y).all()
    err = (y - want).abs().max().item()
    ymax = want.abs().max().item()
    print(f"{case}: max-abs {err:.3e} |y|max {ymax:.4g}")
    assert err < 1e-4 * max(1.0, ymax), (case, err, ymax)
