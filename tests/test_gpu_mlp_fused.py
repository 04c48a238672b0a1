"""The fused block MLP (csrc/mlp_fused.hip: fc1 -> GELU -> fc2 with the hidden
activation kept on-chip, norm1 + FiLM applied to x1 in-kernel; C = 256, H = 512)
against the oracle (oracle/sfno_ref.py block_forward, layers.py:145-178 /
sfnonet.py:359-393) on grids whose pixel count is not a multiple of the
128-pixel tile (ragged last tile), for both filters, a batch of fields with
different FiLM modulations, the latitude-band sharded block (2 and 3 virtual
ranks), and against the unfused fc1 / fc2 GEMM pair (MSFNO_MLP_FUSED=0, in a
child process: the switch is read once per process).
Bar: max-abs < 1e-4 * max(1, |y|)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
if __name__ == "__main__":
    _repo = os.path.dirname(HERE)
    for _d in (HERE, _repo, os.path.join(_repo, "modulated-spherical-fourier-neural-operator_amd")):
        sys.path.insert(0, _d)

import numpy as np  # noqa: E402
import pytest  # noqa: E402
import torch  # noqa: E402

from oracle import sfno_ref  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (filter, nlat, nlon, lmax, B): P = 2112 (tile remainder 64), 4320 (96), 16200 (72)
CASES = [("non-linear", 33, 64, 32, 2), ("linear", 45, 96, 23, 1), ("non-linear", 90, 180, 45, 3)]


def _case(filter_type, nlat, nlon, lmax, B, seed=7):
    C = 256
    cfg = sfno_ref.BlockCfg(filter_type=filter_type)
    p = sfno_ref.make_block_params(C, lmax, lmax + 1, cfg, seed=seed, randomize_affine=True)
    g = torch.Generator().manual_seed(seed + 1)
    x = torch.randn(B, C, nlat, nlon, generator=g)
    gamma = 0.2 * torch.randn(B, C, generator=g)
    beta = 0.2 * torch.randn(B, C, generator=g)
    return cfg, p, x, gamma, beta


def _block(cfg, p, nlat, nlon, lmax):
    from functools import partial

    from msfno_amd.harmonics import InverseRealSHT, RealSHT
    from msfno_amd.sfno import FourierNeuralOperatorBlock_Filmed
    C = 256
    sht = RealSHT(nlat, nlon, lmax=lmax, mmax=lmax + 1, grid="equiangular").float()
    isht = InverseRealSHT(nlat, nlon, lmax=lmax, mmax=lmax + 1, grid="equiangular").float()
    sht.weights = sht.weights * 1e5
    isht.pct = isht.pct / 1e5
    norm = partial(torch.nn.InstanceNorm2d, num_features=C, eps=1e-6, affine=True,
                   track_running_stats=False)
    blk = FourierNeuralOperatorBlock_Filmed(sht, isht, C, filter_type=cfg.filter_type,
                                            mlp_ratio=2.0, norm_layer=(norm, norm),
                                            inner_skip="linear", outer_skip="identity",
                                            mlp_mode="distributed", spectral_layers=3)
    blk.load_state_dict(p, strict=False)
    return blk.eval().to(DEV)


def _native(case):
    cfg, p, x, gamma, beta = _case(*case)
    blk = _block(cfg, p, *case[1:4])
    with torch.no_grad():
        return blk(x.to(DEV), gamma.to(DEV), beta.to(DEV), 0.7).cpu()


@pytest.mark.parametrize("case", CASES, ids=lambda c: f"{c[0]}_{c[1]}x{c[2]}_B{c[4]}")
def test_fused_block_matches_oracle(case):
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    cfg, p, x, gamma, beta = _case(*case)
    y = _native(case)
    sht, isht = sfno_ref.make_transforms(case[1], case[2], case[3], case[3] + 1)
    with torch.no_grad():
        want = sfno_ref.block_forward(p, x, sht, isht, cfg, gamma, beta, 0.7)
    err = (y - want).abs().max().item()
    print(f"{case}: max-abs {err:.3e} |y|max {want.abs().max():.3f}")
    assert err < 1e-4 * max(1.0, want.abs().max().item())


@pytest.mark.parametrize("world", [2, 3])
def test_fused_sharded_block_matches_unsharded(world):
    from msfno_amd.sfno import LatBandBlock, LocalGroup
    case = CASES[2]
    cfg, p, x, gamma, beta = _case(*case)
    blk = _block(cfg, p, *case[1:4])
    x, gamma, beta = x.to(DEV), gamma.to(DEV), beta.to(DEV)
    with torch.no_grad():
        y1 = blk(x, gamma, beta, 0.7)
        shards = [LatBandBlock(blk, r, world) for r in range(world)]
        gens = [s.stages(s.take(x), gamma, beta, 0.7) for s in shards]
        y = LatBandBlock.assemble(shards, LocalGroup.run(gens))
    assert (y - y1).abs().max().item() < 2e-5


def test_fused_equals_unfused_gemm_pair(tmp_path):
    out = str(tmp_path / "unfused.npz")
    r = subprocess.run([sys.executable, os.path.abspath(__file__), out],
                       env=dict(os.environ, MSFNO_MLP_FUSED="0"), cwd=HERE, capture_output=True,
                       text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    other = np.load(out)
    for i, case in enumerate(CASES[:2]):
        y = _native(case)
        y0 = torch.from_numpy(other[f"c{i}"])
        assert (y - y0).abs().max().item() < 2e-5 * max(1.0, y0.abs().max().item())


if __name__ == "__main__":
    np.savez(sys.argv[1], **{f"c{i}": _native(c).numpy() for i, c in enumerate(CASES[:2])})


def test_weight_cache_reuse_and_invalidation():
    """The prepared-weight cache (msfno_block_desc.wcache): the second call reuses the
    images (same output), an in-place weight update (a new _version) rebuilds them
    (the output follows the new weights, equal to a fresh module's)."""
    case = CASES[0]
    cfg, p, x, gamma, beta = _case(*case)
    blk = _block(cfg, p, *case[1:4])
    x, gamma, beta = x.to(DEV), gamma.to(DEV), beta.to(DEV)
    with torch.no_grad():
        y0 = blk(x, gamma, beta, 0.7)
        assert blk._wcache_key is not None
        y1 = blk(x, gamma, beta, 0.7)
        assert torch.equal(y0, y1)
        blk.mlp.fwd[0].weight.mul_(1.25)                     # fused-MLP image
        blk.filter_layer.filter.w[1].mul_(0.8)               # spectral 3M images
        y2 = blk(x, gamma, beta, 0.7)
    p2 = {k: v.clone() for k, v in p.items()}
    p2["mlp.fwd.0.weight"] = p2["mlp.fwd.0.weight"] * 1.25
    p2["filter_layer.filter.w.1"] = p2["filter_layer.filter.w.1"] * 0.8
    fresh = _block(cfg, p2, *case[1:4])
    with torch.no_grad():
        want = fresh(x, gamma, beta, 0.7)
    assert (y2 - y0).abs().max().item() > 1e-3
    assert torch.equal(y2, want)
