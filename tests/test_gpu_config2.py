"""GPU parity at BASELINE config 2 (721x1440, C=256, lmax=360): the fused HIP
block vs the oracle's CPU restatement on identical inputs.  Bar: max-abs < 1e-4."""
import pytest
import torch

from oracle import sfno_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _mine(p, cfg, C, nlat, nlon, lmax, mmax, filmed):
    from functools import partial

    from msfno_amd.harmonics import InverseRealSHT, RealSHT
    from msfno_amd.sfno import FourierNeuralOperatorBlock, FourierNeuralOperatorBlock_Filmed
    sht = RealSHT(nlat, nlon, lmax=lmax, mmax=mmax, grid="equiangular").float()
    isht = InverseRealSHT(nlat, nlon, lmax=lmax, mmax=mmax, grid="equiangular").float()
    sht.weights = sht.weights * 1e5
    isht.pct = isht.pct / 1e5
    norm = partial(torch.nn.InstanceNorm2d, num_features=C, eps=1e-6, affine=True,
                   track_running_stats=False)
    cls = FourierNeuralOperatorBlock_Filmed if filmed else FourierNeuralOperatorBlock
    blk = cls(sht, isht, C, filter_type=cfg.filter_type, mlp_ratio=2.0, norm_layer=(norm, norm),
              inner_skip=cfg.inner_skip, outer_skip=cfg.outer_skip,
              mlp_mode="distributed" if cfg.has_mlp else "none", spectral_layers=3)
    blk.load_state_dict(p, strict=False)
    return blk.eval().to(DEV), sht, isht


@pytest.mark.parametrize("filter_type,C", [("non-linear", 256), ("linear", 32)])
def test_config2_block_matches_oracle(filter_type, C):
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    nlat, nlon, lmax, mmax = 721, 1440, 360, 361
    cfg = sfno_ref.BlockCfg(filter_type=filter_type)
    p = sfno_ref.make_block_params(C, lmax, mmax, cfg, seed=1, randomize_affine=True)
    g = torch.Generator().manual_seed(0)
    x = torch.randn(1, C, nlat, nlon, generator=g)
    gamma = 0.1 * torch.randn(1, C, generator=g)
    beta = 0.1 * torch.randn(1, C, generator=g)
    blk, _, _ = _mine(p, cfg, C, nlat, nlon, lmax, mmax, True)
    with torch.no_grad():
        y = blk(x.to(DEV), gamma.to(DEV), beta.to(DEV), 1.0).cpu()
    del blk
    torch.cuda.empty_cache()
    o_sht, o_isht = sfno_ref.make_transforms(nlat, nlon, lmax, mmax)
    with torch.no_grad():
        want = sfno_ref.block_forward(p, x, o_sht, o_isht, cfg, gamma, beta, 1.0)
    err = (y - want).abs().max().item()
    rms = (y - want).pow(2).mean().sqrt().item()
    print(f"config2 {filter_type} C={C}: max-abs {err:.3e} rms {rms:.3e} |y|max {want.abs().max():.3f}")
    assert err < 1e-4
