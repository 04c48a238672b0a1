"""Build msfno_amd blocks from golden-fixture metadata (shared by CPU + GPU tests)."""
from functools import partial

import torch

from golden_util import wiring_cfg


def make_transforms(meta, rescale=True):
    from msfno_amd.harmonics import InverseRealSHT, RealSHT
    sht = RealSHT(meta["nlat"], meta["nlon"], lmax=meta["lmax"], mmax=meta["mmax"],
                  grid=meta["grid"]).float()
    if "out_nlat" in meta:
        isht = InverseRealSHT(meta["out_nlat"], meta["out_nlon"], lmax=meta["lmax"],
                              mmax=meta["mmax"], grid=meta["out_grid"]).float()
    else:
        isht = InverseRealSHT(meta["nlat"], meta["nlon"], lmax=meta["lmax"], mmax=meta["mmax"],
                              grid=meta["grid"]).float()
    if rescale:  # sfnonet.py:551-555
        sht.weights = sht.weights * 1e5
        isht.pct = isht.pct / 1e5
    return sht, isht


def make_block(meta, params=None):
    from msfno_amd.sfno import FourierNeuralOperatorBlock, FourierNeuralOperatorBlock_Filmed
    sht, isht = make_transforms(meta)
    C = meta["C"]
    inner, outer, has_mlp = wiring_cfg(meta)
    norm = partial(torch.nn.InstanceNorm2d, num_features=C, eps=1e-6, affine=True,
                   track_running_stats=False)
    cls = FourierNeuralOperatorBlock_Filmed if meta["filmed"] else FourierNeuralOperatorBlock
    blk = cls(sht, isht, C, filter_type=meta["filter"], mlp_ratio=2.0, norm_layer=(norm, norm),
              inner_skip=inner, outer_skip=outer,
              mlp_mode="distributed" if has_mlp else "none", spectral_layers=3,
              complex_activation="real", use_complex_kernels=True)
    if params is not None:
        missing, unexpected = blk.load_state_dict(params, strict=False)
        assert not unexpected, unexpected
        assert all(k.endswith((".weights", ".pct")) for k in missing), missing
    blk.eval()
    return blk, sht, isht
