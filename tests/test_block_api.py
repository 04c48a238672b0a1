"""CPU checks of the drop-in block API: constructor signatures, module names and
state-dict keys identical to the reference's (fixture key lists were produced by
the reference modules themselves, tests/golden/make_golden.py)."""
import os

import pytest
import torch

from block_util import make_block
from golden_util import golden_files, load


@pytest.mark.parametrize("path", golden_files()[:12], ids=lambda p: os.path.basename(p)[:-4])
def test_state_dict_keys_match_reference(path):
    meta, params, _, keys = load(path)
    blk, _, _ = make_block(meta, params)
    assert sorted(blk.state_dict().keys()) == sorted(keys)
    for k, v in params.items():
        assert blk.state_dict()[k].shape == v.shape, k


def test_filter_type_dispatch_and_errors():
    from msfno_amd.harmonics import InverseRealSHT, RealSHT
    from msfno_amd.sfno import SpectralAttentionS2, SpectralConvS2, SpectralFilterLayer
    f = RealSHT(16, 32, lmax=16, mmax=17)
    g = InverseRealSHT(16, 32, lmax=16, mmax=17)
    assert isinstance(SpectralFilterLayer(f, g, 8, "non-linear").filter, SpectralAttentionS2)
    assert isinstance(SpectralFilterLayer(f, g, 8, "linear").filter, SpectralConvS2)
    with pytest.raises(NotImplementedError):
        SpectralFilterLayer(f, g, 8, "bogus")
    with pytest.raises(NotImplementedError):
        SpectralFilterLayer(object(), g, 8, "linear")
    # lmax/mmax mismatch is an assertion in the reference (layers.py:364-365)
    g2 = InverseRealSHT(16, 32, lmax=15, mmax=17)
    with pytest.raises(AssertionError):
        SpectralConvS2(f, g2, 8)


def test_linear_filter_weight_shape_and_tril_buffers():
    from msfno_amd.harmonics import InverseRealSHT, RealSHT
    from msfno_amd.sfno import SpectralConvS2
    f = RealSHT(16, 32, lmax=16, mmax=17)
    g = InverseRealSHT(16, 32, lmax=16, mmax=17)
    m = SpectralConvS2(f, g, 4)
    ii, jj = torch.tril_indices(16, 17)
    assert m.w.shape == (4, 4, ii.numel(), 2)
    assert torch.equal(m.ii, ii) and torch.equal(m.jj, jj)


def test_torch_harmonics_style_transforms_are_adopted():
    """A filter built around torch-harmonics-style transforms (here the oracle's
    restatement of torch_harmonics.RealSHT / InverseRealSHT: same attributes and buffer
    names) runs on the native plans over the foreign tables, without copying them; a
    later re-assignment of the foreign buffer (the reference's x1e5 rescale,
    sfnonet.py:551-555) is seen."""
    from msfno_amd.harmonics import InverseRealSHT, RealSHT
    from msfno_amd.sfno import SpectralFilterLayer
    from oracle import sht_ref as S
    f = S.RealSHT(16, 32, lmax=16, mmax=17).float()
    g = S.InverseRealSHT(16, 32, lmax=16, mmax=17).float()
    for kind in ("linear", "non-linear"):
        layer = SpectralFilterLayer(f, g, 8, kind)
        fwd, inv = layer.filter._transforms()
        assert isinstance(fwd, RealSHT) and isinstance(inv, InverseRealSHT)
        assert fwd.weights is f.weights and inv.pct is g.pct
        assert (fwd.nlat, fwd.nlon, fwd.lmax, fwd.mmax) == (16, 32, 16, 17)
    f.weights = f.weights * 1e5
    assert layer.filter._transforms()[0].weights is f.weights
    bad = S.RealSHT(16, 32, lmax=16, mmax=17)
    bad.norm = "schmidt"
    with pytest.raises(NotImplementedError):
        SpectralFilterLayer(bad, g, 8, "linear").filter._transforms()


def test_layer_norm_network_is_refused_at_construction():
    """normalization_layer='layer_norm' (sfnonet.py:482-490, a per-pixel LayerNorm affine)
    is not fused: the mirror refuses it when the network is built, not at its first
    forward."""
    import pytest
    from msfno_amd.sfno import FourierNeuralOperatorNet
    with pytest.raises(NotImplementedError, match="layer_norm"):
        FourierNeuralOperatorNet("cpu", None, img_size=(33, 64), scale_factor=4, in_chans=5,
                                 out_chans=5, embed_dim_sfno=16, num_layers=4,
                                 normalization_layer="layer_norm")
