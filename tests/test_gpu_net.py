"""GPU parity of the network around the block: the native
FourierNeuralOperatorNet[_Filmed] (encoder with pos_embed fused, 4-block stack
across the equiangular -> Gauss -> equiangular grids, in-place big-skip concat,
decoder) against the reference network's own outputs (tests/golden/net/) and
the oracle, plus the standalone native MLP.  Tolerance: max-abs < 1e-4 (×max(1,|y|))."""
import os

import pytest
import torch

from oracle import sfno_ref
from test_oracle_net import NET_FIXTURES, load_net, net_cfg

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _build(meta, params, filmed=False, film_layers=2):
    from msfno_amd.sfno import FourierNeuralOperatorNet, FourierNeuralOperatorNet_Filmed
    kw = dict(filter_type=meta["filter"], img_size=(meta["nlat"], meta["nlon"]),
              scale_factor=meta["scale_factor"], in_chans=meta["in_chans"],
              out_chans=meta["out_chans"], embed_dim_sfno=meta["C"],
              num_layers=meta["num_layers"], spectral_layers=3)
    if filmed:
        net = FourierNeuralOperatorNet_Filmed("cpu", None, film_layers=film_layers,
                                              advanced_logging=False, model_depth=None, **kw)
    else:
        net = FourierNeuralOperatorNet("cpu", None, **kw)
    missing, unexpected = net.load_state_dict(params, strict=False)
    assert not unexpected and all(k.endswith((".weights", ".pct")) for k in missing)
    return net.eval().to(DEV)


@pytest.mark.parametrize("path", NET_FIXTURES, ids=lambda p: os.path.basename(p)[:-4])
def test_net_matches_reference_golden(path):
    meta, params, x, y, _ = load_net(path)
    net = _build(meta, params)
    with torch.no_grad():
        got = net(x.to(DEV)).cpu()
    assert got.shape == y.shape
    assert (got - y).abs().max().item() < 1e-4 * max(1.0, y.abs().max().item())


@pytest.mark.parametrize("path", NET_FIXTURES, ids=lambda p: os.path.basename(p)[:-4])
def test_filmed_net_matches_oracle(path):
    meta, params, x, y, _ = load_net(path)
    net = _build(meta, params, filmed=True, film_layers=2)
    g = torch.Generator().manual_seed(3)
    B, C = x.shape[0], meta["C"]
    gamma = 0.1 * torch.randn(B, 2, C, generator=g)
    beta = 0.1 * torch.randn(B, 2, C, generator=g)
    with torch.no_grad():
        want = sfno_ref.net_forward(params, x, net_cfg(meta), film=(gamma, beta), scale=0.8)
        got = net(x.to(DEV), torch.stack((gamma, beta), dim=1).to(DEV), 0.8).cpu()
    assert (got - want).abs().max().item() < 1e-4 * max(1.0, want.abs().max().item())


def test_native_mlp_concat_and_broadcast_addend():
    from msfno_amd.sfno import MLP
    torch.manual_seed(0)
    m = MLP(in_features=7 + 5, hidden_features=24, out_features=9, output_bias=True).eval()
    x, x2 = torch.randn(2, 7, 6, 10), torch.randn(2, 5, 6, 10)
    add = torch.randn(1, 9, 6, 10)
    p = {f"fwd.{k}": v for k, v in m.fwd.state_dict().items()}
    want = sfno_ref.mlp(torch.cat((x, x2), dim=1), p, prefix="fwd.") + add
    with torch.no_grad():
        got = m.to(DEV).native_forward(x.to(DEV), x2=x2.to(DEV), addend=add.to(DEV)).cpu()
    assert (got - want).abs().max().item() < 1e-5 * max(1.0, want.abs().max().item())
    m2 = MLP(in_features=12, hidden_features=20, out_features=12, output_bias=False).eval()
    xx = torch.randn(3, 12, 5, 8)
    with torch.no_grad():
        want = sfno_ref.mlp(xx, {f"fwd.{k}": v for k, v in m2.fwd.state_dict().items()}, "fwd.")
        got = m2.to(DEV)(xx.to(DEV)).cpu()
    assert (got - want).abs().max().item() < 1e-5 * max(1.0, want.abs().max().item())


def _sharded_net(net, x, world, sst=None, scale=1.0):
    from msfno_amd.sfno import LatBandBlock, LatBandNet, LocalGroup
    shards = [LatBandNet(net, r, world) for r in range(world)]
    gens = [s.stages(s.take(x), sst, scale) for s in shards]
    outs = LocalGroup.run(gens)
    return LatBandBlock.assemble([s.shards[-1] for s in shards], outs)


@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("path", NET_FIXTURES, ids=lambda p: os.path.basename(p)[:-4])
def test_latband_net_matches_reference_golden(path, world):
    """The network forward latitude-band sharded over `world` lock-step virtual ranks
    (LatBandNet: encoder / decoder on each rank's rows, every block a LatBandBlock, the
    resampling blocks chaining the 33x64 and 8x16 band partitions) against the
    reference network's output."""
    meta, params, x, y, _ = load_net(path)
    net = _build(meta, params)
    with torch.no_grad():
        got = _sharded_net(net, x.to(DEV), world).cpu()
    assert (got - y).abs().max().item() < 1e-4 * max(1.0, y.abs().max().item())


@pytest.mark.parametrize("path", NET_FIXTURES, ids=lambda p: os.path.basename(p)[:-4])
def test_latband_filmed_net_matches_unsharded(path):
    meta, params, x, y, _ = load_net(path)
    net = _build(meta, params, filmed=True, film_layers=2)
    g = torch.Generator().manual_seed(3)
    B, C = x.shape[0], meta["C"]
    film = torch.stack((0.1 * torch.randn(B, 2, C, generator=g),
                        0.1 * torch.randn(B, 2, C, generator=g)), dim=1).to(DEV)
    x = x.to(DEV)
    with torch.no_grad():
        want = net(x, film, 0.8)
        got = _sharded_net(net, x, 3, film, 0.8)
    assert (got - want).abs().max().item() < 2e-5 * max(1.0, want.abs().max().item())
