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


def _sharded_net(net, x, world, sst=None, scale=1.0, inner="shard"):
    from msfno_amd.sfno import LatBandBlock, LatBandNet, LocalGroup
    shards = [LatBandNet(net, r, world, inner=inner) for r in range(world)]
    gens = [s.stages(s.take(x), sst, scale) for s in shards]
    outs = LocalGroup.run(gens)
    return LatBandBlock.assemble([s.shards[-1] for s in shards], outs)


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("path", NET_FIXTURES, ids=lambda p: os.path.basename(p)[:-4])
def test_latband_net_replicated_inner_blocks(path, world):
    """LatBandNet(inner="replicate") (the first and last blocks sharded,
    the inner blocks run unsharded on every rank after one all-gather of block 0's
    output rows) against the reference network's output and the all-sharded form."""
    meta, params, x, y, _ = load_net(path)
    net = _build(meta, params)
    x = x.to(DEV)
    with torch.no_grad():
        got = _sharded_net(net, x, world, inner="replicate").cpu()
        sh = _sharded_net(net, x, world).cpu()
    assert (got - y).abs().max().item() < 1e-4 * max(1.0, y.abs().max().item())
    assert (got - sh).abs().max().item() < 2e-5 * max(1.0, y.abs().max().item())


def test_latband_filmed_net_replicated_inner_blocks_matches_unsharded():
    path = NET_FIXTURES[0]
    meta, params, x, y, _ = load_net(path)
    net = _build(meta, params, filmed=True, film_layers=2)
    g = torch.Generator().manual_seed(5)
    B, C = x.shape[0], meta["C"]
    film = torch.stack((0.1 * torch.randn(B, 2, C, generator=g),
                        0.1 * torch.randn(B, 2, C, generator=g)), dim=1).to(DEV)
    x = x.to(DEV)
    with torch.no_grad():
        want = net(x, film, 0.8)
        got = _sharded_net(net, x, 3, film, 0.8, inner="replicate")
    assert (got - want).abs().max().item() < 2e-5 * max(1.0, want.abs().max().item())


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


def _rollout_rank(rank, world, port, path, q, chunks):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.dirname(here),
              os.path.join(os.path.dirname(here), "modulated-spherical-fourier-neural-operator_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    from test_oracle_net import load_net as ld
    from msfno_amd.rollout import Rollout
    from msfno_amd.sfno import LatBandNet, TorchComm
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        meta, params, x, _, _ = ld(path)
        net = _build(meta, params, filmed=True, film_layers=2)
        film, means, stds = _rollout_inputs(meta, x)
        shard = LatBandNet(net, rank, world, comm=TorchComm(), chunks=chunks)
        r = Rollout(shard, means.to(DEV), stds.to(DEV), film=film.to(DEV), scale=0.8)
        x0 = shard.take((x.to(DEV) * stds.to(DEV) + means.to(DEV)).repeat(2, 1, 1, 1))
        outs = [o.cpu().numpy() for _, o in r.run(x0, 3)]
        q.put((rank, (shard.rows_out, outs)))
    finally:
        dist.destroy_process_group()


def _rollout_inputs(meta, x):
    g = torch.Generator().manual_seed(9)
    C, ch = meta["C"], meta["in_chans"]
    B = 2 * x.shape[0]
    film = torch.stack((0.1 * torch.randn(B, 2, C, generator=g),
                        0.1 * torch.randn(B, 2, C, generator=g)), dim=1)
    means = torch.randn(1, ch, 1, 1, generator=g)
    stds = torch.rand(1, ch, 1, 1, generator=g) + 0.5
    return film, means, stds


@pytest.mark.parametrize("chunks", [1, 2])
def test_rollout_of_latband_net_two_processes_gloo(chunks):
    """Rollout driving one rank's LatBandNet (normalise, step, denormalise on the
    rank's rows) in two processes over torch.distributed (gloo), with and without
    the sub-batch pipeline across the whole network, against the unsharded
    Rollout: three 6 h steps of the filmed fixture network."""
    import socket

    import torch.multiprocessing as mp
    from msfno_amd.rollout import Rollout
    path = NET_FIXTURES[0]
    meta, params, x, _, _ = load_net(path)
    net = _build(meta, params, filmed=True, film_layers=2)
    film, means, stds = _rollout_inputs(meta, x)
    x0 = (x.to(DEV) * stds.to(DEV) + means.to(DEV)).repeat(2, 1, 1, 1)
    r = Rollout(net, means.to(DEV), stds.to(DEV), film=film.to(DEV), scale=0.8, graph=False)
    want = [o.cpu() for _, o in r.run(x0, 3)]
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rollout_rank, args=(rk, 2, port, path, q, chunks))
          for rk in range(2)]
    for p in ps:
        p.start()
    try:
        res = dict(q.get(timeout=300) for _ in range(2))
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for i in range(3):
        y = torch.full_like(want[i], float("nan"))
        for rk in range(2):
            rows, parts = res[rk]
            y[:, :, rows] = torch.from_numpy(parts[i])
        sc = max(1.0, want[i].abs().max().item())
        assert (y - want[i]).abs().max().item() < 2e-5 * sc, i
