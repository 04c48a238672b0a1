"""GPU parity of the latitude-band sharded block through the
C-ABI stages (msfno_band_*): W virtual ranks run in lock step on one GPU
(LocalGroup — the all-to-alls become device copies), and the re-assembled
output is compared with the reference golden vectors (max-abs < 1e-4, the
north-star bar) and with the unsharded native block (same kernels, only the
statistics merge order differs: max-abs < 2e-5).  Every golden fixture is
covered: both filters (the linear one with its per-mode weight sharded by
m-set) and the resampling first/last blocks (separate input / output bands)."""
import os

import pytest
import torch

from block_util import make_block
from golden_util import golden_files, load

pytestmark = pytest.mark.gpu
DEV = "cuda"

ALL_BLOCKS = golden_files()


def _sharded(blk, x, gamma, beta, scale, world, row_start=None, m_owner=None):
    from msfno_amd.sfno import LatBandBlock, LocalGroup
    shards = [LatBandBlock(blk, r, world, row_start, m_owner) for r in range(world)]
    gens = [s.stages(s.take(x), gamma, beta, scale) for s in shards]
    return LatBandBlock.assemble(shards, LocalGroup.run(gens))


@pytest.mark.parametrize("world", [1, 2, 3, 5])
@pytest.mark.parametrize("path", ALL_BLOCKS, ids=lambda p: os.path.basename(p)[:-4])
def test_sharded_block_matches_golden(path, world):
    meta, params, arrays, _ = load(path)
    ke = min(n - n // 2 for n in (meta["nlat"], meta.get("out_nlat", meta["nlat"])))
    if ke < world:
        pytest.skip("fewer northern latitude rows than ranks")
    blk, _, _ = make_block(meta, params)
    blk = blk.to(DEV)
    x = arrays["x"].to(DEV)
    g = arrays["gamma"].to(DEV) if meta["filmed"] else None
    b = arrays["beta"].to(DEV) if meta["filmed"] else None
    scale = meta["scale"] if meta["filmed"] else 1.0
    with torch.no_grad():
        y = _sharded(blk, x, g, b, scale, world).cpu()
        y1 = (blk(x, g, b, scale) if meta["filmed"] else blk(x)).cpu()
    want = arrays["y"]
    assert y.shape == want.shape
    assert (y - want).abs().max().item() < 1e-4
    assert (y - y1).abs().max().item() < 2e-5


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("name", ["c1b2_nl_film_middle.npz", "down_lin_film_first.npz",
                                  "mid_nl_film_middle.npz"])
def test_sharded_block_general_layout(name, world, monkeypatch):
    """MSFNO_NO_SYM=1: the tables load in the general (non-folded) layout, so the
    exchange slabs carry each rank's local rows unfolded (2W columns per source)."""
    monkeypatch.setenv("MSFNO_NO_SYM", "1")
    meta, params, arrays, _ = load([p for p in golden_files() if os.path.basename(p) == name][0])
    blk, _, _ = make_block(meta, params)
    blk = blk.to(DEV)
    x = arrays["x"].to(DEV)
    g, b = arrays["gamma"].to(DEV), arrays["beta"].to(DEV)
    with torch.no_grad():
        y = _sharded(blk, x, g, b, meta["scale"], world).cpu()
    assert (y - arrays["y"]).abs().max().item() < 1e-4


def test_sharded_block_custom_partition_with_idle_rank():
    """Uneven bands and a rank that owns no zonal wavenumber."""
    path = [p for p in golden_files() if os.path.basename(p) == "c1b2_nl_film_middle.npz"][0]
    meta, params, arrays, _ = load(path)
    blk, _, _ = make_block(meta, params)
    blk = blk.to(DEV)
    x = arrays["x"].to(DEV)
    nlat, lmax, mmax = meta["nlat"], meta["lmax"], meta["mmax"]
    rows = [0, 3, 11, nlat - nlat // 2]   # bands of the northern half
    own = [(m % 2) if m < min(lmax, mmax) else -1 for m in range(mmax)]   # rank 2 owns none
    with torch.no_grad():
        y = _sharded(blk, x, arrays["gamma"].to(DEV), arrays["beta"].to(DEV), meta["scale"], 3,
                     rows, own).cpu()
    assert (y - arrays["y"]).abs().max().item() < 1e-4


@pytest.mark.parametrize("name", ["c1b2_lin_film_middle.npz", "c1b2_nl_film_middle.npz",
                                  "down_lin_film_first.npz", "up_nl_film_last.npz"])
@pytest.mark.parametrize("chunks", [2, 3])
def test_sharded_block_pipelined_chunks(name, chunks):
    """The sub-batch pipeline (forward(chunks=K)): world 1, the batch split into
    K sub-batches with their own slots / buffers; fields are independent, so each
    equals the golden output of its field."""
    from msfno_amd.sfno import LatBandBlock
    meta, params, arrays, _ = load([p for p in golden_files() if os.path.basename(p) == name][0])
    blk, _, _ = make_block(meta, params)
    blk = blk.to(DEV)
    x = arrays["x"].to(DEV)
    g, b = arrays["gamma"].to(DEV), arrays["beta"].to(DEV)
    reps = 3   # a batch of 3 copies of the fixture batch
    xr, gr, br = x.repeat(reps, 1, 1, 1), g.repeat(reps, 1), b.repeat(reps, 1)
    s = LatBandBlock(blk, 0, 1)
    with torch.no_grad():
        y = s(xr, gr, br, meta["scale"], chunks=chunks).cpu()
    want = arrays["y"].repeat(reps, 1, 1, 1)
    assert (y - want).abs().max().item() < 1e-4


def test_sharded_linear_weight_slice_is_the_rank_modes():
    """The linear filter's weight is sharded by m-set: each rank's slice holds
    exactly the tril modes whose m it owns, and the slices partition the modes."""
    from msfno_amd.sfno import LatBandBlock
    meta, params, arrays, _ = load([p for p in golden_files()
                                    if os.path.basename(p) == "c1_lin_film_middle.npz"][0])
    blk, _, _ = make_block(meta, params)
    blk = blk.to(DEV)
    lmax, mmax = meta["lmax"], meta["mmax"]
    ii, jj = torch.tril_indices(lmax, mmax)
    seen = []
    for r in range(3):
        s = LatBandBlock(blk, r, 3)
        modes = s.plan.linear_modes()
        assert modes == sorted(modes)
        assert all(s.m_owner[int(jj[n])] == r for n in modes)
        w = s._linear_weight(blk.filter_layer.filter.w)
        assert w.shape[2] == len(modes)
        assert torch.equal(w.cpu(), blk.filter_layer.filter.w.detach().cpu()[:, :, modes])
        seen += modes
    assert sorted(seen) == list(range(ii.shape[0]))


@pytest.mark.slow
def test_sharded_block_config2_matches_unsharded():
    """721x1440, C=256, lmax=360, 4 virtual ranks vs the unsharded native block."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    args = bench.parse_args([])
    blk, _, _ = bench.build_block(args, torch.device(DEV))
    gen = torch.Generator().manual_seed(0)
    x = torch.randn(1, 256, 721, 1440, generator=gen).to(DEV)
    g = (0.1 * torch.randn(1, 256, generator=gen)).to(DEV)
    b = (0.1 * torch.randn(1, 256, generator=gen)).to(DEV)
    with torch.no_grad():
        y1 = blk(x, g, b, 1.0)
        y = _sharded(blk, x, g, b, 1.0, 4)
    err = (y - y1).abs().max().item()
    assert err < 2e-5, err


@pytest.mark.slow
def test_sharded_block_config4_geometry_eight_ranks():
    """Config 4's sharding (721x1440, C=256, lmax=360, 8 ranks: bands of 45/46 rows +
    mirrors, W = 48, 8 source blocks in the Legendre GEMMs' K) on 8 lock-step virtual
    ranks, a batch of 2 fields, against the unsharded native block."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    args = bench.parse_args([])
    blk, _, _ = bench.build_block(args, torch.device(DEV))
    gen = torch.Generator().manual_seed(4)
    x = torch.randn(2, 256, 721, 1440, generator=gen).to(DEV)
    g = (0.1 * torch.randn(2, 256, generator=gen)).to(DEV)
    b = (0.1 * torch.randn(2, 256, generator=gen)).to(DEV)
    with torch.no_grad():
        y1 = blk(x, g, b, 1.0)
        y = _sharded(blk, x, g, b, 1.0, 8)
    err = (y - y1).abs().max().item()
    assert err < 2e-5, err


def _dist_rank(rank, world, port, path, q, chunks=1):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for p in (here, os.path.dirname(here),
              os.path.join(os.path.dirname(here), "modulated-spherical-fourier-neural-operator_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    from block_util import make_block as mk
    from golden_util import load as ld
    from msfno_amd.sfno import LatBandBlock, TorchComm
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        meta, params, arrays, _ = ld(path)
        blk, _, _ = mk(meta, params)
        blk = blk.to(DEV)
        shard = LatBandBlock(blk, rank, world)
        x = shard.take(arrays["x"].to(DEV))
        with torch.no_grad():
            y = shard(x, arrays["gamma"].to(DEV), arrays["beta"].to(DEV), meta["scale"],
                      comm=TorchComm(), chunks=chunks)
        q.put((rank, (shard.rows_out, y.cpu().numpy())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,chunks", [("c1b2_nl_film_middle.npz", 1),
                                         ("c1b2_nl_film_middle.npz", 2),
                                         ("c1b2_lin_film_middle.npz", 2),
                                         ("down_nl_film_first.npz", 1)])
def test_sharded_block_two_processes_gloo(name, chunks):
    """Two processes on the one GPU, collectives through torch.distributed (gloo,
    host-staged): exercises TorchComm + the native stages end to end, with and
    without the sub-batch pipeline."""
    import socket

    import torch.multiprocessing as mp
    path = [p for p in golden_files() if os.path.basename(p) == name][0]
    meta, params, arrays, _ = load(path)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_dist_rank, args=(r, 2, port, path, q, chunks)) for r in range(2)]
    for p in ps:
        p.start()
    try:
        res = dict(q.get(timeout=300) for _ in range(2))
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    y = torch.full_like(arrays["y"], float("nan"))
    for r in range(2):
        rows, part = res[r]
        y[:, :, rows] = torch.from_numpy(part)
    assert (y - arrays["y"]).abs().max().item() < 1e-4
