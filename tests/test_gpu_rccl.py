"""The latitude-band path over RCCL itself (torch.distributed backend "nccl"), on the
one GPU a test box has: a world-size-1 process group, so every collective of the N > 1
path — the async all-gather of the norm statistics (all_gather_into_tensor) and the two
uneven all-to-alls (all_to_all_single with split sizes) — runs through RCCL on device
buffers, with the sub-batch pipeline's deferred waits, and the network step is also
captured into a HIP graph with its RCCL collectives and replayed.  The CPU suite covers
the same code on gloo with 2 and 3 processes; this covers the device backend the
driver's multi-GPU bench uses.  Reference: sfnonet.py:537-555 (the sharded transform),
model.py:327-331 (the rollout step)."""
import os
import socket

import pytest
import torch

from golden_util import golden_files, load
from block_util import make_block

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module")
def rccl():
    import torch.distributed as td
    if td.is_initialized():
        pytest.skip("a process group already exists in this process")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    td.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                          device_id=torch.device("cuda", 0))
    assert td.get_backend() == "nccl"
    yield td
    td.destroy_process_group()


@pytest.mark.parametrize("chunks", [1, 3])
@pytest.mark.parametrize("name", ["c1b2_nl_film_middle.npz", "c1b2_lin_film_middle.npz"])
def test_band_block_over_rccl(rccl, name, chunks):
    from msfno_amd.sfno import LatBandBlock, TorchComm
    meta, params, arrays, _ = load([p for p in golden_files() if os.path.basename(p) == name][0])
    blk, _, _ = make_block(meta, params)
    blk = blk.to(DEV)
    reps = 3
    x = arrays["x"].to(DEV).repeat(reps, 1, 1, 1)
    g, b = arrays["gamma"].to(DEV).repeat(reps, 1), arrays["beta"].to(DEV).repeat(reps, 1)
    comm = TorchComm()
    assert not comm.host
    s = LatBandBlock(blk, 0, 1)
    with torch.no_grad():
        y = s(s.take(x), g, b, meta["scale"], comm=comm, chunks=chunks)
        torch.cuda.synchronize()
    want = arrays["y"].repeat(reps, 1, 1, 1)
    err = (LatBandBlock.assemble([s], [y]).cpu() - want).abs().max().item()
    print(f"{name} chunks={chunks} over RCCL: max-abs {err:.3e}")
    assert err < 1e-4


def test_band_net_step_graph_over_rccl(rccl):
    """LatBandNet (sharded blocks) driven over RCCL, eager and as a captured HIP graph
    replayed: the replay equals the eager step."""
    from msfno_amd.sfno import FourierNeuralOperatorNet_Filmed, LatBandNet, TorchComm
    torch.manual_seed(3)
    net = FourierNeuralOperatorNet_Filmed("cpu", None, film_layers=1, advanced_logging=False,
                                          model_depth=None, img_size=(33, 64), scale_factor=4,
                                          in_chans=5, out_chans=5, embed_dim_sfno=16,
                                          num_layers=3, filter_type="non-linear",
                                          spectral_layers=3).eval().to(DEV)
    shard = LatBandNet(net, 0, 1, comm=TorchComm(), chunks=2)
    x = shard.take(torch.randn(2, 5, 33, 64, device=DEV))
    film = 0.1 * torch.randn(2, 2, 1, 16, device=DEV)
    with torch.no_grad():
        eager = shard(x, film, 1.0).clone()
        TorchComm().quiesce()  # the watchdog has reaped the eager step's works
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            y = shard(x, film, 1.0)
        graph.replay()
        torch.cuda.synchronize()
    err = (y - eager).abs().max().item()
    print(f"band net over RCCL: graph replay vs eager max-abs {err:.3e}")
    assert torch.isfinite(eager).all()
    assert err == 0.0
