"""Checkpoint loading (model.py:206-271 semantics) and the rollout driver
(model.py:289-372 without GRIB I/O).  CPU tests cover the loader and the
normalisation; the GPU test checks on-device stepping (graph and eager) against
repeated forward calls."""
import io

import pytest
import torch

from test_oracle_net import NET_FIXTURES, load_net


def _small_net():
    from msfno_amd.sfno import FourierNeuralOperatorNet
    meta, params, x, y, _ = load_net(NET_FIXTURES[0])
    net = FourierNeuralOperatorNet("cpu", None, filter_type=meta["filter"],
                                   img_size=(meta["nlat"], meta["nlon"]),
                                   scale_factor=meta["scale_factor"], in_chans=meta["in_chans"],
                                   out_chans=meta["out_chans"], embed_dim_sfno=meta["C"],
                                   num_layers=meta["num_layers"], spectral_layers=3)
    return net, params, x, meta


def test_load_checkpoint_module_prefix_drop_vars_and_missing_buffers():
    from msfno_amd.rollout import load_checkpoint
    net, params, _, _ = _small_net()
    # an ECMWF-style checkpoint: DDP prefix, a 'ged' entry, the dropped norm
    # vars and no SHT buffers (so the strict load fails and falls back)
    ck = {"module." + k: v.clone() for k, v in params.items()}
    ck["module.ged"] = torch.zeros(1)
    ck["module.norm.weight"] = torch.ones(3)
    buf = io.BytesIO()
    torch.save({"model_state": ck}, buf)
    buf.seek(0)
    with pytest.warns(UserWarning, match="strict=False"):
        net, strict = load_checkpoint(net, buf)
    assert not strict and not net.training
    sd = net.state_dict()
    for k, v in params.items():
        assert torch.equal(sd[k], v), k


def test_load_checkpoint_strict_when_complete():
    from msfno_amd.rollout import load_checkpoint
    net, params, _, _ = _small_net()
    full = {k: v.clone() for k, v in net.state_dict().items()}
    full.update(params)
    net2, strict = load_checkpoint(_small_net()[0], full)
    assert strict
    assert torch.equal(net2.state_dict()["pos_embed"], params["pos_embed"])


def test_normalise_round_trip():
    from msfno_amd.rollout import Rollout
    g = torch.Generator().manual_seed(0)
    means = torch.randn(1, 5, 1, 1, generator=g)
    stds = torch.rand(1, 5, 1, 1, generator=g) + 0.5
    r = Rollout(None, means, stds)
    x = torch.randn(2, 5, 4, 6, generator=g)
    assert torch.allclose(r.normalise(r.normalise(x), reverse=True), x, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("graph", [False, True])
def test_rollout_matches_repeated_forward(graph):
    from msfno_amd.rollout import Rollout
    net, params, x, meta = _small_net()
    net.load_state_dict(params, strict=False)
    net = net.eval().to("cuda")
    g = torch.Generator().manual_seed(1)
    means = torch.randn(1, meta["in_chans"], 1, 1, generator=g).cuda()
    stds = (torch.rand(1, meta["in_chans"], 1, 1, generator=g) + 0.5).cuda()
    x0 = x.cuda() * stds + means
    r = Rollout(net, means, stds, graph=graph)
    outs = [o.clone() for _, o in r.run(x0, 3)]
    with torch.no_grad():
        s = (x0 - means) / stds
        for i in range(3):
            s = net(s)
            want = s * stds + means
            assert (outs[i] - want).abs().max().item() < 1e-5 * max(1.0, want.abs().max().item())
