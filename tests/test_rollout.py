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


class _FilmGen(torch.nn.Module):
    """A stand-in for Film_wrapper (sfnonet.py:863-912): an inner ``film_gen``
    module, output reshaped to (B, 2, film_layers, C)."""

    def __init__(self, n_in, film_layers, C):
        super().__init__()
        self.film_layers, self.C = film_layers, C
        self.film_gen = torch.nn.Linear(n_in, 2 * film_layers * C)

    def forward(self, sst):
        return self.film_gen(sst).reshape(sst.shape[0], 2, self.film_layers, self.C)


def _small_filmed(film_layers=2, with_gen=True, n_sst=6):
    from msfno_amd.sfno import FourierNeuralOperatorNet_Filmed
    meta, params, x, y, _ = load_net(NET_FIXTURES[0])
    gen = _FilmGen(n_sst, film_layers, meta["C"]) if with_gen else None
    net = FourierNeuralOperatorNet_Filmed(
        "cpu", None, film_layers=film_layers, advanced_logging=False, model_depth=None,
        film_gen=gen, filter_type=meta["filter"], img_size=(meta["nlat"], meta["nlon"]),
        scale_factor=meta["scale_factor"], in_chans=meta["in_chans"],
        out_chans=meta["out_chans"], embed_dim_sfno=meta["C"], num_layers=meta["num_layers"],
        spectral_layers=3)
    return net, params, x, meta


def _ecmwf_style(params):
    ck = {"module." + k: v.clone() for k, v in params.items()}
    ck["module.ged"] = torch.zeros(1)
    ck["module.norm.bias"] = torch.zeros(3)
    return {"model_state": ck}


def _film_ck(gen, prefixed):
    sd = {k: v.clone() for k, v in gen.state_dict().items()}  # keys "film_gen.*"
    if not prefixed:
        sd = {k[len("film_gen."):]: v for k, v in sd.items()}
    return {"model_state": sd, "epoch": 3}


@pytest.mark.parametrize("prefixed", [False, True])
def test_filmed_checkpoint_merges_film_gen_and_freezes_sfno(prefixed):
    """model.py:983-1003 (prefix added unless present) and :1021-1023 (only film_gen
    trains)."""
    from msfno_amd.rollout import load_filmed_checkpoint
    net, params, _, meta = _small_filmed()
    src = _FilmGen(6, 2, meta["C"])
    with torch.no_grad():
        src.film_gen.weight.normal_()
    with pytest.warns(UserWarning, match="strict=False"):
        net, strict = load_filmed_checkpoint(net, _ecmwf_style(params),
                                             film_checkpoint=_film_ck(src, prefixed))
    assert not strict and not net.training
    sd = net.state_dict()
    for k, v in params.items():
        assert torch.equal(sd[k], v), k
    assert torch.equal(net.film_gen.film_gen.weight, src.film_gen.weight)
    for name, p in net.named_parameters():
        assert p.requires_grad == ("film_gen" in name), name


def test_filmed_checkpoint_retrain_film_skips_and_unfreezes_the_retrained_layers():
    """--retrain-film (model.py:922-923, 952, 1016-1019): the decoder and the
    'blocks.11 - i' layers keep their fresh weights and stay trainable, the rest
    loads and freezes.  The substring rule is the reference's: 'blocks.1' (film
    layer 10 of 11) would also match blocks.10 and blocks.11."""
    from msfno_amd.rollout import load_filmed_checkpoint, retrain_film_layers
    assert retrain_film_layers(2) == ["film_gen", "decoder", "blocks.11", "blocks.10"]
    net, params, _, meta = _small_filmed(film_layers=2)
    fresh = {k: v.clone() for k, v in net.state_dict().items()}
    # a 12-block checkpoint's trailing-block keys: present in the checkpoint, skipped
    ck = _ecmwf_style(params)
    ck["model_state"]["module.blocks.11.norm0.weight"] = torch.ones(meta["C"])
    with pytest.warns(UserWarning):
        net, _ = load_filmed_checkpoint(net, ck, retrain_film=True, film_layers=2)
    sd = net.state_dict()
    for k, v in params.items():
        if "decoder" in k:
            assert torch.equal(sd[k], fresh[k]), k      # skipped: fresh init kept
        else:
            assert torch.equal(sd[k], v), k
    for name, p in net.named_parameters():
        assert p.requires_grad == any(s in name for s in ("film_gen", "decoder",
                                                          "blocks.11", "blocks.10")), name
    # with a resume checkpoint nothing is skipped (model.py:952)
    net2, _, _, _ = _small_filmed(film_layers=2)
    with pytest.warns(UserWarning):
        net2, _ = load_filmed_checkpoint(net2, _ecmwf_style(params), retrain_film=True,
                                         film_layers=2, resume_checkpoint="resume.pt")
    for k, v in params.items():
        assert torch.equal(net2.state_dict()[k], v), k


def test_filmed_checkpoint_bad_film_weights_load_nothing_like_the_reference():
    from msfno_amd.rollout import load_filmed_checkpoint
    net, params, _, meta = _small_filmed()
    before = net.film_gen.film_gen.weight.clone()
    bad = {"model_state": {"film_gen.other.weight": torch.zeros(2, 2)}}
    with pytest.warns(UserWarning, match="Film Gen"):
        load_filmed_checkpoint(net, _ecmwf_style(params), film_checkpoint=bad)
    assert torch.equal(net.film_gen.film_gen.weight, before)


@pytest.mark.gpu
def test_filmed_ecmwf_checkpoint_runs_like_the_oracle():
    """An ECMWF-style checkpoint (module. prefix, ged, a dropped norm var, no SHT
    buffers) plus a separate FiLM-generator checkpoint loaded into a small
    FourierNeuralOperatorNet_Filmed on the GPU: the output equals
    oracle.net_forward on the same state dict and the generator's modulation."""
    from oracle import sfno_ref
    from test_oracle_net import net_cfg
    from msfno_amd.rollout import load_filmed_checkpoint
    net, params, x, meta = _small_filmed(film_layers=2)
    src = _FilmGen(6, 2, meta["C"])
    with torch.no_grad():
        src.film_gen.weight.mul_(5.0)
    with pytest.warns(UserWarning):
        net, strict = load_filmed_checkpoint(net, _ecmwf_style(params),
                                             film_checkpoint=_film_ck(src, False))
    g = torch.Generator().manual_seed(5)
    sst = torch.randn(x.shape[0], 6, generator=g)
    with torch.no_grad():
        film = src(sst)
        want = sfno_ref.net_forward(params, x, net_cfg(meta), film=(film[:, 0], film[:, 1]),
                                    scale=0.7)
        got = net.to("cuda")(x.cuda(), sst.cuda(), 0.7).cpu()
    assert (got - want).abs().max().item() < 1e-4 * max(1.0, want.abs().max().item())
