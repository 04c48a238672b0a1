"""The oracle's network restatement (oracle/sfno_ref.py:net_forward) against the
reference FourierNeuralOperatorNet outputs (tests/golden/net/, written by
tests/golden/make_golden.py from the reference's own sfnonet.py)."""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import sfno_ref

NET_FIXTURES = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "net", "*.npz")))


def load_net(path):
    d = np.load(path, allow_pickle=False)
    meta = {k[5:]: d[k].item() for k in d.files if k.startswith("meta_")}
    params = {k[3:]: torch.from_numpy(d[k]) for k in d.files if k.startswith("p__")}
    return meta, params, torch.from_numpy(d["x"]), torch.from_numpy(d["y"]), \
        [str(k) for k in d["state_dict_keys"]]


def net_cfg(meta):
    return sfno_ref.NetCfg(img_size=(meta["nlat"], meta["nlon"]), scale_factor=meta["scale_factor"],
                           num_layers=meta["num_layers"], filter_type=meta["filter"])


@pytest.mark.parametrize("path", NET_FIXTURES, ids=lambda p: os.path.basename(p)[:-4])
def test_oracle_net_matches_reference(path):
    meta, params, x, y, _ = load_net(path)
    with torch.no_grad():
        got = sfno_ref.net_forward(params, x, net_cfg(meta))
    assert got.shape == y.shape
    assert (got - y).abs().max().item() < 1e-5 * max(1.0, y.abs().max().item())


def test_net_state_dict_keys_match_reference():
    from msfno_amd.sfno import FourierNeuralOperatorNet
    meta, params, x, y, keys = load_net(NET_FIXTURES[0])
    net = FourierNeuralOperatorNet("cpu", None, filter_type=meta["filter"],
                                   img_size=(meta["nlat"], meta["nlon"]),
                                   scale_factor=meta["scale_factor"], in_chans=meta["in_chans"],
                                   out_chans=meta["out_chans"], embed_dim_sfno=meta["C"],
                                   num_layers=meta["num_layers"], spectral_layers=3)
    assert sorted(net.state_dict().keys()) == sorted(keys)
    for k, v in params.items():
        assert tuple(net.state_dict()[k].shape) == tuple(v.shape), k
