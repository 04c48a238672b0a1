"""FiLM backward: gradients of a loss with respect to the
FiLM modulation (gamma, beta), every SFNO weight frozen, as MSFNO fine-tunes its
FiLM generator (sfnonet.py:787-860: the filmed blocks and the decoder run with
autograd, the blocks before them under no_grad).

The native backward (msfno_block_film_backward / msfno_mlp_backward_input,
through the torch.autograd.Functions of msfno_amd) is checked against torch
autograd through the oracle restatement in fp64 on the CPU, on the reference's
golden block parameters (both filters, middle wiring with the channel MLP and
last wiring without it) and on a small FourierNeuralOperatorNet_Filmed
(film_layers = 1).  Tolerance: max-abs < 1e-4 x max|grad|."""
import os

import pytest
import torch

from block_util import make_block
from golden_util import golden_files, load, wiring_cfg
from oracle import sfno_ref
from oracle import sht_ref as S
from test_oracle_net import NET_FIXTURES, load_net, net_cfg

pytestmark = pytest.mark.gpu
DEV = "cuda"

FILM_CASES = [p for p in golden_files()
              if "_film_" in os.path.basename(p) and "_first" not in os.path.basename(p)]


def _oracle_transforms(meta):
    sht, isht = sfno_ref.make_transforms(meta["nlat"], meta["nlon"], meta["lmax"], meta["mmax"],
                                         meta["grid"], dtype=torch.float64)
    if "out_nlat" in meta:
        isht = S.InverseRealSHT(meta["out_nlat"], meta["out_nlon"], lmax=meta["lmax"],
                                mmax=meta["mmax"], grid=meta["out_grid"]).to(torch.float64)
        isht.pct = isht.pct / 1e5
    return sht, isht


@pytest.mark.parametrize("path", FILM_CASES, ids=lambda p: os.path.basename(p)[:-4])
def test_block_film_grads_match_oracle_autograd(path):
    meta, params, arrays, _ = load(path)
    blk, _, _ = make_block(meta, params)
    blk = blk.to(DEV)
    x, scale = arrays["x"], float(meta["scale"])
    g = torch.Generator().manual_seed(11)
    gamma0, beta0 = arrays["gamma"], arrays["beta"]
    # GPU: native forward + native FiLM backward through autograd
    gamma = gamma0.clone().to(DEV).requires_grad_()
    beta = beta0.clone().to(DEV).requires_grad_()
    y = blk(x.to(DEV), gamma, beta, scale)
    dout = torch.randn(y.shape, generator=g)
    (y * dout.to(DEV)).sum().backward()
    # oracle: torch autograd in fp64
    inner, outer, has_mlp = wiring_cfg(meta)
    cfg = sfno_ref.BlockCfg(filter_type=meta["filter"], inner_skip=inner, outer_skip=outer,
                            has_mlp=has_mlp)
    pd = {k: (v.double() if v.is_floating_point() else v) for k, v in params.items()}
    sht, isht = _oracle_transforms(meta)
    gd = gamma0.double().requires_grad_()
    bd = beta0.double().requires_grad_()
    yd = sfno_ref.block_forward(pd, x.double(), sht, isht, cfg, gd, bd, scale)
    (yd * dout.double()).sum().backward()
    for got, want in ((gamma.grad, gd.grad), (beta.grad, bd.grad)):
        got = got.cpu().double()
        assert got.shape == want.shape
        tol = 1e-4 * max(want.abs().max().item(), 1e-6)
        assert (got - want).abs().max().item() < tol, ((got - want).abs().max().item(), tol)


@pytest.mark.parametrize("path", NET_FIXTURES, ids=lambda p: os.path.basename(p)[:-4])
def test_filmed_net_film_grads_match_oracle_autograd(path):
    """film_layers = 1 (the reference default): the gradient reaches (gamma, beta)
    of the last block through the frozen decoder over cat(x, residual)."""
    from test_gpu_net import _build
    meta, params, x, _, _ = load_net(path)
    net = _build(meta, params, filmed=True, film_layers=1)
    B, C = x.shape[0], meta["C"]
    g = torch.Generator().manual_seed(5)
    film0 = 0.1 * torch.randn(B, 2, 1, C, generator=g)
    film = film0.clone().to(DEV).requires_grad_()
    y = net(x.to(DEV), film, 0.8)
    w = torch.randn(y.shape, generator=g)
    (y * w.to(DEV)).sum().backward()
    pd = {k: (v.double() if v.is_floating_point() else v) for k, v in params.items()}
    fd = film0.double().requires_grad_()
    cfg = net_cfg(meta)
    yd = sfno_ref.net_forward(pd, x.double(), cfg, sfno_ref.make_net_transforms(cfg, torch.float64),
                              film=(fd[:, 0], fd[:, 1]), scale=0.8)
    (yd * w.double()).sum().backward()
    got, want = film.grad.cpu().double(), fd.grad
    assert (got - want).abs().max().item() < 1e-4 * want.abs().max().item()


def test_filmed_block_refuses_input_gradient():
    """dL/dx through a filmed block (film_layers > 1) is not on the MI355X path:
    it raises instead of returning a wrong gradient."""
    path = [p for p in FILM_CASES if os.path.basename(p) == "c1_nl_film_middle.npz"][0]
    meta, params, arrays, _ = load(path)
    blk, _, _ = make_block(meta, params)
    blk = blk.to(DEV)
    x = arrays["x"].to(DEV).requires_grad_()
    y = blk(x, arrays["gamma"].to(DEV), arrays["beta"].to(DEV), 1.0)
    with pytest.raises(NotImplementedError):
        y.sum().backward()
