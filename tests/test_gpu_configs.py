"""GPU parity at the BASELINE.json configurations the golden fixtures cannot hold.

* Linear spectral filter at C=256 (the north-star "per-(l,m) complex spectral
  weight multiply", SpectralConvS2, layers.py:336-427 / contractions.py:37-41):
  the whole block on a 91x180 grid (lmax 45: a 0.54 GB weight the host oracle
  can hold) against the oracle, and the C=256, lmax=360 contraction itself (34 GB
  per-mode weight, drawn on the device) on a sample of modes against an fp64
  einsum of those modes, at the batch sizes that select each kernel variant.
* Config 3 at its real geometry: the 12-block FourierNeuralOperatorNet_Filmed
  (721x1440 equiangular -> 120x240 Legendre-Gauss lmax 120 -> back, C=256,
  73 channels, FiLM on the last block; sfnonet.py:699-860) against
  oracle.sfno_ref.net_forward on the host.
* Config 5 in shape: a 112-step autoregressive rollout (model.py:289-372) of a
  12-block, 73-channel filmed network, stepped by msfno_amd.rollout.Rollout
  (HIP-graph replay) and by the oracle, compared along the whole trajectory.
  The grid is reduced (121x240 -> 30x60) so the host oracle finishes in
  seconds; config 5's 721x1440 geometry per step is config 3's test.

Bar: max-abs < 1e-4 * max(1, |y|) (the north-star tolerance) unless stated."""
import pytest
import torch

from oracle import sfno_ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _threads():
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))


def _block(p, cfg, C, nlat, nlon, lmax, mmax):
    from functools import partial

    from msfno_amd.harmonics import InverseRealSHT, RealSHT
    from msfno_amd.sfno import FourierNeuralOperatorBlock_Filmed
    sht = RealSHT(nlat, nlon, lmax=lmax, mmax=mmax, grid="equiangular").float()
    isht = InverseRealSHT(nlat, nlon, lmax=lmax, mmax=mmax, grid="equiangular").float()
    sht.weights = sht.weights * 1e5
    isht.pct = isht.pct / 1e5
    norm = partial(torch.nn.InstanceNorm2d, num_features=C, eps=1e-6, affine=True,
                   track_running_stats=False)
    blk = FourierNeuralOperatorBlock_Filmed(sht, isht, C, filter_type=cfg.filter_type,
                                            mlp_ratio=2.0, norm_layer=(norm, norm),
                                            inner_skip=cfg.inner_skip, outer_skip=cfg.outer_skip,
                                            mlp_mode="distributed" if cfg.has_mlp else "none",
                                            spectral_layers=3)
    blk.load_state_dict(p, strict=False)
    return blk.eval().to(DEV)


@pytest.mark.parametrize("B", [1, 2])
def test_linear_filter_block_c256_matches_oracle(B):
    """Linear filter, C=256, 91x180 lmax 45: the full filmed block vs the oracle."""
    _threads()
    C, nlat, nlon, lmax, mmax = 256, 91, 180, 45, 46
    cfg = sfno_ref.BlockCfg(filter_type="linear")
    p = sfno_ref.make_block_params(C, lmax, mmax, cfg, seed=5, randomize_affine=True)
    g = torch.Generator().manual_seed(6)
    x = torch.randn(B, C, nlat, nlon, generator=g)
    gamma = 0.1 * torch.randn(B, C, generator=g)
    beta = 0.1 * torch.randn(B, C, generator=g)
    blk = _block(p, cfg, C, nlat, nlon, lmax, mmax)
    with torch.no_grad():
        y = blk(x.to(DEV), gamma.to(DEV), beta.to(DEV), 0.9).cpu()
    o_sht, o_isht = sfno_ref.make_transforms(nlat, nlon, lmax, mmax)
    with torch.no_grad():
        want = sfno_ref.block_forward(p, x, o_sht, o_isht, cfg, gamma, beta, 0.9)
    err = (y - want).abs().max().item()
    print(f"linear C=256 91x180 B={B}: max-abs {err:.3e} |y|max {want.abs().max():.3f}")
    assert err < 1e-4 * max(1.0, want.abs().max().item())


@pytest.fixture(scope="module")
def lmax360_weight():
    """The C=256, lmax=360 per-mode weight (C, C, T, 2), T = |tril(360, 361)| =
    64980: 34.1 GB, drawn on the device with the reference init 0.02*randn
    (layers.py:386-387)."""
    C, T = 256, 360 * 361 // 2
    g = torch.Generator(device=DEV).manual_seed(11)
    w = torch.empty(C, C, T, 2, device=DEV)
    for i in range(C):  # row by row: keeps the generator's temporaries small
        w[i] = 0.02 * torch.randn(C, T, 2, generator=g, device=DEV)
    yield w
    del w
    torch.cuda.empty_cache()


@pytest.mark.parametrize("B", [1, 2, 8])
def test_linear_contraction_c256_lmax360_sampled_modes(lmax360_weight, B):
    """msfno_compl_contract_fwd_c at the config-2 size (the block's linear-filter
    kernel: the LDS-DMA weight stream at B=1, the batched register kernels at
    B=2 / 8) on 97 sampled modes, including the first and last, against an fp64
    einsum of those modes."""
    from msfno_amd.sfno.contractions import compl_contract_fwd_c
    w = lmax360_weight
    C, T = w.shape[0], w.shape[2]
    g = torch.Generator(device=DEV).manual_seed(12 + B)
    a = torch.randn(B, C, T, 2, generator=g, device=DEV)
    y = compl_contract_fwd_c(a, w)
    torch.cuda.synchronize()
    gi = torch.Generator().manual_seed(13)
    modes = torch.cat((torch.tensor([0, 1, T - 2, T - 1]),
                       torch.randint(2, T - 2, (93,), generator=gi))).to(DEV)
    ac = torch.view_as_complex(a[:, :, modes].double().contiguous())
    wc = torch.view_as_complex(w[:, :, modes].double().contiguous())
    want = torch.view_as_real(torch.einsum("bin,kin->bkn", ac, wc))
    got = y[:, :, modes].double()
    err = (got - want).abs().max().item()
    scale = want.abs().max().item()
    print(f"contract C=256 T={T} B={B}: max-abs {err:.3e} |y|max {scale:.3f}")
    assert err < 2e-6 * max(1.0, scale)


def test_config3_net_matches_oracle():
    """Config 3: 12-block FourierNeuralOperatorNet_Filmed at 721x1440, C=256, 73
    channels, film_layers 1 (the reference default), against the oracle."""
    from msfno_amd.sfno import FourierNeuralOperatorNet_Filmed
    _threads()
    torch.manual_seed(21)
    net = FourierNeuralOperatorNet_Filmed("cpu", None, film_layers=1, advanced_logging=False,
                                          model_depth=None, img_size=(721, 1440), in_chans=73,
                                          out_chans=73, embed_dim_sfno=256, num_layers=12,
                                          filter_type="non-linear", spectral_layers=3).eval()
    # reference-shaped parameters: the oracle takes the same state-dict keys
    params = {k: v.detach().clone() for k, v in net.state_dict().items()
              if not k.endswith((".weights", ".pct"))}
    g = torch.Generator().manual_seed(22)
    with torch.no_grad():  # non-trivial norms / biases / position embedding
        for k, v in params.items():
            if k.endswith("norm0.weight") or k.endswith("norm1.weight"):
                v.copy_(1.0 + 0.1 * torch.randn(v.shape, generator=g))
            elif k.endswith(".bias") or k == "pos_embed":
                v.copy_(0.02 * torch.randn(v.shape, generator=g))
    net.load_state_dict(params, strict=False)
    net = net.to(DEV)
    x = torch.randn(1, 73, 721, 1440, generator=g)
    gamma = 0.1 * torch.randn(1, 1, 256, generator=g)
    beta = 0.1 * torch.randn(1, 1, 256, generator=g)
    with torch.no_grad():
        got = net(x.to(DEV), torch.stack((gamma, beta), dim=1).to(DEV), 1.0).cpu()
    del net
    torch.cuda.empty_cache()
    ncfg = sfno_ref.NetCfg(img_size=(721, 1440), scale_factor=6, num_layers=12)
    with torch.no_grad():
        want = sfno_ref.net_forward(params, x, ncfg, film=(gamma, beta), scale=1.0)
    err = (got - want).abs().max().item()
    rms = (got - want).pow(2).mean().sqrt().item()
    print(f"config3 net: max-abs {err:.3e} rms {rms:.3e} |y|max {want.abs().max():.3f}")
    assert got.shape == want.shape == (1, 73, 721, 1440)
    assert err < 1e-4 * max(1.0, want.abs().max().item())


@pytest.mark.parametrize("graph", [True, False])
def test_rollout_112_steps_matches_oracle(graph):
    """Config 5 in shape: 112 six-hour steps (28 days) of a 12-block, 73-channel
    filmed network with normalisation (model.py:273-279), on the device, against
    the oracle iterated on the host.  Every 8th step and the last are compared;
    the rollout's outputs are collected without cloning (each must be its own
    tensor)."""
    from msfno_amd.rollout import Rollout
    from msfno_amd.sfno import FourierNeuralOperatorNet_Filmed
    _threads()
    img, sf, C, ch, steps = (121, 240), 4, 32, 73, 112
    torch.manual_seed(31)
    net = FourierNeuralOperatorNet_Filmed("cpu", None, film_layers=1, advanced_logging=False,
                                          model_depth=None, img_size=img, scale_factor=sf,
                                          in_chans=ch, out_chans=ch, embed_dim_sfno=C,
                                          num_layers=12, filter_type="non-linear",
                                          spectral_layers=3).eval()
    # decoder weights x6.5 over the reference init: with init-scale weights the state
    # collapses to a fixed point within a few steps (a vacuous comparison); at x6.5
    # it keeps moving at O(1) amplitude for all 112 steps without blowing up
    params = {k: (6.5 * v if k.startswith("decoder.") and k.endswith("weight") else v)
              for k, v in net.state_dict().items() if not k.endswith((".weights", ".pct"))}
    net.load_state_dict(params, strict=False)
    net = net.to(DEV)
    g = torch.Generator().manual_seed(32)
    means = torch.randn(1, ch, 1, 1, generator=g)
    stds = torch.rand(1, ch, 1, 1, generator=g) + 0.5
    x0 = torch.randn(1, ch, *img, generator=g) * stds + means
    film = 0.1 * torch.randn(1, 2, 1, C, generator=g)
    r = Rollout(net, means.to(DEV), stds.to(DEV), film=film.to(DEV), scale=1.0, graph=graph)
    outs = [o for _, o in r.run(x0.to(DEV), steps)]
    assert len({o.data_ptr() for o in outs}) == steps
    ncfg = sfno_ref.NetCfg(img_size=img, scale_factor=sf, num_layers=12)
    tr = sfno_ref.make_net_transforms(ncfg)
    check = set(range(0, steps, 8)) | {steps - 1}
    worst = 0.0
    with torch.no_grad():
        s = (x0 - means) / stds
        for i in range(steps):
            s = sfno_ref.net_forward(params, s, ncfg, transforms=tr,
                                     film=(film[:, 0], film[:, 1]), scale=1.0)
            if i in check:
                want = s * stds + means
                err = (outs[i].cpu() - want).abs().max().item() / max(1.0, want.abs().max().item())
                worst = max(worst, err)
                assert err < 1e-4, (i, err)
    print(f"rollout {steps} steps (graph={graph}): worst relative max-abs {worst:.3e}")


def test_config5_geometry_sharded_rollout_eight_ranks():
    """Config 5's multi-GPU form at its real geometry: the 12-block filmed network
    (721x1440 -> 120x240 -> 721x1440, C=256, 73 channels) latitude-band sharded over 8
    lock-step virtual ranks (LatBandNet), stepped autoregressively 3 times, against
    the unsharded network stepped the same way."""
    from msfno_amd.sfno import FourierNeuralOperatorNet_Filmed, LatBandBlock, LatBandNet, LocalGroup
    torch.manual_seed(31)
    net = FourierNeuralOperatorNet_Filmed("cpu", None, film_layers=1, advanced_logging=False,
                                          model_depth=None, img_size=(721, 1440), in_chans=73,
                                          out_chans=73, embed_dim_sfno=256, num_layers=12,
                                          filter_type="non-linear", spectral_layers=3).eval().to(DEV)
    g = torch.Generator().manual_seed(32)
    x = torch.randn(1, 73, 721, 1440, generator=g).to(DEV)
    film = torch.stack((0.1 * torch.randn(1, 1, 256, generator=g),
                        0.1 * torch.randn(1, 1, 256, generator=g)), dim=1).to(DEV)
    shards = [LatBandNet(net, r, 8) for r in range(8)]
    with torch.no_grad():
        want = x
        parts = [s.take(x) for s in shards]
        for _ in range(3):
            want = net(want, film, 1.0)
            parts = LocalGroup.run([s.stages(p, film, 1.0) for s, p in zip(shards, parts)])
        got = LatBandBlock.assemble([s.shards[-1] for s in shards], parts)
    err = (got - want).abs().max().item()
    assert err < 1e-4 * max(1.0, want.abs().max().item()), err


def _bench_block(filter_type="non-linear"):
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    args = bench.parse_args(["--filter", filter_type])
    blk, _, _ = bench.build_block(args, torch.device(DEV))
    return blk


def _sharded_pipelined(blk, x, gamma, beta, scale, world, chunks):
    """`world` lock-step virtual ranks, each running the sub-batch pipeline of
    LatBandBlock.forward(chunks=K) (LocalGroup.run_pipelined: the stages enqueued in
    the same interleaved order as on a real rank)."""
    from msfno_amd.sfno import LatBandBlock, LocalGroup
    shards = [LatBandBlock(blk, r, world) for r in range(world)]
    outs, gens = [], []
    for s in shards:
        o, g = s.chunk_stages(s.take(x), gamma, beta, scale, chunks)
        outs.append(o)
        gens.append(g)
    LocalGroup.run_pipelined(gens)
    return LatBandBlock.assemble(shards, outs)


def test_config4_batch8_eight_ranks_pipelined():
    """Config 4 at its workload: 721x1440, C=256, lmax 360, a batch of 8 fields
    latitude-band sharded over 8 lock-step virtual ranks with the bench's sub-batch
    pipeline (chunks=4: four slots in flight, exchanges interleaved with the other
    sub-batches' stages), against the unsharded block on the same batch."""
    blk = _bench_block()
    gen = torch.Generator(device=DEV).manual_seed(40)
    x = torch.randn(8, 256, 721, 1440, generator=gen, device=DEV)
    g = 0.1 * torch.randn(8, 256, generator=gen, device=DEV)
    b = 0.1 * torch.randn(8, 256, generator=gen, device=DEV)
    with torch.no_grad():
        y1 = blk(x, g, b, 1.0)
        y = _sharded_pipelined(blk, x, g, b, 1.0, 8, 4)
    assert torch.isfinite(y).all()
    err = (y - y1).abs().max().item()
    print(f"config4 B=8 8 ranks chunks=4: max-abs vs unsharded {err:.3e}")
    assert err < 2e-5, err


def test_linear_block_full_grid_c256_properties():
    """The linear filter block at config 2's full size (721x1440, C=256, lmax 360, the
    34 GB per-mode weight): the host oracle cannot hold it, so size-independent
    properties: finite; batch consistency (a batch of 2 equals each field alone: the
    B=1 LDS-DMA weight stream and the batched kernel agree); and 8 lock-step virtual
    ranks (weight sharded by m-set) against the unsharded block."""
    blk = _bench_block("linear")
    gen = torch.Generator(device=DEV).manual_seed(41)
    x = torch.randn(2, 256, 721, 1440, generator=gen, device=DEV)
    g = 0.1 * torch.randn(2, 256, generator=gen, device=DEV)
    b = 0.1 * torch.randn(2, 256, generator=gen, device=DEV)
    with torch.no_grad():
        y2 = blk(x, g, b, 1.0)
        assert torch.isfinite(y2).all()
        scale = max(1.0, y2.abs().max().item())
        for i in range(2):
            y1 = blk(x[i:i + 1], g[i:i + 1], b[i:i + 1], 1.0)
            err = (y1[0] - y2[i]).abs().max().item()
            assert err < 2e-5 * scale, (i, err)
        del y1
        ys = _sharded_pipelined(blk, x, g, b, 1.0, 8, 2)
    err = (ys - y2).abs().max().item()
    print(f"linear C=256 721x1440: sharded-8 vs unsharded {err:.3e} |y|max {scale:.3f}")
    assert err < 2e-5 * scale, err


def test_config5_112_steps_full_geometry():
    """Config 5 at its workload geometry: 112 six-hour steps (28 days) of the
    12-block filmed network at 721x1440 (blocks on the 120x240 Gauss grid), C=256,
    73 channels, with normalisation.  The HIP-graph replayed Rollout is compared
    with eager stepping at every 8th step and the last, and the network
    latitude-band sharded over 8 lock-step virtual ranks (LatBandNet) with one step
    from the same state at each of them plus 9 free-running steps (bar 1e-4 *
    max(1, |y|)).  Decoder weights x2: at this geometry the state then
    keeps moving by O(|y|) per step with |y|max ~ 8-10 for all 112 steps (gain 1
    settles to a fixed point, gain 6.5 grows x1.45 per step to 1e20; scan:
    tools/c5_gain.py, profiles/r03_v2/c5_gain.txt) — both checked below."""
    from msfno_amd.rollout import Rollout
    from msfno_amd.sfno import FourierNeuralOperatorNet_Filmed, LatBandBlock, LatBandNet, LocalGroup
    steps, ch = 112, 73
    torch.manual_seed(51)
    net = FourierNeuralOperatorNet_Filmed("cpu", None, film_layers=1, advanced_logging=False,
                                          model_depth=None, img_size=(721, 1440), in_chans=ch,
                                          out_chans=ch, embed_dim_sfno=256, num_layers=12,
                                          filter_type="non-linear", spectral_layers=3).eval()
    with torch.no_grad():
        for k, v in net.decoder.state_dict().items():
            if k.endswith("weight"):
                v.mul_(2.0)
    net = net.to(DEV)
    g = torch.Generator(device=DEV).manual_seed(52)
    means = torch.randn(1, ch, 1, 1, generator=g, device=DEV)
    stds = torch.rand(1, ch, 1, 1, generator=g, device=DEV) + 0.5
    x0 = torch.randn(1, ch, 721, 1440, generator=g, device=DEV) * stds + means
    film = 0.1 * torch.randn(1, 2, 1, 256, generator=g, device=DEV)
    check = sorted(set(range(0, steps, 8)) | {steps - 1})
    keep = set(check) | {i - 1 for i in check if i > 0}

    def collect(r, x):
        out, prev, moved = {}, None, []
        for i, y in r.run(x, steps):
            if prev is not None:
                moved.append((y - prev).abs().max().item())
            prev = y
            if i in keep:
                out[i] = y.clone()
        return out, moved

    with torch.no_grad():
        ref, moved = collect(Rollout(net, means, stds, film=film, graph=True), x0)
        eager, _ = collect(Rollout(net, means, stds, film=film, graph=False), x0)
        # the state must keep moving (no fixed point) for the comparison to mean anything
        assert min(moved[-16:]) > 1e-3, moved[-16:]
        assert max(v.abs().max().item() for v in ref.values()) < 1e3  # bounded, not blowing up
        shards = [LatBandNet(net, r, 8) for r in range(8)]

        def band_step(x):
            parts = [(s.take(x) - means) / stds for s in shards]
            parts = LocalGroup.run([s.stages(p, film, 1.0) for s, p in zip(shards, parts)])
            return LatBandBlock.assemble([s.shards[-1] for s in shards], parts) * stds + means

        # the sharded network stepped from the unsharded state at every checked step
        # (teacher forcing: the trajectory moves by O(|y|) per step, so two arithmetics
        # that differ in rounding, e.g. the band exchange's k-order, part ways after a
        # few dozen free-running steps), then 8 free-running sharded steps
        worst = 0.0
        for i in check:
            sc = max(1.0, ref[i].abs().max().item())
            e_eager = (eager[i] - ref[i]).abs().max().item() / sc
            e_band = (band_step(ref[i - 1] if i > 0 else x0) - ref[i]).abs().max().item() / sc
            worst = max(worst, e_eager, e_band)
            print(f"config5 step {i}: eager {e_eager:.3e} band (1 step) {e_band:.3e} "
                  f"|y|max {sc:.3e}", flush=True)
            assert e_eager < 1e-4 and e_band < 1e-4, (i, e_eager, e_band)
        parts = [(s.take(x0) - means) / stds for s in shards]
        for i in range(9):
            parts = LocalGroup.run([s.stages(p, film, 1.0) for s, p in zip(shards, parts)])
        y = LatBandBlock.assemble([s.shards[-1] for s in shards], parts) * stds + means
        e_free = (y - ref[8]).abs().max().item() / max(1.0, ref[8].abs().max().item())
        print(f"config5 band free-running 9 steps: {e_free:.3e}")
        assert e_free < 1e-4, e_free
    print(f"config5 112 steps 721x1440: worst relative max-abs {worst:.3e}, "
          f"last-step change {moved[-1]:.3e}")
