"""The network encoder / decoder MLP fused on the x3h engine (csrc/mlp_gen_h.hip:
one launch, hidden activation on-chip, per-pixel power-of-two range scales) against an
fp64 evaluation of the reference MLP (layers.py:145-178; sfnonet.py:513-523 encoder
73 -> 256 -> 256 + pos_embed, 617-629 decoder cat(x, residual) 329 -> 256 -> 73),
next to the two-GEMM x6 path it replaces (MSFNO_MLP_GEN_H=0, in a child process: the
switch is read once per process).

Error measure as tests/test_gpu_gemm_x6.py: |y - y64| / (|W2|·|GELU(W1 x + b1)| + |b2|
+ |addend|), the scale fp32 rounding works on.  Inputs span 1e-3 .. 1e3 per pixel, with
an all-zero pixel, so the per-pixel scales are exercised; P is not a multiple of the
64-pixel tile."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
HERE = os.path.dirname(os.path.abspath(__file__))


def _gelu64(x):
    return 0.5 * x * (1.0 + torch.erf(x / 2 ** 0.5))


# (Cin, Cin2, Hid, Cout, P, B, addend, output_bias)
CASES = [
    (73, 0, 256, 256, 3001, 2, "broadcast", True),   # encoder + pos_embed
    (256, 73, 256, 73, 2145, 2, None, False),        # decoder over cat(x, residual)
    (256, 73, 256, 73, 1000, 1, "batched", True),
    # the persistent encoder kernel (P % 4 == 0): 301 128-pixel tiles per field, two
    # fields -> more tiles than CUs, workgroup ranges crossing the field boundary, a
    # 36-pixel last tile
    (73, 0, 256, 256, 38436, 2, "broadcast", True),
    (73, 0, 256, 256, 38436, 2, None, False),
    (96, 0, 256, 256, 3000, 2, "batched", True),     # Ct = 96: no padded channels
    (73, 0, 256, 256, 60, 3, "broadcast", True),     # one partial 60-pixel tile per field
    (73, 0, 256, 250, 3000, 2, "batched", False),    # Cout 250: output rows past Cout dropped
]
# the persistent kernel's cases (mlp_gen_hp_kernel vs mlp_gen_h_kernel, bitwise)
PCASES = [c for c in CASES if c[1] == 0 and c[4] % 4 == 0]


def _case(Cin, Cin2, Hid, Cout, P, B, addend, bias, seed):
    got, y64, scale = _run(Cin, Cin2, Hid, Cout, P, B, addend, bias, seed)
    return ((got - y64).abs() / scale).max().item(), (got - y64).abs().max().item()


def _run(Cin, Cin2, Hid, Cout, P, B, addend, bias, seed):
    from msfno_amd.sfno import MLP
    torch.manual_seed(seed)
    m = MLP(in_features=Cin + Cin2, hidden_features=Hid, out_features=Cout,
            output_bias=bias).eval()
    with torch.no_grad():
        for p in m.parameters():
            p.copy_(torch.randn_like(p) / p.shape[1] ** 0.5 if p.dim() > 1 else 0.1 * torch.randn_like(p))
    # per-pixel magnitudes 1e-3 .. 1e3, one all-zero pixel
    mag = 10.0 ** (6 * torch.rand(B, 1, 1, P) - 3)
    x = torch.randn(B, Cin, 1, P) * mag
    x[:, :, :, 7] = 0
    x2 = torch.randn(B, Cin2, 1, P) * mag if Cin2 else None
    add = None
    if addend == "broadcast":
        add = torch.randn(1, Cout, 1, P)
    elif addend == "batched":
        add = torch.randn(B, Cout, 1, P)
    sd = {k: v.double() for k, v in m.fwd.state_dict().items()}
    W1, b1 = sd["0.weight"][:, :, 0, 0], sd["0.bias"]
    W2 = sd["2.weight"][:, :, 0, 0]
    b2 = sd["2.bias"] if bias else torch.zeros(Cout, dtype=torch.float64)
    xd = x.double()[:, :, 0, :]
    if Cin2:
        xd = torch.cat([xd, x2.double()[:, :, 0, :]], 1)
    h = _gelu64(torch.einsum("oi,bip->bop", W1, xd) + b1[None, :, None])
    y64 = torch.einsum("oi,bip->bop", W2, h) + b2[None, :, None]
    scale = torch.einsum("oi,bip->bop", W2.abs(), h.abs()) + b2.abs()[None, :, None]
    if add is not None:
        y64 = y64 + add.double()[:, :, 0, :]
        scale = scale + add.double().abs()[:, :, 0, :]
    with torch.no_grad():
        got = m.to(DEV).native_forward(
            x.to(DEV), x2=None if x2 is None else x2.to(DEV),
            addend=None if add is None else add.to(DEV)).double().cpu()[:, :, 0, :]
    assert torch.isfinite(got).all()
    return got, y64, scale


def _errors():
    return [_case(*c, seed=i) for i, c in enumerate(CASES)]


def test_fused_x3h_mlp_matches_fp64_like_x6():
    gen = _errors()
    env = dict(os.environ, MSFNO_MLP_GEN_H="0")
    out = subprocess.run([sys.executable, os.path.abspath(__file__)], env=env, cwd=HERE,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    x6 = json.loads(out.stdout.strip().splitlines()[-1])
    for c, (rg, ag), (rx, ax) in zip(CASES, gen, x6):
        print(f"{c[:6]}: x3h fused rel {rg:.2e} abs {ag:.2e} | x6 two-GEMM rel {rx:.2e} abs {ax:.2e}")
        assert rg < 2e-6, c
        assert rg < 4 * rx + 1e-7, c


@pytest.mark.parametrize("env", [{"MSFNO_MG_P": "0"}, {"MSFNO_MG_PG": "1"}, {"MSFNO_MG_EARLY": "0"}],
                         ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
def test_kernel_variants_equal_default_bitwise(tmp_path, env):
    """mlp_gen_hp_kernel (persistent, pipelined; the default for the encoder shape, PCASES)
    does each output element's arithmetic in the order mlp_gen_h_kernel does, at either
    pixel-group count, and the tile kernel's early addend loads change no arithmetic: every
    case agrees bit for bit with the child process's variant (MSFNO_MG_P=0: the
    one-tile-per-workgroup kernel; MSFNO_MG_PG=1: one 16-pixel group per wave, 8 waves;
    MSFNO_MG_EARLY=0: the addend loaded under the last unit's MFMAs)."""
    dump = tmp_path / "variant.pt"
    out = subprocess.run([sys.executable, os.path.abspath(__file__), "--dump", str(dump)],
                         env=dict(os.environ, **env), cwd=HERE, capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    ref = torch.load(dump, weights_only=True)
    for i, c in enumerate(CASES):
        got = _run(*c, seed=i)[0]
        nd = (got != ref[i]).sum().item()
        print(f"{c[:6]}: {nd} of {got.numel()} differ, max-abs {(got - ref[i]).abs().max().item():.3e}")
        assert nd == 0, c


def test_fused_mlp_stage_is_the_fused_kernel():
    """The stage profiler sees one `mlp_gen` launch per call on the fused path (the
    x6 path records mlp_fc1 / mlp_fc2)."""
    from msfno_amd import _native as N
    from msfno_amd.sfno import MLP
    m = MLP(in_features=73, hidden_features=256, out_features=256).eval().to(DEV)
    x = torch.randn(1, 73, 8, 130, device=DEV)
    N.profile_enable(True)
    try:
        N.profile_collect()
        with torch.no_grad():
            m.native_forward(x)
        st = N.profile_collect()
    finally:
        N.profile_enable(False)
    assert st.get("mlp_gen", (0, 0))[1] == 1 and "mlp_fc1" not in st, st


def test_deferred_last_block_affine_equals_separate_pass():
    """The network's last block (no MLP, no outer skip) leaves its norm1 + FiLM affine to
    the decoder (msfno_block_forward_deferred -> msfno_mlp_forward_affine); the output
    must equal running the block's own affine pass and the plain decoder."""
    from msfno_amd.sfno import FourierNeuralOperatorNet_Filmed
    torch.manual_seed(5)
    net = FourierNeuralOperatorNet_Filmed("cpu", None, film_layers=1, advanced_logging=False,
                                          model_depth=None, img_size=(121, 240), scale_factor=4,
                                          in_chans=73, out_chans=73, embed_dim_sfno=256,
                                          num_layers=3, filter_type="non-linear",
                                          spectral_layers=3).eval()
    with torch.no_grad():
        for k, v in net.state_dict().items():
            if k.endswith("norm1.weight"):
                v.copy_(1.0 + 0.2 * torch.randn_like(v))
            elif k.endswith("norm1.bias"):
                v.copy_(0.1 * torch.randn_like(v))
    net = net.to(DEV)
    x = torch.randn(2, 73, 121, 240, device=DEV)
    mod = 0.1 * torch.randn(2, 2, 1, 256, device=DEV)
    with torch.no_grad():
        assert net._fuse_last_affine(x)
        got = net(x, mod, 1.0)
        h = net.pos_drop(net.encode(x))
        for i, blk in enumerate(net.blocks):
            h = blk(h, mod[:, 0, 0], mod[:, 1, 0], 1.0) if net._filmed(i) else blk(h)
        want = net.decode(h, x)
    err = (got - want).abs().max().item()
    print(f"deferred affine: max-abs {err:.3e}, {(got != want).sum().item()} of {got.numel()} differ")
    assert err <= 1e-6 * want.abs().max().item()


if __name__ == "__main__":
    sys.path.insert(0, HERE)
    import conftest  # noqa: F401  (puts the package on sys.path)
    if len(sys.argv) > 2 and sys.argv[1] == "--dump":
        torch.save([_run(*c, seed=i)[0] for i, c in enumerate(CASES)], sys.argv[2])
    else:
        print(json.dumps(_errors()))
