"""Co-residency: a kernel must give bit-identical results whether or not
MFMA work of another stream shares its CUs.

Round 4 found the row FFT of the 120 x 240 blocks corrupted (real parts of bins 57..63)
whenever skip_h_kernel ran beside it.  The cause: on gfx950 a packed-FP32 VALU op
(v_pk_add/mul/fma_f32) whose src1 feeds the low lane from its high half (op_sel:[0,1])
returns wrong low results in lanes 48..63 while another wave's MFMAs execute on the CU
(tools/gen_pk_opsel_sweep.py, profiles/r05_pk/).  The FFT and spectral units are built
without packed FP32 (csrc/Makefile) and tests/test_isa_audit.py keeps the form out of
the library; this test launches the inner-skip conv (both skip kernels) on one stream
and the SHT of the network's 120 x 240 blocks on another, and requires the SHT outputs
to equal their solo run bit for bit.  Reference: sfnonet.py:366-371 (inner skip), torch-harmonics RealSHT /
InverseRealSHT as called at layers.py:629,638.
"""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _conv(w, b, x, stream=None):
    from msfno_amd import _native as N
    B, Cin, P = x.shape
    Cout = w.shape[0]
    out = torch.empty(B, Cout, P, device=x.device)
    ws = torch.empty(N.lib().msfno_conv1x1_workspace_size(B, Cin, Cout), dtype=torch.uint8,
                     device=x.device)
    s = stream.cuda_stream if stream is not None else N.stream_of(x.device)
    N.check(N.lib().msfno_conv1x1(w.data_ptr(), N.ptr(b), x.data_ptr(), out.data_ptr(), B, Cin,
                                  Cout, P, ws.data_ptr(), ws.numel(), s), "conv1x1")
    return out, ws


@pytest.mark.parametrize("B,Cin,Cout,P", [(2, 256, 256, 120 * 240), (1, 64, 32, 4000),
                                          (3, 256, 256, 1000), (3, 256, 256, 50000),
                                          (1, 256, 256, 1038)])
def test_conv1x1_matches_fp64(B, Cin, Cout, P):
    """The standalone 1x1 conv against fp64; channel magnitudes spread over 1e-3 .. 1e3
    (the per-channel power-of-two scales keep every fp16 term in range).  C = 256 runs
    the persistent skip kernel when P % 4 == 0: P = 50000 gives each workgroup several
    128-pixel tiles that cross field boundaries and end in a partial tile; P = 1038 takes
    the one-tile-per-workgroup kernel."""
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn(B, Cin, P, generator=g, device=DEV)
    x *= torch.logspace(-3, 3, Cin, device=DEV)[None, :, None]
    w = torch.randn(Cout, Cin, generator=g, device=DEV) / Cin ** 0.5
    b = torch.randn(Cout, generator=g, device=DEV)
    y, _ = _conv(w, b, x)
    torch.cuda.synchronize()
    ref = torch.einsum("oi,bip->bop", w.double(), x.double()) + b.double()[None, :, None]
    # scale of the products that meet in each output: sum_i |w| |x|
    mag = torch.einsum("oi,bip->bop", w.double().abs(), x.double().abs())
    err = ((y.double() - ref).abs() / (mag + 1e-30)).max().item()
    print(f"conv1x1 B={B} {Cin}->{Cout} P={P}: max |err| / sum|w x| = {err:.3e}")
    assert err < 2e-6


def test_conv1x1_rejects_small_workspace():
    from msfno_amd import _native as N
    x = torch.zeros(1, 8, 16, device=DEV)
    w = torch.zeros(8, 8, device=DEV)
    out = torch.empty_like(x)
    ws = torch.empty(16, dtype=torch.uint8, device=DEV)
    with pytest.raises(ValueError):
        N.check(N.lib().msfno_conv1x1(w.data_ptr(), None, x.data_ptr(), out.data_ptr(), 1, 8, 8,
                                      16, ws.data_ptr(), ws.numel(), N.stream_of(x.device)),
                "conv1x1")


def _sht_call(plan, fn, src, dst, bc, ws, stream):
    from msfno_amd import _native as N
    N.check(fn(plan.handle, src.data_ptr(), dst.data_ptr(), bc, ws.data_ptr(), ws.numel(),
               stream.cuda_stream), "sht")


@pytest.mark.parametrize("persist", ["0", "1"])
@pytest.mark.parametrize("inverse", [False, True])
def test_sht_beside_skip_conv_is_bitwise(inverse, persist, monkeypatch):
    """persist "0": skip_h_kernel (two 66-KB workgroups per CU, room for an FFT workgroup
    beside them on the same CU); "1": the persistent skip_hp_kernel (the block's default,
    one 142-KB workgroup per CU).  MSFNO_SKIP_P is read on every call."""
    monkeypatch.setenv("MSFNO_SKIP_P", persist)
    from msfno_amd import _native as N
    from msfno_amd.harmonics import InverseRealSHT, RealSHT
    nlat, nlon, lmax = 120, 240, 120
    T = (InverseRealSHT if inverse else RealSHT)(nlat, nlon, lmax=lmax, mmax=lmax + 1,
                                                 grid="legendre-gauss").float().to(DEV)
    plan = T._plan(torch.device(DEV, torch.cuda.current_device()))
    bc = 16 * 256
    g = torch.Generator(device=DEV).manual_seed(11)
    if inverse:
        src = torch.randn(bc, lmax, lmax + 1, 2, generator=g, device=DEV)
        src = torch.view_as_complex(src).contiguous()
        dst = torch.empty(bc, nlat, nlon, device=DEV)
        fn = N.lib().msfno_sht_inverse
    else:
        src = torch.randn(bc, nlat, nlon, generator=g, device=DEV)
        dst = torch.empty(bc, lmax, lmax + 1, dtype=torch.complex64, device=DEV)
        fn = N.lib().msfno_sht_forward
    ws = torch.empty(N.lib().msfno_sht_workspace_size(plan.handle, bc), dtype=torch.uint8,
                     device=DEV)
    # the aggressor: the block's inner skip at C = 256 on 8 fields
    P = nlat * nlon
    x = torch.randn(8, 256, P, generator=g, device=DEV)
    w = torch.randn(256, 256, generator=g, device=DEV) / 16
    b = torch.randn(256, generator=g, device=DEV)
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    _sht_call(plan, fn, src, dst, bc, ws, sa)
    torch.cuda.synchronize()
    ref = dst.clone()
    keep = []
    for rep in range(5):
        dst.zero_()
        torch.cuda.synchronize()
        for _ in range(3):
            keep.append(_conv(w, b, x, stream=sb))
        _sht_call(plan, fn, src, dst, bc, ws, sa)
        torch.cuda.synchronize()
        keep.clear()
        nbad = (torch.view_as_real(dst) != torch.view_as_real(ref)).sum().item() if not inverse \
            else (dst != ref).sum().item()
        print(f"{'inverse' if inverse else 'forward'} SHT beside skip conv, rep {rep}: "
              f"{nbad} values differ")
        assert nbad == 0
