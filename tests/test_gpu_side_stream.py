"""The inner skip on its side stream (api.cpp: forked after the norm0 statistics, joined
before the inverse FFT) changes nothing but the schedule: at config 2's full size
(721x1440, C=256, lmax 360) the block output with the side stream on must equal the
serial one bit for bit, for both filters and at batch 1 and 2.  The skip kernel
(skip_h_kernel) then co-runs with the forward Legendre, the spectral filter and the
inverse Legendre; DESIGN.md §5 records the two kernels it was seen to disturb when
co-resident (the row FFT, and a since-retired S-direct contraction), which the default
schedule never puts beside it.  MSFNO_SIDE_STREAM is read at every call.
Reference: sfnonet.py:227-262 (FourierNeuralOperatorBlock.forward, inner skip)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _run(blk, x, g, b, side):
    saved = os.environ.get("MSFNO_SIDE_STREAM")
    os.environ["MSFNO_SIDE_STREAM"] = side
    try:
        with torch.no_grad():
            y = blk(x, g, b, 1.0).clone()
        torch.cuda.synchronize()
    finally:
        if saved is None:
            os.environ.pop("MSFNO_SIDE_STREAM", None)
        else:
            os.environ["MSFNO_SIDE_STREAM"] = saved
    return y


@pytest.mark.parametrize("filter_type,batch", [("non-linear", 1), ("non-linear", 2), ("linear", 1)])
def test_side_stream_is_bitwise_serial(filter_type, batch):
    from test_gpu_configs import _bench_block
    blk = _bench_block(filter_type)
    gen = torch.Generator(device=DEV).manual_seed(47)
    x = torch.randn(batch, 256, 721, 1440, generator=gen, device=DEV)
    g = 0.1 * torch.randn(batch, 256, generator=gen, device=DEV)
    b = 0.1 * torch.randn(batch, 256, generator=gen, device=DEV)
    ref = _run(blk, x, g, b, "0")
    assert torch.isfinite(ref).all()
    for rep in range(3):
        y = _run(blk, x, g, b, "1")
        nbad = (y != ref).sum().item()
        print(f"{filter_type} B={batch} side rep {rep}: {nbad} differ, "
              f"max-abs {(y - ref).abs().max().item():.3e}")
        assert nbad == 0
