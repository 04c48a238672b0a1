"""The linear filter on S itself (launch_contract_spec: the per-mode contraction reads
the forward Legendre's parity-split triangle through a column map and writes the
inverse's input, no gathered copies) against the gathered form (spec_to_tril ->
compl_contract -> tril_to_spec, MSFNO_LIN_DIRECT=0) at config 2's full size
(721x1440, C=256, lmax 360, the 34 GB per-mode weight), with the inner-skip side
stream on and off (MSFNO_SIDE_STREAM; both switches are read at every call).

The two forms do the same fp32 arithmetic per mode (the same fused multiply-adds in
the same channel order), so the block outputs must agree bit for bit.
Reference: layers.py:408-413 (SpectralConvS2 linear), contractions.py:37-41."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_linear_on_s_equals_gathered_form():
    from test_gpu_configs import _bench_block
    blk = _bench_block("linear")
    gen = torch.Generator(device=DEV).manual_seed(43)
    x = torch.randn(1, 256, 721, 1440, generator=gen, device=DEV)
    g = 0.1 * torch.randn(1, 256, generator=gen, device=DEV)
    b = 0.1 * torch.randn(1, 256, generator=gen, device=DEV)
    out = {}
    saved = {k: os.environ.get(k) for k in ("MSFNO_LIN_DIRECT", "MSFNO_SIDE_STREAM")}
    try:
        for direct in ("0", "1"):
            for side in ("0", "1"):
                os.environ["MSFNO_LIN_DIRECT"] = direct
                os.environ["MSFNO_SIDE_STREAM"] = side
                with torch.no_grad():
                    out[(direct, side)] = blk(x, g, b, 1.0).clone()
                torch.cuda.synchronize()
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    ref = out[("0", "0")]
    assert torch.isfinite(ref).all()
    for key, y in out.items():
        err = (y - ref).abs().max().item()
        nbad = (y != ref).sum().item()
        print(f"direct={key[0]} side={key[1]}: max-abs vs gathered/no-side {err:.3e}, {nbad} differ")
    for key, y in out.items():
        assert torch.equal(y, ref), key
