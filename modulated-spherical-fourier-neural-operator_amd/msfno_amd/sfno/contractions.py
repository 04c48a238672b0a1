"""Complex contraction helpers — mirror of MSFNO/Models/sfno/contractions.py,
backed by HIP kernels (libmsfno).  Tensors use the reference's real-view
layout (last dim = 2: re, im)."""
from __future__ import annotations

import torch

from .. import _native as N


def _c(t, name):
    t = N.require_device_f32(t, name)
    assert t.shape[-1] == 2, f"{name}: expected a real view with trailing dim 2"
    return t


@N.on_input_device
def compl_contract_fwd_c(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """einsum("bin,kin->bkn") on complex views (contractions.py:37-41)."""
    a = _c(a, "a")
    b = _c(b, "b")
    B, Ci, T, _ = a.shape
    Co = b.shape[0]
    assert b.shape[1] == Ci and b.shape[2] == T
    y = torch.empty(B, Co, T, 2, dtype=torch.float32, device=a.device)
    N.check(N.lib().msfno_compl_contract_fwd_c(a.data_ptr(), b.data_ptr(), y.data_ptr(), B, Ci, Co,
                                                T, N.stream_of(a.device)), "compl_contract_fwd_c")
    return y


compl_contract_fwd = compl_contract_fwd_c  # same result (contractions.py:28-33)


@N.on_input_device
def compl_mul2d_fwd_c(a: torch.Tensor, b: torch.Tensor, relu_real: bool = False) -> torch.Tensor:
    """einsum("bixy,io->boxy") on complex views (contractions.py:132-137)."""
    a = _c(a, "a")
    b = _c(b, "b")
    B, Ci = a.shape[0], a.shape[1]
    XY = 1
    for s in a.shape[2:-1]:
        XY *= s
    Co = b.shape[1]
    assert b.shape[0] == Ci
    y = torch.empty(B, Co, *a.shape[2:-1], 2, dtype=torch.float32, device=a.device)
    N.check(N.lib().msfno_compl_mul2d_fwd_c(a.data_ptr(), b.data_ptr(), y.data_ptr(), B, Ci, Co,
                                             XY, int(relu_real), N.stream_of(a.device)),
            "compl_mul2d_fwd_c")
    return y


compl_mul2d_fwd = compl_mul2d_fwd_c  # same result (contractions.py:123-128)
