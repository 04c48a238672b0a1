"""ComplexReLU — mirror of MSFNO/Models/sfno/activations.py:9-51.

On the block's hot path the "real" mode (ReLU of the real part, :42-46) is
fused into the epilogue of the spectral-MLP MFMA GEMM; this module carries the
parameter/buffer layout (``activation.bias``) and the standalone semantics."""
from __future__ import annotations

import torch
from torch import nn


class ComplexReLU(nn.Module):
    def __init__(self, negative_slope=0.0, mode="cartesian", bias_shape=None):
        super().__init__()
        self.mode = mode
        if self.mode in ["modulus", "halfplane"]:
            shape = bias_shape if bias_shape is not None else (1,)
            self.bias = nn.Parameter(torch.zeros(shape, dtype=torch.float32))
        else:
            self.register_buffer("bias", torch.zeros((1), dtype=torch.float32))
        self.negative_slope = negative_slope
        self.act = nn.LeakyReLU(negative_slope=negative_slope)

    def forward(self, z: torch.Tensor) -> torch.Tensor:
        # standalone (non-fused) use only; the fused filter applies it in-kernel
        if self.mode == "real":
            zr = torch.view_as_real(z).clone()
            zr[..., 0] = self.act(zr[..., 0])
            return torch.view_as_complex(zr)
        if self.mode == "cartesian":
            return torch.view_as_complex(self.act(torch.view_as_real(z)))
        if self.mode in ("modulus", "halfplane"):
            raise NotImplementedError(f"ComplexReLU mode {self.mode!r} is not on the MI355X path")
        return z
