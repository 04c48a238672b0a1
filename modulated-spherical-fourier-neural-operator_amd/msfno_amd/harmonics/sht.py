"""Drop-in replacements for ``torch_harmonics.RealSHT`` / ``InverseRealSHT``.

Reference usage: constructed at MSFNO/Models/sfno/sfnonet.py:537-548 with
``.float()``, the buffers ``.weights`` / ``.pct`` rescaled ×1e5 / ÷1e5 at
:551-555, and called as ``forward_transform(x)`` / ``inverse_transform(x)`` at
MSFNO/Models/sfno/layers.py:405,421,629,638.  Attributes read by the reference:
``nlat nlon lmax mmax`` (layers.py:361-365, 569-577).

The tables are computed on the host in fp64 by libmsfno (same recurrence as
torch-harmonics' ``legpoly``) and registered as buffers with the same names and
shapes ``(mmax, lmax, nlat)``; ``forward`` runs entirely on the GPU (HIP
longitude FFT + MFMA Legendre contraction).  Whenever the buffer tensor changes
(``.float()``, the ×1e5 rescale, ``.to(device)``) the device plan re-lays it out
on the next call, so the reference's construction recipe keeps working.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from .. import _native as N

_SUPPORTED_GRIDS = ("equiangular", "legendre-gauss")


def _legendre_table(mmax, lmax, nlat, grid, inverse, csphase):
    t = np.zeros((mmax, lmax, nlat), dtype=np.float64)
    N.check(N.lib().msfno_legendre_table(mmax, lmax, nlat, N.GRID[grid], int(inverse),
                                         int(csphase), t.ctypes.data), "legendre_table")
    return torch.from_numpy(t)


class _SHTBase(nn.Module):
    _buffer_name = "weights"
    _inverse = False

    def _init_common(self, nlat, nlon, lmax, mmax, grid, norm, csphase):
        if grid not in _SUPPORTED_GRIDS:
            raise NotImplementedError(f"Unknown quadrature mode {grid!r} (supported: {_SUPPORTED_GRIDS})")
        if norm != "ortho":
            raise NotImplementedError(f"Unsupported SHT normalisation {norm!r} (only 'ortho')")
        self.nlat, self.nlon, self.grid = nlat, nlon, grid
        self.norm, self.csphase = norm, csphase
        self.lmax = lmax or nlat
        self.mmax = mmax or nlon // 2 + 1
        self._plans = {}

    def _plan(self, device):
        table = getattr(self, self._buffer_name)
        idx = device.index if device.index is not None else torch.cuda.current_device()
        plan = self._plans.get(idx)
        if plan is None:
            plan = N.SHTPlan(self.nlat, self.nlon, self.lmax, self.mmax, self._inverse, idx)
            self._plans[idx] = plan
        key = (table.data_ptr(), table._version, table.dtype, str(table.device))
        if key != plan.key:  # (re)load only when the buffer tensor changed
            t = table
            if t.device != device or t.dtype != torch.float32 or not t.is_contiguous():
                t = t.to(device=device, dtype=torch.float32).contiguous()
            plan.load(t, key)
        return plan

    def __getstate__(self):
        s = self.__dict__.copy()
        s["_plans"] = {}
        return s


class RealSHT(_SHTBase):
    """Forward real SHT: (..., nlat, nlon) fp32 -> (..., lmax, mmax) complex64."""

    _buffer_name = "weights"
    _inverse = False

    def __init__(self, nlat, nlon, lmax=None, mmax=None, grid="equiangular", norm="ortho",
                 csphase=True):
        super().__init__()
        self._init_common(nlat, nlon, lmax, mmax, grid, norm, csphase)
        self.register_buffer("weights", _legendre_table(self.mmax, self.lmax, nlat, grid, False,
                                                        csphase))

    @N.on_input_device
    def forward(self, x):
        assert x.shape[-2] == self.nlat
        assert x.shape[-1] == self.nlon
        x = N.require_device_f32(x, "RealSHT input")
        lead = x.shape[:-2]
        bc = int(np.prod(lead)) if len(lead) else 1
        out = torch.empty(*lead, self.lmax, self.mmax, dtype=torch.complex64, device=x.device)
        plan = self._plan(x.device)
        ws = torch.empty(N.lib().msfno_sht_workspace_size(plan.handle, bc), dtype=torch.uint8,
                         device=x.device)
        N.check(N.lib().msfno_sht_forward(plan.handle, x.data_ptr(), out.data_ptr(), bc,
                                          ws.data_ptr(), ws.numel(), N.stream_of(x.device)),
                "RealSHT.forward")
        return out


class InverseRealSHT(_SHTBase):
    """Inverse real SHT: (..., lmax, mmax) complex64 -> (..., nlat, nlon) fp32."""

    _buffer_name = "pct"
    _inverse = True

    def __init__(self, nlat, nlon, lmax=None, mmax=None, grid="equiangular", norm="ortho",
                 csphase=True):
        super().__init__()
        self._init_common(nlat, nlon, lmax, mmax, grid, norm, csphase)
        self.register_buffer("pct", _legendre_table(self.mmax, self.lmax, nlat, grid, True,
                                                    csphase))

    @N.on_input_device
    def forward(self, x):
        assert x.shape[-2] == self.lmax
        assert x.shape[-1] == self.mmax
        if not x.is_cuda:
            raise ValueError("InverseRealSHT input must be a GPU (HIP) tensor")
        if x.dtype != torch.complex64:
            x = x.to(torch.complex64)
        x = x.contiguous()
        lead = x.shape[:-2]
        bc = int(np.prod(lead)) if len(lead) else 1
        out = torch.empty(*lead, self.nlat, self.nlon, dtype=torch.float32, device=x.device)
        plan = self._plan(x.device)
        ws = torch.empty(N.lib().msfno_sht_workspace_size(plan.handle, bc), dtype=torch.uint8,
                         device=x.device)
        N.check(N.lib().msfno_sht_inverse(plan.handle, x.data_ptr(), out.data_ptr(), bc,
                                          ws.data_ptr(), ws.numel(), N.stream_of(x.device)),
                "InverseRealSHT.forward")
        return out
