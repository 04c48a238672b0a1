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

import weakref

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


# ---- foreign transforms ------------------------------------------------------------
# A block built around torch_harmonics.RealSHT / InverseRealSHT objects (the reference's
# own, sfnonet.py:537-548) runs on the native plans too: adopt() wraps such an object in
# the matching class of this module WITHOUT copying its table.  The wrapper reads the
# foreign buffer (``weights`` / ``pct``) on every call, so the reference's later
# re-assignment of it (the x1e5 rescale, sfnonet.py:551-555, ``.to(device)``) is seen
# exactly as for the native classes.  Accepted: any object with nlat, nlon, lmax, mmax
# and a (mmax, lmax, nlat) table buffer, with norm "ortho" if it says.
_ADOPTED = weakref.WeakKeyDictionary()


class _AdoptedRealSHT(RealSHT):
    def __init__(self, src):
        nn.Module.__init__(self)
        object.__setattr__(self, "_src", src)
        self.nlat, self.nlon, self.lmax, self.mmax = src.nlat, src.nlon, src.lmax, src.mmax
        self.grid = getattr(src, "grid", "equiangular")
        self.norm, self.csphase = "ortho", getattr(src, "csphase", True)
        self._plans = {}

    @property
    def weights(self):
        return self._src.weights


class _AdoptedInverseRealSHT(InverseRealSHT):
    def __init__(self, src):
        nn.Module.__init__(self)
        object.__setattr__(self, "_src", src)
        self.nlat, self.nlon, self.lmax, self.mmax = src.nlat, src.nlon, src.lmax, src.mmax
        self.grid = getattr(src, "grid", "equiangular")
        self.norm, self.csphase = "ortho", getattr(src, "csphase", True)
        self._plans = {}

    @property
    def pct(self):
        return self._src.pct


def adopt(t, inverse: bool):
    """This module's transform for `t`: `t` itself when it already is one, else a
    table-sharing wrapper of a torch-harmonics-style transform (NotImplementedError
    when `t` does not look like one)."""
    ours = InverseRealSHT if inverse else RealSHT
    if isinstance(t, ours):
        return t
    name = "pct" if inverse else "weights"
    kind = "InverseRealSHT" if inverse else "RealSHT"
    tab = getattr(t, name, None)
    if not isinstance(tab, torch.Tensor) or not all(
            hasattr(t, a) for a in ("nlat", "nlon", "lmax", "mmax")):
        raise NotImplementedError(f"expected a {kind} (torch_harmonics or msfno_amd.harmonics), "
                                  f"got {type(t).__name__}")
    if getattr(t, "norm", "ortho") != "ortho":
        raise NotImplementedError(f"Unsupported SHT normalisation {t.norm!r} (only 'ortho')")
    if tuple(tab.shape) != (t.mmax, t.lmax, t.nlat):
        raise NotImplementedError(f"{kind}.{name} must have shape (mmax, lmax, nlat)")
    w = _ADOPTED.get(t)
    if w is None:
        w = (_AdoptedInverseRealSHT if inverse else _AdoptedRealSHT)(t)
        _ADOPTED[t] = w
    return w
