"""ctypes binding of libmsfno.so (the HIP/gfx950 implementation, include/msfno.h).

The library is built in-tree (``make -C csrc`` or ``__graft_entry__.build()``)
and loaded from this package directory.  There is deliberately no fallback:
if the library is missing, every op raises.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (loads the HIP runtime (libamdhip64.so.7) that libmsfno shares)

_HERE = os.path.dirname(os.path.abspath(__file__))
# MSFNO_LIB: another in-tree build of the same library (A/B of two builds in one run)
LIB_PATH = os.environ.get("MSFNO_LIB") or os.path.join(_HERE, "libmsfno.so")

MSFNO_OK = 0
MSFNO_EINVAL = 1
MSFNO_EUNSUPPORTED = 2
MSFNO_EHIP = 3
MSFNO_EWORKSPACE = 4

GRID = {"equiangular": 0, "legendre-gauss": 1}

FILTER_NONLINEAR = 0
FILTER_LINEAR = 1
SKIP_NONE = 0
SKIP_LINEAR = 1
SKIP_IDENTITY = 2

_vp = ctypes.c_void_p
_i = ctypes.c_int
_f = ctypes.c_float
_sz = ctypes.c_size_t


class BlockDesc(ctypes.Structure):
    """Mirror of ``msfno_block_desc`` (include/msfno.h)."""

    _fields_ = [
        ("C", _i), ("filter_type", _i), ("inner_skip", _i), ("outer_skip", _i),
        ("has_mlp", _i), ("mlp_hidden", _i), ("spectral_layers", _i), ("spec_hidden", _i),
        ("norm_eps", _f),
        ("norm0_w", _vp), ("norm0_b", _vp), ("norm1_w", _vp), ("norm1_b", _vp),
        ("spec_w", _vp * 8), ("spec_wout", _vp), ("lin_w", _vp),
        ("skip_w", _vp), ("skip_b", _vp),
        ("fc1_w", _vp), ("fc1_b", _vp), ("fc2_w", _vp), ("fc2_b", _vp),
        ("wcache", _vp), ("wcache_valid", _i),
    ]


class BlockParamGrads(ctypes.Structure):
    """Mirror of ``msfno_block_param_grads`` (include/msfno.h): output pointers of the
    block's parameter gradients, NULL = not wanted."""

    _fields_ = [
        ("norm0_w", _vp), ("norm0_b", _vp), ("spec_w", _vp * 8), ("spec_wout", _vp),
        ("lin_w", _vp), ("skip_w", _vp), ("skip_b", _vp), ("norm1_w", _vp), ("norm1_b", _vp),
        ("fc1_w", _vp), ("fc1_b", _vp), ("fc2_w", _vp), ("fc2_b", _vp),
    ]


class MlpDesc(ctypes.Structure):
    """Mirror of ``msfno_mlp_desc`` (include/msfno.h)."""

    _fields_ = [
        ("Cin", _i), ("Cin2", _i), ("Hid", _i), ("Cout", _i),
        ("fc1_w", _vp), ("fc1_b", _vp), ("fc2_w", _vp), ("fc2_b", _vp),
        ("wcache", _vp), ("wcache_valid", _i),
    ]


class BandIO(ctypes.Structure):
    """Mirror of ``msfno_band_io`` (include/msfno.h)."""

    _fields_ = [
        ("x", _vp), ("gamma", _vp), ("beta", _vp), ("film_scale", _f), ("out", _vp),
        ("send", _vp), ("recv", _vp), ("stats_local", _vp), ("stats_all", _vp),
        ("slot", _i),
    ]


_ip = ctypes.POINTER(_i)
_llp = ctypes.POINTER(ctypes.c_longlong)

# (name, restype, argtypes) — every symbol declared in include/msfno.h
SIGNATURES = [
    ("msfno_last_error", ctypes.c_char_p, []),
    ("msfno_abi_version", _i, []),
    ("msfno_quadrature", _i, [_i, _i, _vp, _vp]),
    ("msfno_legendre_table", _i, [_i, _i, _i, _i, _i, _i, _vp]),
    ("msfno_sht_plan_create", _i, [_i, _i, _i, _i, _i, ctypes.POINTER(_vp)]),
    ("msfno_sht_plan_destroy", _i, [_vp]),
    ("msfno_sht_plan_load_table", _i, [_vp, _vp, _vp]),
    ("msfno_sht_workspace_size", _sz, [_vp, _i]),
    ("msfno_sht_forward", _i, [_vp, _vp, _vp, _i, _vp, _sz, _vp]),
    ("msfno_sht_inverse", _i, [_vp, _vp, _vp, _i, _vp, _sz, _vp]),
    ("msfno_compl_contract_fwd_c", _i, [_vp, _vp, _vp, _i, _i, _i, _i, _vp]),
    ("msfno_compl_mul2d_fwd_c", _i, [_vp, _vp, _vp, _i, _i, _i, ctypes.c_longlong, _i, _vp]),
    ("msfno_conv1x1_workspace_size", _sz, [_i, _i, _i]),
    ("msfno_conv1x1", _i, [_vp, _vp, _vp, _vp, _i, _i, _i, ctypes.c_longlong, _vp, _sz, _vp]),
    ("msfno_block_workspace_size", _sz, [ctypes.POINTER(BlockDesc), _vp, _vp, _i]),
    ("msfno_block_wcache_size", _sz, [ctypes.POINTER(BlockDesc)]),
    ("msfno_block_forward", _i, [ctypes.POINTER(BlockDesc), _vp, _vp, _vp, _vp, _vp, _f, _vp,
                                 _i, _vp, _sz, _vp]),
    ("msfno_block_forward_deferred", _i, [ctypes.POINTER(BlockDesc), _vp, _vp, _vp, _vp, _vp, _f,
                                          _vp, _vp, _i, _vp, _sz, _vp]),
    ("msfno_block_global_conv", _i, [ctypes.POINTER(BlockDesc), _vp, _vp, _vp, _vp, _vp, _i, _vp,
                                     _sz, _vp]),
    ("msfno_filter_forward", _i, [ctypes.POINTER(BlockDesc), _vp, _vp, _vp, _vp, _i, _vp, _sz,
                                  _vp]),
    ("msfno_mlp_wcache_size", _sz, [ctypes.POINTER(MlpDesc)]),
    ("msfno_mlp_workspace_size", _sz, [ctypes.POINTER(MlpDesc), _i, ctypes.c_longlong]),
    ("msfno_mlp_fused_supported", _i, [ctypes.POINTER(MlpDesc)]),
    ("msfno_mlp_forward_affine", _i, [ctypes.POINTER(MlpDesc), _vp, _vp, _vp, _vp, _vp,
                                      ctypes.c_longlong, _vp, _i, ctypes.c_longlong, _vp, _sz,
                                      _vp]),
    ("msfno_mlp_forward", _i, [ctypes.POINTER(MlpDesc), _vp, _vp, _vp, ctypes.c_longlong, _vp, _i,
                               ctypes.c_longlong, _vp, _sz, _vp]),
    ("msfno_block_film_backward_workspace_size", _sz, [ctypes.POINTER(BlockDesc), _vp, _vp, _i]),
    ("msfno_block_film_backward", _i, [ctypes.POINTER(BlockDesc), _vp, _vp, _vp, _vp, _vp, _f,
                                       _vp, _vp, _vp, _i, _vp, _sz, _vp]),
    ("msfno_block_backward_workspace_size", _sz, [ctypes.POINTER(BlockDesc), _vp, _vp, _vp, _vp,
                                                   _i]),
    ("msfno_block_backward", _i, [ctypes.POINTER(BlockDesc), _vp, _vp, _vp, _vp, _vp, _vp, _vp, _f,
                                  _vp, _vp, _vp, _vp, _i, _vp, _sz, _vp]),
    ("msfno_block_backward_params_workspace_size", _sz, [ctypes.POINTER(BlockDesc), _vp, _vp,
                                                          _vp, _vp, _i]),
    ("msfno_block_backward_params", _i, [ctypes.POINTER(BlockDesc), _vp, _vp, _vp, _vp, _vp, _vp,
                                         _vp, _f, _vp, _vp, _vp, _vp,
                                         ctypes.POINTER(BlockParamGrads), _i, _vp, _sz, _vp]),
    ("msfno_mlp_backward_params_workspace_size", _sz, [ctypes.POINTER(MlpDesc), _i,
                                                        ctypes.c_longlong]),
    ("msfno_mlp_backward_params", _i, [ctypes.POINTER(MlpDesc), _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                       _vp, _vp, _i, ctypes.c_longlong, _vp, _sz, _vp]),
    ("msfno_block_backward_hidden_offsets", _i, [ctypes.POINTER(BlockDesc), _vp, _vp, _vp, _vp,
                                                 _i, ctypes.POINTER(_sz), _i,
                                                 ctypes.POINTER(_i)]),
    ("msfno_mlp_backward_input_workspace_size", _sz, [ctypes.POINTER(MlpDesc), _i,
                                                       ctypes.c_longlong]),
    ("msfno_mlp_backward_input", _i, [ctypes.POINTER(MlpDesc), _vp, _vp, _vp, _vp, _i,
                                      ctypes.c_longlong, _vp, _sz, _vp]),
    ("msfno_band_partition", _i, [_i, _i, _i, _i, _ip, _ip]),
    ("msfno_band_exchange_counts", _i, [_i, _i, _i, _i, _ip, _ip, _i, _i, _llp, _llp]),
    ("msfno_band_local_rows", _i, [_i, _i, _i, _ip, _ip, _ip]),
    ("msfno_band_plan_create", _i, [_i, _i, _i, _i, _i, _i, _ip, _ip, ctypes.POINTER(_vp)]),
    ("msfno_band_plan_create2", _i, [_i, _i, _i, _i, _i, _i, _i, _i, _ip, _ip, _ip,
                                     ctypes.POINTER(_vp)]),
    ("msfno_band_plan_exchange_counts", _i, [_vp, _i, _i, _llp, _llp]),
    ("msfno_band_linear_modes", _i, [_vp, _llp, _llp]),
    ("msfno_band_plan_destroy", _i, [_vp]),
    ("msfno_band_plan_load_tables", _i, [_vp, _vp, _vp, _vp]),
    ("msfno_band_workspace_size", _sz, [ctypes.POINTER(BlockDesc), _vp, _i]),
    ("msfno_band_block_stage", _i, [ctypes.POINTER(BlockDesc), _vp, _i, ctypes.POINTER(BandIO),
                                    _i, _vp, _sz, _vp]),
    ("msfno_profile_enable", _i, [_i]),
    ("msfno_profile_mark", _i, [_i, _vp]),
    ("msfno_profile_collect", _i, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(_i)]),
    ("msfno_profile_stage_name", ctypes.c_char_p, [_i]),
]

PROF_NSTAGES = 32


def profile_mark(stage_name: str, stream: int) -> None:
    """Start stage `stage_name` on `stream` (a span lasts to the next mark there)."""
    for i in range(PROF_NSTAGES):
        if lib().msfno_profile_stage_name(i).decode() == stage_name:
            check(lib().msfno_profile_mark(i, stream), "profile_mark")
            return
    raise ValueError(f"unknown profile stage {stage_name!r}")


def profile_enable(on: bool) -> None:
    lib().msfno_profile_enable(int(on))


def profile_collect():
    """{stage_name: (total_ms, launches)} since the last collect (synchronises)."""
    ms = (ctypes.c_double * PROF_NSTAGES)()
    cnt = (_i * PROF_NSTAGES)()
    check(lib().msfno_profile_collect(ms, cnt), "profile_collect")
    out = {}
    for i in range(PROF_NSTAGES):
        if cnt[i]:
            out[lib().msfno_profile_stage_name(i).decode()] = (ms[i], cnt[i])
    return out

_lib = None


def lib():
    """Load libmsfno.so once; raise loudly if it is absent (no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"libmsfno.so not found at {LIB_PATH}; build it with "
                "`make -C modulated-spherical-fourier-neural-operator_amd/csrc` "
                "or `python -c 'import __graft_entry__ as g; g.build()'`")
        L = ctypes.CDLL(LIB_PATH)
        for name, res, args in SIGNATURES:
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int, what: str = "") -> None:
    """Re-raise a C-ABI status with the reference's exception types."""
    if rc == MSFNO_OK:
        return
    msg = lib().msfno_last_error().decode(errors="replace")
    text = f"{what}: {msg}" if what else msg
    if rc == MSFNO_EUNSUPPORTED:
        raise NotImplementedError(text)
    if rc in (MSFNO_EINVAL, MSFNO_EWORKSPACE):
        raise ValueError(text)
    raise RuntimeError(text)


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def on_input_device(fn):
    """Run ``fn`` with its first GPU tensor argument's device as the current HIP
    device: kernels go to the null stream of the *current* device and the C side
    keys its side streams by device, so a module on cuda:1 called while cuda:0 is
    current must switch first."""
    import functools

    @functools.wraps(fn)
    def wrapper(*args, **kwargs):
        for a in list(args) + list(kwargs.values()):
            if isinstance(a, torch.Tensor) and a.is_cuda:
                with torch.cuda.device(a.device):
                    return fn(*args, **kwargs)
        return fn(*args, **kwargs)
    return wrapper


def stream_of(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def require_device_f32(t: torch.Tensor, name: str) -> torch.Tensor:
    if not t.is_cuda:
        raise ValueError(f"{name} must be a GPU (HIP) tensor; libmsfno has no CPU path")
    if t.dtype != torch.float32:
        t = t.float()
    return t.contiguous()


class SHTPlan:
    """Owns one msfno_sht_plan_t (device tables + FFT twiddles)."""

    def __init__(self, nlat, nlon, lmax, mmax, inverse, device):
        self.device = device
        h = _vp()
        with torch.cuda.device(device):
            check(lib().msfno_sht_plan_create(nlat, nlon, lmax, mmax, int(inverse), ctypes.byref(h)),
                  "msfno_sht_plan_create")
        self.handle = h
        self.key = None

    def load(self, table: torch.Tensor, key):
        if key == self.key:
            return
        with torch.cuda.device(self.device):
            check(lib().msfno_sht_plan_load_table(self.handle, table.data_ptr(),
                                                  stream_of(self.device)),
                  "msfno_sht_plan_load_table")
        self._table_ref = table  # keep alive until the relayout kernel has consumed it
        self.key = key

    def __del__(self):
        try:
            if self.handle:
                lib().msfno_sht_plan_destroy(self.handle)
        except Exception:
            pass
