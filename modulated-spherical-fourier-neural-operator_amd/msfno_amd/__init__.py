"""msfno_amd — MI355X (gfx950) SFNO-Block forward path.

Drop-in mirror of the reference's ``MSFNO/Models/sfno`` block API and the
``torch_harmonics`` transforms it uses, executed by hand-written HIP kernels in
``libmsfno.so`` (C-ABI: include/msfno.h) through ctypes.  PyTorch-ROCm is used
for tensor storage and streams only.
"""
from . import _native  # noqa: F401
from . import harmonics  # noqa: F401
from . import sfno  # noqa: F401
from . import rollout  # noqa: F401

__version__ = "0.1.0"
