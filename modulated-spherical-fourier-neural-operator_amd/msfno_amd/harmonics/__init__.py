"""MI355X replacement of the ``torch_harmonics`` surface the reference uses
(``RealSHT``, ``InverseRealSHT``, ``quadrature.legendre_gauss_weights``)."""
from . import quadrature  # noqa: F401
from .sht import InverseRealSHT, RealSHT, adopt  # noqa: F401
