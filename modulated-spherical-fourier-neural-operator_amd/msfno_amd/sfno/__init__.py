"""Mirror of MSFNO/Models/sfno (block, filters, contractions, activations)."""
from .activations import ComplexReLU  # noqa: F401
from .contractions import compl_contract_fwd_c, compl_mul2d_fwd_c  # noqa: F401
from .layers import MLP, DropPath, SpectralAttentionS2, SpectralConvS2, trunc_normal_  # noqa: F401
from .sfnonet import (  # noqa: F401
    FiLM,
    FourierNeuralOperatorBlock,
    FourierNeuralOperatorBlock_Filmed,
    FourierNeuralOperatorNet,
    FourierNeuralOperatorNet_Filmed,
    SpectralFilterLayer,
)
from .latband import (LatBandBlock, LatBandNet, LocalGroup, TorchComm,  # noqa: F401
                      band_partition, exchange_counts, local_rows)
