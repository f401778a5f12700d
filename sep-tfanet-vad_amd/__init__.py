"""MI355X-native Sep-TFAnet^VAD forward path.

Drop-in for the reference's ``model.model.SeparationModel`` (reference ``model/model.py:360-461``):
same constructor kwargs, same state_dict keys, same ``forward(x, inference_kw)`` return tuple and
side attributes; the arithmetic runs in hand-written gfx950 HIP kernels behind the C-ABI library
``libsepvad.so`` (declared in ``include/sepvad.h``).
"""
from .config import (CONFIG_WITH_VAD, CONFIG_WITHOUT_VAD, DEFAULTS, INFERENCE_KW_DEFAULTS,
                     frames, param_spec)
from .model import SeparationModel
from .online import OnlineSaving
from .pit import PITLossWrapper, reorder_source_mse

__all__ = [
    "SeparationModel", "OnlineSaving", "PITLossWrapper", "reorder_source_mse", "CONFIG_WITH_VAD", "CONFIG_WITHOUT_VAD", "DEFAULTS",
    "INFERENCE_KW_DEFAULTS", "param_spec", "frames",
]
