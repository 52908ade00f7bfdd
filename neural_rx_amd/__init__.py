"""MI355X-native CGNN neural-receiver inference engine (theshubh007/neural_rx hot path).

The forward pass runs in hand-written HIP kernels for gfx950 (``csrc/``) behind the C
ABI of ``include/nrx.h``; this package is the Python host layer mirroring the
reference's receiver interfaces (``receiver.py``).
"""
from .config import NRXConfig, ModelSpec, get_config, spec_from_config  # noqa: F401

__all__ = ["NRXConfig", "ModelSpec", "get_config", "spec_from_config"]


def __getattr__(name):
    if name in ("CGNN", "CGNNEngine", "NeuralReceiver", "compute_pe"):
        from . import receiver
        return getattr(receiver, name)
    raise AttributeError(name)
