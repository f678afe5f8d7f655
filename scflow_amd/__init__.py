"""scflow_amd — MI355X-native (gfx950 HIP) implementation of SCFlow's recurrent
correlation-flow hot path, behind the reference's decoder/refiner operator API.

Product path: ``scflow_amd.decoder.SCFlowDecoder`` (drop-in for
``models/decoder/scflow_decoder.py:SCFlowDecoder``) and the modules in
``scflow_amd.modules``, all running on ``lib/libscflow_hip.so`` (C ABI: include/scflow_hip.h).
"""
from .registry import MODELS, Registry  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    # lazy: importing the package must not require torch's GPU stack (CPU-only tests)
    if name in ("SCFlowDecoder",):
        from .decoder import SCFlowDecoder
        return SCFlowDecoder
    if name in ("CorrelationPyramid", "CorrLookup", "MotionEncoder", "ConvGRU", "XHead",
                "MultiClassPoseHead", "ConvModule"):
        from . import modules
        return getattr(modules, name)
    raise AttributeError(name)
