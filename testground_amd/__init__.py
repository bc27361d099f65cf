"""testground_amd — MI355X-native engine for testground's per-packet network.Config enforcement.

The product is ``libtgsim.so`` (HIP kernels for gfx950 behind the C ABI in ``include/tgsim.h``);
this package is its Python host mirror: sdk-go network types (``network``), the engine handle
(``engine``), the sidecar-side Network/handler mirror (``sidecar``) and the storm workload
(``workloads``).
"""
from . import abi, network
from .engine import CABIEngine, Engine, EngineError, EngineUnavailable, load_library, packets

__all__ = ["abi", "network", "CABIEngine", "Engine", "EngineError", "EngineUnavailable",
           "load_library", "packets"]
