"""openr_amd: MI355X-native SPF and route computation for OpenR's Decision module.

The product is the C++ host library ``openr_amd._openr_host`` (drop-in
LinkState / PrefixState / SpfSolver) over ``lib/libopenr_hip.so`` (C ABI in
include/openr_hip.h, hand-written gfx950 kernels). There is no CPU fallback:
if the extension or a GPU is missing, the product path raises.
"""
from __future__ import annotations

import importlib
import os

__all__ = ["host_module", "host_backend", "HIP_LIB_PATH"]

HIP_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libopenr_hip.so")


def host_module():
    """The native host library; raises ImportError if it was not built."""
    try:
        return importlib.import_module("openr_amd._openr_host")
    except ImportError as e:  # fail loudly: no silent fallback
        raise ImportError(
            "openr_amd._openr_host is not built (run `python -m openr_amd.build` or "
            "__graft_entry__.build()): " + str(e)) from e


def host_backend():
    """Facade Backend bound to the HIP product; requires a visible GPU."""
    from .facade import Backend
    mod = host_module()
    if mod.device_count() < 1:
        raise RuntimeError("openr_amd: no HIP device visible; the SPF path runs only on GPU")
    return Backend(mod, "hip")
