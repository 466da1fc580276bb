"""The C-ABI boundary: libopenr_hip loads and exports every symbol that
include/openr_hip.h declares (no compute call: this runs without a GPU)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "openr_hip.h")


def declared_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(orh_[a-z0-9_]+)\s*\(", text)))


@pytest.fixture(scope="module")
def lib():
    from openr_amd import HIP_LIB_PATH
    from openr_amd.build import build_hip_lib
    build_hip_lib()
    return ctypes.CDLL(HIP_LIB_PATH)


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for required in ("orh_create", "orh_destroy", "orh_last_error", "orh_graph_load",
                     "orh_graph_patch_edges", "orh_graph_patch_nodes", "orh_spf_run",
                     "orh_spf_batch", "orh_route_select", "orh_get_counters"):
        assert required in syms


def test_every_declared_symbol_is_exported(lib):
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, f"symbols declared in openr_hip.h but not exported: {missing}"


def test_null_arguments_are_rejected_without_a_device(lib):
    lib.orh_create.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.POINTER(ctypes.c_void_p)]
    assert lib.orh_create(0, 0, None) == -1  # ORH_E_INVALID
    lib.orh_destroy.argtypes = [ctypes.c_void_p]
    assert lib.orh_destroy(None) == -1
    lib.orh_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
    n = ctypes.c_int(-1)
    assert lib.orh_device_count(ctypes.byref(n)) == 0
    assert n.value >= 0


def test_host_module_imports():
    from openr_amd import host_module
    from openr_amd.build import build_host_module
    build_host_module()
    mod = host_module()
    for name in ("LinkState", "AreaLinkStates", "PrefixState", "SpfSolver", "SpfSweep"):
        assert hasattr(mod, name)


def test_route_map_unordered_map_api(tmp_path):
    """DecisionRouteDb::unicastRoutes / DecisionRouteUpdate::
    unicastRoutesToUpdate are 64-shard maps, not std::unordered_map: the
    reference's own call patterns on them (Decision.h:110, RouteUpdate.h:34-41,
    Decision.cpp:148, Fib.cpp:304 / :357-361, NetlinkSocket.cpp:386) compile
    and behave as on std::unordered_map (tests/cxx/route_map_api.cpp)."""
    import subprocess
    exe = tmp_path / "route_map_api"
    subprocess.run(["g++", "-std=c++17", "-O1", "-pthread", "-I" + os.path.join(ROOT, "openr_amd", "csrc", "host"),
                    "-I" + os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "cxx", "route_map_api.cpp"),
                    "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0 and out.stdout.startswith("ok"), (out.returncode, out.stdout)
