"""Shared fixtures.

Backends
--------
``oracle``  CPU restatement of the reference Decision path (oracle/, test
            infrastructure only); runs everywhere.
``hip``     the product: openr_amd's C++ host library over libopenr_hip
            (hand-written gfx950 kernels); needs a GPU, so every test that
            touches it is marked ``gpu``.

Known-answer tests take the ``backend`` fixture and run once per backend:
under ``-m "not gpu"`` against the oracle (pinning it to the reference's own
assertions), under ``-m gpu`` against the HIP product.
"""
import importlib
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# route-DB parity tests run the device route selection at every size (the
# product keeps fewer than 1024 prefixes on the host path by default)
os.environ.setdefault("ORH_DEVICE_SELECT_MIN", "0")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP product path)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def _load_oracle():
    build_dir = os.path.join(ROOT, "oracle", "build")
    mod_path = [p for p in os.listdir(build_dir)] if os.path.isdir(build_dir) else []
    if not any(p.startswith("openr_oracle") for p in mod_path):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    if build_dir not in sys.path:
        sys.path.insert(0, build_dir)
    return importlib.import_module("openr_oracle")


@pytest.fixture(scope="session")
def oracle_mod():
    return _load_oracle()


@pytest.fixture(scope="session")
def oracle(oracle_mod):
    from openr_amd.facade import Backend
    return Backend(oracle_mod, "oracle")


@pytest.fixture(scope="session")
def hip():
    from openr_amd import host_backend
    return host_backend()


@pytest.fixture(params=["oracle", pytest.param("hip", marks=pytest.mark.gpu),
                        pytest.param("hip_default_select", marks=pytest.mark.gpu)])
def backend(request, monkeypatch):
    """hip runs route selection on the device at every size (as set above);
    hip_default_select is the product's own default, where builds of fewer
    than 1,024 prefixes - every reference-sized test - select on the host."""
    if request.param == "hip_default_select":
        monkeypatch.delenv("ORH_DEVICE_SELECT_MIN", raising=False)
        return request.getfixturevalue("hip")
    return request.getfixturevalue(request.param)
