import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cassandra-accord_amd")
for p in (PKG, os.path.join(ROOT, "tests"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C ABI)")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    # build in-tree artefacts once if missing (the GPU box receives the prebuilt .so files)
    if not os.path.exists(os.path.join(PKG, "libaccord_deps.so")):
        subprocess.run(["make", "-C", PKG, "-j8"], check=True, capture_output=True)
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    # a session that runs GPU tests brings torch's HIP runtime up before any test loads the library:
    # a CPU test loading libaccord_deps.so first leaves the later device probe without a device
    if "not gpu" not in (config.getoption("markexpr", "") or ""):
        import torch  # noqa: F401


@pytest.fixture(scope="session")
def gpu_device():
    import torch  # noqa: F401  (device count probe only)
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    n = ctypes.c_int(0)
    if hip.hipGetDeviceCount(ctypes.byref(n)) != 0 or n.value == 0:
        pytest.fail("gpu test without a HIP device")
    return 0
