import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cruise-control_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device and the HIP build of libccmi.so")
    config.addinivalue_line("markers", "slow: larger parity cases")


def _make(path):
    """make under an exclusive lock: pytest-xdist workers reach the session fixtures concurrently."""
    import fcntl
    with open(os.path.join(path, ".make.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-C", path, "-j8"], check=True, capture_output=True)


@pytest.fixture(scope="session")
def oracle_lib():
    _make(os.path.join(REPO, "oracle"))
    from oracle_binding import Oracle

    return Oracle.lib()


@pytest.fixture(scope="session")
def emu_lib():
    """Test-only host emulation of the Device layer (tests/emu) — exercises the engine's host logic on CPU."""
    _make(os.path.join(REPO, "tests", "emu"))
    import ccmi

    return ccmi.Library.get(os.path.join(REPO, "tests", "emu", "libccmi_emu.so"))


@pytest.fixture(scope="session")
def gpu_lib():
    """The product library on a real gfx950 device (fails loudly if absent)."""
    lib_path = os.path.join(REPO, "cruise-control_amd", "libccmi.so")
    if not os.path.exists(lib_path):
        _make(os.path.join(REPO, "cruise-control_amd"))
    import ccmi

    return ccmi.Library.get(lib_path)
