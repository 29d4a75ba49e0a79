"""The C++ unit checks of engine/hostpool.h (tests/cpp/test_hostpool.cpp): built with g++ and run, CPU only."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_hostpool_crews(tmp_path):
    exe = str(tmp_path / "test_hostpool")
    subprocess.run(["g++", "-O1", "-std=c++17", "-pthread", "-I", os.path.join(REPO, "cruise-control_amd", "csrc", "engine"),
                    os.path.join(REPO, "tests", "cpp", "test_hostpool.cpp"), "-o", exe], check=True)
    env = dict(os.environ, CCMI_SYNC_THREADS="4", CCMI_SYNC_CREWS="3")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr
    assert "hostpool ok" in r.stdout
