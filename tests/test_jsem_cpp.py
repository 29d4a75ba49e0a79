"""The C++ unit checks of engine/jsem.h (tests/cpp/test_jsem.cpp): built with g++ and run, CPU only."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_jsem_containers(tmp_path):
    exe = str(tmp_path / "test_jsem")
    subprocess.run(["g++", "-O1", "-std=c++17", "-I", os.path.join(REPO, "cruise-control_amd", "csrc", "engine"),
                    os.path.join(REPO, "tests", "cpp", "test_jsem.cpp"), "-o", exe], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "jsem ok" in r.stdout
