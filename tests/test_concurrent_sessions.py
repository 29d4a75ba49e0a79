"""Many concurrent sessions share the library's host helpers: 8 C1-size what-if sessions run at
once on one GPU, each bit-exact against the C1 golden (the oracle's action log, assignment, leaders and stats), while
the stale-key tree helpers (engine.cpp TreeWorkerPool) stay within their process-wide cap."""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _run(sessions, cap, timeout, stagger=0.0, name="c1"):
    env = dict(os.environ, CCMI_TREE_WORKERS=str(cap), CCMI_TREE_WORKER_MIN="1")
    out = subprocess.run([sys.executable, "-u", os.path.join(HERE, "concurrent_sessions_worker.py"), name, str(sessions),
                          str(stagger)], env=env, capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stderr[-4000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
def test_gpu_eight_concurrent_c1_sessions_within_helper_cap():
    cap = 3
    r = _run(8, cap, 110)
    assert r["actions"] > 0
    assert 1 <= r["peak_helper_threads"] <= cap, r  # the pool was used, and never beyond its cap
    assert r["after"] <= cap  # idle helpers stay parked (no per-session threads left behind)


@pytest.mark.gpu
def test_gpu_staggered_sessions_each_get_a_server():
    """A call that begins while another call's scan server holds the whole device budget: the running server shrinks to
    its share at its next command (Device::ensureServer), so the later session's scans are served too — both bit-exact
    against the C1 golden."""
    r = _run(2, 4, 110, stagger=0.05)
    assert r["actions"] > 0
    assert all(s > 0 for s in r["server_scans"]), r
