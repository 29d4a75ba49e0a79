"""The boundary documentation against the code, and the library's side effects on the caller's thread.

* INTEGRATION.md quotes the ABI version a shim is written against; it must be the one include/ccmi.h defines and the
  library reports (ccmi_abi_version).
* The status-5 (CCMI_E_UNSUPPORTED) cases INTEGRATION.md lists are the ones the engine produces: an optimizedGoals
  member the session does not hold (Goal.optimize(clusterModel, optimizedGoals, options), Goal.java:60-68; exercised
  in test_optimized_goals.py), and the reference's own UnsupportedOperationException mid-optimization. Shared hosts are
  NOT one of them: a CPU / NW_IN / NW_OUT goal on brokers that share a host runs on the device (ABI v8).
* ccmi_session_create / ccmi_optimizations pin the calling thread to the GPU's NUMA node for the call only and restore
  the caller's CPU mask (threadpin.h); CCMI_NUMA_CPULIST stands in for the PCI local_cpulist here.
"""
import os
import re
import subprocess
import sys

import pytest

import ccmi

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _integration():
    return open(os.path.join(REPO, "INTEGRATION.md")).read()


def test_integration_abi_version_matches_header_and_library(emu_lib):
    quoted = re.findall(r"`ccmi_abi_version\(\)` = (\d+)", _integration())
    assert quoted, "INTEGRATION.md quotes no ABI version"
    header = int(re.search(r"#define CCMI_ABI_VERSION (\d+)", open(os.path.join(REPO, "include", "ccmi.h")).read()).group(1))
    assert {int(q) for q in quoted} == {header}
    assert emu_lib.lib.ccmi_abi_version() == header
    # every "(ABI vN)" INTEGRATION.md cites is a version this library has reached
    assert all(int(v) <= header for v in re.findall(r"ABI v(\d+)", _integration()))


def test_integration_status5_cases_are_the_engine_cases():
    text = _integration()
    # no paragraph may send shared-host clusters to the JVM any more
    for para in text.split("\n\n"):
        if "share a host" in para or "shared host" in para.lower():
            assert "No status 5 comes from shared" in para or "status 5" not in para, para
    # the shim's status-5 branch names exactly the two causes the engine has
    assert "a goal in optimizedGoals has no device state" in text
    assert "UnsupportedOperationException" in text


def test_emu_shared_host_cpu_goal_is_not_unsupported(emu_lib, oracle_lib):
    """A chain with CPU / NW_IN / NW_OUT capacity and distribution goals on brokers that share hosts runs (status 0)."""
    from test_hosts import SHARED, _model  # the shared-host builder model

    flat = _model(SHARED)
    cm = ccmi.ClusterModel(flat.desc, device=0, lib=emu_lib, keepalive=flat)
    res = ccmi.GoalOptimizer(ccmi.BalancingConstraint()).optimizations(
        cm, ccmi.goals_from_names(["CpuCapacityGoal", "CpuUsageDistributionGoal", "NetworkOutboundUsageDistributionGoal"]))
    assert len(res.goal_results) == 3


_AFFINITY_SCRIPT = r"""
import os, sys, threading, time, ctypes as C
sys.path.insert(0, {pkg!r}); sys.path.insert(0, {tests!r})
import ccmi
lib = ccmi.Library.get({lib!r})
main_tid = threading.get_native_id()
before = os.sched_getaffinity(0)
seen = set()
stop = False
def sample():  # the driving thread's mask while the call runs
    while not stop:
        for line in open(f"/proc/self/task/{{main_tid}}/status"):
            if line.startswith("Cpus_allowed_list"):
                seen.add(line.split()[1])
        time.sleep(0.0005)
t = threading.Thread(target=sample, daemon=True)
t.start()
buf = ccmi.RandomCluster.generate(lib, num_racks=5, num_brokers=60, num_replicas=30000, num_topics=300)
cm = ccmi.ClusterModel(buf.desc, device=0, lib=lib, keepalive=buf)
after_create = os.sched_getaffinity(0)
ccmi.GoalOptimizer(ccmi.BalancingConstraint()).optimizations(
    cm, ccmi.goals_from_names(["ReplicaDistributionGoal", "DiskUsageDistributionGoal", "CpuUsageDistributionGoal"]))
after_opt = os.sched_getaffinity(0)
del cm
stop = True
t.join()
print(sorted(before) == sorted(after_create) == sorted(after_opt) == sorted(os.sched_getaffinity(0)),
      {pinned!r} in seen)
"""


def test_session_calls_pin_only_for_their_duration(emu_lib):
    """The NUMA pin is scoped to each call: the driving thread runs on the device's CPUs while ccmi_optimizations runs,
    and the caller's CPU mask is the same before and after create, optimize and destroy."""
    cpus = sorted(os.sched_getaffinity(0))
    if len(cpus) < 2:
        pytest.skip("one CPU: nothing to narrow")
    pinned = str(cpus[0])
    code = _AFFINITY_SCRIPT.format(pkg=os.path.join(REPO, "cruise-control_amd"), tests=os.path.join(REPO, "tests"),
                                   lib=os.path.join(REPO, "tests", "emu", "libccmi_emu.so"), pinned=pinned)
    env = dict(os.environ, CCMI_NUMA_CPULIST=pinned)
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    restored, pinned_during = out.stdout.split()
    assert restored == "True"
    assert pinned_during == "True"
