"""Wall time of consecutive C2 proposals in one process (GPU box): sessions made up front (as bench.py does) or one
at a time, optionally after a CCMI_SERVER=0 proposal, to find what makes a later proposal slower than the first."""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cruise-control_amd"))
sys.path.insert(0, REPO)
import ccmi  # noqa: E402
from bench import WORKLOADS, workload_constraint  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c2")
ap.add_argument("--runs", type=int, default=3)
ap.add_argument("--upfront", action="store_true", help="create every session before the first proposal")
ap.add_argument("--launch-pass", action="store_true", help="one CCMI_SERVER=0 proposal first")
ap.add_argument("--timing", action="store_true", help="kernel timing on (as bench.py's warmup)")
ap.add_argument("--torch", action="store_true", help="initialise torch's HIP context first (as bench.py does)")
a = ap.parse_args()
if a.torch:
    import torch
    torch.cuda.set_device(0)
    torch.cuda.synchronize()
props, goal_names, _ = WORKLOADS[a.workload]
lib = ccmi.Library.get()
buf = ccmi.RandomCluster.generate(lib, **props)
goals = ccmi.goals_from_names(goal_names)
opt = ccmi.GoalOptimizer(workload_constraint(a.workload))
if a.launch_pass:
    os.environ["CCMI_SERVER"] = "0"
    s = ccmi.ClusterModel.from_buffers(buf, device=0)
    del os.environ["CCMI_SERVER"]
    t0 = time.perf_counter()
    opt.optimizations(s, goals, None)
    print(f"launch pass {time.perf_counter() - t0:.2f}s", flush=True)
    del s
sessions = [ccmi.ClusterModel.from_buffers(buf, device=0) for _ in range(a.runs)] if a.upfront else None
for i in range(a.runs):
    s = sessions[i] if sessions else ccmi.ClusterModel.from_buffers(buf, device=0)
    if a.timing:
        s.set_kernel_timing(True)
    t0 = time.perf_counter()
    opt.optimizations(s, goals, None)
    dt = time.perf_counter() - t0
    p = s.perf()
    print(f"run {i}: {dt:.2f}s server launches {p.server_launches} scans {p.server_scans} launches {p.scan_launches} "
          f"busy {p.server_busy_ms:.0f} ms", flush=True)
    if not sessions:
        del s
