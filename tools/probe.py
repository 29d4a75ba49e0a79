"""One optimization of a BASELINE workload with per-goal wall time, candidates and device launches (GPU box)."""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cruise-control_amd"))
sys.path.insert(0, REPO)
import ccmi  # noqa: E402
from bench import WORKLOAD_OPTIONS, WORKLOADS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c2")
ap.add_argument("--goals", type=int, default=16)
ap.add_argument("--lib", default=None, help="alternative libccmi build (e.g. tests/emu/libccmi_emu.so on CPU)")
a = ap.parse_args()
props, goals, name = WORKLOADS[a.workload]
lib = ccmi.Library.get(a.lib) if a.lib else ccmi.Library.get()
t0 = time.time()
buf = ccmi.RandomCluster.generate(lib, **props)
t1 = time.time()
cm = ccmi.ClusterModel.from_buffers(buf, device=0)
t2 = time.time()
print(f"{name}: generate {t1 - t0:.2f}s, session {t2 - t1:.2f}s", flush=True)
opts = WORKLOAD_OPTIONS[a.workload]() if a.workload in WORKLOAD_OPTIONS else None
res = ccmi.GoalOptimizer(ccmi.BalancingConstraint()).optimizations(cm, ccmi.goals_from_names(goals[:a.goals]), opts)
t3 = time.time()
for g in res.goal_results:
    print(f"  {g.name:40s} ok={g.succeeded} {g.seconds:8.3f}s cand={g.candidates:>12d} act={g.actions:>7d} "
          f"launches={g.device_launches}", flush=True)
print(f"total {t3 - t2:.2f}s, {res.candidates} candidates, {len(cm.actions())} actions, {len(res.proposals)} proposals")
p = cm.perf()
print(f"perf: scan launches {p.scan_launches} (server {p.server_launches}, chains {p.chain_launches}, cross "
      f"{p.cross_launches}), server scans {p.server_scans} busy {p.server_busy_ms:.1f} ms, host syncs {p.host_syncs}, "
      f"required {p.scan_required} (server {p.server_required}), server payload {p.server_payload_bytes / 1e6:.1f} MB")
