"""One independent what-if proposal of the C1 chain in the CPU restatement (oracle/, test infrastructure) — a worker
process of bench.py's cpu_baseline "what_if_all_cores" leg. Prints {"candidates": n, "seconds": s}."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cruise-control_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

import ccmi  # noqa: E402
from oracle_binding import OracleCluster  # noqa: E402

props = json.loads(sys.argv[1])
goals = json.loads(sys.argv[2])
oc = OracleCluster.random(**props)
t0 = time.perf_counter()
res = oc.optimize(goals, ccmi.BalancingConstraint())
print(json.dumps({"candidates": sum(r.candidates for r in res), "seconds": time.perf_counter() - t0}))
