"""Child process of test_concurrent_sessions.py: S concurrent what-if sessions of one golden case on cuda:0, one host
thread each (GoalOptimizer.java:117-119's precompute pool), with the tree helper pool capped by CCMI_TREE_WORKERS and
forced on for every cluster size (CCMI_TREE_WORKER_MIN=1). A sampler thread counts the library's helper threads
("ccmi-tree" in /proc/self/task/*/comm) while the sessions run. Prints one JSON line."""
import json
import os
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "cruise-control_amd"))
sys.path.insert(0, HERE)

import ccmi  # noqa: E402
from parity import constraint, golden, golden_options  # noqa: E402
from test_oracle_kat import check_against_golden  # noqa: E402


def helper_threads():
    n = 0
    for t in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{t}/comm") as f:
                n += f.read().strip() == "ccmi-tree"
        except OSError:
            pass
    return n


def main():
    name, sessions = sys.argv[1], int(sys.argv[2])
    stagger = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0  # seconds between the sessions' starts
    lib = ccmi.Library.get(os.path.join(os.path.dirname(HERE), "cruise-control_amd", "libccmi.so"))
    g = golden(name)
    bc = constraint(g["resource_balance_percentage"], g.get("max_replicas_per_broker"), g.get("capacity_threshold"))
    buf = ccmi.RandomCluster.generate(lib, **g["props"])
    cms = [ccmi.ClusterModel.from_buffers(buf, device=0) for _ in range(sessions)]
    peak, stop = [0], [False]

    def sample():
        while not stop[0]:
            peak[0] = max(peak[0], helper_threads())
            time.sleep(0.002)

    th = threading.Thread(target=sample, daemon=True)
    th.start()
    opt = ccmi.GoalOptimizer(bc)
    t0 = time.perf_counter()
    def one(i):
        time.sleep(i * stagger)
        return opt.optimizations(cms[i], ccmi.goals_from_names(g["goals"]), golden_options(g))

    with ThreadPoolExecutor(sessions) as pool:
        results = list(pool.map(one, range(sessions)))
    wall = time.perf_counter() - t0
    stop[0] = True
    th.join()
    for cm, res in zip(cms, results):
        check_against_golden(g, cm.actions(), cm.replica_distribution(), cm.leader_distribution(), res.goal_results,
                             res.goal_results[-1].stats, replica_disks=cm.replica_disks())
    print(json.dumps({"sessions": sessions, "peak_helper_threads": peak[0], "after": helper_threads(),
                      "actions": len(cms[0].actions()), "wall_s": wall,
                      "server_scans": [cm.perf().server_scans for cm in cms],
                      "scan_launches": [cm.perf().scan_launches for cm in cms]}))


if __name__ == "__main__":
    main()
