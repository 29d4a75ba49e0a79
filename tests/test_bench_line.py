"""bench.py's offline pieces (no GPU): the committed PMC evidence it prices the roofline line with."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


class _Perf:
    def __init__(self, launches, scans):
        self.server_launches = launches
        self.server_scans = scans


def test_server_traffic_uses_the_profiled_runs_commands_per_launch():
    """HBM bytes per server command = the PMC summary's bytes per scan_server launch over the commands per launch of
    the run the counters came from (its own bench line), whatever this run's launch count is."""
    traffic, src = bench.pmc_server_traffic("c2", _Perf(1, 1))
    assert src is not None and traffic is not None
    with open(os.path.join(REPO, src)) as f:
        k = json.load(f)["kernels"]["scan_server"]
    prof = sorted(p for p in os.listdir(os.path.dirname(os.path.join(REPO, src))) if p.startswith("c2_bench_prof"))
    assert prof, "the PMC summary's own bench line is committed beside it"
    with open(os.path.join(os.path.dirname(os.path.join(REPO, src)), prof[-1])) as f:
        r = json.loads(f.read().strip().splitlines()[-1])["roofline"]
    per_launch = r["server_commands_per_step"] / r["server_launches_per_step"]
    assert abs(traffic - k["hbm_bytes_per_launch"] / per_launch) <= 1e-6 * traffic
    # the same answer for any current-run ratio
    assert bench.pmc_server_traffic("c2", _Perf(990, 108477))[0] == traffic


def test_scan_traffic_summary_is_committed():
    traffic, src = bench.pmc_traffic("c2")
    assert traffic and traffic > 0 and src.startswith("profiles/")
