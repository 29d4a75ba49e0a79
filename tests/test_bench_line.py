"""bench.py's offline pieces (no GPU): the committed PMC evidence it prices the roofline line with."""
import json
import os
import sys

import pytest

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


def _profiled_runs(workload):
    """(round dir, tag) of every committed rocprofv3 run of `workload`: its bench line <workload>_bench_prof_<tag>.json
    next to the kernel-trace stats of the same command, <workload>_kernel_stats_<tag>.csv."""
    import glob
    runs = []
    for line in sorted(glob.glob(os.path.join(REPO, "profiles", "r*", f"{workload}_bench_prof_*.json"))):
        tag = os.path.basename(line)[len(f"{workload}_bench_prof_"):-len(".json")]
        csv = os.path.join(os.path.dirname(line), f"{workload}_kernel_stats_{tag}.csv")
        if os.path.exists(csv):
            runs.append((line, csv))
    return runs


def _avg_ns(csv_path, kernel):
    import csv
    with open(csv_path) as f:
        rows = [r for r in csv.DictReader(f) if r["Name"].split("(")[0] == f"ccmi::{kernel}"]
    assert len(rows) == 1, (csv_path, kernel)
    return float(rows[0]["AverageNs"]), int(rows[0]["Calls"])


@pytest.mark.parametrize("workload,kernel", [("c2", "scan_server"), ("c4", "intra_brokers")])
def test_headline_frac_follows_committed_kernel_stats(workload, kernel):
    """The bench line's headline roofline.frac = algorithmic bytes per launch of the dominant kernel over its average
    launch duration / peak; the same figure recomputed from the rocprofv3 kernel-trace average of the same command
    (committed beside the line) agrees within 10 %."""
    runs = _profiled_runs(workload)
    assert runs, f"no committed {workload} bench line + kernel stats pair under profiles/"
    line_path, csv_path = runs[-1]
    with open(line_path) as f:
        r = json.loads(f.read().strip().splitlines()[-1])["roofline"]
    avg_ns, calls = _avg_ns(csv_path, kernel)
    assert calls > 0
    alg = r["algorithmic_bytes_per_launch"]
    frac = alg / (avg_ns * 1e-9) / 1e9 / r["peak"]
    assert abs(frac - r["frac"]) <= 0.10 * r["frac"], (line_path, frac, r["frac"])
    assert abs(r["avg_launch_us"] * 1e3 - avg_ns) <= 0.10 * avg_ns
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"])
    if kernel == "scan_server":  # the headline is the launch (residency) view, the per-command one secondary
        assert r["resident"]["frac"] == pytest.approx(r["frac"])
        assert r["per_command"]["frac"] > r["frac"]


def _bench_emu(emu_lib, gpus, devices, extra=()):
    import subprocess
    env = dict(os.environ, CCMI_EMU_DEVICES=str(devices))
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--lib", emu_lib.path, "--workload", "c0", "--gpus",
           str(gpus), "--steps", "1", "--warmup", "1", "--no-cpu-baseline", *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_bench_plain_launch_runs_one_session_per_device(emu_lib):
    """`python3 bench.py --gpus 2` without torchrun (the driver's plain form) runs two independent what-if proposals
    per step in one process, one on each of device ordinals 0 and 1 (CPU emulation with two devices), and reports the
    whole job: n_gpus 2, both proposals' candidates."""
    one = _bench_emu(emu_lib, 1, 2)
    two = _bench_emu(emu_lib, 2, 2)
    assert one["n_gpus"] == 1 and one["devices"] == [0]
    assert two["n_gpus"] == 2 and two["devices"] == [0, 1] and two["devices_note"] is None
    # weak scaling: the same proposal on every device, so twice the candidates per step
    assert two["value"] * two["ms_per_step"] == pytest.approx(2 * one["value"] * one["ms_per_step"], rel=1e-9)
    assert two["scaling"] == "weak" and "x2" in two["config"]["parallelism"]


def test_bench_plain_launch_with_fewer_devices_says_so(emu_lib):
    """--gpus 2 on a one-device box: both sessions on ordinal 0, reported as a rehearsal."""
    two = _bench_emu(emu_lib, 2, 1)
    assert two["n_gpus"] == 2 and two["devices"] == [0] and "rehearsal" in two["devices_note"]
