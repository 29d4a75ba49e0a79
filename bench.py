"""Headline benchmark: candidate moves evaluated/s + proposal wall time (BASELINE.json `metric`).

Workload (default, BASELINE.json configs[2] — the configuration the metric is quoted on, and it fits one GPU):
RandomCluster C2 = 100 racks, 10 000 brokers, 999 999 + 20 000 replicas (R = 1 019 999), 10 001 topics, W = 1,
uniform loads, TestConstants seeds; the 16 default goals in default priority order; default BalancingConstraint.
--workload c1 / c3 / c4 / c2_c1goals / c0 select the other BASELINE configs (parity-test cases, not headline lines);
c4 (JBOD, the intra-broker goals) reports the K6 kernel in its roofline.

A "step" is one full GoalOptimizer.optimizations over that cluster (every goal, ClusterModelStats after every goal,
final ExecutionProposals). Each step works on its own device session, uploaded to HBM before the timed region
starts (the session upload — the ClusterModel the caller hands over — is outside the timed region, as the reference
does not time model building either; its time is reported as session_upload_s); K steps = K independent proposals.

value = reference-equivalent candidate moves evaluated/s summed over all ranks (the candidates the reference's
first-fit loops visit), ms_per_step = step wall time = proposal wall time at the default
--requests-per-gpu 1. --requests-per-gpu S runs S independent what-if proposals concurrently per GPU in every step
(one host thread + HIP stream per session, GoalOptimizer's precompute pool); proposal_wall_s is then the mean
per-proposal latency.

Parity: the first timed proposal is checked against the committed oracle golden of the workload (tests/golden/:
action log, final assignment and leaders, per-goal results, every goal's stats within 1e-9) -> "parity".

Multi-GPU: under torchrun (one process per GPU) every rank runs its own independent what-if proposal request by
default (weak scaling, no data-path collective); timing is max over ranks. A plain `python3 bench.py --gpus N` (no
WORLD_SIZE) runs the same N independent proposals per step in one process, one session per device 0..N-1 on its own
host thread, timed from a common start until the slowest device finishes; n_gpus = N and `devices` lists the ordinals
used (fewer devices than N: sessions share them round-robin, flagged in `devices_note`). --sharded instead shards ONE proposal's
candidate space by destination broker over the ranks (strong scaling): every scan's per-rank first-fit keys are
MIN-combined in host shared memory (--combiner shm, the default on one node: no GPU work per combine, so every rank
keeps its scan server) or by an RCCL MIN allreduce (--combiner rccl).

Roofline: the dominant kernels are the candidate scans (scan_cross / scan_pairs / scan_swap / chain_pairs /
chain_rack_rows). Their HIP-event duration is measured during the warmup proposal(s) (events on the engine stream,
outside the timed region); algorithmic bytes = 96 B per candidate the launches had to evaluate (every device list up
to its winner: ccmi_perf_counters.scan_required). traffic = HBM bytes per scan launch from the
committed rocprofv3 PMC summary of this workload. cpu_baseline = the single-threaded C++ restatement (oracle/,
"port") on rank 0 at N = 1 (see cpu_baseline()).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import struct
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "cruise-control_amd"))

import ccmi  # noqa: E402

C1_PROPS = dict(num_racks=20, num_brokers=1000, num_replicas=99999, num_topics=3000)
C2_PROPS = dict(num_racks=100, num_brokers=10000, num_replicas=999999, num_topics=10000)
# C3: RandomSelfHealingTest-style placement (6-arg populate, rack-aware, leader first; RandomCluster.java:119-124)
C3_PROPS = dict(C2_PROPS, num_dead_brokers=500, rack_aware=1, leader_in_first_position=1)
# C4: the C2 cluster on 4 x 75 000 MB logdirs per broker, rack-aware populate (tests/golden/make_golden.py C4_PROPS)
C4_PROPS = dict(C2_PROPS, rack_aware=1, leader_in_first_position=1, jbod=2, num_logdirs=4,
                logdir_capacity=[75000.0] * 4)
C1_GOALS = list(ccmi.C1_GOALS)
DEFAULT_GOALS = list(ccmi.DEFAULT_GOALS)
INTRA_GOALS = list(ccmi.INTRA_BROKER_GOALS)
WORKLOADS = {"c1": (C1_PROPS, C1_GOALS, "C1: 1K brokers x 100K replicas, 5 distribution goals (BASELINE configs[1])"),
             "c2": (C2_PROPS, DEFAULT_GOALS, "C2: 10K brokers x 1M replicas, the 16 default goals (BASELINE configs[2])"),
             "c2_c1goals": (C2_PROPS, C1_GOALS, "C2 cluster with the C1 goal list"),
             "c3": (C3_PROPS, DEFAULT_GOALS, "C3: C2 with brokers 0..499 DEAD, requested destinations 500..1499, the 16 "
                                           "default goals (BASELINE configs[3], RemoveBrokersRunnable options)"),
             "c4": (C4_PROPS, INTRA_GOALS, "C4: JBOD C2 cluster x 4 logdirs, IntraBrokerDiskCapacityGoal + "
                                          "IntraBrokerDiskUsageDistributionGoal with its swap phase (BASELINE configs[4])"),
             "c0": ({}, DEFAULT_GOALS, "C0: TestConstants.BASE_PROPERTIES, the 16 default goals (BASELINE configs[0])")}


def workload_constraint(workload: str) -> "ccmi.BalancingConstraint":
    """Default BalancingConstraint; C4 uses IntraBrokerRebalanceTest's (IntraBrokerRebalanceTest.java:103-111)."""
    bc = ccmi.BalancingConstraint()
    if workload == "c4":
        bc.max_replicas_per_broker = 2000
        bc.set_resource_balance_percentage(1.05)
        bc.set_capacity_threshold(0.8)
    return bc
# Per-workload OptimizationOptions (C3: the 7-arg options RemoveBrokersRunnable.java:107-126 builds)
WORKLOAD_OPTIONS = {"c3": lambda: ccmi.OptimizationOptions(requested_destination_broker_ids=list(range(500, 1500)),
                                                           fast_mode=False)}
# committed oracle goldens of the workloads (tests/golden/make_golden.py)
WORKLOAD_GOLDEN = {"c1": "c1", "c2": "c2_default", "c2_c1goals": "c2_c1goals", "c3": "c3_default", "c4": "c4"}
BYTES_PER_CANDIDATE = 96
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
# candidate-heavy C2 goal the CPU baseline samples on the box (the reference's costliest goal at C2)
C2_SAMPLE_GOAL = "CpuUsageDistributionGoal"


def _sha(ints):
    return hashlib.sha256(struct.pack(f"<{len(ints)}q", *ints)).hexdigest()


def check_parity(workload: str, cm, result) -> dict:
    """The first timed proposal against the workload's committed oracle golden."""
    name = WORKLOAD_GOLDEN.get(workload)
    path = os.path.join(REPO, "tests", "golden", f"{name}.json") if name else None
    if not path or not os.path.exists(path):
        return {"golden": None, "status": "no golden for this workload"}
    with open(path) as f:
        g = json.load(f)
    problems = []
    acts = cm.actions()
    if len(acts) != g["num_actions"]:
        problems.append(f"{len(acts)} actions vs {g['num_actions']}")
    norm = [a[:5] if len(a) == 7 and a[5] == -1 and a[6] == -1 else a for a in acts]  # make_golden.flat_actions
    if _sha([x for a in norm for x in a]) != g["actions_sha256"]:
        problems.append("action log")
    if "replica_disks_sha256" in g and _sha(cm.replica_disks()) != g["replica_disks_sha256"]:
        problems.append("replica disks")
    if _sha(cm.replica_distribution()) != g["replica_distribution_sha256"]:
        problems.append("replica distribution")
    if _sha(cm.leader_distribution()) != g["leader_distribution_sha256"]:
        problems.append("leader distribution")
    worst = 0.0
    for r, e in zip(result.goal_results, g["goals_result"]):
        if (r.name, r.succeeded, r.candidates, r.actions) != (e["name"], e["succeeded"], e["candidates"], e["actions"]):
            problems.append(f"goal {r.name}")
        for k, v in (e.get("stats") or {}).items():
            got = r.stats[k]
            for x, y in zip(got if isinstance(got, list) else [got], v if isinstance(v, list) else [v]):
                if x != y:
                    rel = abs(x - y) / max(abs(y), 1e-300)
                    if abs(x - y) > 1e-12 and rel > worst:
                        worst = rel
    if worst > 1e-9:
        problems.append(f"stats rel {worst:.2e}")
    return {"golden": os.path.relpath(path, REPO), "status": "ok" if not problems else "MISMATCH: " + ", ".join(problems),
            "actions": len(acts), "max_stats_rel_diff": worst,
            "checked": "action log + final assignment + leaders (+ disks for JBOD) (SHA-256), per-goal (name, "
                       "succeeded, candidates, actions), every goal's ClusterModelStats within 1e-9 relative"}


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _c1_chain_procs(n: int):
    """n independent what-if proposals of the C1 chain in the restatement, one child process each
    (tools/cpu_whatif.py); returns [(candidates, seconds)] and the wall time of the whole batch."""
    import subprocess
    cmd = [sys.executable, os.path.join(REPO, "tools", "cpu_whatif.py"), json.dumps(C1_PROPS), json.dumps(C1_GOALS)]
    t0 = time.perf_counter()
    procs = [subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True) for _ in range(n)]
    outs = [json.loads(p.communicate()[0]) for p in procs]
    wall = time.perf_counter() - t0
    if any(p.returncode for p in procs):
        raise RuntimeError("a CPU what-if worker failed")
    return [(o["candidates"], o["seconds"]) for o in outs], wall


def cpu_baseline(lib, buf, workload: str, goal_names, options, gpu_result, device: int, sample_s: float,
                 what_if_procs: int) -> dict:
    """The oracle restatement (oracle/, "port"), single thread, on the GPU box's host cores (rank 0, N = 1):

    * value — a bounded sample of THIS workload: the restatement runs `C2_SAMPLE_GOAL` (the costliest goal) on the
      same cluster for `sample_s` seconds of wall time (its ClusterModelStats calls included, as in the reference);
      the GPU runs the same single-goal optimization to completion beside it (gpu_same_sample).
    * c1_chain — the whole C1 chain (BASELINE configs[1]), 1 thread, next to the GPU's C1 chain.
    * what_if_all_cores — `what_if_procs` independent C1 proposals at once, one process each (the reference's
      precompute pool with num.proposal.precompute.threads = what_if_procs).
    * per_goal_full_chain — the whole chain's per-goal restatement seconds from the committed golden (measured in
      the build container when the golden was generated) beside this run's per-goal GPU seconds.
    """
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle_binding import OracleCluster
    out = {"unit": "candidate moves evaluated/s", "cores": 1, "kind": "port",
           "nproc": os.cpu_count(), "cpu_share": len(os.sched_getaffinity(0)), "cpu_model": _cpu_model(),
           "num.proposal.precompute.threads": 1}
    # (1) bounded sample of the same workload
    goal = {"c2": C2_SAMPLE_GOAL, "c3": C2_SAMPLE_GOAL, "c2_c1goals": C2_SAMPLE_GOAL,
            "c4": "IntraBrokerDiskUsageDistributionGoal"}.get(workload, goal_names[0])
    bc = workload_constraint(workload)
    oc = OracleCluster.from_desc(buf.desc)
    t0 = time.perf_counter()
    done, cands, stats_s = oc.optimize_until([goal], sample_s, bc, options)
    dt = time.perf_counter() - t0
    del oc
    s = ccmi.ClusterModel.from_buffers(buf, device=device)
    r = ccmi.GoalOptimizer(bc).optimizations(s, ccmi.goals_from_names([goal]), options)
    del s
    out["value"] = cands / dt
    out["sample"] = (f"{goal} alone on the {workload.upper()} cluster, restatement stopped after {dt:.1f} s "
                     f"({'completed' if done else 'deadline'}): {cands} candidates, {stats_s:.1f} s of it in "
                     f"ClusterModelStats")
    out["sample_loop_rate"] = cands / max(1e-9, dt - stats_s)
    out["gpu_same_sample"] = {"goal": goal, "seconds": r.seconds, "candidates": r.candidates,
                              "value": r.candidates / r.seconds}
    if workload == "c4":  # the C1-chain comparisons below are about the inter-broker goals
        what_if_procs = 0
    # (2) the whole C1 chain, 1 thread, and the GPU's C1 chain
    if what_if_procs == 0:
        return _per_goal_from_golden(out, workload, gpu_result)
    ((c1c, c1t),), _ = _c1_chain_procs(1)
    b1 = ccmi.RandomCluster.generate(lib, **C1_PROPS)
    s1 = ccmi.ClusterModel.from_buffers(b1, device=device)
    r1 = ccmi.GoalOptimizer(ccmi.BalancingConstraint()).optimizations(s1, ccmi.goals_from_names(C1_GOALS))
    del s1
    out["c1_chain"] = {"restatement_s": c1t, "candidates": c1c, "restatement_value": c1c / c1t,
                       "gpu_s": r1.seconds, "gpu_value": r1.candidates / r1.seconds}
    # (3) independent what-if proposals on all host cores of this box's share
    n = max(1, min(what_if_procs, out["cpu_share"]))
    rs, wall = _c1_chain_procs(n)
    out["what_if_all_cores"] = {"processes": n, "proposals": n, "batch_wall_s": wall,
                                "slowest_proposal_s": max(t for _, t in rs),
                                "value": sum(c for c, _ in rs) / max(t for _, t in rs),
                                "workload": "C1 chain per process (num.proposal.precompute.threads = processes)"}
    return _per_goal_from_golden(out, workload, gpu_result)


def _per_goal_from_golden(out: dict, workload: str, gpu_result) -> dict:
    """(4) per-goal full-chain restatement seconds (golden) beside the GPU's."""
    name = WORKLOAD_GOLDEN.get(workload)
    path = os.path.join(REPO, "tests", "golden", f"{name}.json") if name else None
    if path and os.path.exists(path):
        with open(path) as f:
            g = json.load(f)
        rows = []
        for e, rr in zip(g["goals_result"], gpu_result.goal_results):
            if "seconds" in e:
                rows.append({"goal": e["name"], "candidates": e["candidates"], "restatement_s": round(e["seconds"], 3),
                             "gpu_s": round(rr.seconds, 4)})
        if rows:
            tot = sum(x["restatement_s"] for x in rows)
            out["per_goal_full_chain"] = {
                "source": f"{os.path.relpath(path, REPO)} (restatement timed in the build container, 1 thread)",
                "restatement_total_s": tot, "gpu_total_s": sum(x["gpu_s"] for x in rows),
                "restatement_value": sum(x["candidates"] for x in rows) / tot, "goals": rows}
    return out


SCAN_KERNELS = ("scan_cross", "scan_pairs", "scan_swap", "chain_pairs", "chain_rack_rows")
INTRA_KERNELS = ("intra_brokers",)


def pmc_traffic(workload: str, kernels=SCAN_KERNELS):
    """HBM bytes per scan launch from the newest committed PMC summary of this workload (profiles/rNN/
    <workload>_pmc_summary.json, written by tools/pmc_summary.py from separate rocprofv3 --pmc FETCH_SIZE /
    WRITE_SIZE passes of this same bench command). PMC counters cannot be read inside the timed process."""
    import glob
    paths = sorted(glob.glob(os.path.join(REPO, "profiles", "r*", f"{workload}_pmc_summary.json")))
    if not paths:
        return None, None
    with open(paths[-1]) as f:
        ks = json.load(f)["kernels"]
    n = sum(ks[k]["launches"] for k in kernels if k in ks)
    b = sum(ks[k]["launches"] * ks[k]["hbm_bytes_per_launch"] for k in kernels if k in ks)
    return (b / n if n else None), os.path.relpath(paths[-1], REPO)


def pmc_server_traffic(workload: str, perf):
    """HBM bytes per scan-server command: scan_server's counter bytes per launch in the newest committed PMC summary
    divided by the commands per server launch of the profiled run itself (its bench line, <workload>_bench_prof*.json
    beside the summary; this run's ratio when that is missing). The counters also see the idle workgroups polling."""
    import glob
    paths = sorted(glob.glob(os.path.join(REPO, "profiles", "r*", f"{workload}_pmc_summary.json")))
    if not paths:
        return None, None
    with open(paths[-1]) as f:
        k = json.load(f)["kernels"].get("scan_server")
    if not k or perf.server_launches <= 0:
        return None, None
    per_launch = perf.server_scans / perf.server_launches
    prof = sorted(glob.glob(os.path.join(os.path.dirname(paths[-1]), f"{workload}_bench_prof*.json")))
    if prof:
        try:
            with open(prof[-1]) as f:
                r = json.loads(f.read().strip().splitlines()[-1])["roofline"]
            if r.get("server_launches_per_step"):
                per_launch = r["server_commands_per_step"] / r["server_launches_per_step"]
        except (OSError, ValueError, KeyError, IndexError):
            pass
    return k["hbm_bytes_per_launch"] / per_launch, os.path.relpath(paths[-1], REPO)


def scan_cross_line(perf, workload: str):
    """scan_cross alone: its algorithmic bytes per launch (required candidates x BYTES_PER_CANDIDATE) next to its
    calibrated HBM counter bytes per launch from the committed PMC summary (tools/pmc_calib: FETCH_SIZE x2 holds for
    its 128-B record gathers, profiles/r02/calib_summary.json)."""
    n = max(1, perf.cross_launches)
    alg = perf.cross_required * BYTES_PER_CANDIDATE / n
    traffic, src = pmc_traffic(workload, ("scan_cross",))
    avg_us = perf.cross_kernel_ms * 1e3 / n
    return {"launches_per_step": perf.cross_launches, "avg_launch_us": avg_us,
            "algorithmic_bytes_per_launch": alg, "achieved_gbs": alg / (avg_us * 1e-6) / 1e9 if avg_us > 0 else 0.0,
            "traffic_bytes_per_launch": traffic, "traffic_over_algorithmic": traffic / alg if traffic and alg else None,
            "traffic_source": src}


class GroupSession:
    """The sessions of one shard group (bench --sharded --combiner group): optimized together, one host thread per
    rank; rank 0 stands for the proposal (every rank makes the same decisions)."""

    def __init__(self, ranks):
        from concurrent.futures import ThreadPoolExecutor
        self.ranks = ranks
        self.pool = ThreadPoolExecutor(len(ranks))

    def optimize(self, opt, goals, options):
        return list(self.pool.map(lambda s: opt.optimizations(s, goals, options), self.ranks))[0]

    def __getattr__(self, name):  # perf(), set_kernel_timing(), reset_perf(), ... of rank 0
        return getattr(self.ranks[0], name)


def progress(msg: str) -> None:
    """A progress line on stderr (long runs print one per proposal; stdout carries only the result line)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def optimize(opt, s, goals, options):
    return s.optimize(opt, goals, options) if isinstance(s, GroupSession) else opt.optimizations(s, goals, options)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="N GPUs. Under torchrun (WORLD_SIZE set) one rank per GPU; from a plain launch, N sessions on "
                         "devices 0..N-1 of this process, one host thread each (independent what-if proposals)")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-launch-pass", action="store_true", help="skip the instrumented scan-server-off proposal")
    ap.add_argument("--cpu-sample-seconds", type=float, default=25.0)
    ap.add_argument("--what-if-procs", type=int, default=16)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c2")
    ap.add_argument("--requests-per-gpu", type=int, default=1,
                    help="S concurrent what-if proposals per GPU in every step (one host thread + HIP stream per "
                         "session; the precompute pool of GoalOptimizer.java:117-119). Default 1: one proposal per step")
    ap.add_argument("--combiner", choices=("shm", "rccl", "group"), default="shm",
                    help="--sharded: the per-scan MIN combiner (host shared memory on one node, RCCL, or 'group': ONE "
                         "process drives --gpus N sessions, one per GPU on its own thread, and the scan servers "
                         "combine on the device through a shard group; run without torchrun)")
    ap.add_argument("--sharded", action="store_true",
                    help="N>1: one proposal sharded by destination broker over all ranks (a MIN combine per scan) "
                         "instead of one independent what-if proposal per rank")
    ap.add_argument("--lib", default=None, help=argparse.SUPPRESS)  # tests: the CPU emulation build (tests/emu)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    lib = ccmi.Library.get(args.lib) if args.lib else ccmi.Library.get()
    cuda = torch.cuda.is_available() and not args.lib
    ndev = max(1, lib.device_count())
    # one rank per GPU with the bookkeeping collectives over RCCL; more ranks than GPUs (a rehearsal of the N-rank
    # path on a smaller box) share the cards round-robin and time over gloo (RCCL refuses two ranks on one GPU)
    over_gloo = world > ndev or not cuda
    device = local_rank % ndev if world > 1 else 0
    if cuda:
        torch.cuda.set_device(device)
    if world > 1:
        dist.init_process_group("gloo" if over_gloo else "nccl", init_method="env://")
    if over_gloo and args.sharded and world > 1:
        raise SystemExit("--sharded needs one GPU per rank (each rank's scan server / RCCL combiner holds its GPU)")

    props, goal_names, workload_name = WORKLOADS[args.workload]
    buf = ccmi.RandomCluster.generate(lib, **props)
    goals = ccmi.goals_from_names(goal_names)
    options = WORKLOAD_OPTIONS[args.workload]() if args.workload in WORKLOAD_OPTIONS else None
    opt = ccmi.GoalOptimizer(workload_constraint(args.workload))
    group_mode = args.sharded and args.combiner == "group"
    if group_mode and world > 1:
        raise SystemExit("--combiner group drives every shard from one process: run it without torchrun")
    n_group = max(1, args.gpus) if group_mode else 1
    sharded = (args.sharded and world > 1) or (group_mode and n_group > 1)
    if args.sharded and world == 1 and not group_mode and args.gpus > 1:
        raise SystemExit("--sharded --combiner shm/rccl needs one process per GPU (torchrun); use --combiner group")
    # A plain launch with --gpus N > 1 (no torchrun): N independent what-if proposals per step in THIS process, one
    # per device 0..N-1 (round-robin when the box has fewer), each on its own host thread (ctypes drops the GIL)
    local_devices = ([r % ndev for r in range(args.gpus)] if world == 1 and not group_mode and args.gpus > 1
                     else [device])
    uid = None
    if sharded and not group_mode:  # rank 0's RCCL id / shared-memory name + job nonce reach the other ranks
        obj = [(ccmi.rccl_unique_id(lib) if args.combiner == "rccl" else
                (f"/ccmi_bench_{os.getpid()}_{int(time.time())}", time.time_ns() | 1)) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        uid = obj[0]

    shm_sessions = [0]

    def session(dev=device):
        if group_mode and n_group > 1:  # the group's sessions, rank r on GPU r (round-robin on a smaller box)
            g = ccmi.ShardGroup(n_group, lib)
            ranks = []
            for r in range(n_group):
                x = ccmi.ClusterModel.from_buffers(buf, device=r % ndev)
                x.attach_group(g, r)
                ranks.append(x)
            return GroupSession(ranks)
        s = ccmi.ClusterModel.from_buffers(buf, device=dev)
        if sharded and args.combiner == "rccl":
            s.attach_rccl(rank, world, uid)
        elif sharded:  # one block per session (every rank creates its sessions in the same order)
            shm_sessions[0] += 1
            s.attach_shm(rank, world, f"{uid[0]}_{shm_sessions[0]}", job_nonce=uid[1] + shm_sessions[0])
        return s

    def sync_all():
        if cuda:
            for d in sorted(set(local_devices)):
                torch.cuda.synchronize(d)

    from concurrent.futures import ThreadPoolExecutor
    # Warmup proposals double as the instrumented pass: HIP events around every launched scan kernel and the scan
    # server's in-kernel busy time per command (outside the timed region). Every local device warms up (its first
    # launches load the code object); device 0's session is the instrumented one.
    inst_perf = inst_cands = None
    for w in range(max(1, args.warmup)):
        wss = [session(d) for d in local_devices]
        wss[0].set_kernel_timing(True)
        wss[0].reset_perf()
        if len(wss) == 1:
            rs = [optimize(opt, wss[0], goals, options)]
        else:
            with ThreadPoolExecutor(len(wss)) as wp:
                rs = list(wp.map(lambda s: optimize(opt, s, goals, options), wss))
        inst_perf, inst_cands = wss[0].perf(), rs[0].candidates
        del wss
        progress(f"warmup {w + 1}/{max(1, args.warmup)}: {rs[0].seconds:.2f} s")
    # One more instrumented proposal with the scan server off (a launch per scan): the per-launch kernel times the
    # rocprofv3 trace of the same path can be checked against (rank 0, single GPU, outside the timed region).
    launch_perf = None
    if world == 1 and len(local_devices) == 1 and not args.no_launch_pass and args.workload != "c4" and not group_mode:
        os.environ["CCMI_SERVER"] = "0"
        try:
            ls = session()
        finally:
            del os.environ["CCMI_SERVER"]
        ls.set_kernel_timing(True)
        ls.reset_perf()
        opt.optimizations(ls, goals, options)
        launch_perf = ls.perf()
        del ls
        progress("launch-path proposal done")

    S = max(1, args.requests_per_gpu) if not sharded else 1
    # cluster resident in HBM before timing starts: one session per proposal, [device][step][request]
    t_up = time.perf_counter()
    sessions = [[[session(d) for _ in range(S)] for _ in range(args.steps)] for d in local_devices]
    upload_s = (time.perf_counter() - t_up) / max(1, len(local_devices) * args.steps * S)
    progress(f"{len(local_devices) * args.steps * S} sessions resident; timed region starts")

    def run_device(steps):  # one device's K steps in order, S concurrent proposals per step
        out = []
        pool = ThreadPoolExecutor(S) if S > 1 else None
        try:
            for k, step_sessions in enumerate(steps):
                if pool is None:
                    out.extend(optimize(opt, s, goals, options) for s in step_sessions)
                else:
                    out.extend(pool.map(lambda s: optimize(opt, s, goals, options), step_sessions))
                progress(f"step {k + 1}/{len(steps)}: {out[-1].seconds:.2f} s")
        finally:
            if pool is not None:
                pool.shutdown()
        return out

    dev_pool = ThreadPoolExecutor(len(local_devices)) if len(local_devices) > 1 else None
    sync_all()
    if world > 1:
        dist.barrier()
    sync_all()
    t0 = time.perf_counter()
    if dev_pool is None:
        per_device = [run_device(sessions[0])]
    else:  # every device's thread starts together; the region ends when the slowest finishes (max over devices)
        per_device = list(dev_pool.map(run_device, sessions))
    sync_all()
    if world > 1:
        dist.barrier()
    sync_all()
    elapsed = time.perf_counter() - t0
    if dev_pool is not None:
        dev_pool.shutdown()
    results = [r for rs in per_device for r in rs]

    cands = sum(r.candidates for r in results)
    if world > 1:
        t = torch.tensor([elapsed, float(cands)], dtype=torch.float64, device="cpu" if over_gloo else f"cuda:{device}")
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed, cands = float(tmax[0]), float(t[1])
        if sharded:  # every rank made the same decisions: one proposal's candidates per step
            cands = float(sum(r.candidates for r in results))

    perf = inst_perf
    intra = args.workload == "c4"  # JBOD: the dominant kernel is K6 (intra_brokers)
    if intra:
        launches = max(1, perf.intra_launches)
        scan_avg_ms = perf.intra_kernel_ms / launches
        required_bytes_per_launch = perf.intra_bytes / launches
    elif perf.server_scans > 0:
        # K8 scan_server: one resident launch serves the cross / pair / segment scans; its unit of work is a command
        # and its time per command is measured inside the kernel (s_memrealtime, command seen -> result published)
        launches = max(1, perf.server_scans)
        scan_avg_ms = perf.server_busy_ms / launches
        required_bytes_per_launch = perf.server_required * BYTES_PER_CANDIDATE / launches
    else:
        launches = max(1, perf.scan_launches)
        scan_avg_ms = perf.scan_kernel_ms / launches
        required_bytes_per_launch = perf.scan_required * BYTES_PER_CANDIDATE / launches
    achieved = required_bytes_per_launch / (scan_avg_ms * 1e-3) / 1e9 if scan_avg_ms > 0 else 0.0
    server = perf.server_scans > 0 and not intra
    per_command = None
    if server:
        # The per-command view (in-kernel busy time per command) is kept as a secondary figure; the headline is the
        # rocprof-reproducible one: algorithmic bytes per scan_server LAUNCH over its average launch duration (HIP events
        # from launch to exit on the session stream, the same interval rocprofv3's kernel trace reports, idle polling
        # between the host's commands included).
        per_command = {"avg_us": scan_avg_ms * 1e3, "algorithmic_bytes": required_bytes_per_launch,
                       "achieved": achieved, "frac": achieved / HBM_PEAK_GBS,
                       "note": "in-kernel busy time per command (s_memrealtime, command seen -> result published)"}
        if perf.server_resident_ms > 0:
            launches = max(1, perf.server_launches)
            scan_avg_ms = perf.server_resident_ms / launches
            required_bytes_per_launch = perf.server_required * BYTES_PER_CANDIDATE / launches
            achieved = required_bytes_per_launch / (scan_avg_ms * 1e-3) / 1e9

    if rank != 0:
        dist.destroy_process_group()
        return
    first = results[0]
    parity = check_parity(args.workload, sessions[0][0][0], first)
    traffic, traffic_src = pmc_traffic(args.workload, INTRA_KERNELS if intra else SCAN_KERNELS)
    traffic_unit = "HBM bytes per scan launch"
    if server:
        st, ss = pmc_server_traffic(args.workload, perf)
        if per_command is not None:
            per_command["traffic"] = st
            per_command["traffic_over_algorithmic"] = st / per_command["algorithmic_bytes"] if st else None
        traffic, traffic_src = pmc_traffic(args.workload, ("scan_server",))
        traffic_unit = "HBM bytes per scan_server launch"
    line = {
        "metric": "candidate moves evaluated/s + proposal wall time, 10K brokers/1M replicas",
        "value": cands / elapsed,
        "unit": "candidate moves evaluated/s",
        "n_gpus": n_group if group_mode else world if world > 1 else len(local_devices),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "strong" if sharded else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (RandomCluster restatement, TestConstants seeds)",
        "config": {"workload": workload_name,
                   "brokers": buf.desc.num_brokers, "replicas": buf.desc.num_replicas,
                   "partitions": buf.desc.num_partitions, "topics": buf.desc.num_topics,
                   "goals": goal_names, "parallelism": (f"destination-sharded x{n_group} (one process, shard group: the scan servers MIN-combine "
                                   f"each scan on the device)" if group_mode and sharded else
                                   f"destination-sharded x{world} ({args.combiner} MIN combine per scan)" if sharded
                                   else f"independent what-if per GPU x{max(world, len(local_devices))}"
                                   + ("" if world > 1 or len(local_devices) == 1 else
                                      " (one process, one host thread per device)"))},
        "parity": parity,
        "requests_per_gpu": S,
        "devices": (sorted(set(local_devices)) if world == 1 and not group_mode else None),
        "devices_note": (None if world > 1 or group_mode or len(set(local_devices)) == len(local_devices) else
                         f"{len(local_devices)} sessions on {len(set(local_devices))} device(s): fewer GPUs than "
                         f"--gpus on this box, so sessions share devices round-robin (a rehearsal, not a scaling point)"),
        "proposal_wall_s": sum(r.seconds for r in results) / len(results),
        "session_upload_s": upload_s,
        "timed_region": "GoalOptimizer.optimizations on sessions already resident in HBM (upload excluded)",
        "candidates_per_step": first.candidates,
        "actions_per_step": len(first.actions),
        "proposals_per_step": len(first.proposals),
        "per_goal_gpu_s": {g.name: round(g.seconds, 4) for g in first.goal_results},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_unit": traffic_unit,
                     "traffic_source": traffic_src,
                     "kernel": ("K6 intra_brokers (one wavefront per broker; algorithmic bytes = 17 B per disk + 29 B per "
                                "replica entry read once)" if intra else
                                "K8 scan_server (persistent; per launch: the required candidates of its commands x 96 B "
                                "over the launch's residency, HIP events on the session stream)" if server else
                                "candidate scans (scan_cross/scan_pairs/scan_swap/chain_pairs/chain_rack_rows)"),
                     "avg_launch_us": scan_avg_ms * 1e3,
                     "avg_unit": "per launch",
                     "per_command": per_command,
                     "launches_per_step": perf.intra_launches if intra else perf.scan_launches,
                     "server_launches_per_step": perf.server_launches,
                     "server_commands_per_step": perf.server_scans,
                     # the rocprof-derivable view of the same kernel: algorithmic bytes per scan_server launch over its
                     # residency per launch (HIP events from launch to exit, idle polling included) — what a
                     # rocprofv3 kernel trace's average scan_server duration gives
                     "resident": None if not server or perf.server_resident_ms <= 0 else {
                         "avg_launch_us": perf.server_resident_ms * 1e3 / max(1, perf.server_launches),
                         "algorithmic_bytes_per_launch": perf.server_required * BYTES_PER_CANDIDATE
                         / max(1, perf.server_launches),
                         "achieved": perf.server_required * BYTES_PER_CANDIDATE / (perf.server_resident_ms * 1e-3) / 1e9,
                         "frac": perf.server_required * BYTES_PER_CANDIDATE / (perf.server_resident_ms * 1e-3) / 1e9
                         / HBM_PEAK_GBS,
                         "busy_share": perf.server_busy_ms / perf.server_resident_ms},
                     "server_payload_bytes_per_step": perf.server_payload_bytes,
                     "device_evaluated_candidates_per_s": perf.scan_required / (elapsed / args.steps),
                     "chain_launches_per_step": perf.chain_launches,
                     "algorithmic_bytes_per_launch": required_bytes_per_launch,
                     "traffic_over_algorithmic": (traffic / required_bytes_per_launch
                                                  if traffic and required_bytes_per_launch else None),
                     "required_candidates_per_step": perf.scan_required,
                     "reference_equivalent_candidates_per_step": inst_cands,
                     "stats_avg_launch_us": perf.stats_kernel_ms * 1e3 / max(1, perf.stats_launches),
                     "stats_bytes_per_launch": perf.stats_bytes / max(1, perf.stats_launches),
                     "host_syncs_per_step": perf.host_syncs,
                     "intra_sort": None if not intra else {
                         "launches_per_step": perf.intra_sort_launches,
                         "avg_launch_us": perf.intra_sort_ms * 1e3 / max(1, perf.intra_sort_launches),
                         "note": "K6's per-call entry sort, timed apart from intra_brokers (HIP events)"},
                     "scan_cross": scan_cross_line(launch_perf or perf, args.workload),
                     "launch_path": None if launch_perf is None else {
                         "scan_launches": launch_perf.scan_launches,
                         "avg_scan_launch_us": launch_perf.scan_kernel_ms * 1e3 / max(1, launch_perf.scan_launches),
                         "achieved_gbs": (launch_perf.scan_required * BYTES_PER_CANDIDATE / max(1, launch_perf.scan_launches))
                                         / max(1e-12, launch_perf.scan_kernel_ms * 1e-3 / max(1, launch_perf.scan_launches)) / 1e9,
                         "note": "the same proposal with CCMI_SERVER=0 (one launch per scan), HIP events per launch"}},
        "cpu_baseline": None,
    }
    if world == 1 and len(local_devices) == 1 and not args.no_cpu_baseline:
        progress("cpu baseline")
        line["cpu_baseline"] = cpu_baseline(lib, buf, args.workload, goal_names, options, first, device,
                                            args.cpu_sample_seconds, args.what_if_procs)
    print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()




if __name__ == "__main__":
    main()
