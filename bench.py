"""Headline benchmark: candidate moves evaluated/s + proposal wall time (BASELINE.json `metric`).

Workload (default, BASELINE.json configs[2] — the configuration the metric is quoted on, and it fits one GPU):
RandomCluster C2 = 100 racks, 10 000 brokers, 999 999 + 20 000 replicas (R = 1 019 999), 10 001 topics, W = 1,
uniform loads, TestConstants seeds; the 16 default goals in default priority order; default BalancingConstraint.
--workload c1 / c0 / c2_c1goals select the other BASELINE configs (parity-test cases, not headline lines).

A "step" is one full GoalOptimizer.optimizations over that cluster (every goal, ClusterModelStats after every goal,
final ExecutionProposals). Each step works on its own device session, uploaded to HBM before the timed region
starts; the step count K therefore means K independent proposal computations per GPU.

value = reference-equivalent candidate moves evaluated/s summed over all ranks (the candidates the reference's
first-fit loops would visit), ms_per_step = step wall time = proposal wall time at the default
--requests-per-gpu 1. --requests-per-gpu S runs S independent what-if proposals concurrently per GPU in every step
(one host thread + HIP stream per session, GoalOptimizer's precompute pool); proposal_wall_s is then the mean
per-proposal latency.

Multi-GPU (torchrun, one process per GPU): by default every rank runs its own independent what-if proposal
request (weak scaling, no data-path collective); timing is max over ranks. --sharded instead shards ONE proposal's
candidate space by destination broker over the ranks (one RCCL MIN allreduce per scan, strong scaling).

Roofline: the dominant kernel is the candidate scan. Its HIP-event duration is measured during the warmup
proposal(s) (events on the engine stream, outside the timed region); algorithmic bytes = 96 B per
reference-equivalent candidate. traffic = HBM bytes per scan launch from the committed rocprofv3
PMC summary of this workload. cpu_baseline = the single-threaded C++ restatement (oracle/, "port") on rank 0 at
N = 1: the whole chain for C0/C1, a goal-prefix sample of the chain for C2.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "cruise-control_amd"))

import ccmi  # noqa: E402

C1_PROPS = dict(num_racks=20, num_brokers=1000, num_replicas=99999, num_topics=3000)
C2_PROPS = dict(num_racks=100, num_brokers=10000, num_replicas=999999, num_topics=10000)
# C3: RandomSelfHealingTest-style placement (6-arg populate, rack-aware, leader first; RandomCluster.java:119-124)
C3_PROPS = dict(C2_PROPS, num_dead_brokers=500, rack_aware=1, leader_in_first_position=1)
C1_GOALS = list(ccmi.C1_GOALS)
DEFAULT_GOALS = list(ccmi.DEFAULT_GOALS)
WORKLOADS = {"c1": (C1_PROPS, C1_GOALS, "C1: 1K brokers x 100K replicas, 5 distribution goals (BASELINE configs[1])"),
             "c2": (C2_PROPS, DEFAULT_GOALS, "C2: 10K brokers x 1M replicas, the 16 default goals (BASELINE configs[2])"),
             "c2_c1goals": (C2_PROPS, C1_GOALS, "C2 cluster with the C1 goal list"),
             "c3": (C3_PROPS, DEFAULT_GOALS, "C3: C2 with brokers 0..499 DEAD, requested destinations 500..1499, the 16 "
                                           "default goals (BASELINE configs[3], RemoveBrokersRunnable options)"),
             "c0": ({}, DEFAULT_GOALS, "C0: TestConstants.BASE_PROPERTIES, the 16 default goals (BASELINE configs[0])")}
# Per-workload OptimizationOptions (C3: the 7-arg options RemoveBrokersRunnable.java:107-126 builds)
WORKLOAD_OPTIONS = {"c3": lambda: ccmi.OptimizationOptions(requested_destination_broker_ids=list(range(500, 1500)),
                                                           fast_mode=False)}
BYTES_PER_CANDIDATE = 96
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)


# CPU-baseline sample of the C2 workload: the first goals of the default chain on the same C2 cluster (the whole
# chain takes the single-threaded restatement about an hour: every goal pays ~30 s of ClusterModelStats over the
# T x B topic-replica counts at C2; the first goal alone is ~30 s of CPU work).
C2_CPU_SAMPLE_GOALS = 1


def cpu_baseline(buf, workload: str, goal_names) -> dict:
    """The oracle restatement (oracle/, "port"), single thread, on rank 0 at N=1: the whole chain for C0/C1, a
    goal-prefix sample of the chain for C2 (same cluster, same constraint)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle_binding import OracleCluster

    goals = list(goal_names) if workload in ("c0", "c1") else list(goal_names)[:C2_CPU_SAMPLE_GOALS]
    oc = OracleCluster.from_desc(buf.desc)
    t0 = time.perf_counter()
    opts = WORKLOAD_OPTIONS[workload]() if workload in WORKLOAD_OPTIONS else None
    res = oc.optimize(goals, ccmi.BalancingConstraint(), opts)
    dt = time.perf_counter() - t0
    cands = sum(r.candidates for r in res)
    what = "one full optimizations()" if len(goals) == len(goal_names) else \
        f"optimizations() over the first {len(goals)} goals of the chain ({goals[0]} .. {goals[-1]})"
    return {"value": cands / dt, "unit": "candidate moves evaluated/s", "cores": 1, "kind": "port",
            "sample": f"{what} of the {workload.upper()} workload: {cands} candidates, {len(oc.actions())} actions in "
                      f"{dt:.2f} s by the single-threaded C++ restatement (oracle/)",
            "goals": goals, "wall_s": dt}


SCAN_KERNELS = ("scan_cross", "scan_pairs", "scan_swap")


def pmc_traffic(workload: str):
    """HBM bytes per scan launch from the newest committed PMC summary of this workload (profiles/rNN/
    <workload>_pmc_summary.json, written by tools/pmc_summary.py from separate rocprofv3 --pmc FETCH_SIZE /
    WRITE_SIZE passes of this same bench command). PMC counters cannot be read inside the timed process."""
    import glob
    paths = sorted(glob.glob(os.path.join(REPO, "profiles", "r*", f"{workload}_pmc_summary.json")))
    if not paths:
        return None, None
    with open(paths[-1]) as f:
        ks = json.load(f)["kernels"]
    n = sum(ks[k]["launches"] for k in SCAN_KERNELS if k in ks)
    b = sum(ks[k]["launches"] * ks[k]["hbm_bytes_per_launch"] for k in SCAN_KERNELS if k in ks)
    return (b / n if n else None), os.path.relpath(paths[-1], REPO)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c2")
    ap.add_argument("--requests-per-gpu", type=int, default=1,
                    help="S concurrent what-if proposals per GPU in every step (one host thread + HIP stream per "
                         "session; the precompute pool of GoalOptimizer.java:117-119). Default 1: one proposal per step")
    ap.add_argument("--sharded", action="store_true",
                    help="N>1: one proposal sharded by destination broker over all ranks (RCCL MIN per scan) "
                         "instead of one independent what-if proposal per rank")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", init_method="env://")
    device = local_rank if world > 1 else 0
    torch.cuda.set_device(device)

    lib = ccmi.Library.get()
    props, goal_names, workload_name = WORKLOADS[args.workload]
    buf = ccmi.RandomCluster.generate(lib, **props)
    goals = ccmi.goals_from_names(goal_names)
    options = WORKLOAD_OPTIONS[args.workload]() if args.workload in WORKLOAD_OPTIONS else None
    opt = ccmi.GoalOptimizer(ccmi.BalancingConstraint())
    sharded = args.sharded and world > 1
    uid = None
    if sharded:  # rank 0's RCCL id reaches the other ranks over the default process group
        obj = [ccmi.rccl_unique_id(lib) if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        uid = obj[0]

    def session():
        s = ccmi.ClusterModel.from_buffers(buf, device=device)
        if sharded:
            s.attach_rccl(rank, world, uid)
        return s

    # Warmup proposals double as the instrumented pass: HIP events around every scan kernel on the engine stream
    # (outside the timed region).
    inst_perf = inst_cands = None
    for w in range(max(1, args.warmup)):
        ws = session()
        ws.set_kernel_timing(True)
        ws.reset_perf()
        r = opt.optimizations(ws, goals, options)
        inst_perf, inst_cands = ws.perf(), r.candidates
        del ws

    S = max(1, args.requests_per_gpu) if not sharded else 1
    # cluster resident in HBM before timing starts: one session per proposal
    sessions = [[session() for _ in range(S)] for _ in range(args.steps)]
    pool = None
    if S > 1:
        from concurrent.futures import ThreadPoolExecutor  # ctypes drops the GIL inside ccmi_optimizations
        pool = ThreadPoolExecutor(S)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    results = []
    for step_sessions in sessions:
        if pool is None:
            results.extend(opt.optimizations(s, goals, options) for s in step_sessions)
        else:
            results.extend(pool.map(lambda s: opt.optimizations(s, goals, options), step_sessions))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0

    cands = sum(r.candidates for r in results)
    if world > 1:
        t = torch.tensor([elapsed, float(cands)], dtype=torch.float64, device=f"cuda:{device}")
        tmax = t.clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        elapsed, cands = float(tmax[0]), float(t[1])
        if sharded:  # every rank made the same decisions: one proposal's candidates per step
            cands = float(sum(r.candidates for r in results))

    perf = inst_perf
    scan_avg_ms = perf.scan_kernel_ms / max(1, perf.scan_launches)
    ref_bytes_per_launch = inst_cands * BYTES_PER_CANDIDATE / max(1, perf.scan_launches)
    achieved = ref_bytes_per_launch / (scan_avg_ms * 1e-3) / 1e9 if scan_avg_ms > 0 else 0.0

    if rank != 0:
        dist.destroy_process_group()
        return
    first = results[0]
    traffic, traffic_src = pmc_traffic(args.workload)
    line = {
        "metric": "candidate moves evaluated/s + proposal wall time, 10K brokers/1M replicas",
        "value": cands / elapsed,
        "unit": "candidate moves evaluated/s",
        "n_gpus": world,
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
                   "goals": goal_names, "parallelism": (f"destination-sharded x{world} (RCCL MIN allreduce per scan)" if sharded
                                   else f"independent what-if per GPU x{world}")},
        "requests_per_gpu": S,
        "proposal_wall_s": sum(r.seconds for r in results) / len(results),
        "candidates_per_step": first.candidates,
        "actions_per_step": len(first.actions),
        "proposals_per_step": len(first.proposals),
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_unit": "HBM bytes per scan launch",
                     "traffic_source": traffic_src,
                     "kernel": "scan (scan_cross/scan_pairs/scan_swap)", "avg_launch_us": scan_avg_ms * 1e3,
                     "launches_per_step": perf.scan_launches,
                     "algorithmic_bytes_per_launch": ref_bytes_per_launch,
                     "stats_avg_launch_us": perf.stats_kernel_ms * 1e3 / max(1, perf.stats_launches),
                     "stats_bytes_per_launch": perf.stats_bytes / max(1, perf.stats_launches),
                     "host_syncs_per_step": perf.host_syncs},
        "cpu_baseline": None,
    }
    if world == 1 and not args.no_cpu_baseline:
        line["cpu_baseline"] = cpu_baseline(buf, args.workload, goal_names)
    print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
