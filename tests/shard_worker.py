"""Worker of the multi-process sharded-scan tests (tests/test_shard.py): one process per shard, the MIN combiner either
torch.distributed gloo on 127.0.0.1 (a Python callback) or the library's host shared-memory combiner
(ccmi_session_attach_shm), on the test-only Device emulation or the gfx950 library."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "cruise-control_amd"))


def run(rank, world, port, props, goals, balance, out_dir, lib_path, combiner="gloo", env=None):
    os.environ.update(env or {})
    import torch
    import torch.distributed as dist

    import ccmi
    from parity import constraint

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    calls = [0]

    def combine_min(key):
        calls[0] += 1
        t = torch.tensor([key], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return int(t.item())

    lib = ccmi.Library.get(lib_path)
    buf = ccmi.RandomCluster.generate(lib, **props)
    cm = ccmi.ClusterModel.from_buffers(buf, device=0)
    if combiner == "shm":
        cm.attach_shm(rank, world, f"/ccmi_test_{port}")
    else:
        cm.set_shard(rank, world, combine_min)
    err = None
    res = None
    try:
        res = ccmi.GoalOptimizer(constraint(balance)).optimizations(cm, ccmi.goals_from_names(goals))
    except ccmi.CruiseControlError as e:
        err = f"{type(e).__name__}: {e}"
    out = dict(rank=rank, actions=cm.actions(), replica_distribution=cm.replica_distribution(),
               leader_distribution=cm.leader_distribution(), error=err,
               combines=calls[0] if combiner != "shm" else cm.perf().combines,
               server_launches=cm.perf().server_launches,
               goals=[(g.name, g.succeeded, g.candidates, g.actions) for g in res.goal_results] if res else None,
               device_candidates=sum(g.device_candidates for g in res.goal_results) if res else None)
    with open(os.path.join(out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()
