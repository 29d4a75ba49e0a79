"""Find the first goal whose decisions differ between the product library and the CPU oracle (GPU box debug aid).

    python tools/divergence.py '{"num_topics": 7000}' 3000
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "cruise-control_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import ccmi  # noqa: E402
from oracle_binding import OracleCluster  # noqa: E402
from parity import constraint  # noqa: E402

props = json.loads(sys.argv[1])
max_replicas = int(sys.argv[2]) if len(sys.argv) > 2 else None
lib = ccmi.Library.get()
buf = ccmi.RandomCluster.generate(lib, **props)
goals = list(ccmi.DEFAULT_GOALS)
cm = ccmi.ClusterModel.from_buffers(buf, device=0)
res = ccmi.GoalOptimizer(constraint(1.05, max_replicas)).optimizations(cm, ccmi.goals_from_names(goals))
oc = OracleCluster.from_desc(buf.desc)
ores = oc.optimize(goals, constraint(1.05, max_replicas))
pa, oa = cm.actions(), oc.actions()
n = 0
for r, o in zip(res.goal_results, ores):
    seg_p, seg_o = pa[n:n + r.actions], oa[n:n + o.actions]
    same = (r.candidates, r.actions) == (o.candidates, o.actions) and seg_p == seg_o
    print(f"{r.name:40s} product cand={r.candidates} act={r.actions}  oracle cand={o.candidates} act={o.actions}"
          f"  {'ok' if same else 'DIFF'}", flush=True)
    if not same:
        for i, (x, y) in enumerate(zip(seg_p, seg_o)):
            if x != y:
                print(f"  first differing action #{n + i} (goal-local {i}): product {x} oracle {y}")
                break
        break
    n += r.actions
