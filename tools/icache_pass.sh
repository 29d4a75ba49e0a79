#!/bin/bash
# One rocprofv3 counter pass over one C2 bench step for the instruction cache (SQC_ICACHE_*, SQ_IFETCH) and the
# summed counter values per kernel in gpurun_out/$OUT/icache_summary.json (the per-dispatch CSV stays in /tmp).
#   /usr/local/graft/bin/gpurun --timeout 600 -- 'OUT=r06ic bash tools/icache_pass.sh'
set -euo pipefail
OUT=${OUT:-icache}
DST=gpurun_out/$OUT
mkdir -p "$DST"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
W=/tmp/ccmi_icache
rm -rf "$W"
timeout -s KILL 400 rocprofv3 --pmc ${COUNTERS:-SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH} \
  --output-format csv -d "$W" -o ic -- python3 bench.py --workload c2 --no-cpu-baseline --no-launch-pass --steps 1 \
  --warmup 0 > "$DST/icache_bench.json"
python3 - "$W" > "$DST/icache_summary.json" <<'EOF'
import csv, glob, json, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(float))
n = defaultdict(int)
for path in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    with open(path) as f:
        for row in csv.DictReader(f):
            k = row["Kernel_Name"].split("(")[0].replace("ccmi::", "")
            acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
print(json.dumps({k: dict(v) for k, v in acc.items()}, indent=1, sort_keys=True))
EOF
