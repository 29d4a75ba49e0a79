#!/bin/bash
# XCD-slicing threshold sweep for scan_cross at C2: per threshold, the bench's HIP-event timing (1 warmup = the
# instrumented pass, 1 timed step) and a --pmc FETCH_SIZE pass restricted to scan_cross, summarised per launch.
#   /usr/local/graft/bin/gpurun --timeout 1100 -- 'OUT=r02i bash tools/slice_sweep.sh 2048 512 128'
set -euo pipefail
OUT=${OUT:-sweep}
DST=gpurun_out/$OUT
mkdir -p "$DST"
export TMPDIR=/tmp
for T in "$@"; do
  CCMI_XCD_SLICE_MIN_COLS=$T timeout -k 10 300 python3 bench.py --workload c2 --no-cpu-baseline --steps 1 --warmup 1 \
    > "$DST/bench_$T.json"
  rm -rf /tmp/sweep_$T
  CCMI_XCD_SLICE_MIN_COLS=$T timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex scan_cross \
    --output-format csv -d /tmp/sweep_$T -o s -- python3 bench.py --workload c2 --no-cpu-baseline --steps 1 --warmup 0 \
    > /dev/null
  python3 - "$T" "$DST" <<'PY'
import csv, glob, json, sys
T, dst = sys.argv[1], sys.argv[2]
vals = []
for f in glob.glob(f"/tmp/sweep_{T}/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "scan_cross" in row["Kernel_Name"]:
            vals.append(float(row["Counter_Value"]))
b = json.loads(open(f"{dst}/bench_{T}.json").read().strip().splitlines()[-1])
sc = b["roofline"]["scan_cross"]
out = {"threshold": T, "launches": len(vals), "fetch_x2_bytes_per_launch": 2048.0 * sum(vals) / max(1, len(vals)),
       "algorithmic_bytes_per_launch": sc["algorithmic_bytes_per_launch"], "avg_launch_us": sc["avg_launch_us"],
       "ms_per_step": b["ms_per_step"], "parity": b["parity"]["status"]}
out["fetch_over_algorithmic"] = out["fetch_x2_bytes_per_launch"] / out["algorithmic_bytes_per_launch"]
print(json.dumps(out))
json.dump(out, open(f"{dst}/sweep_{T}.json", "w"))
PY
done
