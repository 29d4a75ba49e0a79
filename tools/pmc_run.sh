#!/bin/bash
# GPU-box evidence for profiles/<round>/: kernel-trace stats and separate FETCH_SIZE / WRITE_SIZE passes, first over
# tools/pmc_calib (known byte counts, scan_cross's access pattern) and then over one C2 bench step. Only the
# summaries are kept under gpurun_out/$OUT (the per-dispatch traces stay in /tmp: they exceed the copy-back cap).
#   /usr/local/graft/bin/gpurun --timeout 1100 -- 'OUT=r02g bash tools/pmc_run.sh'
set -euo pipefail
OUT=${OUT:-pmc}
DST=gpurun_out/$OUT
mkdir -p "$DST"
export TMPDIR=/tmp
W=/tmp/ccmi_pmc
rm -rf "$W"
mkdir -p "$W"
collect() {  # name, pattern -> copies matching CSVs under $W/name to $DST/name_<file>
  find "$W/$1" -name "$2" | while read -r f; do cp "$f" "$DST/$1_$(basename "$f")"; done
}
timeout -s KILL 60 rocprofv3 --kernel-trace --stats --output-format csv -d "$W/calib_trace" -o calib -- \
  ./tools/pmc_calib > "$DST/calib_bytes.json"
collect calib_trace "*stats.csv"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d "$W/calib_$c" -o calib -- ./tools/pmc_calib > /dev/null
  collect "calib_$c" "*counter_collection.csv"
done
python3 tools/pmc_summary.py --calib "$DST/calib_bytes.json" "$DST"/calib_FETCH_SIZE_*counter_collection.csv \
  "$DST"/calib_WRITE_SIZE_*counter_collection.csv > "$DST/calib_summary.json"
if [ "${CALIB_ONLY:-0}" = 1 ]; then exit 0; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$W/c2_trace" -o c2 -- \
  python3 bench.py --workload c2 --no-cpu-baseline --steps 1 --warmup 0 > "$DST/c2_bench_prof.json"
collect c2_trace "*stats.csv"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $c --output-format csv -d "$W/c2_$c" -o c2 -- \
    python3 bench.py --workload c2 --no-cpu-baseline --steps 1 --warmup 0 > /dev/null
done
python3 tools/pmc_summary.py --calib "$DST/calib_summary.json" $(find "$W/c2_FETCH_SIZE" "$W/c2_WRITE_SIZE" \
  -name "*counter_collection.csv") > "$DST/c2_pmc_summary.json"
# C4 (JBOD intra-broker goals, K6): the same three passes
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$W/c4_trace" -o c4 -- \
  python3 bench.py --workload c4 --no-cpu-baseline --steps 1 --warmup 0 > "$DST/c4_bench_prof.json"
collect c4_trace "*stats.csv"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d "$W/c4_$c" -o c4 -- \
    python3 bench.py --workload c4 --no-cpu-baseline --steps 1 --warmup 0 > /dev/null
done
python3 tools/pmc_summary.py --calib "$DST/calib_summary.json" $(find "$W/c4_FETCH_SIZE" "$W/c4_WRITE_SIZE" \
  -name "*counter_collection.csv") > "$DST/c4_pmc_summary.json"
