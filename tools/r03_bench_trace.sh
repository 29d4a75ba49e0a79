#!/bin/bash
# Round-3 bench line plus a rocprofv3 kernel trace + stats of the same bench command (the first two steps of
# tools/r03_final.sh, without the PMC passes).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
make -C cruise-control_amd -j16 > gpurun_out/make.log 2>&1 && make -C oracle -j16 >> gpurun_out/make.log 2>&1 || exit 1
echo "== bench $(date +%T)"
timeout -k 10 900 python -u bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/bench_final.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['parity']['status'])"
echo "== trace $(date +%T)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_final -o bench -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_trace_final.json 2> gpurun_out/bench_trace_final.err || exit $?
f=$(find gpurun_out/prof_final -name '*kernel_trace.csv' | head -1)
python3 tools/trace_hist.py "$f" > gpurun_out/trace_hist_final.txt
find gpurun_out/prof_final -name '*kernel_trace.csv' -delete
head -12 gpurun_out/trace_hist_final.txt
