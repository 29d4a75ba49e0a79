#!/bin/bash
# Round-3 measurement (one gpurun call): the bench line, then a rocprofv3 kernel trace + stats of a short bench run
# (server pass and the scan-server-off launch pass), reduced to a per-kernel duration histogram.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
make -C cruise-control_amd -j16 > gpurun_out/make.log 2>&1 && make -C oracle -j16 >> gpurun_out/make.log 2>&1 || exit 1
echo "== bench $(date +%T)"
timeout -k 10 900 python -u bench.py --steps ${STEPS:-3} --warmup 1 > gpurun_out/bench_${TAG:-r03}.json 2> gpurun_out/bench_${TAG:-r03}.err || exit $?
cat gpurun_out/bench_${TAG:-r03}.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','ms_per_step','parity')}); print(d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline']['launch_path'])"
echo "== trace $(date +%T)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG:-r03} -o bench -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_trace.log 2>&1 || exit $?
f=$(find gpurun_out/prof_${TAG:-r03} -name '*kernel_trace.csv' | head -1)
python3 tools/trace_hist.py "$f" > gpurun_out/trace_hist_${TAG:-r03}.txt
find gpurun_out/prof_${TAG:-r03} -name '*kernel_trace.csv' -delete
cat gpurun_out/trace_hist_${TAG:-r03}.txt | head -40
if [ -n "${PYTEST_K:-}" ]; then
  echo "== pytest -m gpu -k ${PYTEST_K} $(date +%T)"
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -k "${PYTEST_K}" \
    > gpurun_out/pytest_${TAG:-r03}.log 2>&1
  rc=$?; tail -5 gpurun_out/pytest_${TAG:-r03}.log; exit $rc
fi
