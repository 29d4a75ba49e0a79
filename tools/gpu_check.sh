#!/bin/bash
# One GPU-box pass: smoke, GPU parity tests, bench, optional rocprofv3 kernel-trace summary and PMC passes.
# Every GPU step has its own time limit; a crash/abort/timeout (anything but pass/fail) stops the script.
#   env: PYTEST_ARGS, BENCH_ARGS, PROFILE=1, PMC=1, C2=1, SKIP_TESTS=1, SKIP_BENCH=1, PROBE=<workload>
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name exited $rc"; exit $rc; fi
  return $rc
}
make -C cruise-control_amd -j16 > gpurun_out/make.log 2>&1 && make -C oracle -j16 >> gpurun_out/make.log 2>&1 || exit 1
if [ -z "${SKIP_TESTS:-}" ]; then
  step smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}
fi
if [ -n "${PROBE:-}" ]; then
  step probe 900 python -u tools/probe.py --workload "$PROBE"
fi
if [ -z "${SKIP_BENCH:-}" ]; then
  step bench 600 python bench.py ${BENCH_ARGS:-}
fi
if [ -n "${PROFILE:-}" ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o bench -- \
    python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 ${PROF_ARGS:-}
  rm -f gpurun_out/prof/*_kernel_trace.csv  # one row per dispatch: too large to bring back; the stats stay
fi
if [ -n "${PMC:-}" ]; then
  step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o bench -- \
    python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 ${PROF_ARGS:-}
  step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o bench -- \
    python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 ${PROF_ARGS:-}
  python3 tools/pmc_summary.py gpurun_out/pmc_fetch/bench_counter_collection.csv \
    gpurun_out/pmc_write/bench_counter_collection.csv > gpurun_out/pmc_summary.json
  rm -f gpurun_out/pmc_fetch/*_counter_collection.csv gpurun_out/pmc_write/*_counter_collection.csv
fi
if [ -n "${C2:-}" ]; then
  step bench_c2 900 python bench.py --workload c2 --steps 1 --warmup 0
fi
exit 0
