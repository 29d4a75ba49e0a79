#!/bin/bash
# One GPU-box pass: smoke, GPU parity tests, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash/abort/timeout (anything but pass/fail) stops the script.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $name exited $rc"; exit $rc; fi
  return $rc
}
make -C cruise-control_amd -j16 > gpurun_out/make.log 2>&1 && make -C oracle -j16 >> gpurun_out/make.log 2>&1 || exit 1
step smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-}
step bench 600 python bench.py ${BENCH_ARGS:-}
if [ -n "${PROFILE:-}" ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1
fi
exit 0
