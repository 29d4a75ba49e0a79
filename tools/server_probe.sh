#!/bin/bash
# Server correctness (GPU parity subset) and the C2 probe with its perf counters (one gpurun call).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
make -C cruise-control_amd -j16 > gpurun_out/make.log 2>&1 && make -C oracle -j16 >> gpurun_out/make.log 2>&1 || exit 1
step() {
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "stopping: $name exited $rc"; exit $rc; fi
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -k "${PYTEST_K:-}"
CCMI_PROFILE=1 step probe_server 600 python -u tools/probe.py --workload c2
