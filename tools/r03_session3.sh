#!/bin/bash
# One gpurun call: GPU parity subset (PYTEST_K), then the C2 probe with per-goal phases and server stamps.
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
if [ -n "${PYTEST_K:-}" ]; then
  step pytest_s3 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -k "${PYTEST_K}"
fi
CCMI_PROFILE=goal step probe_goal 600 python -u tools/probe.py --workload c2
CCMI_STAMPS=1 CCMI_PROFILE=1 step probe_stamps 600 python -u tools/probe.py --workload c2
grep -E "^total|server stamps" gpurun_out/probe_goal.log gpurun_out/probe_stamps.log
