#!/bin/bash
# Round-5 GPU pass (one gpurun call): smoke, the -m gpu suite, the default C2 bench line. Every GPU step runs under
# its own time limit; anything but success stops the script (no GPU step after a fault, abort or timeout).
#   env: TAG (log names), PYTEST_K (a -k filter), SKIP_TESTS=1, SKIP_BENCH=1, BENCH_ARGS, ENVS (exported for every step),
#        REQ2=1 (bench --requests-per-gpu 2), REHEARSE2=1 (bench --gpus 2 from a plain launch), PROBE=1 (CCMI_PROFILE=goal probe; PROBE_PROFILE, STAMPS=1 for CCMI_STAMPS), ROCPROF=1 (rocprofv3 kernel trace + stats of one bench step)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${TAG:-r05}
for kv in ${ENVS:-}; do export "$kv"; done
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2; shift 2
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/${name}_$T.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc ($(date +%T))"; tail -4 "gpurun_out/${name}_$T.log"
  if [ $rc -ne 0 ]; then echo "stopping: $name exited $rc"; exit $rc; fi
}
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
if [ -z "$SKIP_TESTS" ]; then
  if [ -n "$PYTEST_K" ]; then
    step pytest_gpu 900 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -v --timeout 150 --timeout-method thread -k "$PYTEST_K"
  else
    step pytest_gpu 900 python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -v --timeout 150 --timeout-method thread
  fi
fi
if [ -z "$SKIP_BENCH" ]; then
  echo "== bench ($(date +%T))"
  timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > "gpurun_out/bench_$T.json" 2> "gpurun_out/bench_$T.err"
  rc=$?
  tail -3 "gpurun_out/bench_$T.err"
  [ $rc -eq 0 ] || { echo "stopping: bench exited $rc"; exit $rc; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_$T.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('parity'))"
fi
if [ -n "$REQ2" ]; then  # two concurrent what-if proposals per step on the one GPU (sessions share its server budget)
  step req2 900 python -u bench.py --requests-per-gpu 2 --steps 2 --warmup 1 --no-cpu-baseline --no-launch-pass ${BENCH_ARGS:-}
  tail -1 "gpurun_out/req2_$T.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('req2', d['value'], d['ms_per_step'], d['proposal_wall_s'], d['parity']['status'])"
fi
if [ -n "$REHEARSE2" ]; then  # the driver's plain multi-GPU form on the one-GPU box: two sessions share the card
  step gpus2 900 python -u bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-}
  tail -1 "gpurun_out/gpus2_$T.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d['devices'], d['value'], d['ms_per_step'], d['parity']['status'])"
fi
if [ -n "$PROBE" ]; then  # per-goal phase profile of one C2 optimization
  ( export CCMI_PROFILE=${PROBE_PROFILE:-goal}; [ -n "$STAMPS" ] && export CCMI_STAMPS=1
    step probe 600 python -u tools/probe.py --workload ${WORKLOAD:-c2} ) || exit $?
  grep -E "^total|^perf|stamps\]" "gpurun_out/probe_$T.log"
fi
if [ -n "$ROCPROF" ]; then  # kernel trace + stats of one bench step (the per-dispatch trace stays in /tmp)
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$T -o bench -- \
    python3 -u bench.py --steps ${PROF_STEPS:-1} --warmup 1 --no-cpu-baseline
  mkdir -p gpurun_out/prof_$T && find /tmp/prof_$T -name "*stats.csv" -exec cp {} gpurun_out/prof_$T/ \;
fi
