#!/bin/bash
# K6 check + C2 tree profile, one gpurun call: the JBOD GPU tests, the C4 bench line with its kernel stats, then a C2
# probe with the host phase profile. Every GPU step under its own limit; the first failure stops the script.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${TAG:-k6}
echo "== jbod tests ($(date +%T))"
timeout -k 10 400 python -u -m pytest tests/test_jbod.py -m gpu -x -v --timeout 150 --timeout-method thread \
  > gpurun_out/pytest_jbod_$T.log 2>&1 || { tail -20 gpurun_out/pytest_jbod_$T.log; exit 1; }
tail -2 gpurun_out/pytest_jbod_$T.log
echo "== c4 bench under rocprofv3 ($(date +%T))"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4_$T -o c4 -- \
  python3 -u bench.py --workload c4 --no-cpu-baseline > gpurun_out/c4_bench_$T.json 2> gpurun_out/c4_bench_$T.err \
  || { tail -5 gpurun_out/c4_bench_$T.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/c4_bench_$T.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline'].get('avg_launch_us'), d.get('parity', {}).get('status'))"
echo "== c2 probe ($(date +%T))"
CCMI_PROFILE=1 timeout -k 10 300 python -u tools/probe.py --workload c2 > gpurun_out/probe_$T.log 2>&1 || exit 1
grep -E "^total|tree\.|out\.|tree.build" gpurun_out/probe_$T.log
