#!/bin/bash
# K6 (wavefront per broker) evidence in one gpurun call: the JBOD GPU parity tests, the C4 bench line, and a
# rocprofv3 kernel trace + stats of the same C4 bench command.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
make -C cruise-control_amd -j16 > gpurun_out/make.log 2>&1 && make -C oracle -j16 >> gpurun_out/make.log 2>&1 || exit 1
[ -n "$SKIP_TESTS" ] || { echo "== jbod tests $(date +%T)"
timeout -k 10 600 python -u -m pytest tests/test_jbod.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_jbod.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_jbod.log; [ $rc -eq 0 ] || exit $rc; }
echo "== c4 bench $(date +%T)"
timeout -k 10 300 python -u bench.py --workload c4 --steps 3 --warmup 1 > gpurun_out/c4_bench.json 2> gpurun_out/c4_bench.err || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/c4_bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['parity']['status'], d['roofline'])"
echo "== c4 trace $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o c4 -- \
  python3 bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c4_trace.json 2> gpurun_out/c4_trace.err || exit $?
find gpurun_out/prof_c4 -name '*kernel_trace.csv' -delete
f=$(find gpurun_out/prof_c4 -name '*kernel_stats.csv' | head -1)
grep -E "intra|stats_disks" "$f" | cut -c1-160
