#!/bin/bash
# One gpurun call: smoke, the whole -m gpu suite, then the default bench line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
make -C cruise-control_amd -j16 > gpurun_out/make.log 2>&1 && make -C oracle -j16 >> gpurun_out/make.log 2>&1 || exit 1
echo "== smoke $(date +%T)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_full.log 2>&1 || { tail -5 gpurun_out/smoke_full.log; exit 1; }
echo "== pytest $(date +%T)"
timeout -k 10 780 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_full.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_full.log; [ $rc -eq 0 ] || exit $rc
echo "== bench $(date +%T)"
timeout -k 10 400 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || exit $?
python3 -c "import json; d=json.loads(open('gpurun_out/bench_full.json').read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], d['parity']['status'], r['traffic'], r['traffic_over_algorithmic'], r['frac'])"
