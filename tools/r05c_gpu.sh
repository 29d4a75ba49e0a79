cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r05c
timeout -k 10 300 python -u -m pytest tests/test_concurrent_sessions.py tests/test_jbod.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/r05c/pytest.log 2>&1 || { tail -30 gpurun_out/r05c/pytest.log; exit 1; }
tail -3 gpurun_out/r05c/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r05c_c4 -o c4 -- python3 bench.py --workload c4 --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/r05c/c4_bench_prof.json 2> gpurun_out/r05c/c4_bench_prof.err || exit 1
find /tmp/r05c_c4 -name "*kernel_stats.csv" -exec cp {} gpurun_out/r05c/c4_kernel_stats.csv \;
python3 -c "import json; d=json.loads(open('gpurun_out/r05c/c4_bench_prof.json').read().strip().splitlines()[-1]); r=d['roofline']; print(d['ms_per_step'], r['frac'], r['avg_launch_us'], r['traffic_over_algorithmic'], r['intra_sort'])"
grep intra gpurun_out/r05c/c4_kernel_stats.csv | cut -c1-30,60-
