#!/bin/bash
# C2 measurement pass (one gpurun call): in-kernel phase stamps of the cross/pair scans (CCMI_STAMPS=1) and a
# rocprofv3 kernel trace reduced to a duration histogram by kernel and grid size (tools/trace_hist.py).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
make -C cruise-control_amd -j16 > gpurun_out/make.log 2>&1 || exit 1
echo "== stamps"
CCMI_STAMPS=1 CCMI_PROFILE=1 timeout -k 10 600 python -u tools/probe.py --workload c2 > gpurun_out/probe_stamps.log 2>&1 || exit $?
tail -3 gpurun_out/probe_stamps.log
echo "== trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o probe -- \
  python3 tools/probe.py --workload c2 > gpurun_out/probe_trace.log 2>&1 || exit $?
f=$(find gpurun_out/prof -name '*kernel_trace.csv' | head -1)
python3 tools/trace_hist.py "$f" > gpurun_out/trace_hist.txt
find gpurun_out/prof -name '*kernel_trace.csv' -delete
cat gpurun_out/trace_hist.txt
