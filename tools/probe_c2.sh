#!/bin/bash
# C2 probe only (build, then one optimization with the profiler; extra env passes through), one gpurun call.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
make -C cruise-control_amd -j16 > gpurun_out/make.log 2>&1 || exit 1
echo "== probe ($(date +%T))"
CCMI_PROFILE=1 timeout -k 10 600 python -u tools/probe.py --workload ${WORKLOAD:-c2} > gpurun_out/probe_${TAG:-x}.log 2>&1
rc=$?
echo "== probe rc=$rc"; grep -v "^  #" gpurun_out/probe_${TAG:-x}.log | tail -40
exit $rc
