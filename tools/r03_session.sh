#!/bin/bash
# One gpurun call: C2 probe A/B (tree worker on / off), the bench line + rocprofv3 trace (bench_r03.sh), then the
# GPU tests selected by PYTEST_K.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
AB_ENVS="worker:CCMI_TREE_WORKER=1 noworker:CCMI_X=0" bash tools/ab_probe.sh || exit $?
bash tools/bench_r03.sh
