#!/bin/bash
# One gpurun call: C2 probe determinism (worker, noworker, worker again), then GPU tests selected by PYTEST_K.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
AB_ENVS="w1:CCMI_TREE_WORKER=1 nw:CCMI_X=0 w2:CCMI_TREE_WORKER=1" bash tools/ab_probe.sh || exit $?
if [ -n "${PYTEST_K:-}" ]; then
  echo "== pytest -m gpu -k ${PYTEST_K} $(date +%T)"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread -k "${PYTEST_K}" \
    > gpurun_out/pytest_s2.log 2>&1
  rc=$?; tail -5 gpurun_out/pytest_s2.log; exit $rc
fi
