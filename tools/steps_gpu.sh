#!/bin/bash
# Consecutive-proposal timing variants (tools/steps_probe.py), one gpurun call; stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${TAG:-steps}
i=0
for args in "${@:-}"; do
  i=$((i + 1))
  echo "== variant $i: $args ($(date +%T))"
  timeout -k 10 300 python -u tools/steps_probe.py $args > gpurun_out/${T}_$i.log 2>&1
  rc=$?
  grep -E "^run|^launch" gpurun_out/${T}_$i.log
  [ $rc -eq 0 ] || { echo "stopping: rc=$rc"; tail -5 gpurun_out/${T}_$i.log; exit $rc; }
done
