#!/bin/bash
# The C2 probe under several environments on one box (A/B on the same host): AB_ENVS="NAME:VAR=x,VAR2=y NAME2:..."
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for spec in ${AB_ENVS:-base:CCMI_PROFILE=1}; do
  name=${spec%%:*}; envs=${spec#*:}
  echo "== $name ($envs) $(date +%T)"
  env CCMI_PROFILE=1 $(echo "$envs" | tr ',' ' ') timeout -k 10 600 python -u tools/probe.py --workload ${WORKLOAD:-c2} > gpurun_out/ab_$name.log 2>&1
  rc=$?
  grep -E "^total|^perf|scan.wait|device.scan" gpurun_out/ab_$name.log
  if [ $rc -ne 0 ]; then echo "stopping: $name exited $rc"; tail -5 gpurun_out/ab_$name.log; exit $rc; fi
done
