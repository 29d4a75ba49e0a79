#!/bin/bash
# Same-box A/B over environment settings of one built tree: one C2 probe per setting, in the order given, ROUNDS times
# (2). Each argument is a label=ENV string, e.g.  base=CCMI_SOLO=0  solo=CCMI_SOLO=1  (several variables: a=X=1,Y=2).
# STAMPS=1 adds CCMI_STAMPS. One gpurun call; stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in $(seq 1 ${ROUNDS:-2}); do
  for spec in "$@"; do
    name=${spec%%=*}_$i
    envs=${spec#*=}
    echo "== $name ($envs, $(date +%T))"
    (IFS=','; for kv in $envs; do export "$kv"; done
     [ "${STAMPS:-0}" = 1 ] && export CCMI_STAMPS=1
     CCMI_PROFILE=1 timeout -k 10 300 python -u tools/probe.py --workload c2) > gpurun_out/abe_$name.log 2>&1
    rc=$?
    grep -E "^total|server stamps|row stamps|LeaderReplica" gpurun_out/abe_$name.log | sort -u
    [ $rc -eq 0 ] || { echo "stopping: rc=$rc"; tail -5 gpurun_out/abe_$name.log; exit $rc; }
  done
done
