#!/bin/bash
# Same-box A/B over built trees (directories holding cruise-control_amd/ + tools/probe.py): one C2 proposal each with
# server stamps (STAMPS=0: none), in the order given, ROUNDS times (2). One gpurun call; stops at the first failure. A tree such as ab_prev (a
# `git worktree` of an older commit, built in place) must not be listed in .gpurunignore while it is compared.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in $(seq 1 ${ROUNDS:-2}); do
  for tree in "$@"; do
    name=$(basename "$(cd "$tree" && pwd)")_$i
    echo "== $name ($(date +%T))"
    (cd "$tree" && { [ "${STAMPS:-1}" = 1 ] && export CCMI_STAMPS=1; CCMI_PROFILE=1 timeout -k 10 300 python -u tools/probe.py --workload c2; }) \
      > gpurun_out/abt_$name.log 2>&1
    rc=$?
    grep -E "^total|server stamps|chain stamps" gpurun_out/abt_$name.log | sort -u
    [ $rc -eq 0 ] || { echo "stopping: rc=$rc"; tail -5 gpurun_out/abt_$name.log; exit $rc; }
  done
done
