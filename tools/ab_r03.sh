#!/bin/bash
# Same-box A/B: the round-3 tree (ab_r03/, built from commit 42b8fb8) against the current tree, one C2 proposal each
# with server stamps; alternating, twice. One gpurun call; stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for i in 1 2; do
  for tree in ab_r03 .; do
    name=$( [ "$tree" = . ] && echo cur || echo r03 )_$i
    echo "== $name ($(date +%T))"
    (cd "$tree" && CCMI_STAMPS=1 CCMI_PROFILE=1 timeout -k 10 300 python -u tools/probe.py --workload c2) \
      > gpurun_out/ab_$name.log 2>&1
    rc=$?
    grep -E "^total|server stamps|chain stamps" gpurun_out/ab_$name.log | sort -u
    [ $rc -eq 0 ] || { echo "stopping: rc=$rc"; tail -5 gpurun_out/ab_$name.log; exit $rc; }
  done
done
