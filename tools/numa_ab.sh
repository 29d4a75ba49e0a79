#!/bin/bash
# The C2 probe pinned to the GPU's NUMA node and to another node, alternated (is the bimodal scan round trip a
# placement effect?). One gpurun call:  /usr/local/graft/bin/gpurun --timeout 900 -- 'bash tools/numa_ab.sh'
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
read -r NODE LOCAL REMOTE < <(timeout -k 10 120 python3 tools/numa_probe.py) || exit 1
echo "gpu numa node $NODE; local cpus $LOCAL; remote cpus $REMOTE"
for spec in "local:$LOCAL" "remote:$REMOTE" "local2:$LOCAL" "remote2:$REMOTE" "free:" ; do
  name=${spec%%:*}; cpus=${spec#*:}
  echo "== $name ($cpus) $(date +%T)"
  if [ -n "$cpus" ]; then
    CCMI_PROFILE=1 timeout -k 10 600 taskset -c "$cpus" python3 -u tools/probe.py > "gpurun_out/numa_$name.log" 2>&1
  else
    CCMI_PROFILE=1 timeout -k 10 600 python3 -u tools/probe.py > "gpurun_out/numa_$name.log" 2>&1
  fi
  rc=$?
  grep -E "^total|scan.wait" "gpurun_out/numa_$name.log" | tail -2
  if [ $rc -ne 0 ]; then echo "stopping: $name exited $rc"; tail -5 "gpurun_out/numa_$name.log"; exit $rc; fi
done
