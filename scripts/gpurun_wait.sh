#!/bin/bash
# gpurun, re-submitted only while the pool has no slot / box (status=transient: nothing ran,
# nothing charged); any other outcome (pass, fail, refusal) ends it.
#     bash scripts/gpurun_wait.sh LOG TIMEOUT 'command' [TRIES]
log=$1; to=$2; cmd=$3; tries=${4:-30}
for i in $(seq 1 "$tries"); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  grep -q "status=transient" "$log" || exit 0
  sleep 120
done
