#!/usr/bin/env bash
# Submit one gpurun call, re-submitting only while the pool answers "no box or slot free" (exit 3:
# nothing ran, nothing was charged). Any other outcome -- success, a failed or timed-out command,
# a refusal -- ends the script with that exit code: a GPU step that ran is never repeated.
#   tools/gpurun_when_free.sh LOG TIMEOUT 'command'
log=$1 timeout=$2 cmd=$3
for attempt in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$timeout" -- "$cmd" > "$log" 2>&1
  rc=$?
  [ "$rc" -ne 3 ] && exit "$rc"
  echo "[gpurun_when_free] attempt $attempt: no slot free, waiting" >> "$log.wait"
  sleep 240
done
exit 3
