#!/bin/bash
# tools/gpu.sh <timeout> <log> <command...> — gpurun with up to 4 attempts when
# no box could be acquired (exit 3: nothing ran, nothing charged).
T=$1; LOG=$2; shift 2
for attempt in 1 2 3 4; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > "$LOG" 2>&1
  rc=$?
  if [ $rc -ne 3 ]; then echo "exit $rc" >> "$LOG"; exit $rc; fi
  echo "attempt $attempt: no box (exit 3), waiting" >> "$LOG.retries"
  sleep 60
done
echo "exit 3" >> "$LOG"; exit 3
