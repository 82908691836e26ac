#!/bin/bash
# Run `gpurun -- <cmd>` once a box is free: retries ONLY while gpurun reports
# that nothing ran (no free box / slot, or infrastructure back-off); any run
# that started ends the loop, whatever its outcome.
#   tools/gpurun_when_free.sh <log> <timeout_s> '<command>'
LOG=${1:?log}
TO=${2:?timeout}
CMD=${3:?command}
for attempt in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  if grep -q "no free box\|GPU slot(s) on this pod are busy\|backing off\|stopped responding while being prepared" "$LOG" \
     && ! grep -q "status=ok\|status=fail\|rc=[0-9]" "$LOG"; then
    sleep 120
    continue
  fi
  break
done
tail -3 "$LOG"
