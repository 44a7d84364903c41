#!/bin/bash
# gpurun_retry.sh LOG TIMEOUT CMD... -- submit CMD with gpurun; when no box / slot was free (status
# "transient": nothing ran, nothing charged) wait and submit again, up to MAX_TRIES (12) times, RETRY_SLEEP (200) s apart.  Any other outcome
# (the command ran, whatever its result) ends the loop: a GPU step that failed is never re-run here.
LOG=$1; TO=$2; shift 2
for i in $(seq 1 ${MAX_TRIES:-12}); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$LOG" 2>&1
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$st" != "transient" ]; then echo "attempt $i rc=$rc status=$st"; exit $rc; fi
  sleep ${RETRY_SLEEP:-200}
done
echo "gave up after ${MAX_TRIES:-12} attempts"; exit 3
