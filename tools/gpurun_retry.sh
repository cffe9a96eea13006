#!/bin/bash
# Local wrapper around the gpurun client: re-submits ONLY when the call never
# ran (gpurun status "transient": no box / box lost while being prepared --
# nothing executed, nothing charged), up to 4 times with a pause.  Any call
# that ran, whatever its result, is never repeated.
# usage: tools/gpurun_retry.sh <timeout> '<command>'
t=$1; shift
for i in 1 2 3 4; do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@"
  rc=$?
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$st" != "transient" ] && [ $rc -ne 3 ]; then exit $rc; fi
  echo "[gpurun_retry] transient (attempt $i), retrying in 60 s"
  sleep 60
done
exit $rc
