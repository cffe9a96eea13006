#!/bin/bash
# Local wrapper around the gpurun client: re-submits ONLY when the call never
# ran (gpurun status "transient": no box / box lost while being prepared --
# nothing executed, nothing charged), up to GPURUN_RETRIES (12) times with a pause.  Any call
# that ran, whatever its result, is never repeated.
# usage: tools/gpurun_retry.sh <timeout> '<command>'
t=$1; shift
for i in $(seq 1 ${GPURUN_RETRIES:-12}); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- "$@" 2>&1 | tee /tmp/gpurun_retry_last.log
  rc=${PIPESTATUS[0]}
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$st" != "transient" ] && [ $rc -ne 3 ]; then exit $rc; fi
  # honour the client's back-off ("retry in Ns") when it gives one
  wait=$(python3 -c "import re;m=re.findall(r'retry in (\d+)s',open('/tmp/gpurun_retry_last.log').read());print(int(m[-1])+15 if m else 240)" 2>/dev/null || echo 240)
  echo "[gpurun_retry] transient (attempt $i), retrying in $wait s"
  sleep $wait
done
exit $rc
