#!/bin/bash
# Submit one gpurun call; re-submit only while the call never ran (status "transient": no box,
# box lost while being prepared, slots busy, back-off).  A call that ran is never repeated.
# Usage: bash scripts/gpurun_submit.sh <log> <timeout s> '<command>'
log=$1; to=$2; cmd=$3
cd /root/repo
for i in $(seq 1 40); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$log" 2>&1
  st=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('status'))" 2>/dev/null)
  run=$(python3 -c "import json;print(json.load(open('gpurun_out/.last_call.json')).get('run_s') or 0)" 2>/dev/null)
  if [ "$st" != "transient" ] || [ "$run" != "0.0" -a "$run" != "0" ]; then exit 0; fi
  sleep 150
done
