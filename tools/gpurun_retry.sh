#!/bin/bash
# tools: retry a gpurun call only while the pool reports a transient/no-box status (the command never ran)
out=$1; shift
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun "$@" > $out 2>&1
  st=$(python3 -c "import json;print(json.load(open('/root/repo/gpurun_out/.last_call.json')).get('status'))" 2>/dev/null)
  if [ "$st" != "transient" ] && ! grep -q "retry in\|no free box\|slot(s) on this pod are busy" $out; then exit 0; fi
  if grep -q "status=ok\|status=fail" $out; then exit 0; fi
  sleep 60
done
