#!/bin/bash
# Re-submits a gpurun call only when the infrastructure reports a transient failure
# (nothing ran on the GPU); any real result (pass or fail) is returned as is.
for i in $(seq 1 ${RETRIES:-12}); do
  /usr/local/graft/bin/gpurun "$@"
  rc=$?
  st=$(python3 -c "import json; print(json.load(open('gpurun_out/.last_call.json')).get('status',''))" 2>/dev/null)
  if [ "$st" != "transient" ] && [ $rc -ne 3 ]; then exit $rc; fi
  echo "[retry] transient gpurun failure, waiting 60s ($i)"
  sleep 60
done
exit $rc
