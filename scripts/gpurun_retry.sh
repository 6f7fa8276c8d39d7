#!/bin/bash
# Local helper (runs HERE, not on the GPU box): resubmit a gpurun call only when the
# infrastructure reports a transient failure before the command ran (nothing charged).
# Any real result (ok / fail / timeout / fault) is returned as-is, never retried.
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun "$@" > /tmp/gpurun_last.txt 2>&1
  rc=$?
  if grep -q "status=transient" /tmp/gpurun_last.txt || [ $rc -eq 3 ]; then
    echo "[retry $i] transient infra failure; waiting"; sleep 60; continue
  fi
  cat /tmp/gpurun_last.txt | tail -8
  exit $rc
done
tail -5 /tmp/gpurun_last.txt
exit 3
