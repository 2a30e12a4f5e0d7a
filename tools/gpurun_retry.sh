#!/bin/bash
# retries a gpurun call only while the pool has no slot / box (exit 3:
# nothing ran, nothing charged); any other outcome is final
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[retry] pool busy (attempt $i), waiting 90 s"
  sleep 90
done
exit 3
