#!/bin/bash
# gpurun with retries only when the call never ran (infrastructure: status=transient / exit 3)
LOG=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  timeout 1700 /usr/local/graft/bin/gpurun "$@" > $LOG 2>&1
  rc=$?
  if grep -q "status=transient" $LOG || [ $rc -eq 3 ]; then
    w=$(grep -o "retry in [0-9]*s" $LOG | grep -o "[0-9]*" | head -1)
    sleep $(( ${w:-60} + 10 ))
    continue
  fi
  exit $rc
done
exit $rc
