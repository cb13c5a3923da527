#!/bin/bash
# Host-side helper: submit a gpurun call, re-submitting only while the pool reports that
# nothing ran (status=transient: no free box / slot, infrastructure back-off).  A call that
# ran -- whatever its exit status -- is never repeated.
# usage: gpurun_retry.sh TIMEOUT 'command' LOG [TRIES]
T=$1; CMD=$2; LOG=$3; N=${4:-12}
for i in $(seq 1 $N); do
  /usr/local/graft/bin/gpurun --timeout $T -- "$CMD" > $LOG 2>&1
  rc=$?
  if grep -q "status=transient" $LOG && ! grep -q "status=ok" $LOG; then
    w=$(grep -o "retry in [0-9]*s" $LOG | grep -o "[0-9]*" | tail -1)
    sleep $(( ${w:-60} > 60 ? ${w:-60} + 5 : 60 ))
    continue
  fi
  exit $rc
done
exit 3
