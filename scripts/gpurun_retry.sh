#!/bin/bash
# Host-side helper: submit a gpurun call, re-submitting only while the pool reports that
# nothing ran (status=transient: no free box / slot, infrastructure back-off).  A call that
# ran -- whatever its exit status -- is never repeated.  Before every submission the in-tree
# library must match its sources (hmsc_amd/_lib.py _check_fresh): a tree whose csrc changed
# since the last build waits here instead of shipping a stale library.
# usage: gpurun_retry.sh TIMEOUT 'command' LOG [TRIES]
T=$1; CMD=$2; LOG=$3; N=${4:-12}
R=$(cd "$(dirname "$0")/.." && pwd)
for i in $(seq 1 $N); do
  until (cd "$R" && python -c "from hmsc_amd import _lib; _lib._check_fresh()" 2>/dev/null); do sleep 20; done
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
