#!/bin/bash
# (host-side helper, not a GPU script) retry gpurun only while the pool reports a transient (no box / backoff) status; usage: gpr.sh <outfile> <timeout> <cmd>
out=$1; to=$2; shift 2
for i in $(seq 1 15); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $out 2>&1
  rc=$?
  if grep -q "status=transient" $out && ! grep -q "status=ok\|rc=0\|exit" <(grep "status=" $out | grep -v transient); then
    sleep 60; continue
  fi
  break
done
echo "gpr: tries=$i rc=$rc" >> $out
