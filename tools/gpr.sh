#!/usr/bin/env bash
# usage: gpr.sh <outfile> <timeout> <command>   -- retries only while no box is free (exit 3)
out=$1; lim=$2; shift 2
for i in $(seq 1 200); do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$@" > "$out" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "status=transient" "$out"; then echo "rc=$rc" >> "$out"; exit $rc; fi
  sleep 90
done
echo "gave up" >> "$out"
