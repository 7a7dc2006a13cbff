#!/bin/bash
# Run GPU steps sequentially; stop at the first crash-like exit (fault / abort / timeout), continue
# past ordinary test failures. Usage: scripts/gpu_run.sh "<name>:<timeout>:<cmd>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; to="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name (timeout $to s): $cmd"
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name exit $rc"
  tail -n 25 "gpurun_out/$name.log"
  case $rc in
    0|1|2|5) ;;
    *) echo "=== stopping after crash-like exit $rc"; exit $rc ;;
  esac
done
