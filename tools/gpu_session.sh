#!/bin/bash
# Guarded GPU session: run named steps, each under its own time limit. Continue past ordinary
# failures (exit 1/2: failing tests / usage); stop on anything that looks like a crash or hang
# (>=124: timeout/kill, 134 abort, 139 segv, ...). Logs go to gpurun_out/<name>.log.
# usage: tools/gpu_session.sh "name|seconds|command" ...
set -u
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 2 ] && [ $rc -ne 5 ]; then
    echo "=== stopping: step $name ended with rc=$rc"
    exit $rc
  fi
done
