#!/bin/bash
# Helper for gpurun calls: `source scripts/gpu_steps.sh; step <name> <timeout_s> <cmd...>`.
# Runs each GPU step under its own time limit, logs to gpurun_out/<name>.log, and stops the whole call
# (no further GPU work) after a fault / abort / segfault / timeout; ordinary failures (exit 1, e.g. an
# assertion) let the following steps run.
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then
    echo "fatal rc=$rc in $name: stopping this call" | tee -a gpurun_out/steps.log
    exit $rc
  fi
  return 0
}
