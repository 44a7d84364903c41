#!/bin/bash
# run_steps.sh "<label>:<timeout>:<command>" ... -- runs GPU steps in order; stops at the first
# step whose exit status is not 0/1 (fault, abort, segfault, timeout): nothing more touches the GPU.
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  label="${spec%%:*}"; rest="${spec#*:}"; to="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $label (timeout ${to}s): $cmd"
  timeout -k 10 "$to" bash -c "$cmd" > "gpurun_out/$label.log" 2>&1
  rc=$?
  tail -n ${TAIL:-15} "gpurun_out/$label.log"
  echo "=== $label rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $label"; exit $rc; fi
done
