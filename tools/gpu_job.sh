#!/bin/bash
# Run a sequence of GPU steps on the gpurun box. Each step: "<timeout_s> <name> <command...>".
# A step that fails with exit 1 (test failures) does not stop the job; anything else
# (fault/abort/segfault/timeout) ends it: nothing more touches the GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH="$PWD${PYTHONPATH:+:$PYTHONPATH}"
run() {
  local t=$1; local name=$2; shift 2
  echo "=== $name: $*" | tee -a gpurun_out/job.log
  local start=$(date +%s)
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - start ))s)" | tee -a gpurun_out/job.log
  tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "fatal rc=$rc in $name; stopping"; exit $rc; fi
  return 0
}
