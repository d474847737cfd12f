#!/bin/bash
# GPU-box check script: tests, then benches. Stops on any crash/timeout (rc not 0/1).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
run() {  # run <timeout> <log> <cmd...>
  local t=$1 log=$2; shift 2
  echo "== $* (timeout $t)" | tee -a gpurun_out/summary.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$log" 2>&1
  local rc=$?
  echo "   rc=$rc" | tee -a gpurun_out/summary.log
  tail -5 "gpurun_out/$log" | tee -a gpurun_out/summary.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: rc=$rc" | tee -a gpurun_out/summary.log; exit $rc; fi
  # a GPU fault can surface as a Python exception (rc 1): stop before anything else runs
  if grep -qE "MEMORY_APERTURE_VIOLATION|illegal memory access|HSA_STATUS_ERROR|Memory access fault" "gpurun_out/$log"; then
    echo "STOP: GPU fault reported in $log" | tee -a gpurun_out/summary.log; exit 3
  fi
  return 0
}
