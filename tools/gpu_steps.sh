#!/bin/bash
# Run GPU steps in order; continue past ordinary failures (rc 1/2/5: test
# failures, usage errors) but stop at the first crash, abort or timeout.
mkdir -p gpurun_out
for cmd in "$@"; do
  echo ">>> $cmd"
  bash -c "$cmd"
  rc=$?
  echo "<<< rc=$rc"
  case $rc in 0|1|2|5) ;; *) echo "stopping after rc=$rc"; exit $rc;; esac
done
