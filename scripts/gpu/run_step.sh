#!/bin/bash
# run_step.sh NAME TIMEOUT CMD... : run one GPU step under its own time limit,
# log to gpurun_out/NAME.log, and stop the whole session (exit) on a fault,
# abort, segfault or timeout.  Test failures (rc 1) do not stop the session.
name=$1; shift; tmo=$1; shift
mkdir -p gpurun_out
echo "=== [$name] $(date +%T) $*" | tee -a gpurun_out/session.log
timeout -k 10 "$tmo" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "=== [$name] rc=$rc $(date +%T)" | tee -a gpurun_out/session.log
tail -n 25 "gpurun_out/$name.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
  echo "FATAL step $name rc=$rc: stopping session" | tee -a gpurun_out/session.log
  exit $rc
fi
exit 0
