#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first
# step that times out, aborts, segfaults or is killed (no further GPU step
# after those), continue past ordinary failures.  Usage:
#   bash scripts/gpu_steps.sh SECONDS 'cmd1' SECONDS 'cmd2' ...
mkdir -p gpurun_out
rc_all=0
while [ $# -ge 2 ]; do
    t=$1; cmd=$2; shift 2
    echo "=== [$t s] $cmd"
    timeout -k 10 "$t" bash -c "$cmd"
    rc=$?
    echo "=== rc=$rc"
    case $rc in
        124|137|134|139|143) echo "=== stopping: GPU step ended abnormally"; exit $rc ;;
        0) ;;
        *) rc_all=$rc ;;
    esac
done
exit $rc_all
