#!/bin/bash
# One GPU step of a gpurun call: run "$@" under a time limit, output to gpurun_out/$NAME.log.
# usage: tools/gpu_step.sh NAME SECONDS cmd args...   (stops the chain on failure: use with &&)
name=$1; secs=$2; shift 2
mkdir -p gpurun_out
echo "== $name: $*" >&2
timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "== $name rc=$rc" >&2
tail -5 "gpurun_out/$name.log" >&2
exit $rc
