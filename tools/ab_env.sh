#!/bin/bash
# A/B of one environment switch in one gpurun call: tools/ab_env.sh NAME ROUNDS VAR A B -- cmd args...
# runs cmd with VAR=A and VAR=B alternately, ROUNDS times each; logs gpurun_out/NAME_{A,B}_K.log
set -e
name=$1; rounds=$2; var=$3; va=$4; vb=$5; shift 6
for k in $(seq 1 "$rounds"); do
    for v in "$va" "$vb"; do
        env "$var=$v" tools/gpu_step.sh "${name}_${v}_$k" 400 "$@"
    done
done
