#!/bin/bash
# A/B of two builds of the library in one gpurun call: tools/gpu_ab.sh NAME ROUNDS -- cmd args...
# runs cmd with WQ_LIBRARY=abtest/libwq_base.so and abtest/libwq_new.so alternately, ROUNDS times
# each, logs in gpurun_out/NAME_{base,new}_K.log
set -e
name=$1; rounds=$2; shift 3
for k in $(seq 1 "$rounds"); do
    for v in base new; do
        WQ_LIBRARY=abtest/libwq_$v.so tools/gpu_step.sh ${name}_${v}_$k 400 "$@"
    done
done
