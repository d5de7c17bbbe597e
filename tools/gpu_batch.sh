#!/bin/bash
# One gpurun call's batch of GPU steps (run on the box from the repo root), replacing round 4's
# one-off tools/gpu_batch_r04*.sh. Each step runs under its own time limit through tools/gpu_step.sh
# (log: gpurun_out/<name>.log); the first failing step ends the batch (set -e), so nothing more runs
# on the GPU after a fault, an abort or a time limit.
#
#   tools/gpu_batch.sh STEP [STEP ...]
#     tests              the whole GPU suite                       (t_all)
#     tests=FILE[,FILE]  those GPU test files                       (t_<first file>)
#     smoke              __graft_entry__ build-free smoke           (smoke)
#     bench              the default bench line                     (b_default)
#     bench=ARGS         bench.py with ARGS (commas for spaces)     (b_<args>)
#     kstats=NAME        rocprofv3 kernel stats of the default line (tools/kstats_bench.sh)
#     replay             tools/shard_replay.py, G = 8, shard 0      (replay)
#     replica            tools/replica_slice.py, N = 1 2 4 8        (replica)
#     ab=NAME,ROUNDS,CMD A/B of abtest/libwq_{base,new}.so on CMD  (tools/gpu_ab.sh)
#     run=NAME,SECS,CMD  anything else (commas for spaces)
set -e
export TMPDIR=/tmp
S=tools/gpu_step.sh
PYTEST="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
for step in "$@"; do
  key=${step%%=*}; val=${step#*=}; [ "$key" = "$step" ] && val=""
  case $key in
    tests)   if [ -z "$val" ]; then $S t_all 1100 $PYTEST tests
             else f=${val%%,*}; f=${f##*/}; $S "t_${f%.py}" 900 $PYTEST ${val//,/ }; fi ;;
    smoke)   $S smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)   if [ -z "$val" ]; then $S b_default 400 python bench.py
             else n=${val//[^a-z0-9]/_}; $S "b_${n:0:40}" 400 python bench.py ${val//,/ }; fi ;;
    kstats)  timeout -k 10 420 bash tools/kstats_bench.sh "${val:-default}" > "gpurun_out/ks_${val:-default}.log" 2>&1 ;;
    replay)  $S replay 400 python tools/shard_replay.py --G 8 --rank 0 --ticks 20 ;;
    replica) $S replica 500 python tools/replica_slice.py --n 1 2 4 8 ;;
    ab)      IFS=, read -r n r cmd <<< "$val"; tools/gpu_ab.sh "$n" "$r" -- ${cmd//,/ } ;;
    run)     IFS=, read -r n secs cmd <<< "$val"; $S "$n" "$secs" ${cmd//,/ } ;;
    *)       echo "unknown step $step" >&2; exit 2 ;;
  esac
done
echo batch done
