set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/sr_trace -o r -- python3 $R/tools/shard_replay.py --G 8 --rank 0 --ticks 20 ${REPLAY_ARGS:-} > $R/gpurun_out/sr_trace.log 2>&1
cd $R && python3 tools/trace_gaps.py gpurun_out/sr_trace --marker "${MARKER:-slot_count_kernel}" --out gpurun_out/sr_gaps.json
