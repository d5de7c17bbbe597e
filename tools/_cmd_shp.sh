set -uo pipefail
R=$(pwd); mkdir -p gpurun_out/shp; cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $R/gpurun_out/shp/prof -o r -- python3 $R/tools/sharded_overhead.py --steps 5 > $R/gpurun_out/shp/out.json 2>$R/gpurun_out/shp/err.txt; rc=$?; cat $R/gpurun_out/shp/out.json; exit $rc
