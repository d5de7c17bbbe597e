#!/bin/bash
# Parity + timing after a route-kernel change: routing / full-size / sharded GPU tests, the C3 route
# shapes (tools/tune_route.py) and the default bench line with its kernel stats.
set -uo pipefail
T=${1:-ff}
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_routing.py tests/test_gpu_fullsize.py tests/test_gpu_sharded_native.py tests/test_gpu_multi.py -x -q --timeout 300 --timeout-method thread > $O/${T}_tests.log 2>&1 || { tail -30 $O/${T}_tests.log; exit 1; }
tail -1 $O/${T}_tests.log
timeout -k 10 300 python -u tools/tune_route.py --workload c3 --cfgs 10,8 --rounds 3 --steps 10 > $O/${T}_tune.json 2>&1 || { tail $O/${T}_tune.json; exit 1; }
tail -1 $O/${T}_tune.json
timeout -k 10 300 python -u bench.py > $O/${T}_bench.json 2> $O/${T}_bench.err || { tail $O/${T}_bench.err; exit 1; }
python -c "import json; d=json.loads(open('$O/${T}_bench.json').read().strip().splitlines()[-1]); print('C3', d['ms_per_step'], d['roofline']['frac'], d['value']); c=d['extra']['c2']; print('C2', c['ms_per_step'], c['roofline']['frac']); print('csr_only', d.get('csr_only'))"
