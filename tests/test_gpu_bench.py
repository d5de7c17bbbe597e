"""bench.py's multi-GPU line, rehearsed on one GPU: `bench.py --gpus 2` with no
launcher starts its two ranks itself; WQ_BENCH_ONE_GPU=1 puts both on cuda:0 over gloo (RCCL refuses
two ranks on one GPU). The N = 2 line must carry n_gpus = 2, a real roofline and the same pairs per
tick as the N = 1 line of the same (scaled) C3 tick — the scaling run's line, assembled by the same
code the driver's 8-GPU run uses."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, env=None, timeout=400):
    p = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, (p.returncode, p.stderr[-4000:])
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-4000:]
    return json.loads(lines[0])


def test_bench_two_rank_rehearsal_line_matches_one_rank():
    common = ["--scale", "0.2", "--steps", "3", "--warmup", "1", "--no-cpu-baseline"]
    env = dict(os.environ, WQ_BENCH_ONE_GPU="1")
    env.pop("WORLD_SIZE", None)
    two = _bench("--gpus", "2", *common, env=env)
    one = _bench("--gpus", "1", "--no-extra", *common, env=env)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["config"]["pairs_per_tick"] == one["config"]["pairs_per_tick"] > 0
    assert two["config"]["messages_per_tick"] == one["config"]["messages_per_tick"]
    for line in (one, two):
        rf = line["roofline"]
        assert rf["algorithmic_bytes"] > 0 and rf["frac"] > 0 and rf["achieved"] > 0, rf
        assert line["value"] > 0 and line["ms_per_step"] > 0
    # the per-GPU bytes of the N = 2 line are half the tick's (the same SURVEY §8(d) formula)
    assert abs(two["roofline"]["algorithmic_bytes"] * 2 - one["roofline"]["algorithmic_bytes"]) <= 8
    cube = two["extra"]["cube_hash"]
    assert "error" not in cube, cube
    assert cube["value"] > 0
