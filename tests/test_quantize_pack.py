"""The fused quantise + pack of the slot grouping (wq_device.hpp quantize_pack) against
coord_clamp_dev + pack_key, the functions whose parity the oracle tests pin (cube_area.rs:23-44):
5.5M inputs on the host — exact multiples and their neighbouring doubles around the axis limits
(2^23 cubes, 2^40 units), +-0, subnormals, NaN, inf, saturating values, world ids at the packing
limit, cube sizes from 1 to past 2^40, and random bit patterns."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_quantize_pack_matches_clamp_and_pack(tmp_path):
    exe = tmp_path / "quantize_pack_check"
    subprocess.run([HIPCC, "-O2", "-std=c++17", "-I", os.path.join(ROOT, "include"),
                    "-I", os.path.join(ROOT, "worldql_server_amd", "csrc"),
                    os.path.join(ROOT, "tests", "quantize_pack_check.cpp"), "-o", str(exe)],
                   check=True, capture_output=True, timeout=300)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "mismatches 0" in r.stdout
