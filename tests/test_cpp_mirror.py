"""The C++ host mirror (worldql_server_amd/cpp/world_map.hpp) running the reference's unit tests.

Build (g++, links libwq_router.so) and the host-only sanitize KATs run on CPU; the GPU-backed
AreaMap KATs (area_map.rs:154-254) run under -m gpu.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def binary(tmp_path_factory):
    from worldql_server_amd.build import LIB, build
    if not os.path.exists(LIB):
        build()
    out = str(tmp_path_factory.mktemp("cpp") / "test_world_map")
    libdir = os.path.dirname(LIB)
    # the slices test stages its messages on each device itself: the HIP host API (no device code)
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-Wextra", "-D__HIP_PLATFORM_AMD__",
                           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "worldql_server_amd", "cpp"),
                           "-I", "/opt/rocm/include",
                           os.path.join(ROOT, "tests", "cpp", "test_world_map.cpp"), "-o", out,
                           "-L", libdir, "-lwq_router", f"-Wl,-rpath,{libdir}",
                           "-L", "/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"])
    return out


def test_cpp_mirror_builds_and_sanitize_kats(binary):
    r = subprocess.run([binary, "--host-only"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "host ok" in r.stdout


@pytest.mark.gpu
def test_cpp_mirror_area_map_kats_gpu(binary):
    r = subprocess.run([binary], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("ok")
