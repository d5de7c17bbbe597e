"""Builds libwq_router.so in-tree with hipcc for gfx950 (no JIT cache, no CPU variant).

    python -m worldql_server_amd.build        # incremental
    python -m worldql_server_amd.build --force
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(PKG, "_build")
LIB = os.path.join(PKG, "libwq_router.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

SOURCES = ["wq_route.hip", "wq_global.hip", "wq_query.hip", "wq_table.hip", "wq_delta.hip", "wq_shard.hip", "wq_sharded.hip", "wq_peers.hip", "wq_multi.hip", "wq_router.hip"]
HOST_SOURCES = ["wq_codec.cpp"]
CXX = os.environ.get("CXX", "g++")
HOST_FLAGS = ["-O3", "-fPIC", "-std=c++17", "-pthread", "-Wall"]
HEADERS = ["lane_xchg.hpp", "wq_device.hpp", "wq_internal.hpp", "route_common.hpp", "route_count.hpp", "route_scan.hpp", "route_emit.hpp", "route_tick.hpp", "route_radius.hpp", "route_spill.hpp", "route_gather.hpp", "table_prims.hpp"]
# No fast-math and no FMA contraction: coord_clamp must reproduce Rust's f64 op sequence.
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=off",
         "-fno-fast-math", "-Wall", "-Wno-unused-function", "-Wno-unused-result"]


def _mtime(p):
    return os.path.getmtime(p) if os.path.exists(p) else 0.0


def _jobs() -> int:
    """Parallel compiles: MAX_JOBS when set (16 on the GPU boxes), else the CPUs, at most 8."""
    env = os.environ.get("MAX_JOBS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return max(1, min(8, os.cpu_count() or 1))


def build(force: bool = False, verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    hdr_t = max(_mtime(os.path.join(CSRC, h)) for h in HEADERS)
    hdr_t = max(hdr_t, _mtime(os.path.join(ROOT, "include", "wq_router.h")))
    objs, cmds = [], []
    relink = force or not os.path.exists(LIB)
    for src in SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(BUILD, src.replace(".hip", ".o"))
        objs.append(o)
        if force or _mtime(o) < max(_mtime(s), hdr_t):
            cmds.append([HIPCC, *FLAGS, "-I", os.path.join(ROOT, "include"), "-c", s, "-o", o])
    # host-only C++ (the wire codec): g++, no device code
    codec_h = _mtime(os.path.join(ROOT, "include", "wq_codec.h"))
    for src in HOST_SOURCES:
        s = os.path.join(CSRC, src)
        o = os.path.join(BUILD, src.replace(".cpp", ".o"))
        objs.append(o)
        if force or _mtime(o) < max(_mtime(s), codec_h):
            cmds.append([CXX, *HOST_FLAGS, "-I", os.path.join(ROOT, "include"), "-c", s, "-o", o])
    if cmds:
        relink = True
        for c in cmds:
            if verbose:
                print(" ".join(c), flush=True)
        # the translation units compile independently (wq_route / wq_sharded dominate)
        with ThreadPoolExecutor(max_workers=min(_jobs(), len(cmds))) as pool:
            rcs = list(pool.map(lambda c: subprocess.call(c), cmds))
        for c, rc in zip(cmds, rcs):
            if rc != 0:
                raise subprocess.CalledProcessError(rc, c)
    if relink or any(_mtime(o) > _mtime(LIB) for o in objs):
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-pthread", "-o", LIB, *objs, "-ldl"]
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.check_call(cmd)
    return LIB


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    a = ap.parse_args()
    print(build(force=a.force, verbose=True))
    sys.exit(0)
