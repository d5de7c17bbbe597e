"""VGPRs / occupancy / spills per kernel of one HIP source (compile-time resource usage).
Usage: python tools/occupancy.py worldql_server_amd/csrc/wq_route.hip [...]"""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/tools/", 1)[0]


def usage(src):
    out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17",
                          "-ffp-contract=off", "-fno-fast-math", "-I", ROOT + "/include", "-c", src, "-o",
                          "/tmp/_occ.o", "-Rpass-analysis=kernel-resource-usage"],
                         capture_output=True, text=True).stderr
    rows, name = {}, None
    for line in out.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            name = m.group(1)
            rows[name] = {}
            continue
        m = re.search(r"remark:\s+(VGPRs|Occupancy \[waves/SIMD\]|VGPRs Spill|LDS Size \[bytes/block\]): (\d+)", line)
        if m and name:
            rows[name][{"VGPRs": "vgpr", "VGPRs Spill": "spill"}.get(m.group(1), m.group(1).split()[0])] = int(m.group(2))
    return rows


if __name__ == "__main__":
    for src in sys.argv[1:]:
        for k, v in sorted(usage(src).items()):
            if "rocprim" in k:
                continue
            print(f"{v.get('vgpr', '?'):>4} vgpr {v.get('Occupancy', '?'):>2} waves spill {v.get('spill', 0):>3} "
                  f"lds {v.get('LDS', '?'):>6}  {k[:90]}")
