#!/usr/bin/env python3
"""Per-kernel VGPR / AGPR / scratch / occupancy of a HIP source compiled for gfx950
(hipcc -Rpass-analysis=kernel-resource-usage), one line per kernel.

  [SC_FLAGS="-DX=1"] python scripts/resource_usage.py [kernels.hip] [name-filter]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = os.path.abspath(sys.argv[1]) if len(sys.argv) > 1 else os.path.join(ROOT, "sparsecholesky_amd/csrc/kernels.hip")
filt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-munsafe-fp-atomics",
       "-I" + os.path.join(ROOT, "include"), "-x", "hip", "-c", src, "-o", "/tmp/resource_usage.o",
       "--offload-device-only", "-Rpass-analysis=kernel-resource-usage"] + os.environ.get("SC_FLAGS", "").split()
out = subprocess.run(cmd, capture_output=True, text=True, cwd=os.path.dirname(os.path.abspath(src))).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).split()[0]] = int(m.group(2))
for name, r in rows.items():
    short = re.sub(r"^_ZN2sc\d+", "", name)
    short = re.sub(r"EEEvPK.*$|EvNS_.*$|EEvNS_.*$", "", short)
    if filt and filt not in short:
        continue
    print(f"{short:60s} vgpr {r.get('VGPRs', 0):3d} agpr {r.get('AGPRs', 0):3d} "
          f"scratch {r.get('ScratchSize', 0):4d} occ {r.get('Occupancy', 0)}")
