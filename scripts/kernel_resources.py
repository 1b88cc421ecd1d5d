#!/usr/bin/env python3
"""Register / scratch / LDS use of every k_rc_level instantiation of one translation unit
(hipcc -Rpass-analysis=kernel-resource-usage).  Usage: scripts/kernel_resources.py csrc/rc2dgi_rc_f32b.hip"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "--offload-arch=gfx950",
       "-mllvm", "-disable-promote-alloca-to-lds", "-I", os.path.join(ROOT, "include"), "-c", src, "-o", "/dev/null",
       "-Rpass-analysis=kernel-resource-usage"]
err = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in err.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark: +([\w /\[\]]+?): (\d+)", line)
    if cur and m:
        rows[cur][m.group(1).strip()] = int(m.group(2))
for name, r in rows.items():
    t = re.search(r"k_rc_levelILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELb([01])ELb([01])ELi(\d+)ELi(\d+)ENS_\d(\w+?)ELb([01])", name)
    tag = (f"{t.group(1)}x{t.group(2)}x{t.group(3)} pd{t.group(4)} top{t.group(5)} p2s{t.group(6)} unr{t.group(7)} "
           f"dl{t.group(8)} {t.group(9)} z0{t.group(10)}") if t else name[:60]
    print(f"{tag:55s} sgpr {r.get('TotalSGPRs')} vgpr {r.get('VGPRs')} scratch {r.get('ScratchSize [bytes/lane]')} "
          f"lds {r.get('LDS Size [bytes/block]')} occ {r.get('Occupancy [waves/SIMD]')}")
