#!/usr/bin/env python3
"""Per-kernel resource usage of one source file (VGPRs, AGPRs, spills,
scratch, occupancy) from hipcc's kernel-resource-usage remarks:
  python3 tools/kres.py csrc/fused.hip [filter]   (run from crypto-recommendation_amd/)"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off",
       "-I../include", "-Icsrc", "-x", "hip", "-c", src, "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    if flt in r["name"]:
        print(f'{r.get("VGPRs","?"):>4} v {r.get("AGPRs","?"):>4} a  spill v{r.get("VGPRs Spill","?")} s{r.get("SGPRs Spill","?")}'
              f'  scratch {r.get("ScratchSize [bytes/lane]","?"):>4}  occ {r.get("Occupancy [waves/SIMD]","?")}  {r["name"]}')
