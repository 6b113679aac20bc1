"""Kernel resource report (development tool): VGPRs, scratch, occupancy and LDS of every kernel in
a HIP source, from the compiler's kernel-resource-usage remarks.
usage: python3 tools/kres.py <file.hip> [filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
                      "--cuda-device-only", "-c", src, "-o", "/tmp/kres.o", "-Rpass-analysis=kernel-resource-usage"],
                     capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]|VGPRs Spill): (\S+)", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    else:
        cur[k if k.startswith('VGPRs') else k.split()[0]] = v
for r in rows:
    if flt in r["name"]:
        print(f"{r.get('VGPRs', '?'):>4} vgpr {r.get('VGPRs Spill', '?'):>4} spill {r.get('ScratchSize', '?'):>5} scr "
              f"{r.get('Occupancy', '?'):>2} occ {r.get('LDS', '?'):>6} lds  {r['name'][:90]}")
