#!/usr/bin/env python3
"""Per-kernel resource usage of one .hip file (hipcc -Rpass-analysis=
kernel-resource-usage): VGPRs, AGPRs, spills, occupancy, LDS, one line each.
    python tools/kres.py tmlibrary_amd/csrc/fused_kernels.hip [name-filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC",
                    "-ffp-contract=fast-honor-pragmas", "--offload-arch=gfx950", "-c", src,
                    "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"],
                   capture_output=True, text=True)
cur = None
rows = []
for ln in r.stderr.splitlines():
    m = re.search(r"remark: (.*) \[-Rpass", ln)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
dem = subprocess.run(["c++filt"], input="\n".join(x["name"] for x in rows),
                     capture_output=True, text=True).stdout.splitlines()
for x, d in zip(rows, dem):
    d = re.sub(r"\(.*", "", d).replace("tmh::", "")
    if flt in d:
        print("%-70s vgpr %4s agpr %3s vspill %3s sspill %3s occ %2s lds %6s" % (
            d[:70], x.get("VGPRs"), x.get("AGPRs"), x.get("VGPRs Spill"), x.get("SGPRs Spill"),
            x.get("Occupancy [waves/SIMD]"), x.get("LDS Size [bytes/block]")))
