#!/usr/bin/env python3
"""Per-kernel register / LDS / occupancy table of one HIP source, from the
compiler's kernel-resource-usage remarks (device-only compile for gfx950).

usage: tools/resusage.py go-dsp_amd/csrc/fft_kernels.hip [name-regex] [-D...]
"""
import re
import subprocess
import sys
import os

src = sys.argv[1]
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("-") else None
defs = [a for a in sys.argv[2:] if a.startswith("-D")]
inc = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "include")
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I" + inc,
       "--cuda-device-only", "-c", src, "-o", "/dev/null",
       "-Rpass-analysis=kernel-resource-usage"] + defs + os.environ.get("RESUSAGE_FLAGS", "").split()
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", line)
    if not m:
        continue
    body = m.group(1)
    if body.startswith("Function Name:"):
        name = body.split(":", 1)[1].strip()
        dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        cur = {"name": dem}
        rows.append(cur)
    elif cur is not None and ":" in body:
        k, v = body.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    if pat and not pat.search(r["name"]):
        continue
    print("%-90s vgpr=%-4s agpr=%-3s spill=%-3s lds=%-6s occ=%s" % (
        r["name"][:90], r.get("VGPRs"), r.get("AGPRs"), r.get("VGPRs Spill"),
        r.get("LDS Size [bytes/block]"), r.get("Occupancy [waves/SIMD]")))
