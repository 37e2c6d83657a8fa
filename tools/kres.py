#!/usr/bin/env python3
"""Compact per-kernel resource table of one HIP source (VGPRs / AGPRs / spills / occupancy), from
hipcc's kernel-resource-usage remarks.  Usage: tools/kres.py SRC [extra hipcc flags...]"""
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dct_amd import _build  # noqa: E402

src = sys.argv[1]
flags = _build._flags() + _build.FILE_FLAGS.get(os.path.basename(src), []) + sys.argv[2:]
cmd = [os.path.join(_build.ROCM, "bin", "hipcc")] + flags + ["-x", "hip", "-c", src, "--offload-device-only",
                                                            "-Rpass-analysis=kernel-resource-usage", "-o", "/dev/null"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    print(f"{r.get('VGPRs','?'):>4} agpr {r.get('AGPRs','?'):>3} sspill {r.get('SGPRs Spill','?'):>3} "
          f"vspill {r.get('VGPRs Spill','?'):>3} occ {r.get('Occupancy [waves/SIMD]','?')}  {r['name'][:110]}")
