"""Per-kernel registers / spills / LDS / occupancy from hipcc's resource-usage remarks.

    python tools/resource_usage.py csrc/sgmm_frontier.hip [extra hipcc flags]
(paths relative to the package directory)"""
import re
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent.parent / "deep-reinforcement-learning-based-signal-gated-market-making_amd"
src, extra = sys.argv[1], sys.argv[2:]
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "--offload-arch=gfx950", *extra,
       "-c", "-o", "/tmp/ru.o", src, "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, cwd=PKG, capture_output=True, text=True).stderr
rows, cur = {}, None
for line in out.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = t.split(":", 1)[1].strip()
        rows[cur] = {}
    elif cur and ":" in t:
        k, v = t.split(":", 1)
        rows[cur][k.strip()] = v.strip()
for k, r in rows.items():
    g = r.get
    print(f"{k[:64]:64s} VGPR {g('VGPRs', '?'):>4} AGPR {g('AGPRs', '?'):>3} vspill {g('VGPRs Spill', '?'):>3} "
          f"sspill {g('SGPRs Spill', '?'):>4} LDS {g('LDS Size [bytes/block]', '?'):>6} occ {g('Occupancy [waves/SIMD]', '?')}")
