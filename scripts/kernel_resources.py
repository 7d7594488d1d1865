"""Per-kernel VGPR / scratch / occupancy / LDS of kernels.hip (hipcc
-Rpass-analysis=kernel-resource-usage), as a table.  CPU only."""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
flags = ["-O3", "-std=c++17", "-fno-slp-vectorize", "-DMW_FAST_MATH", "-ffinite-math-only", "-fno-signed-zeros",
         *os.environ.get("EXTRA", "").split()]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", *flags, f"-I{ROOT}/include",
       f"-I{ROOT}/gym-ignition_amd/csrc", "-c", f"{ROOT}/gym-ignition_amd/csrc/kernels.hip",
       "-o", "/tmp/_kr.o", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for key in ("VGPRs", "ScratchSize [bytes/lane]", "Occupancy [waves/SIMD]", "SGPRs Spill", "VGPRs Spill",
                "LDS Size [bytes/block]"):
        m = re.search(re.escape(key) + r": (\d+)", line)
        if m and cur is not None:
            cur[key] = int(m.group(1))
bad = 0
for r in rows:
    name = re.sub(r"^_ZN2mw3dev\d+", "", r["name"])[:60]
    print(f"{name:62s} vgpr={r.get('VGPRs'):4} scratch={r.get('ScratchSize [bytes/lane]'):4} "
          f"occ={r.get('Occupancy [waves/SIMD]')} sgpr_spill={r.get('SGPRs Spill')} vgpr_spill={r.get('VGPRs Spill')} "
          f"lds={r.get('LDS Size [bytes/block]')}")
    bad += (r.get("ScratchSize [bytes/lane]", 0) > 0)
sys.exit(1 if bad else 0)
