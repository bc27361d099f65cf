"""Register, spill and occupancy summary of the engine's kernels (hipcc -Rpass-analysis=kernel-resource-usage),
for a quick check before a GPU run (a VGPR-indexed per-source load once cost k_sim_sparse 126 VGPR
spills).  usage: kernel_resources.py [KERNELS.hip] [extra hipcc flags...]"""
import re
import subprocess
import sys
from pathlib import Path

src = sys.argv[1] if len(sys.argv) > 1 else str(Path(__file__).resolve().parents[1] / "testground_amd/csrc/tgsim_kernels.hip")
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-mllvm",
       "-amdgpu-use-amdgpu-trackers=1", "-mllvm", "-disable-promote-alloca-to-lds", "-Rpass-analysis=kernel-resource-usage", "-c", src, "-o", "/dev/null",
       *sys.argv[2:]]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?):\s+(.*?)\s+\[-Rpass", line)
    if not m:
        continue
    k, v = m.groups()
    if k == "Function Name":
        cur = {"name": re.sub(r"^_ZN5tgsim\d+", "", v)[:40]}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
keys = ["VGPRs", "AGPRs", "SGPRs Spill", "VGPRs Spill", "Occupancy [waves/SIMD]", "LDS Size [bytes/block]"]
print(f"{'kernel':42s}" + "".join(f"{k.split(' [')[0]:>12s}" for k in keys))
for r in rows:
    if r["name"].startswith("k_") or "k_" in r["name"][:8]:
        print(f"{r['name']:42s}" + "".join(f"{r.get(k, '-'):>12s}" for k in keys))
