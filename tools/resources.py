#!/usr/bin/env python3
"""Per-kernel register / scratch / occupancy table of the HIP library
(hipcc -Rpass-analysis=kernel-resource-usage).  usage: resources.py [FILTER]
[-- extra hipcc flags]"""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/tools/", 1)[0]
args = sys.argv[1:]
extra = []
if "--" in args:
    extra = args[args.index("--") + 1:]
    args = args[:args.index("--")]
flt = args[0] if args else ""
base = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c",
        "-ffp-contract=off", "-I", f"{ROOT}/include", "-o", "/dev/null",
        "-Rpass-analysis=kernel-resource-usage"] + extra
# api.hip (non-templated kernels) and the per-NH units (templated kernels)
nhs = [int(x) for x in __import__("os").environ.get("NH", "1,2").split(",")]
cmds = [base + [f"{ROOT}/unipeak_amd/csrc/api.hip"]] + [
    base + [f"-DUPK_NH_TU={k}", f"{ROOT}/unipeak_amd/csrc/nh_tu.hip"] for k in nhs]
out = "\n".join(subprocess.run(c, capture_output=True, text=True).stderr for c in cmds)
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    if cur is None:
        continue
    for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("scratch", r"ScratchSize \[bytes/lane\]: (\d+)"),
                     ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"), ("vspill", r"VGPRs Spill: (\d+)"),
                     ("sspill", r"SGPRs Spill: (\d+)"), ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
        m = re.search(pat, line)
        if m:
            cur[key] = int(m.group(1))
for r in rows:
    n = r["name"]
    d = subprocess.run(["c++filt", n], capture_output=True, text=True).stdout.strip()
    d = re.sub(r"\(.*", "", d).replace("upk::", "")
    if flt in d:
        print(f"{d:48s} vgpr {r.get('vgpr', 0):4d} scratch {r.get('scratch', 0):4d} occ {r.get('occ', 0)} "
              f"vspill {r.get('vspill', 0):3d} sspill {r.get('sspill', 0):3d}")
