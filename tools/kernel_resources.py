"""Per-kernel register / LDS / occupancy table from the compiler's own report.

Compiles each difacto_amd/csrc/*.hip for gfx950 (device only, the Makefile's flags) with
-Rpass-analysis=kernel-resource-usage and prints one markdown row per kernel instantiation:
VGPRs, AGPRs, spilled VGPRs, scratch bytes per lane, static LDS bytes and waves per SIMD.
Usage: python3 tools/kernel_resources.py [regex] > profiles/<round>/kernel_resources.md
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pat = re.compile(sys.argv[1]) if len(sys.argv) > 1 else None
FIELDS = ("VGPRs", "AGPRs", "VGPRs Spill", "ScratchSize [bytes/lane]", "LDS Size [bytes/block]",
          "Occupancy [waves/SIMD]")


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names),
                         capture_output=True, text=True, check=True).stdout.splitlines()
    return out


rows = []
with tempfile.TemporaryDirectory() as td:
    for src in sorted(glob.glob(os.path.join(ROOT, "difacto_amd/csrc/*.hip"))):
        r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC",
                            "-std=c++17", "-ffp-contract=off", "--cuda-device-only", "-c", src,
                            "-o", os.path.join(td, "k.o"),
                            "-Rpass-analysis=kernel-resource-usage"],
                           capture_output=True, text=True)
        cur = None
        for line in r.stderr.splitlines():
            m = re.search(r"remark:\s+Function Name: (\S+)", line)
            if m:
                cur = {"name": m.group(1), "file": os.path.basename(src)}
                rows.append(cur)
                continue
            m = re.search(r"remark:\s+([^:]+): (\S+) \[-Rpass", line)
            if m and cur is not None and m.group(1).strip() in FIELDS:
                cur[m.group(1).strip()] = m.group(2)
names = demangle([r["name"] for r in rows])
print("| kernel | file | VGPRs | AGPRs | VGPR spills | scratch B/lane | LDS B/block | waves/SIMD |")
print("|---|---|---|---|---|---|---|---|")
for r, n in zip(rows, names):
    n = n.split("(")[0].replace("dfx::", "")
    if not n.startswith(("k_", "void k_")):
        continue
    n = n.replace("void ", "")
    if pat and not pat.search(n):
        continue
    print("| %s | %s | %s |" % (n, r["file"], " | ".join(r.get(f, "") for f in FIELDS)))
