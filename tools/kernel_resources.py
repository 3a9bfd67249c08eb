#!/usr/bin/env python3
"""Dump per-kernel VGPR/SGPR/LDS/scratch/occupancy of csrc/kernels/*.hip for gfx950
(hipcc -Rpass-analysis=kernel-resource-usage) as a table."""

import glob
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    rows = []
    for src in sorted(glob.glob(os.path.join(REPO, "csrc", "kernels", "*.hip"))):
        r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", src, "-o",
                            os.devnull, f"-I{os.path.join(REPO, 'csrc', 'kernels')}",
                            "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
        cur = None
        for line in r.stderr.splitlines():
            m = re.search(r"remark: (?:\s*)(Function Name|VGPRs|AGPRs|TotalSGPRs|ScratchSize \[bytes/lane\]|"
                          r"Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (.*?) \[", line)
            if not m:
                continue
            k, v = m.group(1), m.group(2).strip()
            if k == "Function Name":
                cur = {"kernel": v, "file": os.path.basename(src)}
                rows.append(cur)
            elif cur is not None:
                cur[k] = v
    demangle = subprocess.run(["c++filt"], input="\n".join(r["kernel"] for r in rows), capture_output=True,
                              text=True).stdout.splitlines()
    print(f"{'kernel':90s} {'VGPR':>5s} {'AGPR':>5s} {'SGPR':>5s} {'LDS':>6s} {'scratch':>7s} {'waves/SIMD':>10s}")
    for r, name in zip(rows, demangle):
        name = re.sub(r"\(.*", "", name.replace("ddl::(anonymous namespace)::", "").replace("void ", ""))
        print(f"{name[:90]:90s} {r.get('VGPRs', ''):>5s} {r.get('AGPRs', ''):>5s} {r.get('TotalSGPRs', ''):>5s} "
              f"{r.get('LDS Size [bytes/block]', ''):>6s} {r.get('ScratchSize [bytes/lane]', ''):>7s} "
              f"{r.get('Occupancy [waves/SIMD]', ''):>10s}")


if __name__ == "__main__":
    sys.exit(main())
