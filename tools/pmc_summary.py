#!/usr/bin/env python3
"""Per-kernel summary of ``rocprofv3 --pmc ... --kernel-trace --output-format csv`` passes.

    python tools/pmc_summary.py OUT.json DIR [DIR ...]

Each DIR is one counter pass (rocprofv3 collects at most a few counters per block per run, so
FETCH_SIZE / WRITE_SIZE / SQ_* come from separate runs of the same program). For every kernel
name it reports the mean counter value per dispatch, the resources from the dispatch records
(VGPRs, LDS bytes, grid, workgroup size) and the mean kernel duration from the kernel trace.
Derived fields where the counters are present:

* ``hbm_GBps``: (FETCH_SIZE + WRITE_SIZE) KB per dispatch over the mean duration;
* ``waves_per_dispatch`` (SQ_WAVES) and ``occupancy_waves_per_simd``: the waves per SIMD the
  kernel's VGPR/AGPR and LDS allocation allow on gfx950;
* ``valu_per_vmem``: SQ_INSTS_VALU / SQ_INSTS_VMEM_RD (arithmetic intensity in instructions).
"""

from __future__ import annotations

import collections
import csv
import glob
import json
import os
import sys


def _short(name: str) -> str:
    name = name.strip('"')
    if name.startswith("void "):
        name = name[5:]
    for prefix in ("ddl::(anonymous namespace)::", "ddl::"):
        if name.startswith(prefix):
            name = name[len(prefix):]
    return name[:90]


def theoretical_occupancy(e: dict) -> int | None:
    """Waves per SIMD the kernel's resources allow on gfx950 (MI355X_MICROARCH "Register files"):
    min(8, 512 // VGPR+AGPR allocation in granules of 8), and the LDS limit (160 KiB per CU shared
    by the resident workgroups, 4 SIMDs per CU)."""
    regs = e.get("vgpr", 0) + e.get("agpr", 0)
    if not regs or not e.get("workgroup"):
        return None
    alloc = -(-int(regs) // 8) * 8
    waves = min(8, 512 // alloc)
    lds = int(e.get("lds_bytes", 0))
    if lds > 0:
        wgs_per_cu = 163840 // lds
        waves_per_wg = -(-int(e["workgroup"]) // 64)
        waves = min(waves, max(1, wgs_per_cu * waves_per_wg // 4))
    return waves


def load(dirs: list[str]) -> dict:
    counters: dict = collections.defaultdict(lambda: collections.defaultdict(list))
    res: dict = {}
    dur: dict = collections.defaultdict(list)
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    k = _short(row.get("Kernel_Name", "?"))
                    counters[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
                    res[k] = {"vgpr": float(row.get("VGPR_Count") or row.get("Arch_VGPR_Count") or 0),
                              "agpr": float(row.get("Accum_VGPR_Count") or 0),
                              "sgpr": float(row.get("SGPR_Count") or 0),
                              "lds_bytes": float(row.get("LDS_Block_Size") or row.get("Lds_Size") or 0),
                              "grid_threads": float(row.get("Grid_Size") or 0),
                              "workgroup": float(row.get("Workgroup_Size") or 0)}
        for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    try:
                        dur[_short(row["Kernel_Name"])].append(
                            (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-3)
                    except (KeyError, ValueError):
                        pass
    out = {}
    for k, cs in counters.items():
        e = {c: round(sum(v) / len(v), 1) for c, v in cs.items()}
        e.update(res.get(k, {}))
        if dur.get(k):
            e["mean_us"] = round(sum(dur[k]) / len(dur[k]), 2)
            e["dispatches"] = len(dur[k])
        if "FETCH_SIZE" in e and "WRITE_SIZE" in e and e.get("mean_us"):
            e["hbm_GBps"] = round((e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024 / (e["mean_us"] * 1e-6) / 1e9, 1)
        if "SQ_WAVES" in e:
            e["waves_per_dispatch"] = e["SQ_WAVES"]
        occ = theoretical_occupancy(e)
        if occ is not None:
            e["occupancy_waves_per_simd"] = occ
        if e.get("SQ_INSTS_VMEM_RD"):
            e["valu_per_vmem"] = round(e.get("SQ_INSTS_VALU", 0) / e["SQ_INSTS_VMEM_RD"], 2)
        out[k] = e
    return out


def main() -> int:
    if len(sys.argv) < 3:
        print(__doc__)
        return 2
    summary = load(sys.argv[2:])
    with open(sys.argv[1], "w") as f:
        json.dump(summary, f, indent=1)
    for k, e in sorted(summary.items()):
        print(json.dumps({"kernel": k, **{x: e[x] for x in ("mean_us", "hbm_GBps", "vgpr", "lds_bytes",
                                                               "waves_per_dispatch", "occupancy_waves_per_simd",
                                                               "valu_per_vmem") if x in e}}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
