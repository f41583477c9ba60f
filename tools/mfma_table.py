#!/usr/bin/env python3
"""Per-kernel MFMA utilisation and HBM traffic from tools/pmc_mfma.sh passes.

MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x cycles), cycles = GRBM_GUI_ACTIVE / 8
(rocprofv3 sums GRBM over the 8 XCDs; MI355X_MICROARCH.md 'DVFS give-back').  Reads =
2 x FETCH_SIZE (gfx950 calibration, profiles/r02_fetch_calibration.md), writes = WRITE_SIZE
(both KiB in rocprofv3).  Duration: the kernel-trace of the same passes (serialised under PMC).
Rows are split by launch shape (grid threads, dynamic + static LDS bytes): one kernel serves
several linears of different sizes.
usage: python tools/mfma_table.py gpurun_out/pmc_<tag>"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
cnt = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(f)):
        k = (r["Kernel_Name"].split("(")[0], int(r["Grid_Size"]), int(r["LDS_Block_Size"]))
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = k
    for did, cs in per.items():
        for c, v in cs.items():
            cnt[names[did]][c].append(v)
for f in glob.glob(os.path.join(d, "p*", "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        k = (r["Kernel_Name"].split("(")[0],
             int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]), int(r["LDS_Block_Size"]))
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
mean = lambda v: sum(v) / len(v) if v else float("nan")  # noqa: E731
print("| kernel | grid threads | LDS B | dispatches | MFMA instr (F32) | MFMA busy cycles | cycles (GRBM/8) | MFMA busy | HBM read MB | HBM write MB | us (traced, PMC-serialised) |")
print("|---|---|---|---|---|---|---|---|---|---|---|")
for k in sorted(cnt):
    c = cnt[k]
    if "SQ_VALU_MFMA_BUSY_CYCLES" not in c:
        continue
    busy = mean(c["SQ_VALU_MFMA_BUSY_CYCLES"])
    cyc = mean(c.get("GRBM_GUI_ACTIVE", [])) / 8
    util = busy / (1024 * cyc) if cyc else float("nan")
    rd = 2 * mean(c.get("FETCH_SIZE", [])) * 1024 / 1e6
    wr = mean(c.get("WRITE_SIZE", [])) * 1024 / 1e6
    print(f"| `{k[0]}` | {k[1]} | {k[2]} | {len(c['SQ_VALU_MFMA_BUSY_CYCLES'])} | {mean(c.get('SQ_INSTS_VALU_MFMA_F32', [])):.4g} | "
          f"{busy:.4g} | {cyc:.4g} | {100 * util:.1f} % | {rd:.1f} | {wr:.1f} | {mean(dur.get(k, [])):.1f} |")
