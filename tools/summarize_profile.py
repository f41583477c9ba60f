#!/usr/bin/env python3
"""Turn a tools/profile_round.sh output dir into the committed evidence under profiles/.

  python tools/summarize_profile.py gpurun_out/r01a r01a [workload-key]

writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<tag>_summary.md         top kernels per step + bench line + PMC traffic table
  profiles/pmc_traffic.json         per-kernel mean FETCH_SIZE / WRITE_SIZE bytes per launch, under
                                    the bench workload key (bench.workload_key; default: config 2)

Counter units: rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KiB.  gfx950 calibration
(profiles/r02_fetch_calibration.md, tools/proto/fetch_calib.hip): reading 1 GiB once reports
FETCH_SIZE = 0.5 GiB at every load width (4, 8, 12, 16 B per lane); writing 1 GiB reports
WRITE_SIZE = 1.0 GiB.  pmc_traffic.json keeps the raw counters; the tables below and bench.py
report HBM read bytes = 2 x FETCH_SIZE.
"""
import csv
import collections
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


DEFAULT_WK = "egnn_b32_n1024_e4096_L4_lmax4_float32"


def _last_json(path):
    """the last JSON line of a file (the bench line), or None"""
    if not os.path.exists(path):
        return None
    for line in reversed(open(path).read().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    return None


def _timed_region_launches(path, kernel, n):
    """durations (ns) of the last ``n`` launches of ``kernel`` in a rocprofv3 kernel trace: the
    launches of bench.py's timed region (its warm-up launches come first)"""
    if not n or not os.path.exists(path):
        return None
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(path))
         if r["Kernel_Name"].split("(")[0] == kernel]
    return d[-n:] if len(d) >= n else None


def _stats_avg(rows, kernel):
    hit = [r for r in rows if r["Name"].split("(")[0] == kernel]
    return float(hit[0]["AverageNs"]) if hit else float("nan")


def main(src, tag, wk=DEFAULT_WK):
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    bench = open(os.path.join(src, "bench.json")).read().strip().splitlines()[-1]
    b = json.loads(bench)
    tb = _last_json(os.path.join(src, "trace.json"))
    steps_traced = (tb["steps"] + tb["warmup"]) if tb else 7
    rk = b["roofline"]["kernel"].split()[0]
    timed = _timed_region_launches(os.path.join(src, "trace", "run_kernel_trace.csv"), rk,
                                   tb["roofline"]["launches"] if tb else None)
    byts = b["roofline"]["bytes_per_launch"]
    lines = [f"# Profile {tag}", "",
             f"Command: `rocprofv3 --kernel-trace --stats -- python3 bench.py --gpus 1 --steps "
             f"{tb['steps'] if tb else 5} --warmup {tb['warmup'] if tb else 2} --no-cpu-baseline` "
             f"({steps_traced} traced steps); bench line from `python3 bench.py --steps "
             f"{b['steps']} --warmup {b['warmup']}` on the same box.", "",
             f"bench: **{b['value']} {b['unit']}**, {b['ms_per_step']} ms/step; roofline kernel "
             f"{b['roofline']['kernel']}: {b['roofline']['mean_ms']} ms/launch (HIP events), "
             f"{b['roofline']['achieved']} GB/s = {b['roofline']['frac']*100:.1f}% of 8 TB/s", ""]
    if tb and timed:
        tr_ms = sum(timed) / len(timed) / 1e6
        ev_ms = tb["roofline"]["mean_ms"]
        lines += ["## Roofline kernel: HIP events vs the kernel trace", "",
                  f"| measure | {rk} ms/launch | frac of 8 TB/s ({byts:,} B/launch) |", "|---|---|---|",
                  f"| traced run, trace timestamps, the {len(timed)} timed-region launches | "
                  f"{tr_ms:.4f} | {byts / (tr_ms * 1e-3) / 8e12:.4f} |",
                  f"| traced run, HIP events of the same launches (bench line of the traced process: "
                  f"{tb['value']} {tb['unit']}) | {ev_ms:.4f} | {tb['roofline']['frac']:.4f} |",
                  f"| untraced run, HIP events (bench line above) | {b['roofline']['mean_ms']:.4f} | "
                  f"{b['roofline']['frac']:.4f} |",
                  f"| traced run, rocprofv3 --stats average (all launches incl. warm-up) | "
                  f"{_stats_avg(rows, rk) / 1e6:.4f} | {byts / (_stats_avg(rows, rk) * 1e-9) / 8e12:.4f} |", ""]
    lines += [f"kernel time traced: {tot/1e6:.1f} ms = {tot/1e6/steps_traced:.2f} ms/step", "",
             "| % | calls/step | avg us | kernel |", "|---|---|---|---|"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
        lines.append(f"| {float(r['TotalDurationNs'])/tot*100:.1f} | {int(r['Calls'])/steps_traced:.1f} | "
                     f"{float(r['AverageNs'])/1e3:.1f} | `{r['Name'][:80]}` |")
    traffic = collections.defaultdict(dict)
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        p = os.path.join(src, f"pmc_{c}", "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        d = collections.defaultdict(list)
        for r in csv.DictReader(open(p)):
            d[(r["Kernel_Name"].split("(")[0], r["Grid_Size"])].append(float(r["Counter_Value"]) * 1024)
        for (k, g), v in d.items():
            traffic[f"{k}|{g}"][c] = sum(v) / len(v)
    lines += ["", "## HBM traffic per launch (PMC, separate FETCH_SIZE / WRITE_SIZE passes, KiB x 1024; "
              "reads = 2 x FETCH_SIZE, gfx950 calibration)", "",
              "| kernel | grid | FETCH_SIZE MB (raw) | HBM read MB | WRITE MB |", "|---|---|---|---|---|"]
    for key in sorted(traffic, key=lambda k: -sum(traffic[k].values()))[:20]:
        k, g = key.split("|")
        t = traffic[key]
        lines.append(f"| `{k[:60]}` | {g} | {t.get('FETCH_SIZE', 0)/1e6:.1f} | {2 * t.get('FETCH_SIZE', 0)/1e6:.1f} | "
                     f"{t.get('WRITE_SIZE', 0)/1e6:.1f} |")
    open(os.path.join(prof, f"{tag}_summary.md"), "w").write("\n".join(lines) + "\n")
    path = os.path.join(prof, "pmc_traffic.json")
    tab = json.load(open(path)) if os.path.exists(path) else {"unit": "bytes per launch", "workloads": {}}
    if traffic:
        tab["workloads"][wk] = {"source": tag, "kernels": traffic}
        json.dump(tab, open(path, "w"), indent=1, sort_keys=True)
    print("\n".join(lines[:40]))


if __name__ == "__main__":
    main(*sys.argv[1:4])
