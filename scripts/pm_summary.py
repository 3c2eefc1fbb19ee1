"""Per-layer summary of a scripts/r03_pm_prof.sh run of the PredictiveModel forward (bench.py --attack pm):
the last complete forward of the kernel trace and of each PMC pass (dispatch order is deterministic), one
row per launch -- duration, HBM bytes (2 x FETCH_SIZE + WRITE_SIZE, KiB units: MI355X_MICROARCH.md), MFMA
utilisation -- and the forward's total HBM bytes, merged into profiles/traffic.json["pm"] (bench.py's
roofline.traffic, reported when the run's batch equals the profiled one).

  python scripts/pm_summary.py gpurun_out/prof_pm --out profiles/r05_pm [--batch 256]
"""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict

SIMDS = 1024


def forward_slices(names):
    """index ranges [i0, i1) of complete forwards: from one pm_cin1 launch to the next"""
    starts = [i for i, n in enumerate(names) if "pm_cin1" in n]
    return [(a, b) for a, b in zip(starts, starts[1:])]


def trace_last_forward(d):
    rows = []
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if "pm_" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    sl = forward_slices([r["Kernel_Name"] for r in rows])
    i0, i1 = sl[-1]
    return [(r["Kernel_Name"].split("(")[0].replace("void ", "").replace("avc::", ""),
             (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3,
             (int(r["Grid_Size_X"]) // 256, int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]))) for r in rows[i0:i1]]


def pmc_last_forward(d):
    disp = defaultdict(dict)
    name = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "pm_" not in r["Kernel_Name"]:
                continue
            k = int(r["Dispatch_Id"])
            disp[k][r["Counter_Name"]] = disp[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            name[k] = r["Kernel_Name"]
    ids = sorted(disp)
    sl = forward_slices([name[i] for i in ids])
    i0, i1 = sl[-1]
    return [disp[i] for i in ids[i0:i1]]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", required=True)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    tr = trace_last_forward(a.dir)
    passes = [pmc_last_forward(p) for p in sorted(glob.glob(os.path.join(a.dir, "pmc_*")))]
    per = [dict() for _ in tr]
    for ps in passes:
        if len(ps) != len(tr):
            raise SystemExit(f"PMC pass has {len(ps)} launches per forward, trace {len(tr)}")
        for i, c in enumerate(ps):
            per[i].update(c)
    src = None
    log = a.dir.rstrip("/") + ".trace.log"
    if os.path.exists(log):
        m = re.search(r'"libavc": "[^"]*src=([0-9a-f]{16})', open(log).read())
        src = m.group(1) if m else None
    lines = ["| # | kernel | grid | µs | HBM MB | HBM GB/s | MFMA util |", "|---|---|---|---|---|---|---|"]
    tot_us = tot_hbm = 0.0
    for i, ((k, us, g), c) in enumerate(zip(tr, per)):
        hbm = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024 if "FETCH_SIZE" in c and "WRITE_SIZE" in c else None
        gui = c.get("GRBM_GUI_ACTIVE")
        util = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (SIMDS * gui / 8) if gui and "SQ_VALU_MFMA_BUSY_CYCLES" in c else None
        tot_us += us
        tot_hbm += hbm or 0.0
        lines.append(f"| {i} | {k} | {g} | {us:.1f} | {hbm / 1e6 if hbm else float('nan'):.1f} | "
                     f"{hbm / (us * 1e3) if hbm else float('nan'):.0f} | {util if util is not None else float('nan'):.3f} |")
    lines.append(f"| | forward | | {tot_us:.1f} | {tot_hbm / 1e6:.1f} | {tot_hbm / (tot_us * 1e3):.0f} | |")
    txt = "\n".join(lines)
    print(txt)
    with open(a.out + "_summary.md", "w") as fh:
        fh.write(f"# {os.path.basename(a.out)}\n\nlibavc src={src}.  PredictiveModel forward, B={a.batch} windows of "
                 f"[1,80,100], fp32: the last complete forward of `{a.dir}` (kernel trace; PMC passes FETCH_SIZE, "
                 "WRITE_SIZE, MFMA busy).  HBM = 2 x FETCH_SIZE + WRITE_SIZE (KiB).  MFMA util = "
                 "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE/8).\n\n" + txt + "\n")
    tp = os.path.join(os.path.dirname(a.out) or ".", "traffic.json")
    t = json.load(open(tp)) if os.path.exists(tp) else {}
    t["pm"] = {"batch": a.batch, "forward": int(tot_hbm),
               "src": f"{os.path.basename(a.out)}_summary.md (libavc src={src})"}
    json.dump(t, open(tp, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
