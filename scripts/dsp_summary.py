"""Summarise scripts/pmc_dsp.sh (mel2wav back end) into profiles/:
  <round>_mel2wav_kernel_stats.csv   rocprofv3 --stats summary
  <round>_mel2wav_summary.md         per-kernel durations, HBM bytes / launch, LDS counters
  traffic.json["mel2wav"]            HBM bytes per launch (bench.py's roofline.traffic)
HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes), MI355X_MICROARCH.md HBM section."""
import argparse
import csv
import glob
import json
import os
import shutil
import statistics
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(pattern):
    f = glob.glob(pattern, recursive=True)
    if not f:
        raise SystemExit(f"missing {pattern}")
    return f[0]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--round", default="r01")
    a = ap.parse_args()
    prof = os.path.join(ROOT, "profiles")
    shutil.copy(one(f"{a.dir}/trace/**/run_kernel_stats.csv"), os.path.join(prof, f"{a.round}_mel2wav_kernel_stats.csv"))
    dur = defaultdict(list)
    for r in csv.DictReader(open(one(f"{a.dir}/trace/**/run_kernel_trace.csv"))):
        if "dsp_" in r["Kernel_Name"]:
            dur[r["Kernel_Name"].split("(")[0].replace("avc::", "").replace("void ", "").split("<")[0]].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    ctr = defaultdict(lambda: defaultdict(list))
    for i in (1, 2, 3):
        per = defaultdict(dict)
        name = {}
        for r in csv.DictReader(open(one(f"{a.dir}/pmc_{i}/**/run_counter_collection.csv"))):
            d = r["Dispatch_Id"]
            per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            name[d] = r["Kernel_Name"].split("(")[0].replace("avc::", "").replace("void ", "").split("<")[0]
        for d, cs in per.items():
            if "dsp_" in name[d]:
                for c, v in cs.items():
                    ctr[name[d]][c].append(v)
    traffic = {}
    import re
    tl = a.dir.rstrip("/") + ".trace.log"
    m = re.search(r"src=([0-9a-f]{16})", open(tl).read()) if os.path.exists(tl) else None
    lines = [f"# rocprofv3 summary {a.round}: mel2wav back end (B=256 mels 80x128, 100 Griffin-Lim iterations)", "",
             f"libavc src={m.group(1) if m else 'unknown'}.", "",
             "Source: `scripts/pmc_dsp.sh` on one MI355X: `python3 bench.py --attack mel2wav --steps 1 --warmup 0` under "
             "`rocprofv3 --kernel-trace --stats`, plus one run per PMC pass.  HBM = 2*FETCH_SIZE + WRITE_SIZE.", "",
             "| kernel | launches | median us | HBM MB/launch | HBM GB/s | LDS insts/launch | LDS bank confl / LDS active |",
             "|---|---|---|---|---|---|---|"]
    for k, ds in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        c = ctr.get(k, {})
        med = statistics.median(ds)
        hbm = None
        if c.get("FETCH_SIZE") and c.get("WRITE_SIZE"):
            hbm = (2 * statistics.median(c["FETCH_SIZE"]) + statistics.median(c["WRITE_SIZE"])) * 1024
            traffic[k] = int(hbm)
        lds = statistics.median(c["SQ_INSTS_LDS"]) if c.get("SQ_INSTS_LDS") else None
        conf = (statistics.median(c["SQ_LDS_BANK_CONFLICT"]) / max(1.0, statistics.median(c["SQ_ACTIVE_INST_LDS"]))
                if c.get("SQ_LDS_BANK_CONFLICT") and c.get("SQ_ACTIVE_INST_LDS") else None)
        lines.append(f"| {k} | {len(ds)} | {med:.1f} | {hbm / 1e6 if hbm else float('nan'):.2f} | "
                     f"{hbm / (med * 1e-6) / 1e9 if hbm else float('nan'):.0f} | {lds if lds is not None else '-'} | "
                     f"{conf if conf is not None else float('nan'):.3f} |")
    open(os.path.join(prof, f"{a.round}_mel2wav_summary.md"), "w").write("\n".join(lines) + "\n")
    tp = os.path.join(prof, "traffic.json")
    t = json.load(open(tp)) if os.path.exists(tp) else {}
    t["mel2wav"] = traffic
    json.dump(t, open(tp, "w"), indent=1, sort_keys=True)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
