"""Summarise a scripts/pmc_fused.sh run (rocprofv3 kernel trace + PMC passes of avc_bench)
into a per-kernel table: duration (trace), HBM bytes, MFMA utilisation, wave-state split,
LDS bank conflicts, effective clock.

  python scripts/fz_summary.py gpurun_out/fz_p1_a0 [--out profiles/r02_emb_bf16] [--warm N]

MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): busy MFMA
cycles summed over every SIMD of the chip over the SIMD-cycles the dispatch lasted
(GRBM_GUI_ACTIVE is summed over the 8 XCDs: MI355X_MICROARCH.md 'DVFS give-back').  It is
in [0, 1] by construction and independent of the clock.  HBM bytes = 2 x FETCH_SIZE +
WRITE_SIZE (KiB; gfx950 FETCH_SIZE counts half of wide reads, MI355X_MICROARCH.md).
The first --warm dispatches of every kernel (graph capture, cold caches) are skipped.
Round 6: for a short kernel GRBM_GUI_ACTIVE spans more than the dispatch (the counter window's
set-up and drain), which gave "clocks" above the 2.4 GHz maximum; the SIMD-cycles of a dispatch are
therefore min(GRBM_GUI_ACTIVE / 8, trace duration x 2.4 GHz) -- capped rows are marked with * and
their MFMA util is the trace-duration figure (a lower bound if the clock ran below 2.4 GHz).
"""
import argparse
import csv
import glob
import json
import os
import shutil
import statistics
from collections import defaultdict

SIMDS = 1024
CLK_MAX = 2.4     # GHz, MI355X peak engine clock (MI355X_MICROARCH.md)


def short(name):
    n = name.split("(")[0]
    for a, b in (("avc::", ""), ("void ", ""), ("PREC_", "")):
        n = n.replace(a, b)
    return n


def libname(k):
    """rocprof kernel name -> the name libavc's HIP-event profile reports (bench.py keys)."""
    if "<" not in k:
        return k
    base, args = k.split("<", 1)
    first = args.rstrip(">").split(",")[0].strip()
    if first in ("0", "1") and base not in ("se_head_v",):
        return f"{base}<{'bf16' if first == '1' else 'f32'}>"
    return k


def load_counters(d, warm):
    per = defaultdict(lambda: defaultdict(list))     # kernel -> counter -> [values per dispatch]
    for f in sorted(glob.glob(os.path.join(d, "pmc_*", "**", "*counter_collection.csv"), recursive=True)):
        rows = list(csv.DictReader(open(f)))
        seen = defaultdict(int)
        disp = {}
        for r in rows:
            k = short(r["Kernel_Name"])
            key = (r["Dispatch_Id"], k)
            if key not in disp:
                disp[key] = seen[k]
                seen[k] += 1
            if disp[key] < warm:
                continue
            per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return per


def load_trace(d, warm):
    dur = defaultdict(list)
    for f in glob.glob(os.path.join(d, "trace", "**", "*kernel_trace.csv"), recursive=True):
        n = defaultdict(int)
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            n[k] += 1
            if n[k] > warm:
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)   # us
    return dur


def src_hash(d):
    """libavc source hash of the profiled binary (avc_bench logs avc_version() to stderr; the
    trace pass's log sits next to the profile directory as <dir>.trace.log)."""
    import re
    for f in (d.rstrip("/") + ".trace.log",):
        if os.path.exists(f):
            m = re.search(r"libavc [^;\n]*src=([0-9a-f]{16})", open(f).read())
            if m:
                return m.group(1)
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out", default=None, help="prefix for <out>_summary.md / _counters.json / _kernel_stats.csv")
    ap.add_argument("--warm", type=int, default=2)
    ap.add_argument("--pmc-json", default=None, help="merge per-kernel traffic / mfma_util into this file "
                                                      "under --key (read by bench.py)")
    ap.add_argument("--key", default=None, help="e.g. emb, emb_fp32, e2e, fb")
    ap.add_argument("--iters-per-launch", type=int, default=None,
                    help="attack iterations per dispatch of the persistent kernel (se_attack_fused): recorded "
                         "with its row so bench.py reports its traffic per iteration")
    a = ap.parse_args()
    src = src_hash(a.dir)
    per = load_counters(a.dir, a.warm)
    dur = load_trace(a.dir, a.warm)
    rows = []
    out_json = {}
    for k in sorted(dur, key=lambda k: -sum(dur[k])):
        if k.startswith("__amd"):
            continue
        c = {n: statistics.mean(v) for n, v in per.get(k, {}).items() if v}
        us = statistics.median(dur[k])
        gui = c.get("GRBM_GUI_ACTIVE")
        cyc = gui / 8 if gui else None
        capped = cyc is not None and cyc > us * 1e3 * CLK_MAX
        if capped:
            cyc = us * 1e3 * CLK_MAX
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES")
        util = busy / (SIMDS * cyc) if busy is not None and cyc else None
        hbm = None
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            hbm = (2 * c["FETCH_SIZE"] + c["WRITE_SIZE"]) * 1024
        wc = c.get("SQ_WAVE_CYCLES")
        split = {n: c[n] / wc for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY") if wc and n in c}
        lds_conf = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_ACTIVE_INST_LDS"] if c.get("SQ_ACTIVE_INST_LDS") else None
        clk = cyc / (us * 1e3) if cyc else None      # GHz (cycles per ns)
        mf_per = c["SQ_VALU_MFMA_BUSY_CYCLES"] / c["SQ_INSTS_MFMA"] if c.get("SQ_INSTS_MFMA") and busy else None
        d = {"launches": len(dur[k]) + a.warm, "median_us": round(us, 2), "mfma_util": util, "hbm_bytes": hbm,
             "hbm_GBps": hbm / (us * 1e3) if hbm else None, "clock_GHz": clk, "wave_state": split,
             "lds_conflict_cycles_per_lds_cycle": lds_conf, "mfma_busy_per_inst": mf_per, "counters": c,
             "cycles_capped_to_trace": capped}
        out_json[k] = d
        rows.append((k, d))
    lines = ["| kernel | median µs | MFMA util | HBM MB | HBM GB/s | clock GHz | wait / inst-stall / active | LDS conflict |",
             "|---|---|---|---|---|---|---|---|"]
    f = lambda v, p=3: "—" if v is None else f"{v:.{p}f}"
    for k, d in rows:
        ws = d["wave_state"]
        wsf = " / ".join(f(ws.get(n), 2) for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"))
        lines.append(f"| {k} | {d['median_us']} | {f(d['mfma_util'])} | "
                     f"{f(d['hbm_bytes'] / 1e6 if d['hbm_bytes'] else None, 1)} | {f(d['hbm_GBps'], 0)} | "
                     f"{f(d['clock_GHz'], 2)}{'*' if d['cycles_capped_to_trace'] else ''} | {wsf} | {f(d['lds_conflict_cycles_per_lds_cycle'])} |")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out + "_summary.md", "w") as fh:
            fh.write(f"# {os.path.basename(a.out)}\n\nlibavc src={src}.  Source: `{a.dir}` (rocprofv3 kernel trace + PMC passes of "
                     f"avc_bench; first {a.warm} dispatches per kernel skipped).  MFMA util = "
                     "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x min(GRBM_GUI_ACTIVE/8, trace duration x 2.4 GHz)); * = the "
                     "counter window outlasted the dispatch, cycles taken from the trace duration.  HBM = 2 x FETCH_SIZE + "
                     "WRITE_SIZE.  Wave state = fractions of SQ_WAVE_CYCLES." +
                     (f"  `se_attack_fused` (the persistent emb attack) runs {a.iters_per_launch} iterations per "
                      "dispatch: divide its duration and HBM bytes by that for one iteration."
                      if a.iters_per_launch else "") + "\n\n" + txt + "\n")
        json.dump(out_json, open(a.out + "_counters.json", "w"), indent=1)
        st = glob.glob(os.path.join(a.dir, "trace", "**", "*kernel_stats.csv"), recursive=True)
        if st:
            shutil.copy(st[0], a.out + "_kernel_stats.csv")
    if a.pmc_json and a.key:
        db = json.load(open(a.pmc_json)) if os.path.exists(a.pmc_json) else {}
        db[a.key] = {libname(k): {"traffic": d["hbm_bytes"], "mfma_util": d["mfma_util"], "median_us": d["median_us"],
                                  "source": (a.out or a.dir) + "_summary.md", "src": src,
                                  **({"iters_per_launch": a.iters_per_launch}
                                     if a.iters_per_launch and k.startswith("se_attack_fused") else {})}
                     for k, d in rows}
        json.dump(db, open(a.pmc_json, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
