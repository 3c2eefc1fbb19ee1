"""Summarise a scripts/pmc.sh run (rocprofv3 kernel trace + PMC passes of the native
driver) into profiles/:

  <round>_<prec>_kernel_stats.csv   rocprofv3 --stats summary, as written by rocprofv3
  <round>_<prec>_summary.md         per-layer table of one attack iteration (durations
                                    from the kernel trace, HBM bytes / MFMA / LDS counters
                                    from the PMC passes), per-tile-variant averages
  traffic.json                      HBM bytes per launch of each tile variant (read by
                                    bench.py for roofline.traffic)

HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes): MI355X_MICROARCH.md
("HBM" section) -- gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads.

Iteration segmentation: libavc prints its tuned plans (AVC_PRINT_PLAN=1, pmc_tune.log);
an iteration is the dispatch window around an se_head that is followed by a
backward-mode (MODE=1) conv_gemm.
"""
import argparse
import csv
import json
import os
import re
import shutil
import statistics
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANTS_H = os.path.join(ROOT, "attack-vc_amd", "csrc", "avc_gemm_variants.h")


def variant_table():
    """template args (PREC, WM, WN, WGM, WGN, KC) -> variant display name."""
    out = {}
    for m in re.finditer(r'AVC_GEMM_VARIANT\((\d+), PREC_(F32|BF16), (\d+), (\d+), (\d+), (\d+), (\d+), "([^"]+)"\)',
                         open(VARIANTS_H).read()):
        prec = 0 if m.group(2) == "F32" else 1
        out[(prec,) + tuple(int(m.group(i)) for i in range(3, 8))] = m.group(8)
    return out


def short(kname, vt):
    m = re.search(r"conv_gemm<(\d+), (\d+), (\d+), (\d+), (\d+), (\d+), (\d+), (\d+)>", kname)
    if m:
        a = tuple(int(x) for x in m.groups())
        return vt.get(a[:6], "conv_gemm?"), a[6], a[7]   # (variant, mode, stride)
    for k in ("splitk_reduce", "se_head", "attack_init"):
        if k in kname:
            return k, None, None
    return kname.split("(")[0], None, None


def load_plan(path):
    plans = defaultdict(list)
    if not os.path.exists(path):
        return plans
    for line in open(path):
        m = re.match(r"plan (\S+) (\d+) (\S+) (.+?) grid=(\S+) ksplit=(\d+) flop=(\S+)", line)
        if m:
            plans[m.group(1)].append({"layer": m.group(3), "kernel": m.group(4), "grid": m.group(5),
                                      "ksplit": int(m.group(6)), "flop": float(m.group(7))})
    return plans


def iteration_windows(seq, vt, plan):
    """seq: list of kernel names in dispatch order -> list of (lo, hi) dispatch windows."""
    roles = []
    for L in plan:
        roles.append(L["layer"])
        if L["ksplit"] > 1:
            roles.append(L["layer"] + " (reduce)")
    n = len(roles)
    head_pos = next(i for i, r in enumerate(roles) if "head" in r)
    wins = []
    for j, k in enumerate(seq):
        if "se_head" not in k or j + 1 >= len(seq):
            continue
        nxt = short(seq[j + 1], vt)
        if nxt[1] != 1:
            continue
        lo = j - head_pos
        if lo >= 0 and lo + n <= len(seq):
            wins.append((lo, lo + n))
    return wins, roles


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--prec", type=int, default=0)
    ap.add_argument("--round", default="r01")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles"))
    a = ap.parse_args()
    P = a.prec
    pname = "fp32" if P == 0 else "bf16"
    vt = variant_table()
    plans = load_plan(os.path.join(a.dir, f"pmc_tune_p{P}.log"))
    plan = plans["iter" if P == 0 else "iterbf16"]
    os.makedirs(a.out, exist_ok=True)

    stats_src = os.path.join(a.dir, f"prof_p{P}", "run_kernel_stats.csv")
    shutil.copy(stats_src, os.path.join(a.out, f"{a.round}_{pname}_kernel_stats.csv"))

    # kernel trace: durations per iteration position
    tr = sorted(csv.DictReader(open(os.path.join(a.dir, f"prof_p{P}", "run_kernel_trace.csv"))),
                key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in tr]
    wins, roles = iteration_windows(names, vt, plan)
    if not wins:
        raise SystemExit("no iteration windows found")
    dur = defaultdict(list)
    kern = {}
    for lo, hi in wins:
        for p in range(hi - lo):
            r = tr[lo + p]
            dur[p].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
            kern[p] = short(r["Kernel_Name"], vt)
    iter_span = [(int(tr[hi - 1]["End_Timestamp"]) - int(tr[lo]["Start_Timestamp"])) * 1e-3 for lo, hi in wins]

    # PMC passes: per-dispatch counters, same segmentation
    pmc = defaultdict(lambda: defaultdict(list))   # counter -> position -> values
    for i in range(1, 16):
        f = os.path.join(a.dir, f"pmc_p{P}_{i}", "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        per = defaultdict(dict)
        meta = {}
        for r in csv.DictReader(open(f)):
            d = int(r["Dispatch_Id"])
            per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            meta[d] = r["Kernel_Name"]
        ds = sorted(per)
        seq = [meta[d] for d in ds]
        w2, _ = iteration_windows(seq, vt, plan)
        for lo, hi in w2:
            for p in range(hi - lo):
                for c, v in per[ds[lo + p]].items():
                    pmc[c][p].append(v)

    def pm(c, p):
        v = pmc.get(c, {}).get(p)
        return statistics.mean(v) if v else None

    npos = len(roles)
    rows = []
    by_variant = defaultdict(lambda: {"n": 0, "us": 0.0, "bytes": 0.0, "nb": 0, "flop": 0.0})
    flop_pos = {}
    q = 0
    for L in plan:
        flop_pos[q] = L["flop"]
        q += 2 if L["ksplit"] > 1 else 1
    tot = defaultdict(float)
    for p in range(npos):
        us = statistics.median(dur[p])
        fetch, write = pm("FETCH_SIZE", p), pm("WRITE_SIZE", p)
        hbm = (2 * fetch + write) * 1024 if fetch is not None and write is not None else None
        mfma = pm("SQ_VALU_MFMA_BUSY_CYCLES", p)
        busy = pm("GRBM_GUI_ACTIVE", p)
        wait, act, wc = pm("SQ_WAIT_ANY", p), pm("SQ_ACTIVE_INST_ANY", p), pm("SQ_WAVE_CYCLES", p)
        ldsc, ldsa = pm("SQ_LDS_BANK_CONFLICT", p), pm("SQ_ACTIVE_INST_LDS", p)
        hit, miss = pm("TCC_HIT_sum", p), pm("TCC_MISS_sum", p)
        fl = flop_pos.get(p, 0.0)
        v = kern[p][0]
        rows.append((p, roles[p], v, kern[p][1], us, fl / (us * 1e-6) / 1e12 if fl else None,
                     hbm, hbm / (us * 1e-6) / 1e9 if hbm else None,
                     wait / wc if wait is not None and wc else None, act / wc if act is not None and wc else None,
                     ldsc / ldsa if ldsc is not None and ldsa else None,
                     hit / (hit + miss) if hit is not None and miss is not None and hit + miss else None))
        bv = by_variant[v]
        bv["n"] += 1
        bv["us"] += us
        bv["flop"] += fl
        if hbm is not None:
            bv["bytes"] += hbm
            bv["nb"] += 1
        tot["us"] += us
        tot["flop"] += fl
        tot["hbm"] += hbm or 0.0

    f = lambda x, fmt: (fmt % x) if x is not None else "-"
    md = [f"# rocprofv3 summary {a.round}, {pname} emb attack iteration (B=256, T=128)", "",
          "Source: `scripts/pmc.sh` (PREC=%d) on one MI355X; native driver `avc_bench 256 128 N 1 0 %d` "
          "(no Python in the profiled process); tile variants from a prior unprofiled tune run "
          "(AVC_TUNE_FILE)." % (P, P), "",
          f"Iterations in trace: {len(wins)}; median iteration span (first dispatch start -> last end): "
          f"{statistics.median(iter_span):.1f} us; sum of per-launch medians: {tot['us']:.1f} us; "
          f"algorithmic GEMM FLOP/iter {tot['flop']:.4g}; HBM bytes/iter (2*FETCH+WRITE) {tot['hbm'] / 1e6:.1f} MB.",
          "",
          "| pos | layer | kernel | mode | us | TFLOP/s | HBM MB | GB/s | wait/wave | active/wave | LDS confl/LDS | L2 hit |",
          "|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        md.append("| %d | %s | %s | %s | %.1f | %s | %s | %s | %s | %s | %s | %s |" % (
            r[0], r[1], r[2], "-" if r[3] is None else r[3], r[4], f(r[5], "%.1f"),
            f(r[6] / 1e6 if r[6] else None, "%.2f"), f(r[7], "%.0f"), f(r[8], "%.2f"), f(r[9], "%.2f"),
            f(r[10], "%.3f"), f(r[11], "%.2f")))
    md += ["", "## Per tile variant (iteration launches)", "",
           "| kernel | launches/iter | avg us | avg TFLOP/s | HBM bytes/launch |", "|---|---|---|---|---|"]
    traffic = {}
    for v, bv in sorted(by_variant.items(), key=lambda kv: -kv[1]["us"]):
        avg_b = bv["bytes"] / bv["nb"] if bv["nb"] else None
        md.append("| %s | %d | %.1f | %s | %s |" % (v, bv["n"], bv["us"] / bv["n"],
                                                    f(bv["flop"] / (bv["us"] * 1e-6) / 1e12 if bv["flop"] else None,
                                                      "%.1f"), f(avg_b, "%.4g")))
        if avg_b is not None:
            traffic[v] = round(avg_b)
    open(os.path.join(a.out, f"{a.round}_{pname}_summary.md"), "w").write("\n".join(md) + "\n")
    tpath = os.path.join(a.out, "traffic.json")
    allt = json.load(open(tpath)) if os.path.exists(tpath) else {}
    allt.update(traffic)
    json.dump(allt, open(tpath, "w"), indent=1, sort_keys=True)
    print("\n".join(md[:6]))


if __name__ == "__main__":
    main()
