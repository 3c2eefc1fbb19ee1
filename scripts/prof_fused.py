"""Summarise a scripts/pmc_fused.sh run (rocprofv3 kernel trace + PMC passes of the
fused-engine emb attack, native driver) into profiles/:

  <round>_fused_<prec>_kernel_stats.csv   the rocprofv3 --stats summary as written
  <round>_fused_<prec>_summary.md          per kernel: median duration, algorithmic
                                           TFLOP/s, HBM bytes and GB/s, MFMA busy,
                                           wave wait/active split, LDS conflicts, L2 hit
  traffic.json                             HBM bytes per launch per kernel name, keyed by
                                           workload ("emb", "e2e", "fb", "emb_fp32"), in the
                                           kernel names bench.py's roofline uses

HBM bytes per dispatch = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes): on gfx950
FETCH_SIZE counts half the bytes of 16-B-per-lane streaming reads
(MI355X_MICROARCH.md, HBM section); WRITE_SIZE is exact for 16-B stores.
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
# algorithmic FLOP per launch at B=256, T=128 (259,424,256 per utterance
# per direction); the head's dense chain is not counted as conv work
FLOP = {"se_fwd_fused": 259_424_256 * 256, "se_bwd_fused": 259_424_256 * 256,
        # Decoder conv MACs x 2 (avc_vc_host.inc dec_mac): forward 65,798,144, backward 64,225,280
        # MAC per utterance at T0 = 16
        "dec_fwd_fused": 2 * 65_798_144 * 256, "dec_bwd_fused": 2 * 64_225_280 * 256,
        "dense_batched": 2 * 3072 * 128 * 256}
ATTACK = {0: "emb", 1: "e2e", 2: "fb"}


def short(k):
    m = re.search(r"(se_fwd_fused|se_bwd_fused|dec_fwd_fused|dec_bwd_fused)<(\d), (\d)>", k)
    if m:
        return "%s<%s>" % (m.group(1), "f32" if m.group(2) == "0" else "bf16")
    for n in ("se_head_v", "se_head", "attack_init", "dense_batched"):
        if n in k:
            return n
    return k.split("(")[0][:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default=os.path.join(ROOT, "gpurun_out"))
    ap.add_argument("--prec", type=int, default=1)
    ap.add_argument("--attack", type=int, default=0)
    ap.add_argument("--round", default="r01")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles"))
    a = ap.parse_args()
    pname = ("fp32" if a.prec == 0 else "bf16") + ("" if a.attack == 0 else "_" + ATTACK[a.attack])
    base = os.path.join(a.dir, f"fz_p{a.prec}_a{a.attack}")
    os.makedirs(a.out, exist_ok=True)
    shutil.copy(os.path.join(base, "trace", "run_kernel_stats.csv"),
                os.path.join(a.out, f"{a.round}_fused_{pname}_kernel_stats.csv"))
    dur = defaultdict(list)
    for r in csv.DictReader(open(os.path.join(base, "trace", "run_kernel_trace.csv"))):
        dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    cnt = defaultdict(lambda: defaultdict(list))
    for i in range(1, 16):
        f = os.path.join(base, f"pmc_{i}", "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        per = defaultdict(lambda: defaultdict(float))
        name = {}
        for r in csv.DictReader(open(f)):
            d = int(r["Dispatch_Id"])
            per[d][r["Counter_Name"]] += float(r["Counter_Value"])
            name[d] = short(r["Kernel_Name"])
        for d, cs in per.items():
            for c, v in cs.items():
                cnt[name[d]][c].append(v)

    def m(k, c):
        v = cnt[k].get(c)
        return statistics.mean(v) if v else None

    f = lambda x, fmt: (fmt % x) if x is not None else "-"
    md = [f"# rocprofv3 summary {a.round}: fused engine, {pname.split('_')[0]} {ATTACK[a.attack]} attack "
          f"(B=256, T=128)", "",
          f"Source: `PREC={a.prec} ATTACK={a.attack} scripts/pmc_fused.sh` on one MI355X: native driver "
          f"`attack-vc_amd/avc_bench 256 128 <iters> 1 0 {a.prec} {a.attack}` (default engine = fused), "
          "one `--kernel-trace --stats` run plus one run per PMC pass.", "",
          "| kernel | launches | median us | TFLOP/s (alg.) | HBM MB/launch | HBM GB/s | MFMA busy | "
          "wait/wave | active/wave | LDS confl/LDS cyc | L2 hit |",
          "|---|---|---|---|---|---|---|---|---|---|---|"]
    traffic = {}
    for k in sorted(dur, key=lambda k: -sum(dur[k])):
        us = statistics.median(dur[k])
        base_k = k.split("<")[0]
        fl = FLOP.get(base_k)
        fetch, write = m(k, "FETCH_SIZE"), m(k, "WRITE_SIZE")
        hbm = (2 * fetch + write) * 1024 if fetch is not None and write is not None else None
        mf, busy = m(k, "SQ_VALU_MFMA_BUSY_CYCLES"), m(k, "SQ_BUSY_CYCLES")
        wait, act, wc = m(k, "SQ_WAIT_ANY"), m(k, "SQ_ACTIVE_INST_ANY"), m(k, "SQ_WAVE_CYCLES")
        lc, la = m(k, "SQ_LDS_BANK_CONFLICT"), m(k, "SQ_ACTIVE_INST_LDS")
        hit, miss = m(k, "TCC_HIT_sum"), m(k, "TCC_MISS_sum")
        md.append("| %s | %d | %.1f | %s | %s | %s | %s | %s | %s | %s | %s |" % (
            k, len(dur[k]), us, f(fl / (us * 1e-6) / 1e12 if fl else None, "%.1f"),
            f(hbm / 1e6 if hbm else None, "%.2f"), f(hbm / (us * 1e-6) / 1e9 if hbm else None, "%.0f"),
            f(mf / busy if mf is not None and busy else None, "%.3f"),
            f(wait / wc if wait is not None and wc else None, "%.2f"),
            f(act / wc if act is not None and wc else None, "%.2f"),
            f(lc / la if lc is not None and la else None, "%.3f"),
            f(hit / (hit + miss) if hit is not None and miss is not None and hit + miss else None, "%.2f")))
        if hbm is not None:
            traffic[k] = round(hbm)
    md += ["", "MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CYCLES (gfx94x-style ratio; ROCm 7.2 has no "
           "gfx950 derived-counter definitions).  HBM = 2*FETCH_SIZE + WRITE_SIZE."]
    open(os.path.join(a.out, f"{a.round}_fused_{pname}_summary.md"), "w").write("\n".join(md) + "\n")
    tpath = os.path.join(a.out, "traffic.json")
    allt = json.load(open(tpath)) if os.path.exists(tpath) else {}
    if not all(isinstance(v, dict) for v in allt.values()):
        allt = {}                                  # (old flat layout)
    key = ATTACK[a.attack] + ("_fp32" if a.prec == 0 else "")
    allt[key] = traffic
    json.dump(allt, open(tpath, "w"), indent=1, sort_keys=True)
    print("\n".join(md))


if __name__ == "__main__":
    main()
