"""fp32 tolerance calibration (tests/helpers.py TOL_ADV): the GPU's distance from the
reference's float64 run next to the reference's OWN fp32 distance from it.

Inputs (all committed):
  profiles/r04/calib_gpu.npz          libavc fp32 on the MI355X (scripts/calib_dump.py)
  tests/golden/full_T128.npz          the reference's fp32 run (attack_utils.*, make_golden.py)
  tests/golden/full_T128_n100.npz     ... e2e / fb at n = 100
  tests/golden/calib_f64_T128.npz     the reference's arithmetic in float64 (make_calib.py)
Also runs the numpy restatement (oracle/adain_vc.py, fp32) as a second reordering of the same
fp32 arithmetic.  Writes profiles/r04/tol_calibration.{json,md}.

Per case (engine, attack, n): max / mean |x - f64| for x = GPU, reference fp32, oracle fp32, and
the element-wise ratio; at iteration 0 the gradient's relative error and the number of elements
whose gradient SIGN differs from float64 (Adam's first step is ~lr*sign(g) where |g| >> 1e-8).

Usage:  python scripts/tol_calibration.py [--no-oracle]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "attack-vc_amd"), os.path.join(ROOT, "tests")]
G = os.path.join(ROOT, "tests", "golden")


def stats(x, ref):
    d = np.abs(np.asarray(x, np.float64) - ref)
    return float(d.max()), float(d.mean())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpu", default=os.path.join(ROOT, "profiles", "r04", "calib_gpu.npz"))
    ap.add_argument("--no-oracle", action="store_true")
    a = ap.parse_args()
    gpu = dict(np.load(a.gpu))
    z = dict(np.load(os.path.join(G, "full_T128.npz")))
    zn = dict(np.load(os.path.join(G, "full_T128_n100.npz")))
    f64 = dict(np.load(os.path.join(G, "calib_f64_T128.npz")))

    def ref32(kind, n):
        k = f"{kind}_adv_n{n}"
        return z[k] if k in z else zn.get(k)

    orc = {}
    if not a.no_oracle:
        from helpers import cfg_of, model_from_fixture, oracle_weights
        from oracle import adain_vc as oracle
        w = oracle_weights(model_from_fixture(z))
        for kind in ("emb", "e2e", "fb"):
            for n in (10, 100):
                fn = getattr(oracle, f"{kind}_attack")
                args = (z["vc_tgt"], z["adv_tgt"]) if kind == "emb" else (z["vc_src"], z["vc_tgt"], z["adv_tgt"])
                orc[(kind, n)] = fn(w, cfg_of(z), *args, 0.1, n, z[f"{kind}_ptb0"])
                print("oracle", kind, n, flush=True)

    rows = []
    for key in sorted(k for k in gpu if k.endswith("/adv")):
        eng, kind, ns = key.split("/")[:3]
        n = int(ns[1:])
        fk = f"{kind}_adv_n{n}"
        if fk not in f64:
            continue
        r = {"engine": eng, "attack": kind, "n": n}
        r["gpu_max"], r["gpu_mean"] = stats(gpu[key], f64[fk])
        rr = ref32(kind, n)
        if rr is not None:
            r["ref32_max"], r["ref32_mean"] = stats(rr, f64[fk])
            r["gpu_vs_ref32_max"], r["gpu_vs_ref32_mean"] = stats(gpu[key], rr.astype(np.float64))
        if (kind, n) in orc:
            r["oracle32_max"], r["oracle32_mean"] = stats(orc[(kind, n)], f64[fk])
        rows.append(r)
    grads = []
    for eng in ("fused", "layered", "long"):
        for kind in ("emb", "e2e", "fb"):
            k = f"{eng}/{kind}/grad0"
            if k not in gpu:
                continue
            g64 = f64[f"{kind}_grad0"]
            m = np.abs(g64).max()
            r = {"engine": eng, "attack": kind, "max_abs_grad": float(m),
                 "median_abs_grad": float(np.median(np.abs(g64)))}
            for name, g in (("gpu", gpu[k]), ("ref32", z[f"{kind}_grad0"])):
                g = np.asarray(g, np.float64)
                r[f"{name}_rel"] = float(np.abs(g - g64).max() / m)
                flip = np.sign(g) != np.sign(g64)
                r[f"{name}_sign_flips"] = int(flip.sum())
                r[f"{name}_flip_max_abs_grad"] = float(np.abs(g64[flip]).max()) if flip.any() else 0.0
            grads.append(r)
    # where the GPU's n = 10 emb error sits: the gradient there, and the Adam-eps ratio
    where = []
    for eng in ("fused", "layered", "long"):
        k = f"{eng}/emb/n10/adv"
        if k not in gpu:
            continue
        d = np.abs(gpu[k].astype(np.float64) - f64["emb_adv_n10"])
        g64 = f64["emb_grad0"]
        idx = np.argsort(d.ravel())[::-1][:5]
        for i in idx:
            u = np.unravel_index(i, d.shape)
            where.append({"engine": eng, "elem": [int(x) for x in u], "err": float(d[u]),
                          "ref32_err": float(abs(z["emb_adv_n10"][u] - f64["emb_adv_n10"][u])),
                          "abs_grad0": float(abs(g64[u])), "grad0_over_adam_eps": float(abs(g64[u]) / 1e-8)})
    # the frames each error sits in: a ReLU unit whose pre-activation is within fp32 rounding of 0
    # takes the other branch in a differently ordered sum and changes the gradient over its
    # receptive field only (a window of ~12 consecutive frames), where |g| < Adam's eps makes the
    # step linear in g (lr / eps = 1e5 amplification)
    windows = []
    for name, arr, n in [("fused", gpu.get("fused/emb/n10/adv"), 10), ("fused", gpu.get("fused/emb/n100/adv"), 100),
                         ("layered", gpu.get("layered/emb/n100/adv"), 100), ("ref32", z["emb_adv_n100"], 100)]:
        if arr is None:
            continue
        d = np.abs(np.asarray(arr, np.float64) - f64[f"emb_adv_n{n}"])
        thr = 3e-7 if n == 10 else 3e-6
        for b in range(d.shape[0]):
            fr = np.where(d[b].max(0) > thr)[0]
            windows.append({"who": name, "n": n, "utt": b, "threshold": thr, "frames": [int(x) for x in fr],
                            "max": float(d[b].max())})
    out = {"adv": rows, "grad0": grads, "largest_emb_n10": where, "error_frames": windows}
    os.makedirs(os.path.join(ROOT, "profiles", "r04"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "r04", "tol_calibration.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    lines = ["# fp32 tolerance calibration (round 4)", "",
             "Distances from the reference's float64 run (`tests/golden/calib_f64_T128.npz`) of: the GPU (libavc fp32, "
             "`profiles/r04/calib_gpu.npz`), the reference's own fp32 run (the goldens) and the numpy fp32 restatement "
             "(`oracle/adain_vc.py`).  full_T128 inputs, B = 2, T = 128.", "",
             "| engine | attack | n | GPU max | GPU mean | ref fp32 max | ref fp32 mean | oracle fp32 max | GPU vs ref32 max |",
             "|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        lines.append(f"| {r['engine']} | {r['attack']} | {r['n']} | {r['gpu_max']:.2e} | {r['gpu_mean']:.2e} | "
                     f"{r.get('ref32_max', float('nan')):.2e} | {r.get('ref32_mean', float('nan')):.2e} | "
                     f"{r.get('oracle32_max', float('nan')):.2e} | {r.get('gpu_vs_ref32_max', float('nan')):.2e} |")
    lines += ["", "Iteration-0 gradient vs float64 (relative to max |g|; sign flips = elements whose sign differs):", "",
              "| engine | attack | max abs g | GPU rel | GPU flips (max abs g there) | ref32 rel | ref32 flips |",
              "|---|---|---|---|---|---|---|"]
    for r in grads:
        lines.append(f"| {r['engine']} | {r['attack']} | {r['max_abs_grad']:.2e} | {r['gpu_rel']:.2e} | "
                     f"{r['gpu_sign_flips']} ({r['gpu_flip_max_abs_grad']:.1e}) | {r['ref32_rel']:.2e} | "
                     f"{r['ref32_sign_flips']} ({r['ref32_flip_max_abs_grad']:.1e}) |")
    lines += ["", "Largest GPU errors of emb at n = 10 (element [b, mel bin, frame]):", "",
              "| engine | element | GPU err | ref32 err | abs grad0 | abs grad0 / Adam eps |", "|---|---|---|---|---|---|"]
    for r in where:
        lines.append(f"| {r['engine']} | {r['elem']} | {r['err']:.2e} | {r['ref32_err']:.2e} | {r['abs_grad0']:.2e} | "
                     f"{r['grad0_over_adam_eps']:.2f} |")
    lines += ["", "Frames whose error exceeds the threshold (emb; per utterance):", "",
              "| who | n | utt | threshold | frames | max |", "|---|---|---|---|---|---|"]
    for r in windows:
        lines.append(f"| {r['who']} | {r['n']} | {r['utt']} | {r['threshold']:.0e} | {r['frames']} | {r['max']:.2e} |")
    with open(os.path.join(ROOT, "profiles", "r04", "tol_calibration.md"), "w") as fh:
        fh.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
