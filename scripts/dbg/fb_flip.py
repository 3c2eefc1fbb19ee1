"""Localise the fb iteration-0 gradient drift on the CPU.

Runs the float64 oracle's fb iteration 0 on full_T128's inputs with every activation call
instrumented: records each ReLU pre-activation (tagged by call order), lists the ones nearest
zero relative to their layer's scale, then re-runs the float64 gradient with one of those
masks flipped at a time and compares it with the GPU's fp32 grad0 (profiles/r04/calib_gpu.npz).
A flip that brings the float64 gradient to the GPU's within fp32 noise names the unit.

Usage: python scripts/dbg/fb_flip.py [--engine fused|long] [--top 12]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "attack-vc_amd"), os.path.join(ROOT, "tests")]

from helpers import cfg_of, model_from_fixture  # noqa: E402
from oracle import adain_vc as O  # noqa: E402

REC = {"calls": [], "flip": None, "n": 0}


def relu(x):
    i = REC["n"]
    REC["n"] += 1
    REC["calls"].append(x.copy())
    m = x > 0
    if REC["flip"] is not None and REC["flip"][0] == i:
        m = m.copy()
        m[REC["flip"][1]] = ~m[REC["flip"][1]]
    REC.setdefault("masks", {})[i] = m
    return np.where(m, x, 0)


def run_fb_grad0(w, cfg, src, vc, at, p0):
    """fb iteration 0 with the masks of the forward reused in the backward (O's backward
    recomputes act' from the post-activation, so d(y) = y > 0 agrees with the flipped mask)."""
    orig_acts = O.acts

    def acts(c):
        return relu, (lambda y: (y > 0).astype(y.dtype))
    O.acts = acts
    try:
        rec = {}
        REC["n"] = 0
        REC["calls"] = []
        O.attack("fb", w, cfg, src, vc, at, 0.1, 1, p0, record=rec)
        return rec["grad0"], list(REC["calls"])
    finally:
        O.acts = orig_acts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--engine", default="fused")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--utt", type=int, default=0)
    a = ap.parse_args()
    z = dict(np.load(os.path.join(ROOT, "tests/golden/full_T128.npz")))
    zf = np.load(os.path.join(ROOT, "tests/golden/calib_f64_T128.npz"))
    gpu = np.load(os.path.join(ROOT, "profiles/r04/calib_gpu.npz"))[f"{a.engine}/fb/grad0"].astype(np.float64)
    m = model_from_fixture(z)
    w = O.Weights({k: v.detach().numpy() for k, v in m.state_dict().items()}, dtype=np.float64)
    cfg = cfg_of(z)
    u = a.utt
    f64 = [np.asarray(z[k][u:u + 1], np.float64) for k in ("vc_src", "vc_tgt", "adv_tgt", "fb_ptb0")]
    g64, calls = run_fb_grad0(w, cfg, *f64)
    print("float64 grad0 vs calib fixture:", np.abs(g64[0] - zf["fb_grad0"][u]).max())
    gmax = np.abs(g64).max()
    base = np.abs(gpu[u] - g64[0]).max() / gmax
    print(f"GPU vs float64 (utt {u}): {base:.3e} of max|g|")
    # candidates: smallest |pre| / max|pre of that call| -- skip the precompute calls (org / tgt),
    # which come first; the attack's own forward calls are the last len(calls)/... ones
    cand = []
    for i, x in enumerate(calls):
        s = np.abs(x).max()
        if s == 0:
            continue
        r = np.abs(x) / s
        j = np.unravel_index(np.argmin(r), r.shape)
        cand.append((float(r[j]), i, j, x.shape))
    cand.sort()
    print("nearest-zero pre-activations (rel to call max):")
    for r, i, j, sh in cand[:a.top]:
        print(f"  call {i:3d} shape {sh} idx {j} rel {r:.2e}")
    for r, i, j, sh in cand[:a.top]:
        REC["flip"] = (i, j)
        gf, _ = run_fb_grad0(w, cfg, *f64)
        REC["flip"] = None
        e = np.abs(gpu[u] - gf[0]).max() / gmax
        d = np.abs(gf[0] - g64[0]).max() / gmax
        print(f"flip call {i:3d} {j}: float64 moves {d:.3e}; GPU vs flipped {e:.3e}")


if __name__ == "__main__":
    main()


def n10(engine="fused", call=190, idx=(0, 25, 94), n=10):
    """fb at n iterations in float64 with the unit (call, idx) flipped in EVERY iteration's
    forward (the same layer / channel / frame: 79 activation calls per fb iteration after 133
    precompute calls) -- vs the GPU's adv."""
    z = dict(np.load(os.path.join(ROOT, "tests/golden/full_T128.npz")))
    zf = np.load(os.path.join(ROOT, "tests/golden/calib_f64_T128.npz"))
    gpu = np.load(os.path.join(ROOT, "profiles/r04/calib_gpu.npz"))[f"{engine}/fb/n{n}/adv"].astype(np.float64)
    m = model_from_fixture(z)
    w = O.Weights({k: v.detach().numpy() for k, v in m.state_dict().items()}, dtype=np.float64)
    cfg = cfg_of(z)
    f64 = [np.asarray(z[k][0:1], np.float64) for k in ("vc_src", "vc_tgt", "adv_tgt", "fb_ptb0")]
    off = call - 133

    def relu_p(x):
        i = REC["n"]
        REC["n"] += 1
        mk = x > 0
        if i >= 133 and (i - 133) % 79 == off and np.abs(x[idx]) < 1e-6 * np.abs(x).max():
            mk = mk.copy()
            mk[idx] = ~mk[idx]
            REC["nflip"] = REC.get("nflip", 0) + 1
        return np.where(mk, x, 0)
    orig = O.acts
    O.acts = lambda c: (relu_p, (lambda y: (y > 0).astype(y.dtype)))
    try:
        REC["n"] = 0
        advf = O.attack("fb", w, cfg, *f64[:3], 0.1, n, f64[3])
    finally:
        O.acts = orig
    print(f"flips applied: {REC.get('nflip', 0)} of {n} iterations")
    print("GPU vs float64        :", np.abs(gpu[0] - zf[f"fb_adv_n{n}"][0]).max())
    print("GPU vs float64+flip   :", np.abs(gpu[0] - advf[0]).max())
    print("utt 1 GPU vs float64  :", np.abs(gpu[1] - zf[f"fb_adv_n{n}"][1]).max())
