"""Shared test helpers: models from fixtures, oracle weights, tolerances."""
import hashlib
import json
import os

import numpy as np
import torch

import models
from oracle import adain_vc as oracle

# Stated fp32 tolerances (calibrated against fp32-vs-fp64 drift of
# the reference itself).  |adv - ref| is bounded by 2*eps = 0.2 whatever happens,
# so element checks are only meaningful well below that.
TOL_SE_REL = 1e-5        # SpeakerEncoder output, relative to max |emb|
TOL_GRAD_REL = 1e-4      # d loss / d ptb at iteration 0, relative to max |grad|
# e2e / fb chain through the Decoder (fb: SpeakerEncoder -> Decoder -> SpeakerEncoder):
# an fp32 evaluation drifts up to 4.9e-4 (fb, full_T128) / 6.2e-4 (e2e, full_lrelu_T128)
# of max |grad| from the reference's own fp32 run, while a float64 restatement agrees with
# it to ~6e-6 -- isolated elements whose ReLU masks flip between fp32 runs
TOL_GRAD_REL_VC = 1e-3
# e2e / fb iteration-0 gradients vs a float64 restatement, normwise per utterance
# (||g - g64|| / ||g64||).  The objective is ill-conditioned in fp32 at isolated inputs:
# the numpy fp32 restatement of the reference's arithmetic itself reaches 3.4e-3 there
# (scripts/dbg/vc_sweep.py; calibration table in DESIGN.md), while typical
# utterances agree to ~5e-6.  So: every utterance <= 5e-3, the median <= 2e-5.
TOL_VC_GRAD_L2_MAX = 5e-3
TOL_VC_GRAD_L2_MEDIAN = 2e-5
# adv vs the reference's own fp32 run.  Calibrated in round 4 (profiles/r04/tol_calibration.md,
# scripts/tol_calibration.py) against the reference's float64 run of the same attacks
# (tests/golden/calib_f64_T128.npz): at n = 1 every engine is within one fp32 ulp of the golden; by
# n = 10 a differently ordered fp32 sum may flip a ReLU whose pre-activation is within rounding of
# zero, which changes the gradient over that unit's receptive field only (one window of ~12 frames
# of one utterance), and where |grad| < Adam's eps (1e-8; the attacks' gradients are ~1e-8) the step
# is linear in the gradient (lr / eps = 1e5 amplification): the fused engine's 6.2e-6 at n = 10 sits
# on 34 elements, all with |grad| <= 2.5e-8, in frames 76-87 of one utterance.  The reference's own
# fp32 run shows the same mechanism by n = 100 (1.0e-5 vs float64, in the same frame windows).  The
# bounds are ~3x the largest distance any GPU test measured (AVC_TOL_LOG, profiles/r04/tol_log.json):
# max 2.4e-7 / 1.6e-5 / 3.3e-5 / 6.1e-5 and mean 2.3e-9 / 8.9e-8 / 2.1e-7 / 1.4e-6 at n = 1 / 10 / 100 /
# 1500; SURVEY 8(c)'s n = 100 / 1500 bounds are met with room (1e-4; 5e-3, mean 1e-4).
# Round 5: the mean bound at n = 10 is 2e-7.  The fb chain through the Decoder is the worst case: on
# full_lrelu_T128 the reference's OWN fp32 run is 9.3e-8 (mean) from its float64 evaluation (numpy oracle in
# float64 vs the golden; 5.5e-8 for the oracle's fp32), so an independent fp32 evaluation can sit ~2x that
# from the golden (measured 1.37e-7 once every engine computes vc + eps * tanh(ptb) unfused, as the
# reference does).
# Round 6: 2e-7 applies to the e2e / fb chains only (TOL_ADV_MEAN_VC); the emb attack keeps 1e-7.
TOL_ADV = {1: 1e-6, 10: 5e-5, 100: 1e-4, 1500: 5e-4}
TOL_ADV_MEAN = {1: 1e-8, 10: 1e-7, 100: 1e-6, 1500: 5e-6}
TOL_ADV_MEAN_VC = {**TOL_ADV_MEAN, 10: 2e-7}


def check_grad_flip_robust(g, ref, frac=0.05):
    """d loss / d ptb vs a float64 restatement where an isolated ReLU / LeakyReLU mask may flip:
    a pre-activation within fp32 rounding of zero (measured: 4.9e-9 of its layer's max at T=176,
    seed 876, conv_bank k=7, frame 164) takes the other branch in fp32, which changes the
    gradient over that unit's receptive field only (8-80 columns of one utterance, up to 7e-3 of
    max |grad| there).  So: every utterance normwise within TOL_VC_GRAD_L2_MAX, and all but `frac`
    of the elements within TOL_GRAD_REL of max |grad| (a systematic error breaks both)."""
    g = np.asarray(g, np.float64)
    ref = np.asarray(ref, np.float64)
    for u in range(g.shape[0]):
        e = float(np.linalg.norm(g[u] - ref[u]) / np.linalg.norm(ref[u]))
        assert e <= TOL_VC_GRAD_L2_MAX, (u, e)
    off = np.abs(g - ref) > TOL_GRAD_REL * np.abs(ref).max()
    assert off.mean() <= frac, off.mean()


def check_adv(adv, ref, n, kind="emb"):
    """adv vs a reference adv after n iterations; kind "e2e" / "fb" (the chain through the Decoder) takes
    the VC mean bound at n = 10."""
    d = np.abs(np.asarray(adv, np.float64) - np.asarray(ref, np.float64))
    log = os.environ.get("AVC_TOL_LOG")
    if log:   # calibration runs: record every comparison (scripts/tol_calibration.py)
        import inspect
        caller = inspect.stack()[1]
        with open(log, "a") as fh:
            fh.write(json.dumps({"n": n, "max": float(d.max()), "mean": float(d.mean()),
                                 "where": f"{os.path.basename(caller.filename)}:{caller.function}"}) + "\n")
    assert d.max() <= TOL_ADV[n], (n, d.max())
    mean_tol = (TOL_ADV_MEAN_VC if kind in ("e2e", "fb") else TOL_ADV_MEAN)[n]
    assert d.mean() <= mean_tol, (n, kind, d.mean())


def cfg_of(z):
    return json.loads(str(z["config"]))


def state_of(z):
    return {k[2:]: torch.from_numpy(np.asarray(z[k])) for k in z if k.startswith("w/")}


def model_from_fixture(z):
    """Small config: weights stored in the fixture. Full config: seeded init,
    verified against the reference's weight hashes."""
    cfg = cfg_of(z)
    if any(k.startswith("w/") for k in z):
        m = models.AdaInVC(cfg)
        m.load_state_dict(state_of(z))
        return m
    torch.manual_seed(0)
    m = models.AdaInVC(cfg)
    hs = json.loads(str(z["weight_sha256"]))
    for k, v in m.state_dict().items():
        assert hashlib.sha256(v.numpy().tobytes()).hexdigest() == hs[k], k
    return m


def oracle_weights(m):
    return oracle.Weights({k: v.detach().cpu().numpy() for k, v in m.state_dict().items()})


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-30))


def oracle_grad0_instrumented(kind, w, cfg, src, vc, at, p0, flip=None):
    """The oracle's iteration-0 gradient of a `kind` attack (float64 weights/inputs for the
    calibration tests) with every activation call numbered in call order.  Returns (grad0, pre):
    pre[i] is call i's pre-activation.  flip=(i, idx) makes call i's unit idx take the other branch
    of its (Leaky)ReLU -- a pre-activation within rounding of zero evaluated with the other sign: its
    output gets the other sign (the oracle's act' reads the sign of the output, so the backward
    follows); a list of such pairs flips several units.  Test infrastructure for the fb iteration-0
    localisation tests."""
    pre = []
    orig = oracle.acts
    flips = [] if flip is None else ([flip] if isinstance(flip[0], int) else list(flip))

    def acts(c):
        act, dact = orig(c)

        def a(x):
            i = len(pre)
            pre.append(x)
            y = act(x)
            for fi, j in flips:
                if fi == i:
                    y = y.copy()
                    y[j] = act(-x[j]) if x[j] > 0 else -x[j]
            return y
        return a, dact
    oracle.acts = acts
    try:
        rec = {}
        oracle.attack(kind, w, cfg, src, vc, at, 0.1, 1, p0, record=rec)
    finally:
        oracle.acts = orig
    return rec["grad0"], pre


def vc_grad0_explained(kind, model, cfg, ins, g_gpu, rel_ok=1e-5, tol=5e-6, ref64=None):
    """The e2e / fb iteration-0 gradient of ONE utterance (ins: its vc_src, vc_tgt, adv_tgt, ptb0 [1, 80, T])
    vs the reference's arithmetic in float64: within rel_ok of max |g|, or -- the fb / e2e chain funnels a
    Decoder / feedback-encoder unit that takes the other (Leaky)ReLU branch through the 128-wide embedding
    gradients, moving every element of the utterance -- within `tol` of the float64 gradient with one (or two)
    units of the attack iteration's forward flipped, units whose pre-activation is within 1e-6 of its layer's
    max.  Returns (ok, report)."""
    sd = {k: v.detach().cpu().numpy() for k, v in model.state_dict().items()}
    w64 = oracle.Weights(sd, dtype=np.float64)
    f64 = [np.asarray(t, np.float64) for t in ins]
    g64, pre = oracle_grad0_instrumented(kind, w64, cfg, *f64)
    if ref64 is not None:
        assert np.abs(g64 - ref64).max() <= 1e-12 * np.abs(ref64).max()
    gmax = np.abs(g64).max()
    g = np.asarray(g_gpu, np.float64).reshape(g64.shape)
    e0 = float(np.abs(g - g64).max() / gmax)
    if e0 <= rel_ok:
        return True, f"within {e0:.2e} of float64"
    se = cfg["SpeakerEncoder"]
    n_se = len(range(se["bank_scale"], se["bank_size"] + 1, se["bank_scale"])) + 1 + 2 * se["n_conv_blocks"] + \
        2 * se["n_dense_blocks"]
    n_it = n_se + 1 + 2 * cfg["Decoder"]["n_conv_blocks"] + (n_se if kind == "fb" else 0)
    first = len(pre) - n_it
    cand = []
    for i in range(first, len(pre)):
        r = np.abs(pre[i]) / np.abs(pre[i]).max()
        j = np.unravel_index(np.argmin(r), r.shape)
        if r[j] < 1e-6:
            cand.append((float(r[j]), i, j))
    best, rep = None, [f"float64 {e0:.2e}"]
    cand = sorted(cand)
    sets = [[c] for c in cand] + [[a, b] for k, a in enumerate(cand) for b in cand[k + 1:]]   # one flip, then two
    for fs in sets:
        gf, _ = oracle_grad0_instrumented(kind, w64, cfg, *f64, flip=[(i, j) for _, i, j in fs])
        e = float(np.abs(g - gf).max() / gmax)
        rep.append("flip " + " + ".join(f"call {i - first} {tuple(int(v) for v in j)} (|pre| {r:.1e})" for r, i, j in fs) +
                   f": {e:.2e}")
        best = e if best is None else min(best, e)
        if e <= tol:
            break
    return best is not None and best <= tol, "; ".join(rep)
