"""float64 runs of the REAL reference for the fp32 tolerance calibration.

Test infrastructure only; runs in the build container (the reference never leaves it).
Imports the reference's ``models.py`` read-only, builds the full AdaIN-VC config from
``torch.manual_seed(0)`` (the weights full_T128.npz pins by SHA-256), converts the model and
the inputs to float64 and runs the attack loop of attack_utils.py:7-130 (the instrumented
restatement of make_golden.py, asserted there bitwise equal to the reference's own function in
fp32) from each golden's injected ptb0.  Writes calib_f64_T128.npz: adv at n = 1 / 10 / 100
(emb also 1500), grad0 and the loss histories, for emb / e2e / fb.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_calib.py
"""
import argparse
import json
import os
import sys

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))


def loop(kind, model, vc_src, vc_tgt, adv_tgt, eps, ptb0, n_list):
    """attack_utils.py:7-130 (Adam on ptb, eps*tanh reparameterisation, MSE objectives) from an
    injected ptb0; snapshots of vc_tgt + eps*tanh(ptb) after each n in n_list."""
    ptb = ptb0.clone().requires_grad_(True)
    opt = torch.optim.Adam([ptb])
    crit = nn.MSELoss()
    with torch.no_grad():
        if kind == "emb":
            org, tgt = model.speaker_encoder(vc_tgt), model.speaker_encoder(adv_tgt)
        elif kind == "e2e":
            org, tgt = model.inference(vc_src, vc_tgt), model.inference(vc_src, adv_tgt)
        else:
            org, tgt = model.speaker_encoder(model.inference(vc_src, vc_tgt)), model.speaker_encoder(adv_tgt)
    snaps, losses, grad0 = {}, [], None
    for it in range(max(n_list)):
        adv = vc_tgt + eps * ptb.tanh()
        if kind == "emb":
            out = model.speaker_encoder(adv)
        elif kind == "e2e":
            out = model.inference(vc_src, adv)
        else:
            out = model.speaker_encoder(model.inference(vc_src, adv))
        loss = crit(out, tgt) - 0.1 * crit(out, org)
        opt.zero_grad()
        loss.backward()
        if it == 0:
            grad0 = ptb.grad.detach().clone()
        losses.append(loss.item())
        opt.step()
        if it + 1 in n_list:
            snaps[it + 1] = (vc_tgt + eps * ptb.tanh()).detach().clone()
    return snaps, grad0, np.array(losses)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--no-1500", action="store_true")
    a = ap.parse_args()
    sys.dont_write_bytecode = True
    sys.path.insert(0, a.ref)
    import models  # noqa: E402  (reference, read-only)
    torch.set_num_threads(os.cpu_count() or 1)
    z = dict(np.load(os.path.join(HERE, "full_T128.npz")))
    cfg = json.loads(str(z["config"]))
    torch.manual_seed(0)
    model = models.AdaInVC(cfg).double()
    X = {k: torch.from_numpy(z[k]).double() for k in ("vc_src", "vc_tgt", "adv_tgt")}
    out = {"config": z["config"], "weight_sha256": z["weight_sha256"]}
    for kind in ("emb", "e2e", "fb"):
        ns = [1, 10, 100] + ([1500] if kind == "emb" and not a.no_1500 else [])
        advs = {n: [] for n in ns}
        g0s, Ls = [], []
        for b in range(z["vc_tgt"].shape[0]):
            args = [X[k][b:b + 1] for k in ("vc_src", "vc_tgt", "adv_tgt")]
            p0 = torch.from_numpy(z[f"{kind}_ptb0"][b:b + 1]).double()
            snaps, g0, L = loop(kind, model, *args, 0.1, p0, ns)
            for n in ns:
                advs[n].append(snaps[n])
            g0s.append(g0)
            Ls.append(L)
        for n in ns:
            out[f"{kind}_adv_n{n}"] = torch.cat(advs[n]).numpy()
        out[f"{kind}_grad0"] = torch.cat(g0s).numpy()
        out[f"{kind}_losses"] = np.stack(Ls)
        print(kind, "done", flush=True)
    path = os.path.join(HERE, "calib_f64_T128.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path))


if __name__ == "__main__":
    main()
