"""Generate the golden fixtures in tests/golden/ from the REAL reference.

Test infrastructure only.  Runs in the build container (never on the GPU box,
where /root/reference does not exist) and imports the reference's own
``models.py`` and ``attack_utils.py`` read-only from ``--ref`` (default
/root/reference).  Nothing from the reference is copied: only input/output
vectors are written, as .npz data.

Every attack fixture is produced twice and asserted bitwise equal:
  * by calling the reference function itself (attack_utils.emb_attack /
    e2e_attack / fb_attack, attack_utils.py:7-130) after torch.manual_seed(s),
    which makes its unseeded ``zeros_like(x).normal_(0,1)`` draw
    (attack_utils.py:30,68,112) reproducible;
  * by an instrumented loop with the same arithmetic, which additionally
    records the per-iteration loss and the iteration-0 gradient d loss/d ptb.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
import argparse
import hashlib
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))

# Upstream AdaIN-VC config.yaml "model" section (SURVEY.md section 8 header).
FULL_CFG = {
    "SpeakerEncoder": dict(c_in=80, c_h=128, c_out=128, kernel_size=5, bank_size=8,
                           bank_scale=1, c_bank=128, n_conv_blocks=6, n_dense_blocks=6,
                           subsample=[1, 2, 1, 2, 1, 2], act="relu", dropout_rate=0.0),
    "ContentEncoder": dict(c_in=80, c_h=128, c_out=128, kernel_size=5, bank_size=8,
                           bank_scale=1, c_bank=128, n_conv_blocks=6,
                           subsample=[1, 2, 1, 2, 1, 2], act="relu", dropout_rate=0.0),
    "Decoder": dict(c_in=128, c_cond=128, c_h=128, c_out=80, kernel_size=5,
                    n_conv_blocks=6, upsample=[2, 1, 2, 1, 2, 1], act="relu",
                    sn=False, dropout_rate=0.0),
}
# Small config: fast enough for many-iteration pins (SURVEY.md 8(c) "Golden vectors" (1)).
SMALL_CFG = {
    "SpeakerEncoder": dict(c_in=80, c_h=32, c_out=32, kernel_size=5, bank_size=4,
                           bank_scale=1, c_bank=32, n_conv_blocks=2, n_dense_blocks=2,
                           subsample=[1, 2], act="relu", dropout_rate=0.0),
    "ContentEncoder": dict(c_in=80, c_h=32, c_out=32, kernel_size=5, bank_size=4,
                           bank_scale=1, c_bank=32, n_conv_blocks=2,
                           subsample=[1, 2], act="relu", dropout_rate=0.0),
    "Decoder": dict(c_in=32, c_cond=32, c_h=32, c_out=80, kernel_size=5,
                    n_conv_blocks=2, upsample=[2, 1], act="relu",
                    sn=False, dropout_rate=0.0),
}
EPS = 0.1


def sha(t):
    return hashlib.sha256(t.detach().contiguous().numpy().tobytes()).hexdigest()


def instrumented(attack_type, model, vc_src, vc_tgt, adv_tgt, eps, n_iters, seed):
    """Same arithmetic as attack_utils.py:7-130, plus loss/grad recording."""
    import torch.nn as nn
    torch.manual_seed(seed)
    ptb = torch.zeros_like(vc_tgt).normal_(0, 1).requires_grad_(True)
    ptb0 = ptb.detach().clone()
    opt = torch.optim.Adam([ptb])
    crit = nn.MSELoss()
    with torch.no_grad():
        if attack_type == "emb":
            org = model.speaker_encoder(vc_tgt)
            tgt = model.speaker_encoder(adv_tgt)
        elif attack_type == "e2e":
            org = model.inference(vc_src, vc_tgt)
            tgt = model.inference(vc_src, adv_tgt)
        else:
            org = model.speaker_encoder(model.inference(vc_src, vc_tgt))
            tgt = model.speaker_encoder(adv_tgt)
    losses, grad0 = [], None
    for it in range(n_iters):
        adv = vc_tgt + eps * ptb.tanh()
        if attack_type == "emb":
            out = model.speaker_encoder(adv)
        elif attack_type == "e2e":
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
    final = (vc_tgt + eps * ptb.tanh()).detach()
    return dict(ptb0=ptb0, org=org, tgt=tgt, losses=np.array(losses, np.float64),
                grad0=grad0, adv=final)


def run_reference(au, attack_type, model, vc_src, vc_tgt, adv_tgt, eps, n_iters, seed):
    torch.manual_seed(seed)
    if attack_type == "emb":
        out = au.emb_attack(model, vc_tgt, adv_tgt, eps, n_iters)
    elif attack_type == "e2e":
        out = au.e2e_attack(model, vc_src, vc_tgt, adv_tgt, eps, n_iters)
    else:
        out = au.fb_attack(model, vc_src, vc_tgt, adv_tgt, eps, n_iters)
    return out.detach()


def attack_fixture(au, attack_type, model, X, n_list, seeds, prefix, out, keep_losses):
    """Per-utterance (B=1) reference attacks for every n in n_list."""
    B = X["vc_tgt"].shape[0]
    for n in n_list:
        advs, grads, losses, ptb0s, orgs, tgts = [], [], [], [], [], []
        for b in range(B):
            args = [X[k][b:b + 1] for k in ("vc_src", "vc_tgt", "adv_tgt")]
            ins = instrumented(attack_type, model, *args, EPS, n, seeds[b])
            ref = run_reference(au, attack_type, model, *args, EPS, n, seeds[b])
            assert torch.equal(ins["adv"], ref), (attack_type, n, b)
            advs.append(ref)
            grads.append(ins["grad0"])
            losses.append(ins["losses"])
            ptb0s.append(ins["ptb0"])
            orgs.append(ins["org"])
            tgts.append(ins["tgt"])
        out[f"{prefix}{attack_type}_adv_n{n}"] = torch.cat(advs).numpy()
        out[f"{prefix}{attack_type}_grad0"] = torch.cat(grads).numpy()
        out[f"{prefix}{attack_type}_ptb0"] = torch.cat(ptb0s).numpy()
        out[f"{prefix}{attack_type}_org"] = torch.cat(orgs).numpy()
        out[f"{prefix}{attack_type}_tgt"] = torch.cat(tgts).numpy()
        if keep_losses and n == max(n_list):
            out[f"{prefix}{attack_type}_losses_n{n}"] = np.stack(losses)


def make_inputs(B, T, seed):
    """T: one length for all three inputs, or a dict {vc_src, vc_tgt, adv_tgt: frames}."""
    g = torch.Generator().manual_seed(seed)
    lens = T if isinstance(T, dict) else {k: T for k in ("vc_src", "vc_tgt", "adv_tgt")}
    return {k: torch.randn(B, 80, lens[k], generator=g) for k in ("vc_src", "vc_tgt", "adv_tgt")}


def build(models, cfg):
    torch.manual_seed(0)
    m = models.AdaInVC(cfg)
    # The reference never calls .eval() (attack.py:38, data_utils.py:220); with
    # dropout_rate=0 train mode is numerically identical.
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--skip-1500", action="store_true")
    ap.add_argument("--stage", default="all", choices=["all", "base", "long", "long100"],
                    help="long: only the round-2 fixtures (T = 300 with three input lengths; "
                         "e2e / fb at n = 100); long100: only full_T300_n100.npz (round 4)")
    a = ap.parse_args()
    sys.dont_write_bytecode = True
    sys.path.insert(0, a.ref)
    import models  # noqa: E402  (reference, read-only)
    import attack_utils as au  # noqa: E402
    torch.set_num_threads(os.cpu_count() or 1)
    seeds = [1000, 1001]

    if a.stage in ("all", "long"):
        long_fixtures(models, au, seeds)
    if a.stage in ("all", "long100"):
        long100_fixtures(models, au, seeds)
    if a.stage in ("long", "long100"):
        return

    # ---------------- small config -------------------------------------------------
    for T in (32, 33):
        model = build(models, SMALL_CFG)
        X = make_inputs(2, T, seed=T)
        out = {"config": np.array(json.dumps(SMALL_CFG)), "eps": np.float64(EPS), "T": np.int64(T)}
        for k, v in model.state_dict().items():
            out["w/" + k] = v.numpy()
        for k, v in X.items():
            out[k] = v.numpy()
        with torch.no_grad():
            out["se_vc_tgt"] = model.speaker_encoder(X["vc_tgt"]).numpy()
            out["se_adv_tgt"] = model.speaker_encoder(X["adv_tgt"]).numpy()
            mu, log_sigma = model.content_encoder(X["vc_src"])
            out["ce_mu_vc_src"] = mu.numpy()
            out["inference"] = model.inference(X["vc_src"], X["vc_tgt"]).numpy()
        n_emb = [1, 10, 100] if T == 32 else [10]
        attack_fixture(au, "emb", model, X, n_emb, seeds, "", out, keep_losses=True)
        attack_fixture(au, "e2e", model, X, [10], seeds, "", out, keep_losses=True)
        attack_fixture(au, "fb", model, X, [10], seeds, "", out, keep_losses=True)
        if T == 32:
            # Batched call of the reference itself (mean-reduced loss over the batch):
            # pins reduction="mean" semantics of a [B,80,T] input.
            torch.manual_seed(seeds[0])
            out["emb_batched_adv_n10"] = au.emb_attack(
                model, X["vc_tgt"], X["adv_tgt"], EPS, 10).detach().numpy()
            torch.manual_seed(seeds[0])
            out["emb_batched_ptb0"] = torch.zeros_like(X["vc_tgt"]).normal_(0, 1).numpy()
        path = os.path.join(HERE, f"small_T{T}.npz")
        np.savez_compressed(path, **out)
        print("wrote", path, os.path.getsize(path))

    # ---------------- full config (weights regenerated from seed 0; pinned by hash) ---
    for T in (128, 127):
        model = build(models, FULL_CFG)
        X = make_inputs(2, T, seed=T)
        out = {"config": np.array(json.dumps(FULL_CFG)), "eps": np.float64(EPS), "T": np.int64(T)}
        hashes = {k: sha(v) for k, v in model.state_dict().items()}
        sums = {k: float(v.double().sum()) for k, v in model.state_dict().items()}
        out["weight_sha256"] = np.array(json.dumps(hashes))
        out["weight_sum"] = np.array(json.dumps(sums))
        for k, v in X.items():
            out[k] = v.numpy()
        with torch.no_grad():
            out["se_vc_tgt"] = model.speaker_encoder(X["vc_tgt"]).numpy()
            out["se_adv_tgt"] = model.speaker_encoder(X["adv_tgt"]).numpy()
            out["inference"] = model.inference(X["vc_src"], X["vc_tgt"]).numpy()
        if T == 128:
            n_emb = [1, 10, 100] + ([] if a.skip_1500 else [1500])
            attack_fixture(au, "emb", model, X, n_emb, seeds, "", out, keep_losses=True)
            attack_fixture(au, "e2e", model, X, [10], seeds, "", out, keep_losses=True)
            attack_fixture(au, "fb", model, X, [10], seeds, "", out, keep_losses=True)
        else:
            attack_fixture(au, "emb", model, X, [10], seeds, "", out, keep_losses=True)
        path = os.path.join(HERE, f"full_T{T}.npz")
        np.savez_compressed(path, **out)
        print("wrote", path, os.path.getsize(path))


def long_fixtures(models, au, seeds):
    """Round 2: real utterance lengths.  full_T300.npz -- vc_tgt 300 frames (the long
    engine), vc_src 280 and adv_tgt 260 (every input its own length, as attack.py loads them):
    emb / e2e / fb adv at n = 10, grad0, losses, SE(vc_tgt) and inference(vc_src, vc_tgt).
    full_T128_n100.npz -- the e2e / fb attacks at n = 100 on full_T128's inputs."""
    model = build(models, FULL_CFG)
    hashes = {k: sha(v) for k, v in model.state_dict().items()}
    X = make_inputs(2, {"vc_src": 280, "vc_tgt": 300, "adv_tgt": 260}, seed=300)
    out = {"config": np.array(json.dumps(FULL_CFG)), "eps": np.float64(EPS), "T": np.int64(300),
           "weight_sha256": np.array(json.dumps(hashes))}
    for k, v in X.items():
        out[k] = v.numpy()
    with torch.no_grad():
        out["se_vc_tgt"] = model.speaker_encoder(X["vc_tgt"]).numpy()
        out["se_adv_tgt"] = model.speaker_encoder(X["adv_tgt"]).numpy()
        out["inference"] = model.inference(X["vc_src"], X["vc_tgt"]).numpy()
    for kind in ("emb", "e2e", "fb"):
        attack_fixture(au, kind, model, X, [10], seeds, "", out, keep_losses=True)
    path = os.path.join(HERE, "full_T300.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path))

    X = make_inputs(2, 128, seed=128)              # full_T128.npz's inputs
    out = {"config": np.array(json.dumps(FULL_CFG)), "eps": np.float64(EPS), "T": np.int64(128),
           "weight_sha256": np.array(json.dumps(hashes))}
    for kind in ("e2e", "fb"):
        attack_fixture(au, kind, model, X, [100], seeds, "", out, keep_losses=True)
    path = os.path.join(HERE, "full_T128_n100.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path))


def long100_fixtures(models, au, seeds):
    """Round 4: full_T300_n100.npz -- full_T300.npz's inputs (vc_src 280, vc_tgt 300, adv_tgt 260
    frames, seed 300) attacked for 100 iterations by emb / e2e / fb: adv at n = 100, grad0 and the
    whole loss history (the long engine at the horizon of SURVEY 8(c)'s n = 100 tolerance)."""
    model = build(models, FULL_CFG)
    hashes = {k: sha(v) for k, v in model.state_dict().items()}
    X = make_inputs(2, {"vc_src": 280, "vc_tgt": 300, "adv_tgt": 260}, seed=300)
    out = {"config": np.array(json.dumps(FULL_CFG)), "eps": np.float64(EPS), "T": np.int64(300),
           "weight_sha256": np.array(json.dumps(hashes))}
    for kind in ("emb", "e2e", "fb"):
        attack_fixture(au, kind, model, X, [100], seeds, "", out, keep_losses=True)
    for k in list(out):   # the inputs and targets live in full_T300.npz (same seed); keep vectors only
        if k.endswith(("_org", "_tgt")) and not k.startswith(("vc_", "adv_")):
            del out[k]
    path = os.path.join(HERE, "full_T300_n100.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path))


if __name__ == "__main__":
    main()
