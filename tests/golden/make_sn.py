"""Spectral-norm Decoder fixture (sn=True) from the REAL reference -> tests/golden/full_sn_T128.npz.

Test infrastructure only; runs in the build container and imports the reference's ``models.py`` /
``attack_utils.py`` read-only (nothing of it is copied: the .npz holds input / output vectors).

The reference wraps every Decoder layer in torch.nn.utils.spectral_norm when the config says
sn=True (models.py:382) and never calls .eval() (data_utils.py:200-223, attack.py:38), so every
Decoder forward runs one power iteration and updates the layers' weight_u / weight_v buffers --
inside the attack loop too (attack_utils.py:35-43, 117-125).  The fixture pins that:
  * the model: FULL_CFG with Decoder sn=True, torch.manual_seed(0) (weights AND the initial u / v
    draws pinned by per-tensor SHA-256);
  * inference(vc_src, vc_tgt) of a fresh model and the u / v after it;
  * e2e / fb attacks at n = 10 per utterance, each from a fresh copy of the model (the power
    iteration does not depend on the data, so every utterance sees the same sigma sequence):
    adv, grad0, the loss history, ptb0, and the u / v after the attack.  Each attack is produced by
    the reference function itself and by make_golden.py's instrumented loop (bitwise equal).

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_sn.py
"""
import copy
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import EPS, FULL_CFG, instrumented, make_inputs, run_reference, sha  # noqa: E402

SN_CFG = json.loads(json.dumps(FULL_CFG))
SN_CFG["Decoder"]["sn"] = True


def uv(model):
    """weight_u / weight_v of every Decoder layer, state_dict order."""
    return {k: v.detach().clone().numpy() for k, v in model.decoder.state_dict().items() if k.endswith(("_u", "_v"))}


def main(ref="/root/reference"):
    sys.dont_write_bytecode = True
    sys.path.insert(0, ref)
    import attack_utils as au  # noqa: E402  (reference, read-only)
    import models  # noqa: E402
    torch.set_num_threads(os.cpu_count() or 1)
    torch.manual_seed(0)
    model = models.AdaInVC(SN_CFG)
    sd = model.state_dict()
    out = {"config": np.array(json.dumps(SN_CFG)), "eps": np.float64(EPS), "T": np.int64(128),
           "weight_sha256": np.array(json.dumps({k: sha(v) for k, v in sd.items()}))}
    X = make_inputs(2, 128, seed=128)
    for k, v in X.items():
        out[k] = v.numpy()
    for k, v in uv(model).items():
        out["uv0/" + k] = v
    m = copy.deepcopy(model)
    with torch.no_grad():
        out["inference"] = m.inference(X["vc_src"], X["vc_tgt"]).numpy()
    for k, v in uv(m).items():
        out["uv_inference/" + k] = v
    seeds = [1000, 1001]
    for kind in ("e2e", "fb"):
        advs, grads, losses, ptb0s = [], [], [], []
        for b in range(2):
            args = [X[k][b:b + 1] for k in ("vc_src", "vc_tgt", "adv_tgt")]
            ins = instrumented(kind, copy.deepcopy(model), *args, EPS, 10, seeds[b])
            mr = copy.deepcopy(model)
            ref_adv = run_reference(au, kind, mr, *args, EPS, 10, seeds[b])
            assert torch.equal(ins["adv"], ref_adv), (kind, b)
            advs.append(ref_adv)
            grads.append(ins["grad0"])
            losses.append(ins["losses"])
            ptb0s.append(ins["ptb0"])
            if b == 0:
                for k, v in uv(mr).items():
                    out[f"uv_{kind}/" + k] = v
            else:   # the power iteration is data-independent: every utterance ends in the same state
                for k, v in uv(mr).items():
                    assert np.array_equal(out[f"uv_{kind}/" + k], v), k
        out[f"{kind}_adv_n10"] = torch.cat(advs).numpy()
        out[f"{kind}_grad0"] = torch.cat(grads).numpy()
        out[f"{kind}_ptb0"] = torch.cat(ptb0s).numpy()
        out[f"{kind}_losses_n10"] = np.stack(losses)
    path = os.path.join(HERE, "full_sn_T128.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path))


if __name__ == "__main__":
    main(*(sys.argv[1:2]))
