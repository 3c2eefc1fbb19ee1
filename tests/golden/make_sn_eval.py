"""Spectral-norm Decoder in EVAL mode from the REAL reference -> tests/golden/full_sn_eval_T128.npz.

Test infrastructure only; runs in the build container and imports the reference's ``models.py`` /
``attack_utils.py`` read-only (the .npz holds input / output vectors only).

The reference itself never calls .eval() (make_sn.py pins that train-mode path).  A user who does --
e.g. because a Decoder with dropout_rate > 0 is refused in training mode -- gets torch's eval-mode
spectral_norm hook: no power iteration, sigma = u . (W v) from the stored weight_u / weight_v, the
buffers unchanged.  This fixture pins that path on full_sn_T128's model (seed 0) and inputs:
  * inference(vc_src, vc_tgt) of the eval-mode model (u / v as initialised) and, to make the stored
    state non-trivial, inference again after one train-mode forward moved u / v;
  * the e2e attack at n = 10 per utterance in eval mode (the Decoder's weights then stay fixed):
    adv and ptb0 (the reference function's own run), grad0 (make_golden.py's instrumented loop, bitwise
    the same adv);
  * the u / v after all of it (must equal the ones before each eval-mode call).

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_sn_eval.py
"""
import copy
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import EPS, instrumented, make_inputs, run_reference, sha  # noqa: E402
from make_sn import SN_CFG, uv  # noqa: E402


def main(ref="/root/reference"):
    import json
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
    m = copy.deepcopy(model).eval()
    u0 = uv(m)
    with torch.no_grad():
        out["inference_eval"] = m.inference(X["vc_src"], X["vc_tgt"]).numpy()
    for k, v in uv(m).items():
        assert np.array_equal(v, u0[k]), k            # eval mode leaves the buffers alone
    m.train()
    with torch.no_grad():
        m.inference(X["vc_src"], X["vc_tgt"])          # one power iteration: u / v move
    m.eval()
    u1 = uv(m)
    for k, v in u1.items():
        out["uv1/" + k] = v
    with torch.no_grad():
        out["inference_eval_uv1"] = m.inference(X["vc_src"], X["vc_tgt"]).numpy()
    seeds = [2000, 2001]
    advs, ptb0s, grads = [], [], []
    for b in range(2):
        args = [X[k][b:b + 1] for k in ("vc_src", "vc_tgt", "adv_tgt")]
        mr = copy.deepcopy(model).eval()
        advs.append(run_reference(au, "e2e", mr, *args, EPS, 10, seeds[b]))
        ins = instrumented("e2e", copy.deepcopy(model).eval(), *args, EPS, 10, seeds[b])
        assert torch.equal(ins["adv"], advs[-1])                 # the same arithmetic, plus the gradient
        ptb0s.append(ins["ptb0"])
        grads.append(ins["grad0"])
        for k, v in uv(mr).items():
            assert np.array_equal(v, u0[k]), k
    out["e2e_adv_n10_eval"] = torch.cat(advs).detach().numpy()
    out["e2e_ptb0_eval"] = torch.cat(ptb0s).numpy()
    out["e2e_grad0_eval"] = torch.cat(grads).numpy()
    path = os.path.join(HERE, "full_sn_eval_T128.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path))


if __name__ == "__main__":
    main(*(sys.argv[1:2]))
