"""Golden fixture for the LeakyReLU variant of the AdaIN-VC config (act="lrelu" in every
module, models.py:107-118 get_act) from the REAL reference: tests/golden/full_lrelu_T128.npz.

Test infrastructure only (build container).  Same procedure as make_golden.py (whose
instrumented loop and fixture helpers it reuses): weights regenerated from
torch.manual_seed(0) and pinned by per-tensor SHA-256, inputs seeded, attack vectors
asserted bitwise-equal to the reference's own attack_utils functions.  The fused GPU
kernels run this config on their generic (runtime-activation) shapes.

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_lrelu.py
"""
import argparse
import copy
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    a = ap.parse_args()
    sys.dont_write_bytecode = True
    sys.path.insert(0, a.ref)
    import models  # noqa: E402  (reference, read-only)
    import attack_utils as au  # noqa: E402
    torch.set_num_threads(os.cpu_count() or 1)
    cfg = copy.deepcopy(mg.FULL_CFG)
    for k in cfg:
        cfg[k]["act"] = "lrelu"
    T = 128
    model = mg.build(models, cfg)
    X = mg.make_inputs(2, T, seed=331)
    out = {"config": np.array(json.dumps(cfg)), "eps": np.float64(mg.EPS), "T": np.int64(T)}
    out["weight_sha256"] = np.array(json.dumps({k: mg.sha(v) for k, v in model.state_dict().items()}))
    for k, v in X.items():
        out[k] = v.numpy()
    with torch.no_grad():
        out["se_vc_tgt"] = model.speaker_encoder(X["vc_tgt"]).numpy()
        out["inference"] = model.inference(X["vc_src"], X["vc_tgt"]).numpy()
    seeds = [2000, 2001]
    for kind in ("emb", "e2e", "fb"):
        mg.attack_fixture(au, kind, model, X, [10], seeds, "", out, keep_losses=True)
    path = os.path.join(HERE, "full_lrelu_T128.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path))


if __name__ == "__main__":
    main()
