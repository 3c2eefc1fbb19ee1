"""GPU side of the fp32 tolerance calibration (tests/helpers.py TOL_ADV).

Runs the reference-golden cases of tests/golden/full_T128.npz through libavc in fp32 on
cuda:0 -- emb at n = 1 / 10 / 100 / 1500, e2e and fb at n = 1 / 10 / 100 -- on every engine
that runs the standard shape (fused, layered for emb, long forced), and writes the adversarial
mels, the iteration-0 gradients and the loss histories to gpurun_out/calib_gpu.npz.
scripts/tol_calibration.py then sets them beside the reference's own fp32 run (the goldens)
and its float64 run (tests/golden/calib_f64_T128.npz) on the CPU.

Usage (GPU box):  python scripts/calib_dump.py [out.npz]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "attack-vc_amd"), os.path.join(ROOT, "tests")]

import attack_utils  # noqa: E402
from avc_native import context_for  # noqa: E402
from helpers import model_from_fixture  # noqa: E402

FN = {"emb": attack_utils.emb_attack, "e2e": attack_utils.e2e_attack, "fb": attack_utils.fb_attack}


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "calib_gpu.npz")
    dev = torch.device("cuda:0")
    z = dict(np.load(os.path.join(ROOT, "tests", "golden", "full_T128.npz")))
    m = model_from_fixture(z).to(dev)
    t = {k: torch.from_numpy(z[k]).to(dev) for k in ("vc_src", "vc_tgt", "adv_tgt")}
    ctx = context_for(m.speaker_encoder, dev)
    res = {}
    for engine in ("fused", "layered", "long"):
        ctx.set_engine(engine)
        for kind, ns in (("emb", (1, 10, 100, 1500)), ("e2e", (1, 10, 100)), ("fb", (1, 10, 100))):
            if kind != "emb" and engine == "layered":
                continue    # the VC attacks need the fused or long shape
            p0 = torch.from_numpy(z[f"{kind}_ptb0"]).to(dev)
            for n in ns:
                if kind == "emb":
                    adv, info = FN[kind](m, t["vc_tgt"], t["adv_tgt"], 0.1, n, ptb0=p0, return_info=True)
                else:
                    adv, info = FN[kind](m, t["vc_src"], t["vc_tgt"], t["adv_tgt"], 0.1, n, ptb0=p0,
                                         return_info=True)
                key = f"{engine}/{kind}/n{n}"
                res[key + "/adv"] = adv.detach().cpu().numpy()
                res[key + "/losses"] = info["losses"].cpu().numpy()
                if n == 1:
                    res[f"{engine}/{kind}/grad0"] = info["grad0"].cpu().numpy()
                print(key, flush=True)
    ctx.set_engine("auto")
    os.makedirs(os.path.dirname(out_path), exist_ok=True)
    np.savez_compressed(out_path, **res)
    print("wrote", out_path)


if __name__ == "__main__":
    main()
