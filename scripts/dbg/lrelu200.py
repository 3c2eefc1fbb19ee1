"""Diagnostic: long-engine grad0 vs float64 oracle at T=200 (lrelu / relu), with and without a
prior se_forward at the attack's shape (workspace reuse)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "attack-vc_amd"), os.path.join(ROOT, "tests")]
import numpy as np, torch
import attack_utils, avc_native
from helpers import model_from_fixture, cfg_of, rel
from oracle import adain_vc as oracle
DEV = torch.device("cuda:0")
for name in ("full_lrelu_T128", "full_T128"):
    z = dict(np.load(os.path.join(ROOT, "tests/golden", name + ".npz")))
    cfg = cfg_of(z)
    for T in (200, 300, 176, 208):
        for prior in (False, True):
            m = model_from_fixture(z).to(DEV)
            sd = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
            w64 = oracle.Weights(sd, dtype=np.float64)
            ctx = avc_native.context_for(m.speaker_encoder, DEV)
            g = torch.Generator().manual_seed(700 + T)
            vc, p0 = (torch.randn(2, 80, T, generator=g) for _ in range(2))
            at = torch.randn(2, 80, T - 21, generator=g)
            if prior:
                ctx.se_forward(vc.to(DEV))
            _, info = attack_utils.emb_attack(m, vc.to(DEV), at.to(DEV), 0.1, 1, ptb0=p0.to(DEV), return_info=True)
            rec = {}
            oracle.emb_attack(w64, cfg, vc.double().numpy(), at.double().numpy(), 0.1, 1, p0.double().numpy(), record=rec)
            gg = info["grad0"].cpu().numpy()
            d = np.abs(gg - rec["grad0"]) / np.abs(rec["grad0"]).max()
            bad = np.argwhere(d > 1e-4)
            cols = sorted(set(int(x) for x in bad[:, 2]))[:20]
            utts = sorted(set(int(x) for x in bad[:, 0]))
            print(f"{name} T={T} prior={prior} rel={d.max():.3e} nbad={len(bad)} utts={utts} cols={cols}", flush=True)
            del ctx, m
            avc_native._ctx_cache.clear()
