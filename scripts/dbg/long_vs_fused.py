"""Debug: where do the fused and long engines differ at T <= 128 (fp32)?"""
import sys
import numpy as np
import torch
sys.path.insert(0, "attack-vc_amd"); sys.path.insert(0, "."); sys.path.insert(0, "tests")
import avc_native, helpers
z = np.load("tests/golden/full_T128.npz")
m = helpers.model_from_fixture(z).to("cuda:0")
ctx = avc_native.context_for(m.speaker_encoder, torch.device("cuda:0"))
for T in (128, 100, 64):
    g = torch.Generator().manual_seed(300 + T)
    vc, at, p0 = (torch.randn(3, 80, T, generator=g).cuda() for _ in range(3))
    out = {}
    for eng in ("fused", "long"):
        ctx.set_engine(eng)
        e = ctx.se_forward(vc)
        adv, L, g0 = ctx.emb_attack(vc, at, p0, 0.1, 1, want_losses=True, want_grad0=True)
        out[eng] = dict(e=e, L=L, g0=g0, adv=adv)
    for k in ("e", "L", "g0", "adv"):
        a, b = out["fused"][k], out["long"][k]
        d = (a - b).abs()
        idx = np.unravel_index(int(d.argmax()), tuple(d.shape))
        print(T, k, "equal" if torch.equal(a, b) else "DIFF", float(d.max()), "n_diff", int((d > 0).sum()), "at", idx, flush=True)
