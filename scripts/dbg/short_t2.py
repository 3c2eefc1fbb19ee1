import sys, os
R = os.path.join(os.path.dirname(__file__), "..", "..")
for p in (R, os.path.join(R, "attack-vc_amd"), os.path.join(R, "tests")):
    sys.path.insert(0, p)
import torch, numpy as np
from helpers import model_from_fixture
import avc_native
z = dict(np.load(os.path.join(R, "tests", "golden", "full_T128.npz")))
DEV = torch.device("cuda:0")
m = model_from_fixture(z).to(DEV)
ctx = avc_native.context_for(m.speaker_encoder, DEV)
for T in (12, 16, 17):
    for B in (1, 2, 4):
        x = torch.randn(B, 80, T, generator=torch.Generator().manual_seed(T)).to(DEV)
        ctx.set_engine("layered"); ref = ctx.se_forward(x)
        ctx.set_engine("fused")
        outs = [ctx.se_forward(x) for _ in range(3)]
        d = [float((o - ref).abs().max() / ref.abs().max()) for o in outs]
        per = ((outs[0] - ref).abs().amax(1) / ref.abs().max()).tolist()
        print(T, B, "runs", [f"{v:.1e}" for v in d], "per-utt", [f"{v:.1e}" for v in per], flush=True)
        ctx.set_engine("fused")
        a, L, g = ctx.emb_attack(x, x.flip(0), x * 0.5, 0.1, 1, want_grad0=True)
        ctx.set_engine("layered")
        a2, L2, g2 = ctx.emb_attack(x, x.flip(0), x * 0.5, 0.1, 1, want_grad0=True)
        print("   grad0 rel", f"{float((g - g2).abs().max() / g2.abs().max()):.1e}", flush=True)
