"""bf16-mode head diagnostic: losses / grad0 of a 1-3 iteration emb attack, fp32 vs bf16."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "attack-vc_amd"), os.path.join(ROOT, "tests")]
import avc_native
from helpers import model_from_fixture
z = np.load(os.path.join(ROOT, "tests/golden/full_T128.npz"))
DEV = torch.device("cuda:0")
m = model_from_fixture(z).to(DEV)
ctx = avc_native.context_for(m.speaker_encoder, DEV)
g = torch.Generator().manual_seed(77)
vc, at, p0 = (torch.randn(4, 80, 128, generator=g).to(DEV) for _ in range(3))
r = {}
for prec in ("fp32", "bf16"):
    for gr in (True, False):
        a, l, g0 = ctx.emb_attack(vc, at, p0, 0.1, 3, precision=prec, want_losses=True, want_grad0=True, use_graph=gr)
        r[prec, gr] = (a.cpu().numpy(), l.cpu().numpy(), g0.cpu().numpy())
        print(prec, "graph" if gr else "eager", "losses", l.cpu().numpy()[:, :2].ravel(), "|g0|", np.abs(g0.cpu().numpy()).max())
with torch.no_grad():
    e = m.speaker_encoder(vc).cpu().numpy()
    print("torch emb[0,:4]", e[0, :4])
a, b = r["fp32", True][2].reshape(4, -1), r["bf16", True][2].reshape(4, -1)
print("cos", (a * b).sum(1) / np.linalg.norm(a, axis=1) / np.linalg.norm(b, axis=1))
