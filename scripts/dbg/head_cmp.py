"""bf16 emb attack, fused MFMA head vs the separate VALU head (AVC_FUSE_HEAD=0) vs fp32: loss and grad0."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "attack-vc_amd"), os.path.join(ROOT, "tests")]
import avc_native
from helpers import model_from_fixture
DEV = torch.device("cuda:0")
z = dict(np.load(os.path.join(ROOT, "tests", "golden", "full_T128.npz")))
m = model_from_fixture(z).to(DEV)
g = torch.Generator().manual_seed(41)
vc, at, p0 = (torch.randn(6, 80, 128, generator=g).to(DEV) for _ in range(3))
def mk():
    c = avc_native.Context(avc_native.se_config(m.speaker_encoder), avc_native.flat_weights(m.speaker_encoder), 0)
    c.set_engine("fused")
    return c
c1 = mk()
res = {}
for n in (1, 12):
    res[("mfma", n)] = c1.emb_attack(vc, at, p0, 0.1, n, precision="bf16", want_losses=True, want_grad0=True)
    res[("f32", n)] = c1.emb_attack(vc, at, p0, 0.1, n, precision="fp32", want_losses=True, want_grad0=True)
os.environ["AVC_FUSE_HEAD"] = "0"
c2 = mk()
for n in (1, 12):
    res[("valu", n)] = c2.emb_attack(vc, at, p0, 0.1, n, precision="bf16", want_losses=True, want_grad0=True)
def rel(a, b):
    a = a.double().reshape(6, -1); b = b.double().reshape(6, -1)
    return ((a - b).norm(dim=1) / b.norm(dim=1)).cpu().numpy()
for n in (1, 12):
    for x, y in (("mfma", "valu"), ("mfma", "f32"), ("valu", "f32")):
        A, B = res[(x, n)], res[(y, n)]
        print(f"n={n} {x} vs {y}: grad0 rel {np.array2string(rel(A[2], B[2]), precision=2)}  "
              f"loss rel {float(((A[1] - B[1]) / B[1]).abs().max()):.2e}  adv max {float((A[0] - B[0]).abs().max()):.2e}")
print("losses n=1", res[("mfma", 1)][1].cpu().numpy(), res[("valu", 1)][1].cpu().numpy(), res[("f32", 1)][1].cpu().numpy())
