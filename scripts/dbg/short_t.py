import sys, os
R = os.path.join(os.path.dirname(__file__), "..", "..")
for p in (R, os.environ.get("AVC_PKG", os.path.join(R, "attack-vc_amd")), os.path.join(R, "tests")):
    sys.path.insert(0, p)
import torch, numpy as np
from helpers import model_from_fixture, oracle_weights, rel, cfg_of
from oracle import adain_vc as oracle
import avc_native
z = dict(np.load(os.path.join(R, "tests", "golden", "full_T128.npz")))
DEV = torch.device("cuda:0")
m = model_from_fixture(z).to(DEV)
ctx = avc_native.context_for(m.speaker_encoder, DEV)
W = oracle_weights(m)
for T in (9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 20, 24, 31, 32):
    x = torch.randn(3, 80, T, generator=torch.Generator().manual_seed(T))
    ctx.set_engine("fused")
    e = ctx.se_forward(x.to(DEV)).cpu().numpy()
    eo, _ = oracle.se_forward(W, cfg_of(z)["SpeakerEncoder"], x.numpy())
    print(T, f"{rel(e, eo):.2e}", flush=True)
