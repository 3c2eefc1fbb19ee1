"""Debug: which precision / split breaks shard invariance on the fused engine."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "attack-vc_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import torch, numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
from helpers import model_from_fixture
import avc_native
z = dict(np.load(os.path.join(os.path.dirname(__file__), "..", "..", "tests", "golden", "full_T128.npz")))
DEV = torch.device("cuda:0")
m = model_from_fixture(z).to(DEV)
ctx = avc_native.context_for(m.speaker_encoder, DEV)
g = torch.Generator().manual_seed(31)
vc, at, p0 = (torch.randn(20, 80, 128, generator=g).to(DEV) for _ in range(3))
for prec in ("fp32", "bf16"):
    for n in (0, 1, 12):
        a, L, _ = ctx.emb_attack(vc, at, p0, 0.1, n, precision=prec, want_losses=n > 0)
        for cut in (7, 8):
            lo, L1, _ = ctx.emb_attack(vc[:cut], at[:cut], p0[:cut], 0.1, n, precision=prec, want_losses=n > 0)
            hi, L2, _ = ctx.emb_attack(vc[cut:], at[cut:], p0[cut:], 0.1, n, precision=prec, want_losses=n > 0)
            d = (torch.cat([lo, hi]) - a).abs().amax(dim=(1, 2))
            dl = (torch.cat([L1, L2], 1) - L).abs().amax(0) if n > 0 else None
            print(prec, "n", n, "cut", cut, "adv diff per utt", [f"{x:.1e}" for x in d.tolist()],
                  "loss diff", None if dl is None else [f"{x:.1e}" for x in dl.tolist()])
