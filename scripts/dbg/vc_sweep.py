"""e2e / fb iteration-0 gradients, GPU vs numpy oracle (fp32 and fp64), per utterance,
over lengths and seeds: separates isolated fp32 ReLU-mask flips from systematic errors."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'attack-vc_amd'), ROOT]
import numpy as np, torch
from helpers import *
from oracle import adain_vc as oracle
import attack_utils
DEV = torch.device("cuda:0")
z = dict(np.load(os.path.join(ROOT, 'tests/golden/full_T128.npz')))
m = model_from_fixture(z)
sd = {k: v.detach().numpy() for k, v in m.state_dict().items()}
w32, w64 = oracle.Weights(sd, np.float32), oracle.Weights(sd, np.float64)
cfg = cfg_of(z)
md = m.to(DEV)
d = lambda t: t.to(DEV)
for T in [int(x) for x in sys.argv[1].split(",")]:
    for seed in range(int(sys.argv[2])):
        g = torch.Generator().manual_seed(1000 * T + seed)
        src, vc, at, p0 = (torch.randn(2, 80, T, generator=g) for _ in range(4))
        for kind in sys.argv[3].split(","):
            r32, r64 = {}, {}
            oracle.attack(kind, w32, cfg, src.numpy(), vc.numpy(), at.numpy(), 0.1, 1, p0.numpy(), record=r32)
            a = lambda t: t.numpy().astype(np.float64)
            oracle.attack(kind, w64, cfg, a(src), a(vc), a(at), 0.1, 1, a(p0), record=r64)
            fn = attack_utils.e2e_attack if kind == "e2e" else attack_utils.fb_attack
            _, info = fn(md, d(src), d(vc), d(at), 0.1, 1, ptb0=d(p0), return_info=True)
            gg = info["grad0"].cpu().numpy()
            print(f"T={T} seed={seed} {kind}: gpu-vs-64 " + " ".join(f"{rel(gg[u], r64['grad0'][u]):.1e}" for u in range(2)) +
                  "  o32-vs-64 " + " ".join(f"{rel(r32['grad0'][u], r64['grad0'][u]):.1e}" for u in range(2)), flush=True)
