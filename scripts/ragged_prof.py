"""Profiled process for the mixed-length line's PMC passes (scripts/pmc_ragged.sh): the workload of
`bench.py --lengths LO:HI` (same model seed, same lengths, vc and ptb0 as rank 0 at N=1; drawn target embeddings), ITERS iterations of
ONE ragged embedding attack (avc_emb_attack_ragged) in the longest-first order attack_many uses.  Prints
libavc's version line (`libavc ... src=...`) to stderr like avc_bench, so fz_summary.py stamps the source.

  python3 scripts/ragged_prof.py LO HI [ITERS] [B]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "attack-vc_amd"))
sys.path.insert(0, ROOT)

import avc_native  # noqa: E402
import models  # noqa: E402
from bench import FULL_CFG  # noqa: E402


def main():
    lo, hi = int(sys.argv[1]), int(sys.argv[2])
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 256
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = models.AdaInVC(FULL_CFG).to(dev)
    g = torch.Generator().manual_seed(2)
    lens = torch.randint(lo, hi + 1, (B,), generator=g).tolist()
    gi = torch.Generator().manual_seed(3)
    vc = [torch.randn(80, t, generator=gi).to(dev) for t in lens]
    p0 = [torch.randn(80, t, generator=gi).to(dev) for t in lens]
    ctx = avc_native.context_for(model.speaker_encoder, dev)
    # target embeddings drawn, not computed: the per-length se_forward launches would mix B=1 long-engine
    # forwards into the attack kernels' statistics (the targets do not change the attack's work)
    te = torch.randn(B, 128, generator=gi).to(dev) * 0.1
    order = sorted(range(B), key=lambda i: (-lens[i], i))
    print(avc_native.lib().avc_version().decode(), file=sys.stderr, flush=True)
    outs, _, _ = ctx.emb_attack_ragged([vc[i] for i in order], te[order], [p0[i] for i in order], 0.1, iters,
                                       precision="bf16")
    torch.cuda.synchronize()
    assert all(torch.isfinite(o).all() for o in outs)
    print(f"ragged_prof: B={B} lengths [{lo}, {hi}] mean {sum(lens) / B:.1f} frames, {iters} iterations: ok",
          file=sys.stderr, flush=True)


if __name__ == "__main__":
    main()
