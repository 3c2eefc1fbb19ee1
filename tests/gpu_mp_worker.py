"""One rank of tests/test_gpu_multiproc.py: a separate process running libavc's HIP path on
its contiguous shard (shard.shard_slice), host-side gather over gloo, result saved by rank 0.
Not a test module; started as a child process by the test."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "attack-vc_amd"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

import attack_utils  # noqa: E402
import models  # noqa: E402
import shard  # noqa: E402
from bench import FULL_CFG  # noqa: E402


def inputs(total, T):
    g = torch.Generator().manual_seed(5)
    vc, at, src = (torch.randn(total, 80, T, generator=g) for _ in range(3))
    p0 = torch.randn(total, 80, T, generator=torch.Generator().manual_seed(6))
    return vc, at, src, p0


def run(kind, vc, at, src, p0, dev, n_iters, precision):
    torch.manual_seed(0)
    m = models.AdaInVC(FULL_CFG).eval().to(dev)
    args = [t.to(dev) for t in (vc, at, src, p0)]
    if kind == "emb":
        return attack_utils.emb_attack(m, args[0], args[1], 0.1, n_iters, ptb0=args[3], precision=precision)
    return attack_utils.fb_attack(m, args[2], args[0], args[1], 0.1, n_iters, ptb0=args[3], precision=precision)


def main():
    kind, total, T, n_iters, precision, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), \
        sys.argv[5], sys.argv[6]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)          # every rank on the one GPU of the box
    torch.cuda.set_device(dev)
    vc, at, src, p0 = inputs(total, T)
    sl = shard.shard_slice(total, rank, world)
    adv = run(kind, vc[sl], at[sl], src[sl], p0[sl], dev, n_iters, precision).detach().cpu()
    full = shard.gather_shards(adv, total, dist)
    t = shard.max_over_ranks(float(rank), dist)
    if rank == 0:
        assert t == world - 1
        np.save(out, full.numpy())
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
