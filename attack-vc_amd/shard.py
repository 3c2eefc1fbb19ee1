"""Multi-GPU data parallelism for the attack: the workload is embarrassingly
parallel over utterances (no cross-utterance op in the SpeakerEncoder, loss or
Adam), so a batch is split into contiguous shards, one per GPU,
with no data-path collective.

Two drivers:
  * one process per GPU (torchrun; bench.py): `shard_slice` picks the rank's
    utterances, `max_over_ranks` / `gather_shards` are the only collectives
    (timing and the final host-side gather);
  * one process, several GPUs (`attack_multi_gpu`, emb / e2e / fb): one host
    thread per device, each with its own libavc context and stream, results
    gathered on the first device.
"""
import threading
from typing import List, Optional, Sequence

import torch


def shard_slice(total: int, rank: int, world: int) -> slice:
    """Contiguous, as-even-as-possible shard of `total` utterances for `rank`."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, extra = divmod(total, world)
    lo = rank * base + min(rank, extra)
    return slice(lo, lo + base + (1 if rank < extra else 0))


def max_over_ranks(value: float, dist=None, device=None) -> float:
    """Max of a per-rank scalar (the elapsed time of a timed region)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_shards(shard: torch.Tensor, total: int, dist=None) -> torch.Tensor:
    """All-gather contiguous shards (possibly of unequal size) into [total, ...]."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return shard
    world = dist.get_world_size()
    sizes = [shard_slice(total, r, world).stop - shard_slice(total, r, world).start for r in range(world)]
    mx = max(sizes)
    pad = torch.zeros((mx,) + tuple(shard.shape[1:]), dtype=shard.dtype, device=shard.device)
    pad[: shard.shape[0]] = shard
    outs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad)
    return torch.cat([o[:n] for o, n in zip(outs, sizes)], dim=0)


def attack_multi_gpu(kind: str, model_per_device: Sequence[torch.nn.Module], vc_src: Optional[torch.Tensor],
                     vc_tgt: torch.Tensor, adv_tgt: torch.Tensor, eps: float, n_iters: int,
                     ptb0: Optional[torch.Tensor] = None, precision: str = "fp32") -> torch.Tensor:
    """emb / e2e / fb attack (attack_utils.py:51-86 / 7-48 / 89-130) over len(model_per_device)
    GPUs from one process: one host thread per device, each attacking a contiguous utterance
    shard with its own libavc context and stream; the results are gathered on the first
    device.  model_per_device[i] must live on its own device; inputs may live anywhere.
    Utterance b of the result equals a single-GPU attack of utterance b (the shards share
    nothing).  This is configs[3]'s path (fb, B = 2048 over 8 GPUs) without torchrun."""
    import attack_utils

    if kind not in ("emb", "e2e", "fb"):
        raise ValueError(f"unknown attack {kind!r}")
    if kind != "emb" and vc_src is None:
        raise ValueError("e2e / fb attacks need vc_src")
    devs = [next(m.parameters()).device for m in model_per_device]
    B = vc_tgt.shape[0]
    if ptb0 is None:
        # drawn on the first model's device, as the reference draws it on the attack's device
        # (attack_utils.py:68): a seeded caller gets the single-GPU perturbation bit for bit
        ptb0 = torch.zeros(vc_tgt.shape, dtype=torch.float32, device=devs[0]).normal_(0, 1)
    outs: List[Optional[torch.Tensor]] = [None] * len(devs)
    errs: List[BaseException] = []

    def work(i: int):
        try:
            sl = shard_slice(B, i, len(devs))
            if sl.stop <= sl.start:
                return
            d = devs[i]
            with torch.cuda.device(d):
                if kind == "emb":
                    o = attack_utils.emb_attack(model_per_device[i], vc_tgt[sl].to(d), adv_tgt[sl].to(d), eps,
                                                n_iters, ptb0=ptb0[sl].to(d), precision=precision)
                else:
                    fn = attack_utils.e2e_attack if kind == "e2e" else attack_utils.fb_attack
                    o = fn(model_per_device[i], vc_src[sl].to(d), vc_tgt[sl].to(d), adv_tgt[sl].to(d), eps, n_iters,
                           ptb0=ptb0[sl].to(d), precision=precision)
                torch.cuda.current_stream(d).synchronize()
            outs[i] = o.detach()
        except BaseException as e:  # re-raised on the calling thread
            errs.append(e)

    threads = [threading.Thread(target=work, args=(i,)) for i in range(len(devs))]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errs:
        raise errs[0]
    return torch.cat([o.to(devs[0]) for o in outs if o is not None], dim=0).requires_grad_(True)


def emb_attack_multi_gpu(model_per_device: Sequence[torch.nn.Module], vc_tgt: torch.Tensor, adv_tgt: torch.Tensor,
                         eps: float, n_iters: int, ptb0: Optional[torch.Tensor] = None,
                         precision: str = "fp32") -> torch.Tensor:
    """emb_attack over len(model_per_device) GPUs from one process (attack_multi_gpu)."""
    return attack_multi_gpu("emb", model_per_device, None, vc_tgt, adv_tgt, eps, n_iters, ptb0, precision)
