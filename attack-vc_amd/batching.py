"""Length-bucketed batching for real data (hard part 4).

The reference attacks one utterance per call, at the length its wav gave it
(/root/reference/attack.py:41-56 loads vc_tgt, adv_tgt and vc_src from three files).  Reflect
padding, ceil-mode pooling and InstanceNorm statistics all depend on that length
(models.py:10-30, 206, 176), so utterances of different lengths cannot be zero-padded into one
batch.  `attack_many` therefore

  1. embeds every adv_tgt once, grouped by ITS length (the reference embeds adv_tgt on its own,
     attack_utils.py:74-75 / 117-119), one batched SpeakerEncoder forward per distinct length;
  2. groups the attacked utterances into buckets of equal shape -- T of vc_tgt for the emb
     attack, (T of vc_tgt, T of vc_src) for e2e / fb -- cut into chunks of at most `max_batch`;
  3. deals the chunks to the devices (largest first, each to the device with the least work so
     far: B x T x n_iters), one host thread per device, each with its own libavc context and
     stream (no collective: the attacks share nothing);
  4. returns the adversarial mels in input order.

Every chunk runs the same per-utterance arithmetic as a single-utterance call (the kernels are
batch-invariant, tests/test_gpu_parity.py::test_batch_shard_invariance), so utterance i of the
result equals attack_utils.*_attack on utterance i alone, bit for bit.

ragged=True (emb attack): instead of one batch per length, ONE ragged batch per chunk of up to
max_batch utterances of ANY lengths (avc_emb_attack_ragged: every SpeakerEncoder pass is one launch,
each workgroup its own utterance length, on the long engine), longest first so that neighbouring
workgroups -- dealt round-robin over the 8 XCDs -- carry similar work.  With real data's spread of
lengths the per-length buckets are mostly of one or two utterances (a handful of the 256 CUs busy);
the ragged batch keeps every CU busy.  Utterance i then equals its single-utterance attack on the long
engine (AVC_ENGINE_LONG) bit for bit -- the fused engine's result too in fp32, where the two engines
are bitwise equal (tests/test_gpu_long.py).  libavc caches one
workspace (buffers, plans, captured graphs) per shape, and attack_many sizes that cache to the
shapes it uses, so a second call over the same lengths re-plans nothing (avc_ws_stats).
"""
import threading
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from avc_native import check_no_train_dropout, context_for, vc_context_for


def buckets(keys: Sequence, max_batch: int) -> List[List[int]]:
    """Indices grouped by equal key, each group in input order and cut into chunks of at most
    max_batch; chunks ordered by key of first appearance."""
    if max_batch < 1:
        raise ValueError("max_batch must be >= 1")
    groups: Dict = {}
    for i, k in enumerate(keys):
        groups.setdefault(k, []).append(i)
    out = []
    for idx in groups.values():
        for s in range(0, len(idx), max_batch):
            out.append(idx[s:s + max_batch])
    return out


def assign(costs: Sequence[float], n_dev: int) -> List[List[int]]:
    """Greedy longest-processing-time assignment of jobs (by cost) to n_dev devices; each device's
    list keeps ascending job order."""
    load = [0.0] * n_dev
    own: List[List[int]] = [[] for _ in range(n_dev)]
    for j in sorted(range(len(costs)), key=lambda j: (-costs[j], j)):
        d = min(range(n_dev), key=lambda d: (load[d], d))
        load[d] += costs[j]
        own[d].append(j)
    return [sorted(o) for o in own]


def _mel(name: str, t: torch.Tensor) -> torch.Tensor:
    if t.dim() == 3 and t.shape[0] == 1:
        t = t[0]
    if t.dim() != 2:
        raise ValueError(f"{name}: expected one [80, T] mel per utterance, got {tuple(t.shape)}")
    return t


def attack_many(kind: str, model_per_device: Sequence[torch.nn.Module], vc_tgts: Sequence[torch.Tensor],
                adv_tgts: Sequence[torch.Tensor], eps: float, n_iters: int,
                vc_srcs: Optional[Sequence[torch.Tensor]] = None, ptb0s: Optional[Sequence[torch.Tensor]] = None,
                precision: str = "fp32", max_batch: int = 256, ragged: bool = False) -> List[torch.Tensor]:
    """emb / e2e / fb attack (attack_utils.py:51-86 / 7-48 / 89-130) of a list of utterances of any
    lengths: vc_tgts[i] [80, T_i], adv_tgts[i] [80, T'_i], vc_srcs[i] [80, S_i] (e2e / fb).
    Returns [vc_tgts[i] + eps * tanh(ptb_i)] ([80, T_i] each, on the first model's device).
    ptb0s[i] ([80, T_i]) as the reference's N(0,1) draw; drawn per utterance in input order on
    the first model's device when omitted (attack_utils.py:68)."""
    if kind not in ("emb", "e2e", "fb"):
        raise ValueError(f"unknown attack {kind!r}")
    n = len(vc_tgts)
    if len(adv_tgts) != n or (vc_srcs is not None and len(vc_srcs) != n) or (ptb0s is not None and len(ptb0s) != n):
        raise ValueError("vc_tgts, adv_tgts, vc_srcs and ptb0s must have one entry per utterance")
    if kind != "emb" and vc_srcs is None:
        raise ValueError("e2e / fb attacks need vc_srcs")
    if n == 0:
        return []
    devs = [next(m.parameters()).device for m in model_per_device]
    for m in model_per_device:
        check_no_train_dropout(m.speaker_encoder)
    vc_tgts = [_mel("vc_tgt", t) for t in vc_tgts]
    adv_tgts = [_mel("adv_tgt", t) for t in adv_tgts]
    vc_srcs = None if vc_srcs is None else [_mel("vc_src", t) for t in vc_srcs]
    if ptb0s is None:
        ptb0s = [torch.zeros(t.shape, dtype=torch.float32, device=devs[0]).normal_(0, 1) for t in vc_tgts]
    ptb0s = [_mel("ptb0", t) for t in ptb0s]
    for i in range(n):
        if ptb0s[i].shape != vc_tgts[i].shape:
            raise ValueError(f"utterance {i}: ptb0 {tuple(ptb0s[i].shape)} != vc_tgt {tuple(vc_tgts[i].shape)}")

    if ragged and kind != "emb":
        raise ValueError("ragged batches are built for the emb attack only")
    # the attack chunks: equal (T, S) within a chunk -- or, ragged, any lengths, longest first
    keys = [(vc_tgts[i].shape[1], vc_srcs[i].shape[1] if vc_srcs is not None else 0) for i in range(n)]
    if ragged:
        order = sorted(range(n), key=lambda i: (-keys[i][0], i))
        chunks = [order[s:s + max_batch] for s in range(0, n, max_batch)]
    else:
        chunks = buckets(keys, max_batch)
    owner = assign([sum(keys[i][0] for i in c) * max(n_iters, 1) for c in chunks], len(devs))
    # per device: the adv_tgt embeddings it needs, grouped by adv_tgt length
    need = [sorted({i for j in owner[d] for i in chunks[j]}) for d in range(len(devs))]
    results: List[Optional[torch.Tensor]] = [None] * n
    errs: List[BaseException] = []

    def work(d: int):
        try:
            if not owner[d]:
                return
            dev = devs[d]
            m = model_per_device[d]
            with torch.cuda.device(dev):
                ctx = context_for(m.speaker_encoder, dev) if kind == "emb" else vc_context_for(m, dev)
                adv_groups = buckets([adv_tgts[i].shape[1] for i in need[d]], max_batch)
                # distinct shapes this device runs: embeddings, attacks (+ their forward plans);
                # the cache holds them all, so a repeated call over the same lengths re-plans nothing
                shapes = {(len(g), adv_tgts[need[d][g[0]]].shape[1]) for g in adv_groups}
                shapes |= {(len(chunks[j]), keys[chunks[j][0]][0]) if not ragged else tuple(chunks[j]) for j in owner[d]}
                # e2e / fb: the ContentEncoder / Decoder workspaces are keyed by (B, T, T_src) and share
                # the cap with the SpeakerEncoder ones
                vc_shapes = {(len(chunks[j]),) + tuple(keys[chunks[j][0]]) for j in owner[d]} if kind != "emb" else set()
                ctx.set_ws_cache(min(64, max(6, max(len(shapes), len(vc_shapes)) + 2)))
                emb: Dict[int, torch.Tensor] = {}
                for g in adv_groups:
                    ids = [need[d][k] for k in g]
                    x = torch.stack([adv_tgts[i] for i in ids]).to(dev, torch.float32).contiguous()
                    e = ctx.se_forward(x)
                    for k, i in enumerate(ids):
                        emb[i] = e[k]
                for j in owner[d]:
                    ids = chunks[j]
                    if ragged:
                        te = torch.stack([emb[i] for i in ids]).contiguous()
                        outs, _, _ = ctx.emb_attack_ragged([vc_tgts[i].to(dev, torch.float32) for i in ids], te,
                                                           [ptb0s[i].to(dev, torch.float32) for i in ids], eps, n_iters,
                                                           precision=precision)
                        for k, i in enumerate(ids):
                            results[i] = outs[k]
                        continue
                    vc = torch.stack([vc_tgts[i] for i in ids]).to(dev, torch.float32).contiguous()
                    p0 = torch.stack([ptb0s[i] for i in ids]).to(dev, torch.float32).contiguous()
                    te = torch.stack([emb[i] for i in ids]).contiguous()
                    if kind == "emb":
                        out, _, _ = ctx.emb_attack(vc, None, p0, eps, n_iters, precision=precision, tgt_emb=te)
                    else:
                        src = torch.stack([vc_srcs[i] for i in ids]).to(dev, torch.float32).contiguous()
                        out, _, _ = ctx.vc_attack(kind, src, vc, None, p0, eps, n_iters, precision=precision,
                                                  tgt_emb=te)
                    for k, i in enumerate(ids):
                        results[i] = out[k]
                torch.cuda.current_stream(dev).synchronize()
        except BaseException as e:  # re-raised on the calling thread
            errs.append(e)

    threads = [threading.Thread(target=work, args=(d,)) for d in range(len(devs))]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errs:
        raise errs[0]
    return [r.to(devs[0]) for r in results]
