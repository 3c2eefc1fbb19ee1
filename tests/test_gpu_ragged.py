"""GPU: the ragged embedding attack (avc_emb_attack_ragged; batching.attack_many(ragged=True)).

Real utterances arrive at their own lengths (/root/reference/attack.py:41-56, data_utils.py:65-118);
each length has its own reflect padding, ceil-mode pooling and time-mean (models.py:10-30, 275-343),
so per-length buckets of real data hold one or two utterances and leave the GPU idle.  The ragged
batch runs every length in ONE launch per pass (the long engine, per-workgroup length and packed
offsets).  What it must equal: every utterance, bit for bit, its own single-utterance attack on the long
engine (same kernels, same per-utterance arithmetic) -- adv, the loss history and the iteration-0
gradient -- in both precisions; in fp32 that is also the fused engine's result for T <= 128 (the long
and fused engines are bitwise equal there, test_gpu_long.py), i.e. attack_utils.emb_attack's."""
import pytest
import torch

import attack_utils
import avc_native
import batching
from helpers import model_from_fixture

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
LENS = [600, 300, 201, 129, 128, 100, 77, 64, 33]


@pytest.fixture(scope="module")
def full(golden):
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")
    m = model_from_fixture(golden("full_T128")).to(DEV)
    ctx = avc_native.context_for(m.speaker_encoder, DEV)
    yield m, ctx
    ctx.set_engine("auto")


def _utts(lens, seed):
    g = torch.Generator().manual_seed(seed)
    vc = [torch.randn(80, t, generator=g).to(DEV) for t in lens]
    at = [torch.randn(80, max(40, t - 23), generator=g).to(DEV) for t in lens]
    p0 = [torch.randn(80, t, generator=g).to(DEV) for t in lens]
    return vc, at, p0


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_ragged_equals_single_utterance_long(full, prec):
    """55 iterations (one captured 50-iteration graph + 5 launches): adv, losses and grad0 of every
    utterance equal its own long-engine attack bitwise; a second call re-plans nothing."""
    m, ctx = full
    ctx.set_engine("auto")
    vc, at, p0 = _utts(LENS, 11)
    te = torch.cat([ctx.se_forward(a[None]) for a in at])
    outs, L, g0 = ctx.emb_attack_ragged(vc, te, p0, 0.1, 55, precision=prec, want_losses=True, want_grad0=True)
    torch.cuda.synchronize()
    s1 = ctx.ws_stats()
    again, _, _ = ctx.emb_attack_ragged(vc, te, p0, 0.1, 55, precision=prec)
    torch.cuda.synchronize()
    s2 = ctx.ws_stats()
    for k in ("builds", "replans", "captures", "evictions"):
        assert s2[k] == s1[k], (k, s1, s2)
    ctx.set_engine("long")
    try:
        for b, T in enumerate(LENS):
            assert outs[b].shape == (80, T)
            assert torch.equal(outs[b], again[b])
            ref, Lr, gr = ctx.emb_attack(vc[b][None], None, p0[b][None], 0.1, 55, precision=prec, want_losses=True,
                                         want_grad0=True, tgt_emb=te[b:b + 1])
            assert torch.equal(outs[b], ref[0]), (T, float((outs[b] - ref[0]).abs().max()))
            assert torch.equal(L[:, b], Lr[:, 0]), T
            assert torch.equal(g0[b], gr[0]), T
            assert float((outs[b] - vc[b]).abs().max()) <= 0.1 + 1e-6
    finally:
        ctx.set_engine("auto")


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_ragged_fused_runtime_lengths(full, prec, monkeypatch):
    """Every length in (64, 128]: the ragged batch runs on the fused runtime-length kernels (se_*_fused<*, 16>,
    per-workgroup length and offset; bf16: the persistent kernel) -- each utterance equals its own attack on the
    same kernels (AVC_FUSED_RT_FORCE=1 so T = 128 runs them too) bit for bit; AVC_RAGGED_FUSED=0 keeps the long
    engine, which is checked to be a different path (its timing stamps)."""
    m, _ = full
    lens = [128, 127, 120, 113, 100, 97, 80, 65]
    monkeypatch.setenv("AVC_FUSED_RT_FORCE", "1")
    ctx = avc_native.Context(avc_native.se_config(m.speaker_encoder), avc_native.flat_weights(m.speaker_encoder),
                             DEV.index or 0)
    vc, at, p0 = _utts(lens, 14)
    te = torch.cat([ctx.se_forward(a[None]) for a in at])
    ctx.ktime_start()
    outs, L, g0 = ctx.emb_attack_ragged(vc, te, p0, 0.1, 55, precision=prec, want_losses=True, want_grad0=True)
    kt = ctx.ktime_stop()
    assert not any(k.startswith("lz_") for k in kt), kt
    for b, T in enumerate(lens):
        ref, Lr, gr = ctx.emb_attack(vc[b][None], None, p0[b][None], 0.1, 55, precision=prec, want_losses=True,
                                     want_grad0=True, tgt_emb=te[b:b + 1])
        assert torch.equal(outs[b], ref[0]), (T, float((outs[b] - ref[0]).abs().max()))
        assert torch.equal(L[:, b], Lr[:, 0]), T
        assert torch.equal(g0[b], gr[0]), T
    monkeypatch.setenv("AVC_RAGGED_FUSED", "0")
    c2 = avc_native.Context(avc_native.se_config(m.speaker_encoder), avc_native.flat_weights(m.speaker_encoder),
                            DEV.index or 0)
    c2.ktime_start()
    c2.emb_attack_ragged(vc, te, p0, 0.1, 3, precision=prec)
    assert any(k.startswith("lz_se_bwd") for k in c2.ktime_stop())


def test_attack_many_ragged(full):
    """attack_many(ragged=True): chunks of any lengths (longest first), results in input order; fp32 equals
    attack_utils.emb_attack per utterance (fused engine for T <= 128, long above) bit for bit."""
    m, ctx = full
    lens = [64, 300, 128, 77, 450, 33, 129, 200, 96, 128, 600, 90]
    vc, at, p0 = _utts(lens, 12)
    out = batching.attack_many("emb", [m], vc, at, 0.1, 12, ptb0s=p0, max_batch=5, ragged=True)
    for i, T in enumerate(lens):
        ref = attack_utils.emb_attack(m, vc[i][None], at[i][None], 0.1, 12, ptb0=p0[i][None]).detach()[0]
        assert out[i].shape == (80, T)
        assert torch.equal(out[i], ref), (i, T, float((out[i] - ref).abs().max()))
    out16 = batching.attack_many("emb", [m, m], vc, at, 0.1, 12, ptb0s=p0, precision="bf16", max_batch=4, ragged=True)
    ctx.set_engine("long")
    try:
        for i in range(len(lens)):
            ref = attack_utils.emb_attack(m, vc[i][None], at[i][None], 0.1, 12, ptb0=p0[i][None],
                                          precision="bf16").detach()[0]
            assert torch.equal(out16[i], ref), i
    finally:
        ctx.set_engine("auto")


def test_ragged_rejects_bad_input(full):
    m, ctx = full
    vc, at, p0 = _utts([100, 5], 13)
    te = torch.zeros(2, 128, device=DEV)
    with pytest.raises(RuntimeError, match="too short"):
        ctx.emb_attack_ragged(vc, te, p0, 0.1, 2)
    with pytest.raises(RuntimeError, match="ptb0 lengths"):
        ctx.emb_attack_ragged(vc[:1], te[:1], [p0[0][:, :50]], 0.1, 2)
    with pytest.raises(ValueError, match="emb attack only"):
        batching.attack_many("e2e", [m], vc, at, 0.1, 2, vc_srcs=vc, ragged=True)
