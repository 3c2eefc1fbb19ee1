"""GPU parity of the fused per-utterance engine (csrc/avc_fused.hip) against the
layered GEMM engine, the CPU oracle and the reference's golden vectors, through
the C ABI.  The golden tests in test_gpu_parity.py run the full AdaIN-VC config
on the default engine (fused); here both engines are pinned explicitly."""
import numpy as np
import pytest
import torch

import attack_utils
import avc_native
from helpers import TOL_GRAD_REL, TOL_SE_REL, cfg_of, check_adv, model_from_fixture, oracle_weights, rel
from oracle import adain_vc as oracle

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


@pytest.fixture(scope="module")
def full(golden):
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")
    z = golden("full_T128")
    m = model_from_fixture(z).to(DEV)
    ctx = avc_native.context_for(m.speaker_encoder, DEV)
    yield z, m, ctx
    ctx.set_engine("auto")


def test_engine_selection(full, golden):
    z, m, ctx = full
    assert ctx.engine_for(128) == "fused" and ctx.engine_for(9) == "fused"
    assert ctx.engine_for(129) == "long"             # LDS images are sized for T <= 128: chunked above
    small = model_from_fixture(golden("small_T32")).to(DEV)
    sctx = avc_native.context_for(small.speaker_encoder, DEV)
    assert sctx.engine_for(32) == "layered"          # c_h = 32: not the fused engine's shape
    with pytest.raises(RuntimeError, match="fused engine needs"):
        sctx.set_engine("fused")


@pytest.mark.parametrize("T", [128, 127, 100, 64, 33, 17, 9])
def test_fused_se_forward_vs_oracle(full, T):
    """SpeakerEncoder(x) on the fused engine vs the numpy oracle, odd/short T
    included (reflect pads of 1..4 rows, ceil-mode pooling tails)."""
    z, m, ctx = full
    g = torch.Generator().manual_seed(100 + T)
    x = torch.randn(5, 80, T, generator=g)
    ctx.set_engine("fused")
    e = ctx.se_forward(x.to(DEV)).cpu().numpy()
    eo, _ = oracle.se_forward(oracle_weights(m), cfg_of(z)["SpeakerEncoder"], x.numpy())
    assert rel(e, eo) <= TOL_SE_REL, (T, rel(e, eo))


@pytest.mark.parametrize("T", [128, 127, 45, 9])
def test_fused_vs_layered_attack(full, T):
    """The two engines on identical inputs: fp32 sums in different orders, so
    agreement within the stated fp32 tolerances, not bitwise."""
    z, m, ctx = full
    g = torch.Generator().manual_seed(200 + T)
    vc, at, p0 = (torch.randn(3, 80, T, generator=g).to(DEV) for _ in range(3))
    out = {}
    for eng in ("fused", "layered"):
        ctx.set_engine(eng)
        adv, L, g0 = ctx.emb_attack(vc, at, p0, 0.1, 10, want_losses=True, want_grad0=True)
        out[eng] = (adv.cpu().numpy(), L.cpu().numpy(), g0.cpu().numpy())
    ctx.set_engine("auto")
    check_adv(out["fused"][0], out["layered"][0], 10)
    assert rel(out["fused"][2], out["layered"][2]) <= TOL_GRAD_REL
    np.testing.assert_allclose(out["fused"][1], out["layered"][1], rtol=2e-4, atol=1e-8)


@pytest.mark.parametrize("engine", ["fused", "layered"])
def test_golden_full_both_engines(full, engine):
    """The reference's own emb_attack outputs (tests/golden/full_T128.npz, made by
    attack_utils.emb_attack itself) reproduced on each engine."""
    z, m, ctx = full
    ctx.set_engine(engine)
    for n in (1, 10, 100):
        adv, L, g0 = ctx.emb_attack(_dev(z["vc_tgt"]), _dev(z["adv_tgt"]), _dev(z["emb_ptb0"]), 0.1, n,
                                    want_losses=True, want_grad0=True)
        check_adv(adv.cpu().numpy(), z[f"emb_adv_n{n}"], n)
        assert rel(g0.cpu().numpy(), z["emb_grad0"]) <= TOL_GRAD_REL
    ctx.set_engine("auto")


def test_golden_full_T127_fused(full, golden):
    z127 = golden("full_T127")
    z, m, ctx = full
    ctx.set_engine("fused")
    adv, _, g0 = ctx.emb_attack(_dev(z127["vc_tgt"]), _dev(z127["adv_tgt"]), _dev(z127["emb_ptb0"]), 0.1, 10,
                                want_grad0=True)
    check_adv(adv.cpu().numpy(), z127["emb_adv_n10"], 10)
    assert rel(g0.cpu().numpy(), z127["emb_grad0"]) <= TOL_GRAD_REL
    ctx.set_engine("auto")


def test_fused_bf16_vs_fp32(full):
    """bf16 operands on the fused engine track its fp32 run (SURVEY.md 8(c) bf16
    bounds: gradient cosine >= 0.99; adv within 2e-2 after 100 iterations)."""
    z, m, ctx = full
    ctx.set_engine("fused")
    g = torch.Generator().manual_seed(77)
    vc, at, p0 = (torch.randn(4, 80, 128, generator=g).to(DEV) for _ in range(3))
    a32, _, g32 = ctx.emb_attack(vc, at, p0, 0.1, 100, want_grad0=True)
    a16, _, g16 = ctx.emb_attack(vc, at, p0, 0.1, 100, precision="bf16", want_grad0=True)
    ctx.set_engine("auto")
    a = g16.cpu().numpy().reshape(4, -1).astype(np.float64)
    b = g32.cpu().numpy().reshape(4, -1).astype(np.float64)
    cos = (a * b).sum(1) / np.linalg.norm(a, axis=1) / np.linalg.norm(b, axis=1)
    assert cos.min() >= 0.99, cos
    assert float((a16 - a32).abs().max()) <= 2e-2


def test_fused_deterministic_and_shard_invariant(full):
    z, m, ctx = full
    ctx.set_engine("fused")
    g = torch.Generator().manual_seed(31)
    vc, at, p0 = (torch.randn(20, 80, 128, generator=g).to(DEV) for _ in range(3))
    for prec in ("fp32", "bf16"):
        a, _, _ = ctx.emb_attack(vc, at, p0, 0.1, 12, precision=prec)
        b, _, _ = ctx.emb_attack(vc, at, p0, 0.1, 12, precision=prec)
        assert torch.equal(a, b)
        lo, _, _ = ctx.emb_attack(vc[:7], at[:7], p0[:7], 0.1, 12, precision=prec)
        hi, _, _ = ctx.emb_attack(vc[7:], at[7:], p0[7:], 0.1, 12, precision=prec)
        assert torch.equal(torch.cat([lo, hi]), a)
    ctx.set_engine("auto")


def test_bf16_objective_after_1500(full):
    """SURVEY.md 8(c) bf16 bound at the bench's n_iters: the final objective
    MSE(SE(adv), SE(adv_tgt)) of the bf16 attack is within 5 % (relative) of the fp32
    attack's, per utterance (elements of adv may differ: Adam normalises each element's
    step, so near-zero gradients wander)."""
    z, m, ctx = full
    ctx.set_engine("fused")
    g = torch.Generator().manual_seed(15)
    vc, at, p0 = (torch.randn(4, 80, 128, generator=g).to(DEV) for _ in range(3))
    a32, _, _ = ctx.emb_attack(vc, at, p0, 0.1, 1500)
    a16, _, _ = ctx.emb_attack(vc, at, p0, 0.1, 1500, precision="bf16")
    ctx.set_engine("auto")
    tgt = ctx.se_forward(at)
    l32 = ((ctx.se_forward(a32) - tgt) ** 2).mean(1)
    l16 = ((ctx.se_forward(a16) - tgt) ** 2).mean(1)
    l0 = ((ctx.se_forward(vc) - tgt) ** 2).mean(1)
    assert (l32 < l0).all() and (l16 < l0).all()          # both attacks made progress
    assert float(((l16 - l32).abs() / l32).max()) <= 0.05, (l16, l32)


def test_bf16_vs_fp32_at_bench_size(full):
    """The headline configuration itself (BASELINE configs[1]: B=256, T=128, n_iters=1500, eps=0.1):
    the bf16 attack against the fp32 one (the reference's arithmetic) over all 256 utterances.
    Element-wise the two adv tensors drift apart (Adam normalises every element's step, so elements
    with near-zero gradients wander; bench.py reports max |adv16 - adv32| ~ 0.11 of the 2 eps range),
    so the check is on what the attack is for: every utterance's objective MSE(SE(adv), SE(adv_tgt))
    decreases under both, and the bf16 objective is close to the fp32 one (thresholds ~4x the
    distribution observed on MI355X, printed)."""
    z, m, ctx = full
    ctx.set_engine("fused")
    g = torch.Generator().manual_seed(256)
    vc, at, p0 = (torch.randn(256, 80, 128, generator=g).to(DEV) for _ in range(3))
    a32, _, _ = ctx.emb_attack(vc, at, p0, 0.1, 1500)
    a16, _, _ = ctx.emb_attack(vc, at, p0, 0.1, 1500, precision="bf16")
    ctx.set_engine("auto")
    assert float((a16 - vc).abs().max()) <= 0.1 + 1e-6 and float((a32 - vc).abs().max()) <= 0.1 + 1e-6
    tgt = ctx.se_forward(at)
    l0 = ((ctx.se_forward(vc) - tgt) ** 2).mean(1)
    l32 = ((ctx.se_forward(a32) - tgt) ** 2).mean(1)
    l16 = ((ctx.se_forward(a16) - tgt) ** 2).mean(1)
    rel = ((l16 - l32).abs() / l32).cpu()
    d = (a16 - a32).abs().flatten().cpu()
    q = torch.quantile(rel, torch.tensor([0.5, 0.9, 0.99]))
    qe = torch.quantile(d[torch.randperm(d.numel(), generator=torch.Generator().manual_seed(0))[:1000000]],
                        torch.tensor([0.5, 0.99, 0.999]))
    print(f"objective rel diff median {q[0]:.4f} p90 {q[1]:.4f} p99 {q[2]:.4f} max {rel.max():.4f}; "
          f"|adv16-adv32| median {qe[0]:.2e} p99 {qe[1]:.2e} p99.9 {qe[2]:.2e} max {d.max():.3f}; "
          f"objective decrease fp32 {float((l32 / l0).mean()):.3f} bf16 {float((l16 / l0).mean()):.3f}")
    assert (l32 < l0).all() and (l16 < l0).all()
    # observed on MI355X: rel diff median 0.0022, p99 0.0093, max 0.0112; |adv16 - adv32| median
    # 4.3e-4, p99.9 0.024; mean objective ratio 0.244 under both
    assert float(q[0]) <= 0.01 and float(rel.max()) <= 0.05
    assert float(qe[0]) <= 2e-3
    assert abs(float((l16 / l0).mean()) - float((l32 / l0).mean())) <= 0.01


def test_fused_head_matches_separate_head(full, monkeypatch):
    """The bf16 emb attack runs the head chain (dense blocks, output Linear, loss and its
    backward) inside se_fwd_fused (se_head_fused); AVC_FUSE_HEAD=0 plans the separate
    se_head_v launch instead.  Same per-element arithmetic in the same order, so adv, the
    per-iteration losses (handed to the backward through a [B] buffer) and grad0 are
    bitwise equal."""
    z, m, ctx = full
    g = torch.Generator().manual_seed(41)
    vc, at, p0 = (torch.randn(6, 80, 128, generator=g).to(DEV) for _ in range(3))
    ctx.set_engine("fused")
    a, L, g0 = ctx.emb_attack(vc, at, p0, 0.1, 12, precision="bf16", want_losses=True, want_grad0=True)
    ctx.set_engine("auto")
    monkeypatch.setenv("AVC_FUSE_HEAD", "0")
    sep = avc_native.Context(avc_native.se_config(m.speaker_encoder), avc_native.flat_weights(m.speaker_encoder),
                             DEV.index or 0)
    sep.set_engine("fused")
    a2, L2, g02 = sep.emb_attack(vc, at, p0, 0.1, 12, precision="bf16", want_losses=True, want_grad0=True)
    assert torch.isfinite(L).all() and L.abs().sum() > 0
    assert torch.equal(a, a2)
    assert torch.equal(L, L2)
    assert torch.equal(g0, g02)
