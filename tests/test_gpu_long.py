"""GPU parity of the long-utterance engine (csrc/avc_long.hip): any T, the fused engine's
kernels family with the activations chunked through global scratch.

  * T <= 128, engine forced to "long": the same MFMA K loops, summation orders and fold
    arithmetic as the fused engine, so the fp32 attack is BITWISE equal to the fused one,
    and the reference's own golden vectors (tests/golden/full_T128.npz) are reproduced;
  * T in {129, 200, 257, 600} (AUTO picks "long" above 128): SpeakerEncoder(x), the emb
    attack's iteration-0 gradient and 10-iteration adv against the float64 oracle;
  * reference-generated goldens at T = 300 (tests/golden/full_T300.npz at n = 10,
    full_T300_n100.npz at n = 100);
  * bf16 vs fp32, determinism and shard invariance at T = 300."""
import os

import numpy as np
import pytest
import torch

import attack_utils
import avc_native
from helpers import (TOL_GRAD_REL, TOL_GRAD_REL_VC, TOL_SE_REL, TOL_VC_GRAD_L2_MAX, TOL_VC_GRAD_L2_MEDIAN, cfg_of,
                     check_adv, model_from_fixture, rel)
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
    sd = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    yield z, m, ctx, oracle.Weights(sd, dtype=np.float64)
    ctx.set_engine("auto")


def test_engine_selection_long(full):
    z, m, ctx, _ = full
    ctx.set_engine("auto")
    assert ctx.engine_for(128) == "fused"
    assert ctx.engine_for(129) == "long" and ctx.engine_for(600) == "long"
    ctx.set_engine("long")
    assert ctx.engine_for(64) == "long"
    ctx.set_engine("auto")


@pytest.mark.parametrize("T", [128, 100, 64, 33])
def test_long_equals_fused_bitwise(full, T):
    """T <= 128: long and fused run identical arithmetic in identical order."""
    z, m, ctx, _ = full
    g = torch.Generator().manual_seed(300 + T)
    vc, at, p0 = (torch.randn(3, 80, T, generator=g).to(DEV) for _ in range(3))
    out = {}
    for eng in ("fused", "long"):
        ctx.set_engine(eng)
        e = ctx.se_forward(vc)
        adv, L, g0 = ctx.emb_attack(vc, at, p0, 0.1, 5, want_losses=True, want_grad0=True)
        out[eng] = (e, adv, L, g0)
    ctx.set_engine("auto")
    for a, b in zip(out["fused"], out["long"]):
        assert torch.equal(a, b), float((a - b).abs().max())


def test_long_golden_T128(full):
    """The reference's emb_attack outputs at T = 128 reproduced by the long engine."""
    z, m, ctx, _ = full
    ctx.set_engine("long")
    for n in (1, 10, 100):
        adv, _, g0 = ctx.emb_attack(_dev(z["vc_tgt"]), _dev(z["adv_tgt"]), _dev(z["emb_ptb0"]), 0.1, n,
                                    want_grad0=True)
        check_adv(adv.cpu().numpy(), z[f"emb_adv_n{n}"], n)
        assert rel(g0.cpu().numpy(), z["emb_grad0"]) <= TOL_GRAD_REL
    ctx.set_engine("auto")


@pytest.mark.parametrize("T", [129, 200, 257, 600])
def test_long_se_forward_vs_oracle(full, T):
    z, m, ctx, w64 = full
    g = torch.Generator().manual_seed(400 + T)
    x = torch.randn(3, 80, T, generator=g)
    e = ctx.se_forward(x.to(DEV)).cpu().numpy()
    eo, _ = oracle.se_forward(w64, cfg_of(z)["SpeakerEncoder"], x.double().numpy())
    assert rel(e, eo) <= TOL_SE_REL, (T, rel(e, eo))


@pytest.mark.parametrize("T", [129, 200, 257, 600])
def test_long_emb_attack_vs_oracle(full, T):
    """grad0 (relative 1e-4) and the 10-iteration adv (fp32 tolerances of SURVEY 8(c)) vs the
    float64 oracle; adv_tgt of another length on the way (the *_emb entry point)."""
    z, m, ctx, w64 = full
    g = torch.Generator().manual_seed(500 + T)
    vc, p0 = (torch.randn(2, 80, T, generator=g) for _ in range(2))
    at = torch.randn(2, 80, T - 37, generator=g)
    adv, info = attack_utils.emb_attack(m, vc.to(DEV), at.to(DEV), 0.1, 10, ptb0=p0.to(DEV), return_info=True)
    rec = {}
    ref = oracle.emb_attack(w64, cfg_of(z), vc.double().numpy(), at.double().numpy(), 0.1, 10, p0.double().numpy(),
                            record=rec)
    assert rel(info["grad0"].cpu().numpy(), rec["grad0"]) <= TOL_GRAD_REL, rel(info["grad0"].cpu().numpy(), rec["grad0"])
    check_adv(adv.detach().cpu().numpy(), ref, 10)
    np.testing.assert_allclose(info["losses"].cpu().numpy().T, rec["losses"], rtol=2e-4, atol=1e-9)


def test_long_golden_T300(full, golden):
    """Made by the reference's own attack_utils.emb_attack at T = 300 (make_golden.py)."""
    path = os.path.join(os.path.dirname(__file__), "golden", "full_T300.npz")
    if not os.path.exists(path):
        pytest.fail("tests/golden/full_T300.npz missing")
    zl = golden("full_T300")
    z, m, ctx, _ = full
    adv, L, g0 = ctx.emb_attack(_dev(zl["vc_tgt"]), _dev(zl["adv_tgt"]), _dev(zl["emb_ptb0"]), 0.1, 10,
                                want_losses=True, want_grad0=True)
    check_adv(adv.cpu().numpy(), zl["emb_adv_n10"], 10)
    assert rel(g0.cpu().numpy(), zl["emb_grad0"]) <= TOL_GRAD_REL
    e = ctx.se_forward(_dev(zl["vc_tgt"])).cpu().numpy()
    assert rel(e, zl["se_vc_tgt"]) <= TOL_SE_REL


def test_long_bf16_tracks_fp32(full):
    z, m, ctx, _ = full
    g = torch.Generator().manual_seed(77)
    vc, at, p0 = (torch.randn(3, 80, 300, generator=g).to(DEV) for _ in range(3))
    a32, _, g32 = ctx.emb_attack(vc, at, p0, 0.1, 100, want_grad0=True)
    a16, _, g16 = ctx.emb_attack(vc, at, p0, 0.1, 100, precision="bf16", want_grad0=True)
    a = g16.cpu().numpy().reshape(3, -1).astype(np.float64)
    b = g32.cpu().numpy().reshape(3, -1).astype(np.float64)
    cos = (a * b).sum(1) / np.linalg.norm(a, axis=1) / np.linalg.norm(b, axis=1)
    assert cos.min() >= 0.99, cos
    assert float((a16 - a32).abs().max()) <= 2e-2


def test_long_deterministic_and_shard_invariant(full):
    z, m, ctx, _ = full
    g = torch.Generator().manual_seed(31)
    vc, at, p0 = (torch.randn(9, 80, 300, generator=g).to(DEV) for _ in range(3))
    for prec in ("fp32", "bf16"):
        a, _, _ = ctx.emb_attack(vc, at, p0, 0.1, 6, precision=prec)
        b, _, _ = ctx.emb_attack(vc, at, p0, 0.1, 6, precision=prec)
        assert torch.equal(a, b)
        lo, _, _ = ctx.emb_attack(vc[:4], at[:4], p0[:4], 0.1, 6, precision=prec)
        hi, _, _ = ctx.emb_attack(vc[4:], at[4:], p0[4:], 0.1, 6, precision=prec)
        assert torch.equal(torch.cat([lo, hi]), a)


@pytest.mark.parametrize("kind", ["e2e", "fb"])
def test_long_vc_golden_T300(full, golden, kind):
    """e2e / fb attacks made by the reference at vc_src 280, vc_tgt 300, adv_tgt 260 frames:
    the ContentEncoder (280 frames), the Decoder (35 -> 280 frames), the fb SpeakerEncoder
    over the decoder output and the attacked SpeakerEncoder (300) all on the long engine."""
    zl = golden("full_T300")
    z, m, ctx, _ = full
    fn = attack_utils.e2e_attack if kind == "e2e" else attack_utils.fb_attack
    adv, info = fn(m, _dev(zl["vc_src"]), _dev(zl["vc_tgt"]), _dev(zl["adv_tgt"]), 0.1, 10,
                   ptb0=_dev(zl[f"{kind}_ptb0"]), return_info=True)
    check_adv(adv.detach().cpu().numpy(), zl[f"{kind}_adv_n10"], 10, kind=kind)
    assert rel(info["grad0"].cpu().numpy(), zl[f"{kind}_grad0"]) <= TOL_GRAD_REL_VC
    np.testing.assert_allclose(info["losses"].cpu().numpy().T, zl[f"{kind}_losses_n10"], rtol=2e-4, atol=1e-9)


@pytest.mark.parametrize("kind", ["emb", "e2e", "fb"])
def test_long_golden_T300_n100(full, golden, kind):
    """The reference's own 100-iteration attacks at vc_src 280 / vc_tgt 300 / adv_tgt 260 frames
    (tests/golden/full_T300_n100.npz, make_golden.py --stage long100): the long engine at the
    SURVEY 8(c) n = 100 fp32 tolerances (adv max 1e-3 / mean 1e-6), grad0 and the whole loss
    history (rtol 2e-4)."""
    zl, zn = golden("full_T300"), golden("full_T300_n100")
    z, m, ctx, _ = full
    fn = {"emb": attack_utils.emb_attack, "e2e": attack_utils.e2e_attack, "fb": attack_utils.fb_attack}[kind]
    args = (_dev(zl["vc_tgt"]), _dev(zl["adv_tgt"])) if kind == "emb" else \
        (_dev(zl["vc_src"]), _dev(zl["vc_tgt"]), _dev(zl["adv_tgt"]))
    adv, info = fn(m, *args, 0.1, 100, ptb0=_dev(zn[f"{kind}_ptb0"]), return_info=True)
    check_adv(adv.detach().cpu().numpy(), zn[f"{kind}_adv_n100"], 100, kind=kind)
    assert rel(info["grad0"].cpu().numpy(), zn[f"{kind}_grad0"]) <= (TOL_GRAD_REL if kind == "emb" else TOL_GRAD_REL_VC)
    np.testing.assert_allclose(info["losses"].cpu().numpy().T, zn[f"{kind}_losses_n100"], rtol=2e-4, atol=1e-9)


def test_long_inference_golden_T300(full, golden):
    zl = golden("full_T300")
    z, m, ctx, _ = full
    out = m.inference(_dev(zl["vc_src"]), _dev(zl["vc_tgt"])).cpu().numpy()
    assert out.shape == zl["inference"].shape
    assert rel(out, zl["inference"]) <= 1e-4, rel(out, zl["inference"])


@pytest.mark.parametrize("Ts", [129, 200, 600])
def test_long_vc_vs_oracle(full, Ts):
    """Long ContentEncoder / Decoder lengths vs the float64 oracle: inference and the e2e / fb
    iteration-0 gradients per utterance (normwise, helpers.TOL_VC_GRAD_*)."""
    z, m, ctx, w64 = full
    g = torch.Generator().manual_seed(600 + Ts)
    src = torch.randn(4, 80, Ts, generator=g)
    vc, at, p0 = (torch.randn(4, 80, 160, generator=g) for _ in range(3))
    out = m.inference(src.to(DEV), vc.to(DEV)).cpu().numpy()
    ref = oracle.inference(w64, cfg_of(z), src.double().numpy(), vc.double().numpy())
    assert out.shape == ref.shape == (4, 80, 8 * ((Ts + 7) // 8))
    assert rel(out, ref) <= 1e-4, rel(out, ref)
    for kind in ("e2e", "fb"):
        rec = {}
        getattr(oracle, f"{kind}_attack")(w64, cfg_of(z), src.double().numpy(), vc.double().numpy(),
                                          at.double().numpy(), 0.1, 1, p0.double().numpy(), record=rec)
        fn = attack_utils.e2e_attack if kind == "e2e" else attack_utils.fb_attack
        _, info = fn(m, src.to(DEV), vc.to(DEV), at.to(DEV), 0.1, 1, ptb0=p0.to(DEV), return_info=True)
        gg = info["grad0"].cpu().numpy().astype(np.float64)
        e = [float(np.linalg.norm(gg[u] - rec["grad0"][u]) / np.linalg.norm(rec["grad0"][u])) for u in range(4)]
        assert max(e) <= TOL_VC_GRAD_L2_MAX and float(np.median(e)) <= 5 * TOL_VC_GRAD_L2_MEDIAN, (kind, e)


def test_long_vc_forced_equals_fused(full):
    """T = 128 e2e with every component forced onto the long engine vs the fused engine."""
    z, m, ctx, _ = full
    g = torch.Generator().manual_seed(88)
    src, vc, at, p0 = (torch.randn(2, 80, 128, generator=g).to(DEV) for _ in range(4))
    a_f, i_f = attack_utils.e2e_attack(m, src, vc, at, 0.1, 3, ptb0=p0, return_info=True)
    ctx.set_engine("long")
    try:
        a_l, i_l = attack_utils.e2e_attack(m, src, vc, at, 0.1, 3, ptb0=p0, return_info=True)
    finally:
        ctx.set_engine("auto")
    assert rel(i_l["grad0"].cpu().numpy(), i_f["grad0"].cpu().numpy()) <= TOL_GRAD_REL_VC
    check_adv(a_l.detach().cpu().numpy(), a_f.detach().cpu().numpy(), 10)
