"""GPU parity of the voice-conversion path (ContentEncoder + Decoder, csrc/avc_vc.hip)
through the C ABI: AdaInVC.inference and the e2e / feedback attacks against the
reference's own outputs (tests/golden/full_T*.npz, made by the reference's
attack_utils / models on CPU)."""
import numpy as np
import pytest
import torch

import attack_utils
from helpers import TOL_GRAD_REL, TOL_GRAD_REL_VC, TOL_VC_GRAD_L2_MAX, TOL_VC_GRAD_L2_MEDIAN, cfg_of, check_adv, model_from_fixture, oracle_weights, rel
from oracle import adain_vc as oracle

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TOL_DEC_REL = 1e-4       # Decoder output relative to max |out| (six InstanceNorms deep, fp32)


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


@pytest.fixture(scope="module")
def full(golden):
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")
    z = golden("full_T128")
    return z, model_from_fixture(z).to(DEV)


@pytest.mark.parametrize("name", ["full_T128", "full_T127"])
def test_inference_golden(full, golden, name):
    """model.inference(vc_src, vc_tgt) (models.py:472-489) vs the reference's output;
    T = 127 exercises the ceil-mode ContentEncoder and a 128-frame decoder output."""
    z = golden(name)
    _, m = full
    out = m.inference(_dev(z["vc_src"]), _dev(z["vc_tgt"])).cpu().numpy()
    assert out.shape == z["inference"].shape
    assert rel(out, z["inference"]) <= TOL_DEC_REL, rel(out, z["inference"])


@pytest.mark.parametrize("kind", ["e2e", "fb"])
def test_vc_attack_golden(full, kind):
    """e2e_attack / fb_attack (attack_utils.py:7-48, 89-130) after 10 iterations, the
    iteration-0 gradient and the per-iteration losses vs the reference's."""
    z, m = full
    fn = attack_utils.e2e_attack if kind == "e2e" else attack_utils.fb_attack
    adv, info = fn(m, _dev(z["vc_src"]), _dev(z["vc_tgt"]), _dev(z["adv_tgt"]), 0.1, 10,
                   ptb0=_dev(z[f"{kind}_ptb0"]), return_info=True)
    check_adv(adv.detach().cpu().numpy(), z[f"{kind}_adv_n10"], 10, kind=kind)
    assert rel(info["grad0"].cpu().numpy(), z[f"{kind}_grad0"]) <= (TOL_GRAD_REL_VC if kind != "emb" else TOL_GRAD_REL)
    np.testing.assert_allclose(info["losses"].cpu().numpy().T, z[f"{kind}_losses_n10"], rtol=2e-4, atol=1e-9)


@pytest.mark.parametrize("kind", ["e2e", "fb"])
def test_vc_attack_bf16_tracks_fp32(full, kind):
    z, m = full
    g = torch.Generator().manual_seed(5)
    src, vc, at, p0 = (torch.randn(3, 80, 128, generator=g).to(DEV) for _ in range(4))
    fn = attack_utils.e2e_attack if kind == "e2e" else attack_utils.fb_attack
    a32, i32 = fn(m, src, vc, at, 0.1, 20, ptb0=p0, return_info=True)
    a16, i16 = fn(m, src, vc, at, 0.1, 20, ptb0=p0, precision="bf16", return_info=True)
    a = i16["grad0"].cpu().numpy().reshape(3, -1).astype(np.float64)
    b = i32["grad0"].cpu().numpy().reshape(3, -1).astype(np.float64)
    cos = (a * b).sum(1) / np.linalg.norm(a, axis=1) / np.linalg.norm(b, axis=1)
    assert cos.min() >= 0.99, cos
    assert float((a16 - a32).detach().abs().max()) <= 2e-2


@pytest.mark.parametrize("kind", ["e2e", "fb"])
def test_vc_bf16_objective_after_1500(full, kind):
    """SURVEY.md 8(c) bf16 bound at the bench horizon (n_iters = 1500) for e2e / fb: the final
    objective term the attack drives down -- MSE(inference(src, adv), inference(src, adv_tgt))
    (e2e, attack_utils.py:41) or MSE(SE(inference(src, adv)), SE(adv_tgt)) (fb, 123-124) -- of
    the bf16 attack is within 5 % (relative) of the fp32 attack's, per utterance, and both
    attacks made progress."""
    z, m = full
    g = torch.Generator().manual_seed(21 if kind == "e2e" else 22)
    src, vc, at, p0 = (torch.randn(4, 80, 128, generator=g).to(DEV) for _ in range(4))
    fn = attack_utils.e2e_attack if kind == "e2e" else attack_utils.fb_attack
    a32 = fn(m, src, vc, at, 0.1, 1500, ptb0=p0).detach()
    a16 = fn(m, src, vc, at, 0.1, 1500, ptb0=p0, precision="bf16").detach()

    def objective(x):
        out = m.inference(src, x)
        if kind == "e2e":
            return ((out - m.inference(src, at)) ** 2).mean((1, 2))
        se = m.speaker_encoder
        return ((se(out) - se(at)) ** 2).mean(1)
    l0, l32, l16 = objective(vc), objective(a32), objective(a16)
    assert (l32 < l0).all() and (l16 < l0).all(), (l0, l32, l16)
    assert float(((l16 - l32).abs() / l32).max()) <= 0.05, (l16, l32)


@pytest.mark.parametrize("kind", ["e2e", "fb"])
def test_vc_attack_deterministic_and_shard_invariant(full, kind):
    z, m = full
    g = torch.Generator().manual_seed(9)
    src, vc, at, p0 = (torch.randn(10, 80, 128, generator=g).to(DEV) for _ in range(4))
    fn = attack_utils.e2e_attack if kind == "e2e" else attack_utils.fb_attack
    a = fn(m, src, vc, at, 0.1, 6, ptb0=p0).detach()
    b = fn(m, src, vc, at, 0.1, 6, ptb0=p0).detach()
    assert torch.equal(a, b)
    lo = fn(m, src[:3], vc[:3], at[:3], 0.1, 6, ptb0=p0[:3]).detach()
    hi = fn(m, src[3:], vc[3:], at[3:], 0.1, 6, ptb0=p0[3:]).detach()
    assert torch.equal(torch.cat([lo, hi]), a)


@pytest.mark.parametrize("T", [100, 64])
def test_vc_generic_length_vs_oracle(full, T):
    """T = 100 (ContentEncoder 13 frames -> Decoder 104) and T = 64 (8 -> 64): the generic
    kernel shapes vs the float64 numpy oracle -- inference output and the e2e / fb
    iteration-0 gradients of 4 seeded utterances (normwise, see helpers.TOL_VC_GRAD_*)."""
    z, m = full
    g = torch.Generator().manual_seed(T)
    src, vc, at, p0 = (torch.randn(4, 80, T, generator=g) for _ in range(4))
    sd = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    w64 = oracle.Weights(sd, dtype=np.float64)
    cfg = cfg_of(z)
    f64 = [t.numpy().astype(np.float64) for t in (src, vc, at, p0)]
    out = m.inference(src.to(DEV), vc.to(DEV)).cpu().numpy()
    ref = oracle.inference(w64, cfg, f64[0], f64[1])
    assert out.shape == ref.shape == (4, 80, 8 * ((T + 7) // 8))
    assert rel(out, ref) <= TOL_DEC_REL, rel(out, ref)
    for kind in ("e2e", "fb"):
        rec = {}
        getattr(oracle, f"{kind}_attack")(w64, cfg, *f64[:3], 0.1, 1, f64[3], record=rec)
        fn = attack_utils.e2e_attack if kind == "e2e" else attack_utils.fb_attack
        _, info = fn(m, src.to(DEV), vc.to(DEV), at.to(DEV), 0.1, 1, ptb0=p0.to(DEV), return_info=True)
        gg = info["grad0"].cpu().numpy().astype(np.float64)
        e = [float(np.linalg.norm(gg[u] - rec["grad0"][u]) / np.linalg.norm(rec["grad0"][u])) for u in range(4)]
        assert max(e) <= TOL_VC_GRAD_L2_MAX and float(np.median(e)) <= TOL_VC_GRAD_L2_MEDIAN, (kind, e)


def test_vc_small_config_rejected(golden):
    """c_h = 32 (tests/golden/small_T32.npz) is not the fused engine's shape: loud error,
    no fallback."""
    m = model_from_fixture(golden("small_T32")).to(DEV)
    x = torch.zeros(1, 80, 32, device=DEV)
    with pytest.raises(RuntimeError):
        attack_utils.e2e_attack(m, x, x, x, 0.1, 1)


@pytest.mark.parametrize("kind", ["emb", "e2e", "fb"])
def test_graph_tail_matches_eager(full, kind):
    """The attack loop replays a captured graph of 50 iterations plus plain launches for the
    n_iters % 50 tail (csrc/avc_api.hip graph_replay): at n = 103 (two graphs + three launches),
    bf16, the adversarial output and the whole per-iteration loss history equal the eager
    (one launch per kernel) run bitwise."""
    from avc_native import context_for, vc_context_for
    _, m = full
    g = torch.Generator().manual_seed(11)
    src, vc, at, p0 = (torch.randn(2, 80, 128, generator=g).to(DEV) for _ in range(4))
    if kind == "emb":
        ctx = context_for(m.speaker_encoder, DEV)
        run = lambda gr: ctx.emb_attack(vc, at, p0, 0.1, 103, precision="bf16", use_graph=gr, want_losses=True)
    else:
        ctx = vc_context_for(m, DEV)
        run = lambda gr: ctx.vc_attack(kind, src, vc, at, p0, 0.1, 103, precision="bf16", use_graph=gr,
                                       want_losses=True)
    a, la, _ = run(True)
    b, lb, _ = run(False)
    assert torch.equal(a, b)
    assert la.shape[0] == 103 and torch.equal(la, lb)
