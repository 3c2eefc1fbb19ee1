"""GPU parity: libavc's HIP path vs the reference's golden vectors and the CPU
oracle, through the C ABI (avc_native -> libavc.so).  All tests need an MI355X."""
import numpy as np
import pytest
import torch

import attack_utils
import avc_native
from helpers import TOL_ADV, TOL_GRAD_REL, TOL_SE_REL, cfg_of, check_adv, model_from_fixture, oracle_weights, rel
from oracle import adain_vc as oracle

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


@pytest.fixture(scope="module")
def gpu():
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")
    avc_native.lib()
    return DEV


@pytest.mark.parametrize("name", ["small_T32", "small_T33", "full_T128", "full_T127"])
def test_se_forward_golden(gpu, golden, name):
    z = golden(name)
    m = model_from_fixture(z).to(gpu)
    for key, x in (("se_vc_tgt", "vc_tgt"), ("se_adv_tgt", "adv_tgt")):
        e = m.speaker_encoder(_dev(z[x])).cpu().numpy()
        assert rel(e, z[key]) <= TOL_SE_REL, (name, key, rel(e, z[key]))


@pytest.mark.parametrize("name,ns", [("small_T32", [1, 10, 100]), ("small_T33", [10]),
                                     ("full_T128", [1, 10, 100, 1500]), ("full_T127", [10])])
def test_emb_attack_golden(gpu, golden, name, ns):
    z = golden(name)
    m = model_from_fixture(z).to(gpu)
    for n in ns:
        adv, info = attack_utils.emb_attack(m, _dev(z["vc_tgt"]), _dev(z["adv_tgt"]), 0.1, n,
                                            ptb0=_dev(z["emb_ptb0"]), return_info=True)
        check_adv(adv.detach().cpu().numpy(), z[f"emb_adv_n{n}"], n)
        g0 = info["grad0"].cpu().numpy()
        assert rel(g0, z["emb_grad0"]) <= TOL_GRAD_REL, rel(g0, z["emb_grad0"])
        key = f"emb_losses_n{n}"
        if key in z:
            np.testing.assert_allclose(info["losses"].cpu().numpy().T, z[key], rtol=2e-4, atol=1e-8)


def test_emb_attack_batched_mean(gpu, golden):
    z = golden("small_T32")
    m = model_from_fixture(z).to(gpu)
    adv = attack_utils.emb_attack(m, _dev(z["vc_tgt"]), _dev(z["adv_tgt"]), 0.1, 10,
                                  ptb0=_dev(z["emb_batched_ptb0"]), reduction="mean")
    check_adv(adv.detach().cpu().numpy(), z["emb_batched_adv_n10"], 10)


def test_emb_attack_draws_ptb_like_reference(gpu, golden):
    """Without ptb0, emb_attack consumes the RNG exactly like attack_utils.py:68."""
    z = golden("small_T32")
    m = model_from_fixture(z).to(gpu)
    vc, at = _dev(z["vc_tgt"][:1]), _dev(z["adv_tgt"][:1])
    torch.manual_seed(7)
    a = attack_utils.emb_attack(m, vc, at, 0.1, 3)
    torch.manual_seed(7)
    p0 = torch.zeros_like(vc).normal_(0, 1)
    b = attack_utils.emb_attack(m, vc, at, 0.1, 3, ptb0=p0)
    assert torch.equal(a, b)
    assert a.requires_grad


def test_oracle_parity_random(gpu):
    """Seeded synthetic inputs at sizes the oracle finishes in seconds; also
    B not a multiple of the head's 16-utterance tile and an odd T."""
    cfg = cfg_of_small()
    torch.manual_seed(3)
    import models
    m = models.AdaInVC(cfg)
    w = oracle_weights(m)
    m = m.to(gpu)
    g = torch.Generator().manual_seed(11)
    B, T = 17, 45
    vc, at, p0 = (torch.randn(B, 80, T, generator=g) for _ in range(3))
    e = m.speaker_encoder(vc.to(gpu)).cpu().numpy()
    eo, _ = oracle.se_forward(w, cfg["SpeakerEncoder"], vc.numpy())
    assert rel(e, eo) <= TOL_SE_REL
    adv = attack_utils.emb_attack(m, vc.to(gpu), at.to(gpu), 0.1, 10, ptb0=p0.to(gpu))
    ref = oracle.emb_attack(w, cfg, vc.numpy(), at.numpy(), 0.1, 10, p0.numpy())
    check_adv(adv.detach().cpu().numpy(), ref, 10)


def cfg_of_small():
    import json
    import os
    from conftest import GOLDEN
    return json.loads(str(np.load(os.path.join(GOLDEN, "small_T32.npz"))["config"]))


def test_minimum_length_and_errors(gpu, golden):
    z = golden("full_T128")
    m = model_from_fixture(z).to(gpu)
    x = torch.randn(2, 80, 9, device=gpu)        # shortest T the full config accepts
    e = m.speaker_encoder(x)
    w = oracle_weights(m)
    eo, _ = oracle.se_forward(w, cfg_of(z)["SpeakerEncoder"], x.cpu().numpy())
    assert rel(e.cpu().numpy(), eo) <= TOL_SE_REL
    with pytest.raises(RuntimeError, match="too short"):
        m.speaker_encoder(torch.randn(1, 80, 8, device=gpu))
    with pytest.raises(RuntimeError, match="MI355X"):
        attack_utils.emb_attack(m, torch.randn(1, 80, 32), torch.randn(1, 80, 32), 0.1, 1)


def test_batch_shard_invariance(gpu, golden):
    """Per-utterance independence: attacking a batch equals attacking its two
    halves separately, bit for bit (what multi-GPU sharding relies on)."""
    z = golden("full_T128")
    m = model_from_fixture(z).to(gpu)
    g = torch.Generator().manual_seed(5)
    B, T = 48, 128
    vc, at, p0 = (torch.randn(B, 80, T, generator=g).to(gpu) for _ in range(3))
    full = attack_utils.emb_attack(m, vc, at, 0.1, 20, ptb0=p0).detach()
    h = B // 2
    lo = attack_utils.emb_attack(m, vc[:h], at[:h], 0.1, 20, ptb0=p0[:h]).detach()
    hi = attack_utils.emb_attack(m, vc[h:], at[h:], 0.1, 20, ptb0=p0[h:]).detach()
    assert torch.equal(torch.cat([lo, hi]), full)


def test_graph_and_eager_agree(gpu, golden):
    z = golden("small_T32")
    m = model_from_fixture(z).to(gpu)
    ctx = avc_native.context_for(m.speaker_encoder, gpu)
    args = (_dev(z["vc_tgt"]), _dev(z["adv_tgt"]), _dev(z["emb_ptb0"]), 0.1, 55)   # one 50-iteration graph + 5
    a, _, _ = ctx.emb_attack(*args, use_graph=True)
    b, _, _ = ctx.emb_attack(*args, use_graph=False)
    assert torch.equal(a, b)


def test_full_size_properties(gpu, golden):
    """B=256, T=128 (the bench workload): determinism across calls, the
    perturbation bound |adv - vc| <= eps, and the embedding loss decreasing."""
    z = golden("full_T128")
    m = model_from_fixture(z).to(gpu)
    g = torch.Generator().manual_seed(1)
    B, T = 256, 128
    vc, at = (torch.randn(B, 80, T, generator=g).to(gpu) for _ in range(2))
    p0 = torch.randn(B, 80, T, generator=torch.Generator().manual_seed(123)).to(gpu)
    a, info = attack_utils.emb_attack(m, vc, at, 0.1, 50, ptb0=p0, return_info=True)
    b = attack_utils.emb_attack(m, vc, at, 0.1, 50, ptb0=p0)
    assert torch.equal(a, b)
    assert float((a - vc).abs().max()) <= 0.1 + 1e-6
    L = info["losses"].cpu().numpy()
    assert np.all(L[-1] < L[0])
    # spot-check 2 utterances of the batch against the oracle
    w = oracle_weights(m)
    idx = [0, 255]
    ref = oracle.emb_attack(w, cfg_of(z), vc[idx].cpu().numpy(), at[idx].cpu().numpy(), 0.1, 50,
                            p0[idx].cpu().numpy())
    d = np.abs(a[idx].detach().cpu().numpy() - ref)
    assert d.max() <= 1e-3 and d.mean() <= 1e-6
    # the bench's own precision: bf16 MFMA operands at B = 256
    a16, info16 = attack_utils.emb_attack(m, vc, at, 0.1, 50, ptb0=p0, precision="bf16", return_info=True)
    b16 = attack_utils.emb_attack(m, vc, at, 0.1, 50, ptb0=p0, precision="bf16")
    assert torch.equal(a16, b16)
    assert float((a16 - vc).abs().max()) <= 0.1 + 1e-6
    L16 = info16["losses"].cpu().numpy()
    assert np.all(L16[-1] < L16[0])
    assert float((a16 - a).abs().max()) <= 2e-2          # SURVEY 8(c) bf16 adv bound (n <= 100)


def test_bf16_mode_tracks_fp32(gpu, golden):
    """bf16 MFMA operands (fp32 accumulate, fp32 Adam state): SURVEY.md 8(c)
    tolerances - one-step gradient cosine >= 0.99 vs the reference, adv within
    2e-2 at n=100, final embedding loss within 5% of the fp32 reference's."""
    z = golden("full_T128")
    m = model_from_fixture(z).to(gpu)
    adv, info = attack_utils.emb_attack(m, _dev(z["vc_tgt"]), _dev(z["adv_tgt"]), 0.1, 100,
                                        ptb0=_dev(z["emb_ptb0"]), precision="bf16", return_info=True)
    g = info["grad0"].cpu().numpy().reshape(2, -1).astype(np.float64)
    r = z["emb_grad0"].reshape(2, -1).astype(np.float64)
    cos = (g * r).sum(1) / np.linalg.norm(g, axis=1) / np.linalg.norm(r, axis=1)
    assert cos.min() >= 0.99, cos
    assert np.abs(adv.detach().cpu().numpy() - z["emb_adv_n100"]).max() <= 2e-2
    L = info["losses"].cpu().numpy().T[:, -1]
    Lref = z["emb_losses_n1500"][:, 99]      # iteration 99 of the same trajectory
    assert np.all(np.abs(L - Lref) <= 0.05 * np.abs(Lref)), (L, Lref)


def test_bf16_batch_shard_invariance(gpu, golden):
    z = golden("full_T128")
    m = model_from_fixture(z).to(gpu)
    g = torch.Generator().manual_seed(9)
    vc, at, p0 = (torch.randn(32, 80, 128, generator=g).to(gpu) for _ in range(3))
    full = attack_utils.emb_attack(m, vc, at, 0.1, 10, ptb0=p0, precision="bf16").detach()
    lo = attack_utils.emb_attack(m, vc[:16], at[:16], 0.1, 10, ptb0=p0[:16], precision="bf16").detach()
    hi = attack_utils.emb_attack(m, vc[16:], at[16:], 0.1, 10, ptb0=p0[16:], precision="bf16").detach()
    assert torch.equal(torch.cat([lo, hi]), full)


def test_multi_gpu_driver_matches_single(gpu, golden):
    """shard.emb_attack_multi_gpu (one host thread per device) == one call; run
    here with the same device listed twice (the box has one GPU)."""
    import shard
    z = golden("small_T32")
    m = model_from_fixture(z).to(gpu)
    g = torch.Generator().manual_seed(4)
    vc, at, p0 = (torch.randn(5, 80, 32, generator=g).to(gpu) for _ in range(3))
    one = attack_utils.emb_attack(m, vc, at, 0.1, 8, ptb0=p0).detach()
    two = shard.emb_attack_multi_gpu([m, m], vc, at, 0.1, 8, ptb0=p0).detach()
    assert torch.equal(one, two)
    # configs[3]'s attack (fb) through the same driver on the full config
    zf = golden("full_T128")
    mf = model_from_fixture(zf).to(gpu)
    src, vc, at, p0 = (torch.randn(5, 80, 64, generator=g).to(gpu) for _ in range(4))
    one = attack_utils.fb_attack(mf, src, vc, at, 0.1, 4, ptb0=p0).detach()
    two = shard.attack_multi_gpu("fb", [mf, mf], src, vc, at, 0.1, 4, ptb0=p0).detach()
    assert torch.equal(one, two)


def test_pgd_update_matches_restatement(gpu, golden):
    """--update pgd (opt-in, north_star's sign-grad + eps-clamp; parity unpinned against the
    reference, which has no such attack): the GPU emb attack equals the CPU restatement of the
    mode (tests/test_oracle_golden.pgd_attack_np) except where a sign flips on a near-zero
    gradient, stays in the eps ball, and is deterministic."""
    from test_oracle_golden import pgd_attack_np
    z = golden("small_T32")
    m = model_from_fixture(z).to(gpu)
    args = (_dev(z["vc_tgt"]), _dev(z["adv_tgt"]), 0.1, 20)
    a = attack_utils.emb_attack(m, *args, ptb0=_dev(z["emb_ptb0"]), update="pgd", pgd_step=5e-3).detach()
    b = attack_utils.emb_attack(m, *args, ptb0=_dev(z["emb_ptb0"]), update="pgd", pgd_step=5e-3).detach()
    assert torch.equal(a, b)
    a = a.cpu().numpy()
    assert np.abs(a - z["vc_tgt"]).max() <= 0.1 + 1e-6
    ref = pgd_attack_np(oracle_weights(m), cfg_of(z), z["vc_tgt"], z["adv_tgt"], 0.1, 20, z["emb_ptb0"], 5e-3)
    d = np.abs(a - ref)
    assert np.mean(d <= 1e-5) >= 0.99, np.mean(d <= 1e-5)


def test_fp32_error_sits_on_near_zero_gradients(gpu, golden):
    """The fp32 tolerance calibration (tests/helpers.py TOL_ADV; profiles/r04/tol_calibration.md) as a
    test: the fused emb attack at n = 10 vs the reference's float64 run (calib_f64_T128.npz, made by
    tests/golden/make_calib.py) -- within TOL_ADV[10], mean at the reference's own fp32 level, and every
    element off by more than 3e-6 has |d loss / d ptb| below Adam's eps (1e-8: the regime where the
    step is linear in the gradient) and lies in one window of <= 16 frames of its utterance (the
    receptive field of a ReLU that flipped), not spread over the mel."""
    z, zf = golden("full_T128"), golden("calib_f64_T128")
    m = model_from_fixture(z).to(gpu)
    adv = attack_utils.emb_attack(m, _dev(z["vc_tgt"]), _dev(z["adv_tgt"]), 0.1, 10,
                                  ptb0=_dev(z["emb_ptb0"])).detach().cpu().numpy().astype(np.float64)
    d = np.abs(adv - zf["emb_adv_n10"])
    assert d.max() <= TOL_ADV[10], d.max()
    assert d.mean() <= 5e-8, d.mean()
    big = d > 3e-6
    if big.any():
        assert np.abs(zf["emb_grad0"])[big].max() < 1e-8
        for b in range(d.shape[0]):
            fr = np.where(big[b].any(0))[0]
            if fr.size:
                assert fr.max() - fr.min() < 16, (b, fr)
