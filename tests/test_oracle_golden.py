"""CPU: pin the numpy oracle (oracle/adain_vc.py) against vectors produced by the
real reference (tests/golden/make_golden.py), and pin our AdaInVC parameter
tree / seeded init against the reference's (weight hashes)."""
import hashlib
import json

import numpy as np
import pytest
import torch

import models
from helpers import TOL_GRAD_REL, TOL_GRAD_REL_VC, TOL_SE_REL, cfg_of, check_adv, model_from_fixture, oracle_weights, rel
from oracle import adain_vc as oracle


@pytest.mark.parametrize("name", ["small_T32", "small_T33", "full_T128", "full_T127"])
def test_speaker_encoder_forward(golden, name):
    z = golden(name)
    m = model_from_fixture(z)
    w = oracle_weights(m)
    se = cfg_of(z)["SpeakerEncoder"]
    for key, x in (("se_vc_tgt", "vc_tgt"), ("se_adv_tgt", "adv_tgt")):
        e, _ = oracle.se_forward(w, se, z[x])
        assert rel(e, z[key]) <= TOL_SE_REL


@pytest.mark.parametrize("name", ["small_T32", "small_T33", "full_T128", "full_T127"])
def test_inference_forward(golden, name):
    z = golden(name)
    w = oracle_weights(model_from_fixture(z))
    out = oracle.inference(w, cfg_of(z), z["vc_src"], z["vc_tgt"])
    assert rel(out, z["inference"]) <= 1e-5


@pytest.mark.parametrize("name,ns", [("small_T32", [1, 10, 100]), ("small_T33", [10]),
                                     ("full_T128", [1, 10]), ("full_T127", [10])])
def test_emb_attack(golden, name, ns):
    z = golden(name)
    w = oracle_weights(model_from_fixture(z))
    cfg = cfg_of(z)
    for n in ns:
        rec = {}
        adv = oracle.emb_attack(w, cfg, z["vc_tgt"], z["adv_tgt"], 0.1, n, z["emb_ptb0"], record=rec)
        check_adv(adv, z[f"emb_adv_n{n}"], n)
        assert rel(rec["grad0"], z["emb_grad0"]) <= TOL_GRAD_REL
        if f"emb_losses_n{n}" in z:
            np.testing.assert_allclose(rec["losses"], z[f"emb_losses_n{n}"], rtol=1e-4, atol=1e-9)


def test_emb_attack_batched_mean(golden):
    """The reference called on a [2,80,T] tensor == reduction="mean"."""
    z = golden("small_T32")
    w = oracle_weights(model_from_fixture(z))
    adv = oracle.emb_attack(w, cfg_of(z), z["vc_tgt"], z["adv_tgt"], 0.1, 10, z["emb_batched_ptb0"],
                            reduction="mean")
    check_adv(adv, z["emb_batched_adv_n10"], 10)


@pytest.mark.slow
def test_emb_attack_full_n100(golden):
    z = golden("full_T128")
    w = oracle_weights(model_from_fixture(z))
    adv = oracle.emb_attack(w, cfg_of(z), z["vc_tgt"], z["adv_tgt"], 0.1, 100, z["emb_ptb0"])
    check_adv(adv, z["emb_adv_n100"], 100)


def test_seeded_init_matches_reference(golden):
    """Our module tree draws the reference's default-init weights bit for bit."""
    z = golden("full_T128")
    hs = json.loads(str(z["weight_sha256"]))
    torch.manual_seed(0)
    sd = models.AdaInVC(cfg_of(z)).state_dict()
    assert list(sd.keys()) == list(hs.keys())
    for k, v in sd.items():
        assert hashlib.sha256(v.numpy().tobytes()).hexdigest() == hs[k], k


def test_small_state_dict_layout(golden):
    z = golden("small_T32")
    m = models.AdaInVC(cfg_of(z))
    keys = [k[2:] for k in z if k.startswith("w/")]
    assert list(m.state_dict().keys()) == keys
    for k, v in m.state_dict().items():
        assert tuple(v.shape) == z["w/" + k].shape


def test_pool_ceil_mode_edge():
    """F.avg_pool1d(k=2, ceil_mode=True) on [0..4] -> [0.5, 2.5, 4.0]."""
    x = np.arange(5, dtype=np.float32)[None, None, :]
    np.testing.assert_array_equal(oracle.avg_pool_ceil(x, 2)[0, 0], [0.5, 2.5, 4.0])


def test_reflect_pad_adjoint():
    """<P x, y> == <x, P^T y> for every bank/conv pad pair."""
    rng = np.random.default_rng(0)
    for k in range(1, 9):
        pl, pr = oracle.bank_pads(k)
        x = rng.standard_normal((2, 3, 11))
        y = rng.standard_normal((2, 3, 11 + pl + pr))
        lhs = (oracle.reflect_pad(x, pl, pr) * y).sum()
        rhs = (x * oracle.reflect_pad_backward(y, pl, pr, 11)).sum()
        assert abs(lhs - rhs) < 1e-9


def test_torch_cpu_baseline_is_reference_arithmetic(golden):
    """bench.py's CPU baseline (oracle/torch_cpu.py) reproduces the reference bitwise."""
    from oracle import torch_cpu
    z = golden("small_T32")
    m = model_from_fixture(z)
    sd = m.state_dict()
    for b in range(2):
        out = torch_cpu.emb_attack(sd, cfg_of(z), torch.from_numpy(z["vc_tgt"][b:b + 1]),
                                   torch.from_numpy(z["adv_tgt"][b:b + 1]), 0.1, 10,
                                   torch.from_numpy(z["emb_ptb0"][b:b + 1]))
        assert torch.equal(out, torch.from_numpy(z["emb_adv_n10"][b:b + 1]))


@pytest.mark.parametrize("name", ["small_T32", "small_T33", "full_T128"])
@pytest.mark.parametrize("kind", ["e2e", "fb"])
def test_vc_attacks(golden, name, kind):
    """e2e / fb attacks (attack_utils.py:7-48, 89-130): numpy Decoder backward and the
    attack loops vs the reference's 10-iteration outputs, grad0 and losses."""
    z = golden(name)
    if f"{kind}_adv_n10" not in z:
        pytest.skip("fixture has no VC attack vectors")
    w = oracle_weights(model_from_fixture(z))
    rec = {}
    adv = getattr(oracle, f"{kind}_attack")(w, cfg_of(z), z["vc_src"], z["vc_tgt"], z["adv_tgt"], 0.1, 10,
                                            z[f"{kind}_ptb0"], record=rec)
    check_adv(adv, z[f"{kind}_adv_n10"], 10, kind=kind)
    assert rel(rec["grad0"], z[f"{kind}_grad0"]) <= (TOL_GRAD_REL_VC if kind != "emb" else TOL_GRAD_REL)
    np.testing.assert_allclose(rec["losses"], z[f"{kind}_losses_n10"], rtol=1e-4, atol=1e-9)


@pytest.mark.slow
@pytest.mark.parametrize("kind", ["e2e", "fb"])
def test_vc_attacks_full_n100(golden, kind):
    """The reference's 100-iteration e2e / fb runs (full_T128_n100.npz, inputs of full_T128.npz)
    reproduced by the fp32 restatement: adv at SURVEY 8(c)'s n = 100 tolerances, grad0, losses."""
    z = golden("full_T128")
    zn = golden("full_T128_n100")
    w = oracle_weights(model_from_fixture(z))
    rec = {}
    adv = getattr(oracle, f"{kind}_attack")(w, cfg_of(z), z["vc_src"], z["vc_tgt"], z["adv_tgt"], 0.1, 100,
                                            zn[f"{kind}_ptb0"], record=rec)
    check_adv(adv, zn[f"{kind}_adv_n100"], 100, kind=kind)
    assert rel(rec["grad0"], zn[f"{kind}_grad0"]) <= TOL_GRAD_REL_VC
    np.testing.assert_allclose(rec["losses"], zn[f"{kind}_losses_n100"], rtol=2e-4, atol=1e-9)


def test_decoder_backward_is_adjoint():
    """<d out, J d cond> == <J^T d out, d cond> for the numpy Decoder (finite differences
    in float64 on a tiny random decoder)."""
    rng = np.random.default_rng(1)
    C, cfg = 8, dict(n_conv_blocks=2, upsample=[2, 1])
    sd = {"decoder.in_conv_layer.weight": rng.standard_normal((C, C, 1)), "decoder.in_conv_layer.bias": rng.standard_normal(C),
          "decoder.out_conv_layer.weight": rng.standard_normal((5, C, 1)), "decoder.out_conv_layer.bias": rng.standard_normal(5)}
    for l, up in enumerate(cfg["upsample"]):
        sd[f"decoder.first_conv_layers.{l}.weight"] = rng.standard_normal((C, C, 5)) * 0.3
        sd[f"decoder.first_conv_layers.{l}.bias"] = rng.standard_normal(C)
        sd[f"decoder.second_conv_layers.{l}.weight"] = rng.standard_normal((C * up, C, 5)) * 0.3
        sd[f"decoder.second_conv_layers.{l}.bias"] = rng.standard_normal(C * up)
        for q in (2 * l, 2 * l + 1):
            sd[f"decoder.conv_affine_layers.{q}.weight"] = rng.standard_normal((2 * C, 4)) * 0.5
            sd[f"decoder.conv_affine_layers.{q}.bias"] = rng.standard_normal(2 * C)
    w = oracle.Weights(sd, dtype=np.float64)
    z, cond = rng.standard_normal((2, C, 7)), rng.standard_normal((2, 4))
    st = []
    out = oracle.dec_forward(w, cfg, z, cond, st=st)
    g = rng.standard_normal(out.shape)
    gc = oracle.dec_backward(w, cfg, st, g)
    d = rng.standard_normal(cond.shape)
    h = 1e-6
    fd = ((oracle.dec_forward(w, cfg, z, cond + h * d) - oracle.dec_forward(w, cfg, z, cond - h * d)) * g).sum() / (2 * h)
    assert abs(fd - (gc * d).sum()) <= 1e-6 * max(1.0, abs(fd))


@pytest.mark.parametrize("kind", ["e2e", "fb"])
def test_torch_cpu_vc_baseline_matches_reference(golden, kind):
    """bench.py's e2e / fb CPU baseline (oracle/torch_cpu.vc_attack) vs the reference's outputs."""
    from oracle import torch_cpu
    z = golden("small_T32")
    sd = model_from_fixture(z).state_dict()
    out = torch_cpu.vc_attack(kind, sd, cfg_of(z), torch.from_numpy(z["vc_src"][:1]), torch.from_numpy(z["vc_tgt"][:1]),
                              torch.from_numpy(z["adv_tgt"][:1]), 0.1, 10, torch.from_numpy(z[f"{kind}_ptb0"][:1]))
    check_adv(out.numpy(), z[f"{kind}_adv_n10"][:1], 10, kind=kind)


def test_predictive_model_oracle_and_init(golden):
    """PredictiveModel (models/predictive_model.py:53-110): our module tree draws the
    reference's seeded init (hashes), and the numpy oracle reproduces the reference's eval
    forward on both window shapes of tests/golden/predictive.npz."""
    import predictive_model
    from oracle import predictive
    z = golden("predictive")
    torch.manual_seed(0)
    m = predictive_model.PredictiveModel()
    hs = json.loads(str(z["init_sha256"]))
    sd = m.state_dict()
    for k, h in hs.items():
        assert hashlib.sha256(sd[k].numpy().tobytes()).hexdigest() == h, k
    sdn = {k: v.numpy() for k, v in sd.items()}
    sdn.update({k[2:]: z[k] for k in z if k.startswith("p/")})
    for xk, yk in (("x", "y"), ("x_odd", "y_odd")):
        out = predictive.forward(sdn, z[xk])
        assert out.shape == z[yk].shape
        assert rel(out, z[yk]) <= 1e-5, rel(out, z[yk])


def test_torch_cpu_pm_baseline_matches_reference(golden):
    """bench.py's PredictiveModel CPU baseline (oracle/torch_cpu.pm_forward) vs the reference."""
    import predictive_model
    from oracle import torch_cpu
    z = golden("predictive")
    torch.manual_seed(0)
    sd = predictive_model.PredictiveModel().state_dict()
    for k in z:
        if k.startswith("p/"):
            sd[k[2:]].copy_(torch.from_numpy(z[k]))
    with torch.no_grad():
        out = torch_cpu.pm_forward(sd, torch.from_numpy(z["x"]))
    assert rel(out.numpy(), z["y"]) <= 1e-6


@pytest.mark.parametrize("kind", ["emb", "e2e", "fb"])
def test_lrelu_config(golden, kind):
    """act="lrelu" everywhere (models.py:107-118): the oracle's LeakyReLU forward and
    derivative vs the reference's outputs (tests/golden/full_lrelu_T128.npz)."""
    z = golden("full_lrelu_T128")
    w = oracle_weights(model_from_fixture(z))
    cfg = cfg_of(z)
    if kind == "emb":
        e, _ = oracle.se_forward(w, cfg["SpeakerEncoder"], z["vc_tgt"])
        assert rel(e, z["se_vc_tgt"]) <= TOL_SE_REL
        assert rel(oracle.inference(w, cfg, z["vc_src"], z["vc_tgt"]), z["inference"]) <= 1e-5
    rec = {}
    adv = oracle.attack(kind, w, cfg, z["vc_src"], z["vc_tgt"], z["adv_tgt"], 0.1, 10, z[f"{kind}_ptb0"], record=rec)
    check_adv(adv, z[f"{kind}_adv_n10"], 10, kind=kind)
    assert rel(rec["grad0"], z[f"{kind}_grad0"]) <= (TOL_GRAD_REL_VC if kind != "emb" else TOL_GRAD_REL)


def test_long_mixed_lengths_fixture(golden):
    """full_T300.npz (round 2): vc_src 280, vc_tgt 300, adv_tgt 260 frames, made by the
    reference itself: the oracle's SE / inference and its emb / e2e / fb attacks (n = 10)
    at these lengths."""
    z = golden("full_T300")
    w = oracle_weights(model_from_fixture(z))
    cfg = cfg_of(z)
    assert z["vc_src"].shape[2] == 280 and z["vc_tgt"].shape[2] == 300 and z["adv_tgt"].shape[2] == 260
    e, _ = oracle.se_forward(w, cfg["SpeakerEncoder"], z["vc_tgt"])
    assert rel(e, z["se_vc_tgt"]) <= TOL_SE_REL
    out = oracle.inference(w, cfg, z["vc_src"], z["vc_tgt"])
    assert out.shape == z["inference"].shape and rel(out, z["inference"]) <= 1e-5
    for kind in ("emb", "e2e", "fb"):
        rec = {}
        fn = getattr(oracle, f"{kind}_attack")
        args = (z["vc_tgt"], z["adv_tgt"]) if kind == "emb" else (z["vc_src"], z["vc_tgt"], z["adv_tgt"])
        adv = fn(w, cfg, *args, 0.1, 10, z[f"{kind}_ptb0"], record=rec)
        check_adv(adv, z[f"{kind}_adv_n10"], 10, kind=kind)
        assert rel(rec["grad0"], z[f"{kind}_grad0"]) <= (TOL_GRAD_REL if kind == "emb" else TOL_GRAD_REL_VC)
        np.testing.assert_allclose(rec["losses"], z[f"{kind}_losses_n10"], rtol=2e-4, atol=1e-9)


def pgd_attack_np(w, cfg, vc_tgt, adv_tgt, eps, n_iters, ptb0, step):
    """CPU restatement of the opt-in PGD update (include/avc.h AVC_UPDATE_PGD) for the emb
    attack: delta0 = eps*tanh(ptb0); delta <- clamp(delta - step*sign(dL/d delta), -eps, eps).
    Not the reference's update (parity unpinned): only the mode's own definition."""
    se = cfg["SpeakerEncoder"]
    dt = vc_tgt.dtype.type
    org, _ = oracle.se_forward(w, se, vc_tgt)
    tgt, _ = oracle.se_forward(w, se, adv_tgt)
    d = dt(eps) * np.tanh(ptb0.astype(vc_tgt.dtype))
    n_el = int(np.prod(org.shape[1:]))
    for _ in range(n_iters):
        out, st = oracle.se_forward(w, se, vc_tgt + d)
        g = oracle.se_backward(w, se, st, oracle.emb_loss_grad(out, tgt, org, n_el))
        d = np.clip(d - dt(step) * np.sign(g), -eps, eps).astype(vc_tgt.dtype)
    return vc_tgt + d


def test_pgd_restatement_properties(golden):
    """The PGD restatement stays inside the eps ball and lowers the embedding objective."""
    z = golden("small_T32")
    w = oracle_weights(model_from_fixture(z))
    cfg = cfg_of(z)
    adv = pgd_attack_np(w, cfg, z["vc_tgt"], z["adv_tgt"], 0.1, 20, z["emb_ptb0"], 5e-3)
    assert np.abs(adv - z["vc_tgt"]).max() <= 0.1 + 1e-6
    se = cfg["SpeakerEncoder"]
    tgt, _ = oracle.se_forward(w, se, z["adv_tgt"])
    e0, _ = oracle.se_forward(w, se, z["vc_tgt"] + 0.1 * np.tanh(z["emb_ptb0"]))
    e1, _ = oracle.se_forward(w, se, adv)
    assert ((e1 - tgt) ** 2).mean() < ((e0 - tgt) ** 2).mean()


def test_module_forwards_oracle(golden):
    """ContentEncoder.forward (mu, log_sigma), Decoder.forward and the PredictiveModel block chain
    of the reference (tests/golden/modules.npz, make_modules.py) reproduced by the restatements."""
    from oracle import predictive as po
    zm = golden("modules")
    hs = json.loads(str(zm["weight_sha256"]))
    torch.manual_seed(0)
    m = models.AdaInVC(cfg_of(zm))
    for k, v in m.state_dict().items():
        assert hashlib.sha256(v.numpy().tobytes()).hexdigest() == hs[k], k
    w = oracle_weights(m)
    cfg = cfg_of(zm)
    for T in (128, 300):
        mu, ls = oracle.ce_forward(w, cfg["ContentEncoder"], zm[f"ce_x_T{T}"], log_sigma=True)
        assert rel(mu, zm[f"ce_mu_T{T}"]) <= 1e-5 and rel(ls, zm[f"ce_log_sigma_T{T}"]) <= 1e-5
    for Tz in (16, 37):
        out = oracle.dec_forward(w, cfg["Decoder"], zm[f"dec_z_T{Tz}"], zm[f"dec_cond_T{Tz}"])
        assert rel(out, zm[f"dec_out_T{Tz}"]) <= 1e-5
    zp = golden("predictive")
    import predictive_model
    torch.manual_seed(0)
    pm = predictive_model.PredictiveModel()
    sd = {k: v.numpy().copy() for k, v in pm.state_dict().items()}
    for k in zp:
        if k.startswith("p/"):
            sd[k[2:]] = zp[k]
    # block by block, each fed the reference's output of the previous block: a block's own
    # numerics only (chained, an isolated PReLU / LeakyReLU sign flip at a near-zero
    # pre-activation amplifies through the later blocks)
    h = zm["pm_x"]
    for i, (_, _, st) in enumerate(po.DOWN):
        p = f"down_blocks.{i}.conv."
        y = po.conv2d_reflect(h, sd[p + "1.weight"], sd[p + "1.bias"], st)
        sc = sd[p + "2.weight"] / np.sqrt(sd[p + "2.running_var"] + np.float32(1e-5))
        y = (y - sd[p + "2.running_mean"][None, :, None, None]) * sc[None, :, None, None] + sd[p + "2.bias"][None, :, None, None]
        y = np.where(y >= 0, y, sd[p + "3.weight"][0] * y)
        assert rel(y, zm[f"pm_down{i}"]) <= 1e-5, (i, rel(y, zm[f"pm_down{i}"]))
        h = zm[f"pm_down{i}"]
    for i in range(len(po.UP)):
        p = f"up_blocks.{i}.conv_transpose.0."
        y = po.conv_transpose2d(h, sd[p + "weight"], sd[p + "bias"])
        y = np.where(y >= 0, y, np.float32(0.2) * y)
        assert rel(y, zm[f"pm_up{i}"]) <= 1e-5, (i, rel(y, zm[f"pm_up{i}"]))
        h = zm[f"pm_up{i}"]


def test_spectral_norm_decoder_oracle(golden):
    """sn=True Decoder (models.py:382; tests/golden/make_sn.py, made by the real reference): the seeded
    build reproduces the reference's weights and initial u / v (hashes), and the oracle's train-mode
    power iteration (oracle.spectral_norm_step, one per Decoder forward) reproduces inference, the e2e /
    fb attacks at n = 10 (adv, grad0, losses) and the u / v the reference's buffers hold afterwards."""
    z = golden("full_sn_T128")
    m = model_from_fixture(z)                       # asserts the per-tensor hashes (weights, u, v)
    assert m.decoder.sn and hasattr(m.decoder.in_conv_layer, "weight_orig")
    sd = {k: v.detach().numpy() for k, v in m.state_dict().items()}
    cfg = cfg_of(z)

    def uv_err(w, tag):
        return max(float(np.abs(w.d["decoder." + k.split("/", 1)[1]] - z[k]).max()) for k in z if k.startswith(tag + "/"))
    w = oracle.Weights(sd)
    out = oracle.inference(w, cfg, z["vc_src"], z["vc_tgt"])
    assert rel(out, z["inference"]) <= 1e-5
    assert uv_err(w, "uv_inference") <= 1e-6
    for kind in ("e2e", "fb"):
        w, rec = oracle.Weights(sd), {}
        adv = oracle.attack(kind, w, cfg, z["vc_src"], z["vc_tgt"], z["adv_tgt"], 0.1, 10, z[f"{kind}_ptb0"], record=rec)
        check_adv(adv, z[f"{kind}_adv_n10"], 10, kind=kind)
        assert rel(rec["grad0"], z[f"{kind}_grad0"]) <= TOL_GRAD_REL_VC
        np.testing.assert_allclose(rec["losses"], z[f"{kind}_losses_n10"], rtol=2e-4, atol=1e-9)
        assert uv_err(w, f"uv_{kind}") <= 1e-6        # 1 (fb) / 2 (e2e) precompute forwards + 10 iterations


def test_spectral_norm_eval_oracle(golden):
    """The eval-mode hook (tests/golden/make_sn_eval.py, the real reference after .eval()): no power
    iteration, sigma from the stored u / v -- inference at the initial and at a moved u / v, and the e2e
    attack at n = 10 (the Decoder's weights then fixed); the buffers never change."""
    z = golden("full_sn_eval_T128")
    m = model_from_fixture(z)
    sd = {k: v.detach().numpy() for k, v in m.state_dict().items()}
    cfg = cfg_of(z)
    w = oracle.Weights(dict(sd))
    w.sn_train = False
    u0 = {k: v.copy() for k, v in w.d.items() if k.endswith(("_u", "_v"))}
    assert rel(oracle.inference(w, cfg, z["vc_src"], z["vc_tgt"]), z["inference_eval"]) <= 1e-5
    for k, v in u0.items():
        assert np.array_equal(w.d[k], v), k
    w1 = oracle.Weights(dict(sd))
    w1.sn_train = False
    for k in z:
        if k.startswith("uv1/"):
            w1.d["decoder." + k.split("/", 1)[1]] = z[k]
    assert rel(oracle.inference(w1, cfg, z["vc_src"], z["vc_tgt"]), z["inference_eval_uv1"]) <= 1e-5
    w = oracle.Weights(dict(sd))
    w.sn_train = False
    adv = oracle.attack("e2e", w, cfg, z["vc_src"], z["vc_tgt"], z["adv_tgt"], 0.1, 10, z["e2e_ptb0_eval"])
    check_adv(adv, z["e2e_adv_n10_eval"], 10, kind="e2e")
