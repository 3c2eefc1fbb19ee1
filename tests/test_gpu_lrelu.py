"""GPU parity of the LeakyReLU AdaIN-VC variant (act="lrelu", models.py:107-118) against
the reference's outputs (tests/golden/full_lrelu_T128.npz): the fused kernels' generic
shapes with a runtime activation (the standard shape is compiled for ReLU only)."""
import os

import numpy as np
import pytest
import torch

import attack_utils
import avc_native
from helpers import TOL_GRAD_REL, TOL_GRAD_REL_VC, TOL_SE_REL, check_adv, model_from_fixture, rel

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


@pytest.fixture(scope="module")
def lrelu(golden):
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")
    z = golden("full_lrelu_T128")
    return z, model_from_fixture(z).to(DEV)


def test_lrelu_forward(lrelu):
    z, m = lrelu
    ctx = avc_native.context_for(m.speaker_encoder, DEV)
    assert ctx.engine_for(128) == "fused"
    assert rel(ctx.se_forward(_dev(z["vc_tgt"])).cpu().numpy(), z["se_vc_tgt"]) <= TOL_SE_REL
    assert rel(m.inference(_dev(z["vc_src"]), _dev(z["vc_tgt"])).cpu().numpy(), z["inference"]) <= 1e-4


@pytest.mark.parametrize("kind", ["emb", "e2e", "fb"])
def test_lrelu_attacks(lrelu, kind):
    z, m = lrelu
    t = {k: _dev(z[k]) for k in ("vc_src", "vc_tgt", "adv_tgt", f"{kind}_ptb0")}
    if kind == "emb":
        adv, info = attack_utils.emb_attack(m, t["vc_tgt"], t["adv_tgt"], 0.1, 10, ptb0=t["emb_ptb0"], return_info=True)
    else:
        fn = attack_utils.e2e_attack if kind == "e2e" else attack_utils.fb_attack
        adv, info = fn(m, t["vc_src"], t["vc_tgt"], t["adv_tgt"], 0.1, 10, ptb0=t[f"{kind}_ptb0"], return_info=True)
    check_adv(adv.detach().cpu().numpy(), z[f"{kind}_adv_n10"], 10, kind=kind)
    g = info["grad0"].cpu().numpy()
    if kind == "emb":
        assert rel(g, z[f"{kind}_grad0"]) <= TOL_GRAD_REL
    elif rel(g, z[f"{kind}_grad0"]) > TOL_GRAD_REL_VC:
        # the e2e / fb iteration-0 gradient is ill-conditioned at isolated units: the distance must be one
        # LeakyReLU unit within rounding of zero taking the other slope (helpers.vc_grad0_explained)
        from helpers import cfg_of, vc_grad0_explained
        for u in range(g.shape[0]):
            ok, rep = vc_grad0_explained(kind, m, cfg_of(z), [z[k][u:u + 1] for k in ("vc_src", "vc_tgt", "adv_tgt",
                                                                                    f"{kind}_ptb0")], g[u:u + 1])
            print(f"utterance {u}: {rep}")
            if not ok and os.path.isdir("gpurun_out"):
                np.save(f"gpurun_out/lrelu_{kind}_grad0.npy", g)
            assert ok, (u, rep)


@pytest.mark.parametrize("T", [300, 200])
def test_lrelu_long_engine_vs_oracle(lrelu, T):
    """LeakyReLU(0.01) on the long engine (T > 128: csrc/avc_long.hip's epilogues and its act'
    from the ballot words) vs the float64 oracle: SpeakerEncoder(x), the emb attack's grad0 /
    10-iteration adv / losses, inference, and the e2e / fb iteration-0 gradients (normwise per
    utterance, helpers.TOL_VC_GRAD_*).  vc_src / adv_tgt of other lengths on the way."""
    from helpers import TOL_VC_GRAD_L2_MAX, TOL_VC_GRAD_L2_MEDIAN, cfg_of, check_grad_flip_robust
    from oracle import adain_vc as oracle
    z, m = lrelu
    ctx = avc_native.context_for(m.speaker_encoder, DEV)
    assert ctx.engine_for(T) == "long"
    cfg = cfg_of(z)
    assert cfg["SpeakerEncoder"]["act"] == "lrelu"
    sd = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    w64 = oracle.Weights(sd, dtype=np.float64)
    g = torch.Generator().manual_seed(700 + T)
    vc, p0 = (torch.randn(2, 80, T, generator=g) for _ in range(2))
    at = torch.randn(2, 80, T - 21, generator=g)
    src = torch.randn(2, 80, T + 11, generator=g)
    d = lambda t: t.to(DEV)
    f64 = lambda t: t.double().numpy()
    e = ctx.se_forward(d(vc)).cpu().numpy()
    eo, _ = oracle.se_forward(w64, cfg["SpeakerEncoder"], f64(vc))
    assert rel(e, eo) <= TOL_SE_REL, rel(e, eo)
    adv, info = attack_utils.emb_attack(m, d(vc), d(at), 0.1, 10, ptb0=d(p0), return_info=True)
    rec = {}
    ref = oracle.emb_attack(w64, cfg, f64(vc), f64(at), 0.1, 10, f64(p0), record=rec)
    # mask flips at near-zero pre-activations (helpers.check_grad_flip_robust): seed 900's
    # utterance 1 at T = 200 has one, 2.8e-3 of max |grad| over columns 1-12
    check_grad_flip_robust(info["grad0"].cpu().numpy(), rec["grad0"])
    check_adv(adv.detach().cpu().numpy(), ref, 10)
    np.testing.assert_allclose(info["losses"].cpu().numpy().T, rec["losses"], rtol=2e-4, atol=1e-9)
    out = m.inference(d(src), d(vc)).cpu().numpy()
    ro = oracle.inference(w64, cfg, f64(src), f64(vc))
    assert out.shape == ro.shape and rel(out, ro) <= 1e-4, rel(out, ro)
    for kind in ("e2e", "fb"):
        rec = {}
        getattr(oracle, f"{kind}_attack")(w64, cfg, f64(src), f64(vc), f64(at), 0.1, 1, f64(p0), record=rec)
        fn = attack_utils.e2e_attack if kind == "e2e" else attack_utils.fb_attack
        _, info = fn(m, d(src), d(vc), d(at), 0.1, 1, ptb0=d(p0), return_info=True)
        gg = info["grad0"].cpu().numpy().astype(np.float64)
        err = [float(np.linalg.norm(gg[u] - rec["grad0"][u]) / np.linalg.norm(rec["grad0"][u])) for u in range(2)]
        # two utterances only (no meaningful median): each within the isolated-flip bound.  At T = 200
        # utterance 1 carries the SpeakerEncoder flip above (e2e 2.3e-4) and fb's second encoder pass
        # over the 216-frame decoder output adds its own (4.1e-4 / 6.8e-4); T = 300: <= 2e-5
        assert max(err) <= TOL_VC_GRAD_L2_MAX, (kind, err)
