"""GPU parity of the spectral-norm Decoder (sn=True, models.py:382) against the REAL reference's run
(tests/golden/full_sn_T128.npz, tests/golden/make_sn.py): the reference never calls .eval(), so every
Decoder forward -- the attack's precomputed targets and each iteration -- runs torch's spectral_norm
hook in train mode (one power iteration, weight_orig / sigma, u / v updated in place).  libavc runs
sn_power + sn_scale before each Decoder forward; the module's weight_u / weight_v buffers are loaded
before and written back after every call (avc_native.Context._sn_call).

Tolerances: the fp32 ones of tests/helpers.py (adv TOL_ADV[10], grad0 TOL_GRAD_REL_VC, loss history
rtol 2e-4); the Decoder output 1e-4 of its max (the fused Decoder's own bound); u / v 1e-5 (fp32 power
iteration in another summation order than torch's sgemv)."""
import copy

import numpy as np
import pytest
import torch

import attack_utils
import models
from helpers import TOL_ADV_MEAN_VC, TOL_GRAD_REL_VC, cfg_of, check_adv, model_from_fixture, rel
from oracle import adain_vc as oracle

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
FN = {"e2e": attack_utils.e2e_attack, "fb": attack_utils.fb_attack}


@pytest.fixture(scope="module")
def sn(golden):
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")
    z = golden("full_sn_T128")
    m = model_from_fixture(z)          # weights and initial u / v pinned by the reference's hashes
    assert m.decoder.sn
    return z, m


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _uv_err(model, z, tag):
    sd = model.decoder.state_dict()
    return max(float(np.abs(sd[k.split("/", 1)[1]].cpu().numpy() - z[k]).max()) for k in z if k.startswith(tag + "/"))


def test_sn_inference(sn):
    z, m0 = sn
    m = copy.deepcopy(m0).to(DEV)
    assert _uv_err(m, z, "uv0") == 0.0
    out = m.inference(_dev(z["vc_src"]), _dev(z["vc_tgt"])).cpu().numpy()
    assert rel(out, z["inference"]) <= 1e-4, rel(out, z["inference"])
    assert _uv_err(m, z, "uv_inference") <= 1e-5          # one power iteration, written back


@pytest.mark.parametrize("kind", ["e2e", "fb"])
def test_sn_attack_golden(sn, kind):
    """attack_utils.{e2e,fb}_attack at n = 10 on the sn=True model vs the reference's own run: adv, grad0,
    the loss history, and the u / v left in the module (e2e: 2 precompute + 10 Decoder forwards; fb 1 + 10)."""
    z, m0 = sn
    m = copy.deepcopy(m0).to(DEV)
    adv, info = FN[kind](m, _dev(z["vc_src"]), _dev(z["vc_tgt"]), _dev(z["adv_tgt"]), 0.1, 10,
                         ptb0=_dev(z[f"{kind}_ptb0"]), return_info=True)
    check_adv(adv.detach().cpu().numpy(), z[f"{kind}_adv_n10"], 10, kind=kind)
    assert rel(info["grad0"].cpu().numpy(), z[f"{kind}_grad0"]) <= TOL_GRAD_REL_VC
    np.testing.assert_allclose(info["losses"].cpu().numpy().T, z[f"{kind}_losses_n10"], rtol=2e-4, atol=1e-9)
    assert _uv_err(m, z, f"uv_{kind}") <= 1e-5


@pytest.mark.parametrize("kind", ["e2e", "fb"])
def test_sn_bf16_and_state_carries_over(sn, kind):
    """The bench precision on the sn=True model (B = 8, n = 20): deterministic from the same u / v,
    |adv - vc| <= eps, within SURVEY 8(c)'s bf16 bound (2e-2) of the fp32 attack from the same state, and
    the state carries over between calls as in the reference: a second call starts from the u / v the
    first left, i.e. equals the same call on a model given those buffers.  (No loss-decrease check: the
    power iteration changes the Decoder every forward, so the objective moves under the attack -- the
    reference's own fp32 e2e loss rises from -2.2e-3 to 5.6e-3 over 10 iterations in full_sn_T128.npz.)"""
    z, m0 = sn
    g = torch.Generator().manual_seed(88)
    src, vc, at, p0 = (torch.randn(8, 80, 128, generator=g).to(DEV) for _ in range(4))
    m1, m2, m4 = (copy.deepcopy(m0).to(DEV) for _ in range(3))
    a1 = FN[kind](m1, src, vc, at, 0.1, 20, ptb0=p0, precision="bf16").detach()
    a2 = FN[kind](m2, src, vc, at, 0.1, 20, ptb0=p0, precision="bf16").detach()
    a4 = FN[kind](m4, src, vc, at, 0.1, 20, ptb0=p0).detach()
    assert torch.equal(a1, a2)
    assert float((a1 - vc).abs().max()) <= 0.1 + 1e-6
    assert float((a1 - a4).abs().max()) <= 2e-2, float((a1 - a4).abs().max())
    assert _uv_err(m1, z, "uv0") > 0                      # the buffers moved
    state = {k: v.clone() for k, v in m1.decoder.state_dict().items()}
    b1 = FN[kind](m1, src, vc, at, 0.1, 20, ptb0=p0, precision="bf16").detach()   # from the advanced u / v
    m3 = copy.deepcopy(m0).to(DEV)
    m3.decoder.load_state_dict(state)
    b3 = FN[kind](m3, src, vc, at, 0.1, 20, ptb0=p0, precision="bf16").detach()
    assert torch.equal(b1, b3), float((b1 - b3).abs().max())
    for k, v in m3.decoder.state_dict().items():          # and both leave the same u / v
        assert torch.equal(v, m1.decoder.state_dict()[k]), k


def test_sn_eval_mode(golden):
    """After .eval() (tests/golden/make_sn_eval.py, the real reference in eval mode): no power iteration,
    sigma = u . (W v) from the stored u / v, the buffers untouched -- inference at the initial and at a
    moved u / v, and the e2e attack at n = 10 against the reference's adv."""
    z = golden("full_sn_eval_T128")
    m0 = model_from_fixture(z)
    m = copy.deepcopy(m0).to(DEV).eval()
    before = {k: v.clone() for k, v in m.decoder.state_dict().items()}
    out = m.inference(_dev(z["vc_src"]), _dev(z["vc_tgt"])).cpu().numpy()
    assert rel(out, z["inference_eval"]) <= 1e-4, rel(out, z["inference_eval"])
    out2 = m.inference(_dev(z["vc_src"]), _dev(z["vc_tgt"])).cpu().numpy()
    assert np.array_equal(out, out2)                       # no state moved between the calls
    for k, v in m.decoder.state_dict().items():
        assert torch.equal(v, before[k]), k
    with torch.no_grad():
        for k in z:
            if k.startswith("uv1/"):
                m.decoder.state_dict()[k.split("/", 1)[1]].copy_(_dev(z[k]))
    out = m.inference(_dev(z["vc_src"]), _dev(z["vc_tgt"])).cpu().numpy()
    assert rel(out, z["inference_eval_uv1"]) <= 1e-4, rel(out, z["inference_eval_uv1"])
    m = copy.deepcopy(m0).to(DEV).eval()
    adv, info = attack_utils.e2e_attack(m, _dev(z["vc_src"]), _dev(z["vc_tgt"]), _dev(z["adv_tgt"]), 0.1, 10,
                                        ptb0=_dev(z["e2e_ptb0_eval"]), return_info=True)
    g0, ref0 = info["grad0"].cpu().numpy(), z["e2e_grad0_eval"]
    assert rel(g0, ref0) <= TOL_GRAD_REL_VC, rel(g0, ref0)
    for k, v in m.decoder.state_dict().items():
        assert torch.equal(v.cpu(), m0.decoder.state_dict()[k].cpu()), k
    # The same attack with the eval-mode weights (weight_orig / u.(W v), oracle.spectral_norm_step) baked into a
    # plain sn=False Decoder: isolates the eval-mode hook from the attack's own fp32 conditioning.  On this input
    # the e2e objective takes an fp32 ReLU flip between iterations 5 and 10 (scripts/dbg/sn_eval_diag.py: GPU vs
    # float64 5.7e-6 at n = 5, 7.3e-5 at n = 10 -- the baked plain Decoder equally, 7.25e-5), so adv at n = 10 is
    # held to 2e-4 of the reference's run (mean within the VC bound) and to 1e-5 of the baked model.
    wo = oracle.Weights({k: v.detach().cpu().numpy() for k, v in m0.state_dict().items()})
    wo.sn_train = False
    oracle.spectral_norm_step(wo)
    cfg2 = cfg_of(z)
    cfg2["Decoder"] = dict(cfg2["Decoder"], sn=False)
    mb = models.AdaInVC(cfg2)
    mb.load_state_dict({k: (torch.from_numpy(np.ascontiguousarray(wo.d[k])) if k.startswith("decoder.")
                            else m0.state_dict()[k]) for k in mb.state_dict()})
    mb = mb.to(DEV)
    adv_b = attack_utils.e2e_attack(mb, _dev(z["vc_src"]), _dev(z["vc_tgt"]), _dev(z["adv_tgt"]), 0.1, 10,
                                    ptb0=_dev(z["e2e_ptb0_eval"]))
    assert float((adv - adv_b).abs().max()) <= 1e-5, float((adv - adv_b).abs().max())
    d = np.abs(adv.detach().cpu().numpy().astype(np.float64) - z["e2e_adv_n10_eval"])
    assert d.mean() <= TOL_ADV_MEAN_VC[10] and d.max() <= 2e-4, (d.mean(), d.max())
    # and back in train mode the hook iterates again (the buffers move)
    m.train()
    m.inference(_dev(z["vc_src"]), _dev(z["vc_tgt"]))
    assert any(not torch.equal(v.cpu(), m0.decoder.state_dict()[k].cpu())
               for k, v in m.decoder.state_dict().items() if k.endswith(("_u", "_v")))
