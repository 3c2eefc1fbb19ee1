"""GPU parity when the attack's inputs have different lengths, as real utterances do.

The reference never requires vc_src, vc_tgt and adv_tgt to match: attack.py:49-56 builds
each from its own wav; emb_attack embeds adv_tgt on its own (attack_utils.py:74-75);
inference(vc_src, .) takes its output length from vc_src (models.py:472-489).  Here the
library gets them through the *_emb entry points (adv_tgt embedded by avc_se_forward
first) and is compared with the float64 numpy oracle, which handles any lengths."""
import numpy as np
import pytest
import torch

import attack_utils
from helpers import TOL_GRAD_REL, TOL_VC_GRAD_L2_MAX, TOL_VC_GRAD_L2_MEDIAN, cfg_of, model_from_fixture, rel
from oracle import adain_vc as oracle

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TOL_DEC_REL = 1e-4


@pytest.fixture(scope="module")
def full(golden):
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")
    z = golden("full_T128")
    m = model_from_fixture(z).to(DEV)
    sd = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    return z, m, oracle.Weights(sd, dtype=np.float64)


def _inputs(seed, B, lens):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(B, 80, t, generator=g) for t in lens]


@pytest.mark.parametrize("Tt,Ta", [(100, 120), (64, 33)])
def test_emb_attack_other_adv_length(full, Tt, Ta):
    z, m, w64 = full
    vc, at, p0 = _inputs(Tt + Ta, 3, (Tt, Ta, Tt))
    adv, info = attack_utils.emb_attack(m, vc.to(DEV), at.to(DEV), 0.1, 10, ptb0=p0.to(DEV), return_info=True)
    rec = {}
    ref = oracle.emb_attack(w64, cfg_of(z), vc.double().numpy(), at.double().numpy(), 0.1, 10, p0.double().numpy(),
                            record=rec)
    assert adv.shape == vc.shape
    assert rel(info["grad0"].cpu().numpy(), rec["grad0"]) <= TOL_GRAD_REL
    d = np.abs(adv.detach().cpu().numpy() - ref)
    assert d.max() <= 1e-4 and d.mean() <= 1e-7, (d.max(), d.mean())


def test_inference_other_tgt_length(full):
    z, m, w64 = full
    src, tgt = _inputs(7, 2, (100, 64))
    out = m.inference(src.to(DEV), tgt.to(DEV)).cpu().numpy()
    ref = oracle.inference(w64, cfg_of(z), src.double().numpy(), tgt.double().numpy())
    assert out.shape == ref.shape == (2, 80, 104)
    assert rel(out, ref) <= TOL_DEC_REL, rel(out, ref)


@pytest.mark.parametrize("kind", ["e2e", "fb"])
def test_vc_attack_three_lengths(full, kind):
    """vc_src 96 frames, vc_tgt 112, adv_tgt 80: iteration-0 gradient per utterance vs the
    float64 oracle (normwise, helpers.TOL_VC_GRAD_*), and the loss trajectory."""
    z, m, w64 = full
    src, vc, at, p0 = _inputs(11 if kind == "e2e" else 12, 4, (96, 112, 80, 112))
    fn = attack_utils.e2e_attack if kind == "e2e" else attack_utils.fb_attack
    adv, info = fn(m, src.to(DEV), vc.to(DEV), at.to(DEV), 0.1, 3, ptb0=p0.to(DEV), return_info=True)
    rec = {}
    getattr(oracle, f"{kind}_attack")(w64, cfg_of(z), src.double().numpy(), vc.double().numpy(),
                                      at.double().numpy(), 0.1, 3, p0.double().numpy(), record=rec)
    assert adv.shape == vc.shape
    g = info["grad0"].cpu().numpy().astype(np.float64)
    e = [float(np.linalg.norm(g[u] - rec["grad0"][u]) / np.linalg.norm(rec["grad0"][u])) for u in range(4)]
    assert max(e) <= TOL_VC_GRAD_L2_MAX and float(np.median(e)) <= TOL_VC_GRAD_L2_MEDIAN, e
    np.testing.assert_allclose(info["losses"].cpu().numpy().T, rec["losses"], rtol=1e-3, atol=1e-9)


def test_mismatched_batch_rejected(full):
    z, m, _ = full
    vc, at = _inputs(3, 2, (64, 64))
    with pytest.raises(RuntimeError, match="batch"):
        attack_utils.emb_attack(m, vc.to(DEV), at[:1].to(DEV), 0.1, 1)


def test_train_mode_dropout_rejected(full):
    """The reference leaves the model in train mode (attack.py:38): with dropout_rate > 0 its
    loop is random; libavc refuses such a module instead of silently differing."""
    import models
    cfg = cfg_of(full[0])
    cfg["SpeakerEncoder"] = dict(cfg["SpeakerEncoder"], dropout_rate=0.5)
    torch.manual_seed(0)
    m = models.AdaInVC(cfg).to(DEV)
    x = torch.zeros(1, 80, 64, device=DEV)
    with pytest.raises(NotImplementedError, match="dropout"):
        attack_utils.emb_attack(m, x, x, 0.1, 1)
    m.eval()                                   # eval: dropout is the identity -> allowed
    attack_utils.emb_attack(m, x, x, 0.1, 1)
