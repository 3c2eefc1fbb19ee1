"""GPU parity of the LeakyReLU AdaIN-VC variant (act="lrelu", models.py:107-118) against
the reference's outputs (tests/golden/full_lrelu_T128.npz): the fused kernels' generic
shapes with a runtime activation (the standard shape is compiled for ReLU only)."""
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
    check_adv(adv.detach().cpu().numpy(), z[f"{kind}_adv_n10"], 10)
    assert rel(info["grad0"].cpu().numpy(), z[f"{kind}_grad0"]) <= (TOL_GRAD_REL_VC if kind != "emb" else TOL_GRAD_REL)
