"""GPU: module-level forwards the reference exposes besides the attacks, through libavc, against
the reference's own outputs (tests/golden/modules.npz, make_modules.py):
ContentEncoder.forward -> (mu, log_sigma) (/root/reference/models.py:181-210), Decoder.forward
(403-435), each on the fused (T <= 128) and the long engine."""
import numpy as np
import pytest
import torch

import models
from helpers import cfg_of, rel

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


@pytest.fixture(scope="module")
def mod(golden):
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")
    zm = golden("modules")
    torch.manual_seed(0)
    return zm, models.AdaInVC(cfg_of(zm)).to(DEV)


@pytest.mark.parametrize("T", [128, 300])
def test_content_encoder_forward(mod, T):
    zm, m = mod
    mu, ls = m.content_encoder(_dev(zm[f"ce_x_T{T}"]))
    assert mu.shape == zm[f"ce_mu_T{T}"].shape and ls.shape == zm[f"ce_log_sigma_T{T}"].shape
    assert rel(mu.cpu().numpy(), zm[f"ce_mu_T{T}"]) <= 1e-4, rel(mu.cpu().numpy(), zm[f"ce_mu_T{T}"])
    assert rel(ls.cpu().numpy(), zm[f"ce_log_sigma_T{T}"]) <= 1e-4


@pytest.mark.parametrize("Tz", [16, 37])
def test_decoder_forward(mod, Tz):
    zm, m = mod
    out = m.decoder(_dev(zm[f"dec_z_T{Tz}"]), _dev(zm[f"dec_cond_T{Tz}"]))
    assert out.shape == zm[f"dec_out_T{Tz}"].shape
    assert rel(out.cpu().numpy(), zm[f"dec_out_T{Tz}"]) <= 1e-4, rel(out.cpu().numpy(), zm[f"dec_out_T{Tz}"])


def test_module_forward_compose_to_inference(mod):
    """Decoder(ContentEncoder(src)[0], SpeakerEncoder(tgt)) == AdaInVC.inference, bitwise."""
    zm, m = mod
    src = _dev(zm["ce_x_T128"])
    tgt = torch.flip(src, dims=[0])
    mu, _ = m.content_encoder(src)
    out = m.decoder(mu, m.speaker_encoder(tgt))
    assert torch.equal(out, m.inference(src, tgt))


def test_standalone_module_refuses():
    ce = models.ContentEncoder(**models_cfg()["ContentEncoder"]).to(DEV)
    with pytest.raises(RuntimeError, match="AdaInVC"):
        ce(torch.zeros(1, 80, 64, device=DEV))


def models_cfg():
    import bench
    return bench.FULL_CFG
