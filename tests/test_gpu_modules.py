"""GPU: module-level forwards the reference exposes besides the attacks, through libavc, against
the reference's own outputs (tests/golden/modules.npz, make_modules.py):
ContentEncoder.forward -> (mu, log_sigma) (/root/reference/models.py:181-210), Decoder.forward
(403-435), each on the fused (T <= 128) and the long engine."""
import ctypes

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


def test_predictive_blocks_forward(golden):
    """DownSamplingBlock / UpSamplingBlock.forward (models/predictive_model.py:28-29, 50-51) of the
    reference's PredictiveModel (weights of tests/golden/predictive.npz), each block fed the
    reference's output of the previous one; the chain of blocks + tanh equals the whole forward."""
    import predictive_model
    zm, zp = golden("modules"), golden("predictive")
    torch.manual_seed(0)
    pm = predictive_model.PredictiveModel()
    sd = pm.state_dict()
    for k in zp:
        if k.startswith("p/"):
            sd[k[2:]] = torch.from_numpy(zp[k])
    pm.load_state_dict(sd)
    pm = pm.eval().to(DEV)
    h = zm["pm_x"]
    names = [f"pm_down{i}" for i in range(7)] + [f"pm_up{i}" for i in range(5)]
    blocks = list(pm.down_blocks) + list(pm.up_blocks)
    for blk, name in zip(blocks, names):
        y = blk(_dev(h)).cpu().numpy()
        assert y.shape == zm[name].shape, name
        assert rel(y, zm[name]) <= 1e-5, (name, rel(y, zm[name]))
        h = zm[name]
    x = _dev(zm["pm_x"])
    chain = x
    for blk in blocks:
        chain = blk(chain)
    full = pm(x)
    assert full.shape == chain.shape
    assert float((torch.tanh(chain) - full).abs().max()) <= 1e-4


def test_predictive_block_wrong_channels():
    """A block fed the wrong channel count raises like torch's Conv2d shape check instead of reading
    past the input (the C ABI checks Cin too)."""
    import avc_native
    import predictive_model
    torch.manual_seed(0)
    pm = predictive_model.PredictiveModel().eval().to(DEV)
    ctx = avc_native.pm_context_for(pm, DEV)
    with pytest.raises(RuntimeError, match="channels"):
        pm.down_blocks[3](torch.zeros(1, 32, 20, 13, device=DEV))
    x = torch.zeros(1, 32, 20, 13, device=DEV)
    rc = avc_native.lib().avc_pm_block_forward(ctx.h, 3, ctypes.c_void_p(x.data_ptr()), 1, 32, 20, 13,
                                               ctypes.c_void_p(x.data_ptr()), None)
    assert rc != 0 and b"channels" in avc_native.lib().avc_last_error()
