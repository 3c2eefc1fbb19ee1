"""GPU parity of the VSMask mel loop (libavc avc_vsmask_protect / avc_vsmask_apply_header,
/root/reference/vsmask.py:177-208, utils/audio.py:77-116, models/header_model.py:70-95)
against the numpy restatement oracle/vsmask.py.

  * bit-exact: the loop restatement in float32 fed with libavc's own per-window predictor
    outputs (the PredictiveModel is batch-invariant bitwise, test_gpu_predictive.py) must
    equal the GPU protect_mel exactly -- gather, window order, crop, band edges, clamp;
  * end to end: against the restatement in float64 with the float64 PredictiveModel oracle
    (pinned by the reference's own outputs in tests/golden/predictive.npz), TOL_VSM_ABS.
"""
import numpy as np
import pytest
import torch

import avc_native
import predictive_model
import vsmask
from oracle import predictive as po
from oracle import vsmask as vo

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TOL_VSM_ABS = 2e-6      # protected log-mel, fp32 predictor vs float64 (outputs are tanh-bounded sums)


@pytest.fixture(scope="module")
def pm(golden):
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")
    z = golden("predictive")
    torch.manual_seed(0)
    m = predictive_model.PredictiveModel()
    sd = m.state_dict()
    for k in z:
        if k.startswith("p/"):
            sd[k[2:]].copy_(torch.from_numpy(z[k]))
    sd64 = {k: v.detach().numpy().astype(np.float64) for k, v in m.state_dict().items() if v.is_floating_point()}
    return m.eval().to(DEV), sd64


def _inputs(B, T, seed, Th=100):
    g = torch.Generator().manual_seed(seed)
    mel = torch.randn(B, 1, 80, T, generator=g) * 0.5 - 1.0
    hdr = (torch.rand(1, 1, 80, Th, generator=g) - 0.5) * 0.2
    return mel, hdr


@pytest.mark.parametrize("B,T,W,S", [(1, 100, 100, 10), (2, 101, 100, 10), (2, 237, 100, 10),
                                     (1, 400, 100, 10), (3, 180, 100, 7), (1, 260, 120, 16)])
def test_vsmask_combine_bitexact(pm, B, T, W, S):
    m, _ = pm
    mel, hdr = _inputs(B, T, T + W + S)
    melg, hdrg = mel.to(DEV), hdr.to(DEV)
    ctx = avc_native.pm_context_for(m, DEV)
    out = ctx.protect(melg, hdrg, W, S, 0.1, 0.05, 0.08).cpu().numpy()
    nw = vo.n_windows(T, W, S)
    assert avc_native.vsmask_windows(T, W, S) == nw
    if nw:
        wins = torch.stack([melg[b, :, :, S * k:S * k + W] for b in range(B) for k in range(nw)])
        ys = ctx.forward(wins).cpu().numpy().reshape(B, nw, 1, *ctx.out_shape(80, W))
    it = iter(range(nw))

    def pred(w):            # called once per window in loop order, on all B utterances
        k = next(it)
        return ys[:, k]
    ref = vo.protect_mel(mel.numpy(), hdr.numpy(), pred, W, S, 0.1, 0.05, 0.08)
    assert np.array_equal(out, ref), np.abs(out - ref).max()


@pytest.mark.parametrize("T", [150, 263])
def test_vsmask_vs_float64_oracle(pm, T):
    m, sd64 = pm
    mel, hdr = _inputs(1, T, 7 * T)
    vs = vsmask.VSMask(None, None, device="cuda:0")
    vs.predictive_model = m
    vs.header.header = hdr.to(DEV)
    out = vs.protect_mel(mel.to(DEV)).cpu().numpy()
    ref = vo.protect_mel(mel.numpy().astype(np.float64), hdr.numpy().astype(np.float64),
                         lambda w: po.forward(sd64, w))
    assert np.abs(out - ref).max() <= TOL_VSM_ABS, np.abs(out - ref).max()
    # the band clamp is active: some perturbation saturates at each band's epsilon
    d = out - mel.numpy()
    assert np.isclose(np.abs(d[0, 0, :24]).max(), 0.1, atol=1e-6)


def test_vsmask_shapes_and_cli(pm, tmp_path):
    m, _ = pm
    mel, hdr = _inputs(1, 130, 5)
    torch.save(m.state_dict(), tmp_path / "pm.pt")
    torch.save(hdr, tmp_path / "hdr.pt")
    vs = vsmask.VSMask(str(tmp_path / "pm.pt"), str(tmp_path / "hdr.pt"), device="cuda:0")
    x4 = mel.to(DEV)
    o4 = vs.protect_mel(x4)
    o3 = vs.protect_mel(x4[:, 0])                   # the 3-D [1, F, T] mel waveform_to_mel returns
    o2 = vs.protect_mel(x4[0, 0])
    assert o3.shape == (1, 80, 130) and o2.shape == (80, 130)
    assert torch.equal(o4[:, 0], o3) and torch.equal(o4[0, 0], o2)
    np.save(tmp_path / "mel.npy", mel[0].numpy())
    vsmask.main(["--predictive_model", str(tmp_path / "pm.pt"), "--header", str(tmp_path / "hdr.pt"),
                 "--input", str(tmp_path / "mel.npy"), "--output", str(tmp_path / "out.npy")])
    assert np.array_equal(np.load(tmp_path / "out.npy"), o3.cpu().numpy())


def test_apply_header_bitexact():
    g = torch.Generator().manual_seed(3)
    hdr = (torch.rand(1, 1, 80, 100, generator=g) - 0.5)
    h = vsmask.UniversalPerturbationHeader(device="cuda:0")
    h.header = hdr.to(DEV)
    for T in (40, 100, 211):
        mel = torch.rand(2, 1, 80, T, generator=g) * 2 - 1
        out = h.apply_header(mel.to(DEV)).cpu().numpy()
        assert np.array_equal(out, vo.apply_header(mel.numpy(), hdr.numpy()))


def test_vsmask_errors(pm):
    m, _ = pm
    ctx = avc_native.pm_context_for(m, DEV)
    mel = torch.zeros(1, 1, 80, 150, device=DEV)
    with pytest.raises(RuntimeError):
        ctx.protect(mel, torch.zeros(1, 1, 79, 100, device=DEV))     # header bins != mel bins
    with pytest.raises(RuntimeError):
        ctx.protect(mel, None, 100, 0)                               # future_step 0 (range() step)
    with pytest.raises(RuntimeError):
        ctx.protect(mel[0], None)                                    # not [B, 1, F, T]
    with pytest.raises(RuntimeError, match="too small"):
        ctx.protect(mel, None, 64, 16)                               # window too short for the predictor
    out = ctx.protect(mel, None)                                     # no header: zero mel stays bounded
    assert torch.isfinite(out).all()
