"""GPU: the 8-wave bf16 SpeakerEncoder engine (csrc/avc_fused8.hip) against the 4-wave one.

At the config.yaml shape and T = 128 the bf16 SE passes run se_fwd8 / se_bwd8 (two waves per SIMD,
each wave half of a layer's frames); AVC_FZ8=0 plans the 4-wave se_fwd_fused / se_bwd_fused.  Every
output element is accumulated by one wave with the same MFMA sequence over K, the reflect-pad
adjoint folds the same pad sums, the cross-wave reduction adds the same partials in the same order
and the head / Adam tails do the same per-element arithmetic, so the two engines agree BITWISE:
adversarial mels, per-iteration losses, grad0 and embeddings, for the emb attack (head fused in the
forward) and for e2e / fb (head backward fused in the SE backward; fb's SE(dec) hands its input
gradient on)."""
import pytest
import torch

import avc_native
from helpers import model_from_fixture

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def full(golden):
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")
    return model_from_fixture(golden("full_T128")).to(DEV)


def _ctx(m, fz8: str, monkeypatch, vc=False):
    monkeypatch.setenv("AVC_FZ8", fz8)
    ctx = avc_native.Context(avc_native.se_config(m.speaker_encoder), avc_native.flat_weights(m.speaker_encoder),
                             DEV.index or 0)
    if vc:
        mods = (m.content_encoder, m.decoder)
        flat = torch.cat([v.detach().reshape(-1).to("cpu", torch.float32) for md in mods
                          for v in md.state_dict().values()])
        ctx.attach_vc(avc_native.ce_config(m.content_encoder), avc_native.dec_config(m.decoder), flat)
    return ctx


@pytest.mark.parametrize("B,iters", [(6, 12), (256, 55)])
def test_emb_attack_8wave_bitwise(full, monkeypatch, B, iters):
    """B = 256 is the bench batch (one utterance per CU); 55 iterations = one captured 50-iteration
    graph + 5 launches."""
    g = torch.Generator().manual_seed(80 + B)
    vc, at, p0 = (torch.randn(B, 80, 128, generator=g).to(DEV) for _ in range(3))
    c8 = _ctx(full, "1", monkeypatch)
    a8, L8, g8 = c8.emb_attack(vc, at, p0, 0.1, iters, precision="bf16", want_losses=True, want_grad0=True)
    c4 = _ctx(full, "0", monkeypatch)
    a4, L4, g4 = c4.emb_attack(vc, at, p0, 0.1, iters, precision="bf16", want_losses=True, want_grad0=True)
    torch.cuda.synchronize()
    assert torch.isfinite(L8).all() and float(L8[-1].mean()) < float(L8[0].mean())
    assert torch.equal(L8, L4), float((L8 - L4).abs().max())
    assert torch.equal(g8, g4), float((g8 - g4).abs().max())
    assert torch.equal(a8, a4), float((a8 - a4).abs().max())


def test_emb_attack_8wave_is_planned(full, monkeypatch):
    """The bf16 plan at T = 128 names the 8-wave kernels (and only them); AVC_FZ8=0 the 4-wave."""
    g = torch.Generator().manual_seed(90)
    vc, at, p0 = (torch.randn(4, 80, 128, generator=g).to(DEV) for _ in range(3))
    for flag, fwd, bwd in (("1", "se_fwd8<bf16>", "se_bwd8<bf16>"), ("0", "se_fwd_fused<bf16>", "se_bwd_fused<bf16>")):
        c = _ctx(full, flag, monkeypatch)
        c.set_profiling(True)
        c.emb_attack(vc, at, p0, 0.1, 3, precision="bf16", use_graph=False)
        torch.cuda.synchronize()
        _, per = c.profile()
        assert fwd in per and bwd in per, (flag, sorted(per))
        c.set_profiling(False)


def test_se_forward_bf16_embedding_unchanged(full, monkeypatch):
    """Plain embeddings are fp32 (se_forward): the 8-wave switch must not touch them."""
    g = torch.Generator().manual_seed(91)
    x = torch.randn(5, 80, 128, generator=g).to(DEV)
    e8 = _ctx(full, "1", monkeypatch).se_forward(x)
    e4 = _ctx(full, "0", monkeypatch).se_forward(x)
    assert torch.equal(e8, e4)


@pytest.mark.parametrize("kind", ["e2e", "fb"])
def test_vc_attack_8wave_bitwise(full, monkeypatch, kind):
    """e2e / fb in bf16: SE(adv) forward (head mode 2) + its backward (head mode 3); fb also
    SE(dec) forward (head mode 1) + backward handing d loss / d dec on."""
    g = torch.Generator().manual_seed(92 if kind == "e2e" else 93)
    src, vc, at, p0 = (torch.randn(4, 80, 128, generator=g).to(DEV) for _ in range(4))
    c8 = _ctx(full, "1", monkeypatch, vc=True)
    a8, L8, g8 = c8.vc_attack(kind, src, vc, at, p0, 0.1, 7, precision="bf16", want_losses=True, want_grad0=True)
    c4 = _ctx(full, "0", monkeypatch, vc=True)
    a4, L4, g4 = c4.vc_attack(kind, src, vc, at, p0, 0.1, 7, precision="bf16", want_losses=True, want_grad0=True)
    torch.cuda.synchronize()
    assert torch.isfinite(L8).all()
    assert torch.equal(L8, L4), float((L8 - L4).abs().max())
    assert torch.equal(g8, g4), float((g8 - g4).abs().max())
    assert torch.equal(a8, a4), float((a8 - a4).abs().max())
