"""GPU: the standard-shape kernels at runtime lengths (se_*_fused<*, 16>; round 6).

Real utterances of 65-127 frames used to run on the shape-generic instances (SH = 8: runtime bank loop,
4-deep weight ring, unfused head), about twice a 128-frame utterance's cost per iteration.  The config.yaml
model at any T in (64, 128] has the 128-frame kernels' fragment classes (8, 8, 4, 4, 2, 2, 1 -- upper
bounds of its layer lengths), so those kernels run it with the frame counts as runtime values.  The
per-element arithmetic (GEMM K order, epilogues, pooling tails, fused head, Adam) is the generic
instances', so the two must agree BIT FOR BIT -- adv, the loss history and grad0 -- in both precisions,
for the emb attack and for the e2e / fb attacks (whose SpeakerEncoder passes use them too).
AVC_FUSED_RT=0 plans the generic instances (read when a workspace is planned: a fresh context)."""
import pytest
import torch

import attack_utils
import avc_native
from helpers import model_from_fixture

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def full(golden):
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")
    return model_from_fixture(golden("full_T128")).to(DEV)


def _ctx(m):
    return avc_native.Context(avc_native.se_config(m.speaker_encoder), avc_native.flat_weights(m.speaker_encoder),
                              DEV.index or 0)


@pytest.mark.parametrize("T", [127, 120, 113, 100, 65])
@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_std_rt_equals_generic_emb(full, T, prec, monkeypatch):
    m = full
    g = torch.Generator().manual_seed(9000 + T)
    vc, at, p0 = (torch.randn(6, 80, T, generator=g).to(DEV) for _ in range(3))
    a = _ctx(m)
    r1 = a.emb_attack(vc, at, p0, 0.1, 55, precision=prec, want_losses=True, want_grad0=True)
    monkeypatch.setenv("AVC_FUSED_RT", "0")
    b = _ctx(m)
    r2 = b.emb_attack(vc, at, p0, 0.1, 55, precision=prec, want_losses=True, want_grad0=True)
    for x, y in zip(r1, r2):
        assert torch.equal(x, y), float((x - y).abs().max())
    e1, e2 = a.se_forward(vc), b.se_forward(vc)
    assert torch.equal(e1, e2)


@pytest.mark.parametrize("kind", ["e2e", "fb"])
def test_std_rt_equals_generic_vc(full, kind, monkeypatch):
    """e2e / fb, bf16, T = 120 (content length 15) and vc_src of 104 frames: the SpeakerEncoder passes on the
    runtime-length standard kernels equal the generic ones bitwise (the Decoder runs its generic kernels
    either way)."""
    m = full
    g = torch.Generator().manual_seed(9100)
    src = torch.randn(3, 80, 104, generator=g).to(DEV)
    vc, at, p0 = (torch.randn(3, 80, 120, generator=g).to(DEV) for _ in range(3))
    fn = attack_utils.e2e_attack if kind == "e2e" else attack_utils.fb_attack
    a1, i1 = fn(m, src, vc, at, 0.1, 12, ptb0=p0, precision="bf16", return_info=True)
    monkeypatch.setenv("AVC_FUSED_RT", "0")
    import copy
    m2 = copy.deepcopy(m)                     # a fresh model object: its own (re-planned) libavc contexts
    a2, i2 = fn(m2, src, vc, at, 0.1, 12, ptb0=p0, precision="bf16", return_info=True)
    assert torch.equal(a1, a2), float((a1 - a2).abs().max())
    assert torch.equal(i1["grad0"], i2["grad0"])
    assert torch.equal(i1["losses"], i2["losses"])
