"""GPU: the persistent emb attack kernel (se_attack_fused; round 6).

The bf16 emb attack at the standard shape runs all its iterations in ONE launch: each workgroup runs its
utterance's forward (+ fused head) and backward (+ Adam) back to back, with the step counter read once per
launch and advanced by fz_step_add after it.  The per-element arithmetic is the per-pass kernels' (the same
device functions), so the result must equal the per-pass launches (AVC_PERSIST=0) BIT FOR BIT: adv, the
loss history and grad0 -- across graph-sized and odd iteration counts, repeated calls on one workspace, and
a batch of more workgroups than the chip holds at once (B > 256: the later workgroups start after earlier
ones finished, which must not see an advanced step counter)."""
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


def _ctx(m):
    return avc_native.Context(avc_native.se_config(m.speaker_encoder), avc_native.flat_weights(m.speaker_encoder),
                              DEV.index or 0)


@pytest.mark.parametrize("B,n,T", [(6, 55, 128), (5, 1, 128), (300, 3, 128), (6, 55, 120), (4, 7, 97)])
def test_persistent_equals_per_pass(full, B, n, T, monkeypatch):
    """T = 128: the standard kernels; T = 120 / 97: the runtime-length ones (shape 16)."""
    g = torch.Generator().manual_seed(9300 + B + n + T)
    vc, at, p0 = (torch.randn(B, 80, T, generator=g).to(DEV) for _ in range(3))
    a = _ctx(full)
    a.ktime_start()
    r1 = a.emb_attack(vc, at, p0, 0.1, n, precision="bf16", want_losses=True, want_grad0=True)
    kt = a.ktime_stop()
    assert kt.get("se_attack_fused<bf16>", (0, 0))[0] == 1, kt          # one launch for the whole call
    assert "se_bwd_fused<bf16>" not in kt, kt
    again = a.emb_attack(vc, at, p0, 0.1, n, precision="bf16", want_losses=True, want_grad0=True)
    monkeypatch.setenv("AVC_PERSIST", "0")
    b = _ctx(full)
    r2 = b.emb_attack(vc, at, p0, 0.1, n, precision="bf16", want_losses=True, want_grad0=True)
    for x, y, z in zip(r1, r2, again):
        assert torch.equal(x, y), float((x - y).abs().max())
        assert torch.equal(x, z)
    assert float((r1[0] - vc).abs().max()) <= 0.1 + 1e-6
