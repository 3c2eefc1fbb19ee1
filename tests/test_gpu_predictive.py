"""GPU parity of the VSMask PredictiveModel forward (csrc/avc_pm.hip)
against the reference's own outputs (tests/golden/predictive.npz) through the C ABI."""
import numpy as np
import pytest
import torch

import predictive_model
from helpers import rel

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TOL_PM_REL = 1e-5        # output (tanh-bounded) relative to max |y|, fp32


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
    return z, m.eval().to(DEV)


@pytest.mark.parametrize("xk,yk", [("x", "y"), ("x_odd", "y_odd")])
def test_predictive_golden(pm, xk, yk):
    z, m = pm
    out = m(torch.from_numpy(z[xk]).to(DEV)).cpu().numpy()
    assert out.shape == z[yk].shape
    assert rel(out, z[yk]) <= TOL_PM_REL, rel(out, z[yk])


def test_predictive_batch_invariant(pm):
    """B=256 windows: each equals its own B=1 run bitwise (per-window arithmetic only)."""
    z, m = pm
    g = torch.Generator().manual_seed(11)
    x = torch.randn(256, 1, 80, 100, generator=g).to(DEV)
    y = m(x)
    assert y.shape == (256, 1, 95, 63) and torch.isfinite(y).all()
    for i in (0, 77, 255):
        assert torch.equal(m(x[i:i + 1]), y[i:i + 1])


def test_predictive_rejects_train_mode_and_bad_shapes(pm):
    z, m = pm
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 2, 80, 100, device=DEV))
    m.train()
    try:
        with pytest.raises(RuntimeError, match="eval"):
            m(torch.zeros(1, 1, 80, 100, device=DEV))
    finally:
        m.eval()


def test_predictive_edge_kernels_bitwise(pm, monkeypatch):
    """The first (Cin = 1) and last (Cout = 1) layers run on pm_cin1 / pm_cout1, which repeat
    pm_conv's per-output arithmetic (same fma chain, same K slices summed in order): the whole
    forward equals the all-pm_conv one (AVC_PM_EDGE=0) bit for bit, odd window shapes included."""
    z, m = pm
    g = torch.Generator().manual_seed(12)
    for shape in ((37, 1, 80, 100), (3, 1, 72, 90)):
        x = torch.randn(*shape, generator=g).to(DEV)
        y1 = m(x)
        monkeypatch.setenv("AVC_PM_EDGE", "0")
        y0 = m(x)
        monkeypatch.delenv("AVC_PM_EDGE")
        torch.cuda.synchronize()
        assert torch.equal(y0, y1), float((y0 - y1).abs().max())
