"""Diagnostic: pm_mfma split-K tickets vs pm_reduce, same inputs, B = 256 and B = 1."""
import os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "attack-vc_amd"), ROOT]
import predictive_model
torch.manual_seed(0)
m = predictive_model.PredictiveModel().eval().cuda()
x = torch.randn(256, 1, 80, 100, generator=torch.Generator().manual_seed(3)).cuda()
def run(t, xx):
    os.environ["AVC_PM_TICKET"] = t
    y = m(xx); torch.cuda.synchronize(); return y
a = run("1", x); b = run("0", x); a2 = run("1", x)
print("B=256 ticket vs reduce: max", float((a - b).abs().max()), "n diff", int((a != b).sum()), "ticket rerun equal", bool(torch.equal(a, a2)))
for i in (0, 1, 255):
    s1 = run("1", x[i:i+1]); s0 = run("0", x[i:i+1])
    print(f"B=1 window {i}: ticket vs reduce max {float((s1 - s0).abs().max()):.3e}; ticket vs batched {float((s1 - a[i:i+1]).abs().max()):.3e}; reduce vs batched(reduce) {float((s0 - b[i:i+1]).abs().max()):.3e}")
