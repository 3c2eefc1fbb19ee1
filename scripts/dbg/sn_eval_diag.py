"""Diagnostic: the e2e attack on the eval-mode sn=True Decoder vs the same model with the eval-mode weights
(weight_orig / sigma) baked into a plain Decoder, vs the float64 oracle, at n = 1, 2, 5, 10."""
import copy, json, os, sys
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "attack-vc_amd"), ROOT]
import attack_utils, models
from helpers import model_from_fixture, cfg_of
from oracle import adain_vc as oracle
DEV = torch.device("cuda:0")
z = dict(np.load(os.path.join(ROOT, "tests/golden/full_sn_eval_T128.npz")))
m0 = model_from_fixture(z)
sd = {k: v.detach().numpy() for k, v in m0.state_dict().items()}
cfg = cfg_of(z)
# baked: plain Decoder with weight = weight_orig / sigma (torch's eval-mode compute_weight)
cfg2 = json.loads(json.dumps(cfg)); cfg2["Decoder"]["sn"] = False
mb = models.AdaInVC(cfg2)
wo = oracle.Weights(dict(sd)); wo.sn_train = False
oracle.spectral_norm_step(wo)            # eval-mode weights: weight_orig / (u . W v), fp32
sd2 = {k: (torch.from_numpy(np.ascontiguousarray(wo.d[k])) if k.startswith("decoder.") else m0.state_dict()[k])
       for k in mb.state_dict()}
mb.load_state_dict(sd2)
d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)
ins = [d(z[k]) for k in ("vc_src", "vc_tgt", "adv_tgt", "e2e_ptb0_eval")]
w64 = oracle.Weights(dict(sd), dtype=np.float64); w64.sn_train = False
for n in (1, 2, 5, 10):
    me = copy.deepcopy(m0).to(DEV).eval()
    a_sn, i_sn = attack_utils.e2e_attack(me, *ins[:3], 0.1, n, ptb0=ins[3], return_info=True)
    a_bk, i_bk = attack_utils.e2e_attack(copy.deepcopy(mb).to(DEV), *ins[:3], 0.1, n, ptb0=ins[3], return_info=True)
    rec = {}
    f = lambda a: np.asarray(a, np.float64)
    a64 = oracle.attack("e2e", w64, cfg, f(z["vc_src"]), f(z["vc_tgt"]), f(z["adv_tgt"]), 0.1, n, f(z["e2e_ptb0_eval"]), record=rec)
    g64 = rec["grad0"]
    e = lambda a: float(np.abs(a.detach().cpu().numpy() - a64).max())
    eg = lambda i: float(np.abs(i["grad0"].cpu().numpy() - g64).max() / np.abs(g64).max())
    print(f"n={n}: adv sn-eval vs f64 {e(a_sn):.2e} (grad0 {eg(i_sn):.2e}); baked vs f64 {e(a_bk):.2e} (grad0 {eg(i_bk):.2e}); "
          f"sn-eval vs baked {float((a_sn - a_bk).abs().max()):.2e}; losses sn {i_sn['losses'][:, 0].tolist()[:3]} "
          f"baked {i_bk['losses'][:, 0].tolist()[:3]} f64 {list(rec['losses'][0][:3]) if np.ndim(rec['losses'])==2 else list(rec['losses'][:3])}", flush=True)
