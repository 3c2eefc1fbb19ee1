"""Drop-in replacement for /root/reference/attack.py (attack.py:10-114) on MI355X.

Same positional arguments and flags as the reference:

  python attack.py MODEL_DIR VC_TGT ADV_TGT OUTPUT [--vc_src SRC] [--eps 0.1]
                   [--n_iters 1500] [--attack_type {e2e,emb,fb}]

plus `--precision {fp32,bf16}` (default fp32, the reference's arithmetic) and the opt-in
`--update pgd [--pgd_step S]` (sign-gradient step + eps-clamp, include/avc.h AVC_UPDATE_PGD;
default `adam`, the reference's update).  The
wav -> mel front end, the attack loop and the Griffin-Lim back end all run in
libavc's HIP kernels (data_utils.py / attack_utils.py of this package); the
output is written as 16-bit PCM WAV like soundfile's default.
"""
import argparse

import torch

from attack_utils import e2e_attack, emb_attack, fb_attack
from data_utils import denormalize, file2mel, load_model, mel2wav, normalize, write_wav


def main(model_dir: str, vc_src: str, vc_tgt: str, adv_tgt: str, output: str, eps: float, n_iters: int,
         attack_type: str, precision: str = "fp32", update: str = "adam", pgd_step: float = 1e-3):
    """attack.py:10-75."""
    assert attack_type == "emb" or vc_src is not None
    model, config, attr, device = load_model(model_dir)

    vc_tgt = file2mel(vc_tgt, **config["preprocess"])
    adv_tgt = file2mel(adv_tgt, **config["preprocess"])
    vc_tgt = normalize(vc_tgt, attr)
    adv_tgt = normalize(adv_tgt, attr)
    vc_tgt = torch.from_numpy(vc_tgt).float().T.unsqueeze(0).to(device)
    adv_tgt = torch.from_numpy(adv_tgt).float().T.unsqueeze(0).to(device)

    if attack_type != "emb":
        vc_src = file2mel(vc_src, **config["preprocess"])
        vc_src = normalize(vc_src, attr)
        vc_src = torch.from_numpy(vc_src).float().T.unsqueeze(0).to(device)

    kw = dict(precision=precision, update=update, pgd_step=pgd_step)
    if attack_type == "e2e":
        adv_inp = e2e_attack(model, vc_src, vc_tgt, adv_tgt, eps, n_iters, **kw)
    elif attack_type == "emb":
        adv_inp = emb_attack(model, vc_tgt, adv_tgt, eps, n_iters, **kw)
    elif attack_type == "fb":
        adv_inp = fb_attack(model, vc_src, vc_tgt, adv_tgt, eps, n_iters, **kw)
    else:
        raise NotImplementedError()

    adv_inp = adv_inp.squeeze(0).T
    adv_inp = denormalize(adv_inp.data.cpu().numpy(), attr)
    adv_inp = mel2wav(adv_inp, **config["preprocess"])
    write_wav(output, adv_inp, config["preprocess"]["sample_rate"])


def build_parser() -> argparse.ArgumentParser:
    """attack.py:77-113."""
    p = argparse.ArgumentParser()
    p.add_argument("model_dir", type=str, help="The directory of model files.")
    p.add_argument("vc_tgt", type=str,
                   help="The target utterance to be defended, providing vocal timbre in voice conversion.")
    p.add_argument("adv_tgt", type=str, help="The target used in adversarial attack.")
    p.add_argument("output", type=str, help="The output defended utterance.")
    p.add_argument("--vc_src", type=str, default=None,
                   help="The source utterance providing linguistic content in voice conversion "
                        "(required in end-to-end and feedback attack).")
    p.add_argument("--eps", type=float, default=0.1, help="The maximum amplitude of the perturbation.")
    p.add_argument("--n_iters", type=int, default=1500,
                   help="The number of iterations for updating the perturbation.")
    p.add_argument("--attack_type", type=str, choices=["e2e", "emb", "fb"], default="emb",
                   help="The type of adversarial attack to use (end-to-end, embedding, or feedback attack).")
    p.add_argument("--precision", type=str, choices=["fp32", "bf16"], default="fp32",
                   help="Arithmetic of the attack loop (fp32 = the reference's).")
    p.add_argument("--update", type=str, choices=["adam", "pgd"], default="adam",
                   help="Perturbation update: adam (the reference's tanh + Adam) or pgd (opt-in sign-gradient "
                        "step + eps-clamp).")
    p.add_argument("--pgd_step", type=float, default=1e-3, help="Step size of the pgd update.")
    return p


if __name__ == "__main__":
    main(**vars(build_parser().parse_args()))
