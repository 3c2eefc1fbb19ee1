"""Drop-in replacement for /root/reference/attack_utils.py on MI355X.

Same function names, argument order and meaning as the reference:

  emb_attack(model, vc_tgt, adv_tgt, eps, n_iters)            attack_utils.py:51-86
  e2e_attack(model, vc_src, vc_tgt, adv_tgt, eps, n_iters)    attack_utils.py:7-48
  fb_attack(model, vc_src, vc_tgt, adv_tgt, eps, n_iters)     attack_utils.py:89-130

`model` is any module with the reference's AdaInVC tree (the reference's own
models.AdaInVC or ours in models.py).  The per-iteration loop (tanh
reparameterisation, SpeakerEncoder forward, MSE loss, input-gradient backward,
Adam step) runs entirely inside libavc's HIP kernels; this module only draws
the initial perturbation exactly like the reference and hands device pointers
over the C ABI (avc_native.py).

Differences from the reference, all documented in DESIGN.md:
  * no tqdm bar (the loop never returns to the host between iterations);
  * weight .grad of the model is not touched (the reference accumulates unused
    weight gradients);
  * a [B,80,T] batch is B independent attacks by default
    (reduction="independent"); reduction="mean" reproduces the reference called
    on the batched tensor (its MSE mean over the whole batch);
  * vc_src, vc_tgt and adv_tgt may have different lengths (attack.py loads each
    from its own wav), exactly as in the reference;
  * a module with dropout_rate > 0 in training mode is refused (the reference
    would apply random dropout inside the loop; see check_no_train_dropout).
"""
from typing import Optional

import torch
import torch.nn as nn

from avc_native import check_no_train_dropout, context_for, vc_context_for


def _draw_ptb(vc_tgt: torch.Tensor) -> torch.Tensor:
    # attack_utils.py:68 — same generator, device and call, so a seeded caller
    # gets the reference's perturbation bit for bit.
    return torch.zeros_like(vc_tgt).normal_(0, 1)


def emb_attack(model: nn.Module, vc_tgt: torch.Tensor, adv_tgt: torch.Tensor, eps: float, n_iters: int,
               *, ptb0: Optional[torch.Tensor] = None, reduction: str = "independent",
               precision: str = "fp32", return_info: bool = False, update: str = "adam", pgd_step: float = 1e-3):
    """Embedding attack: perturb vc_tgt so SpeakerEncoder(vc_tgt + eps*tanh(ptb))
    approaches SpeakerEncoder(adv_tgt) and leaves SpeakerEncoder(vc_tgt)
    (attack_utils.py:51-86).  Returns vc_tgt + eps*tanh(ptb) ([B,80,T], fp32).

    Keyword extensions: ptb0 (explicit initial perturbation), reduction,
    precision ("fp32"), return_info (also return {"losses": [n_iters,B],
    "grad0": d loss/d ptb at iteration 0}), update ("adam", the reference's; "pgd": the
    opt-in sign-gradient + eps-clamp update of include/avc.h AVC_UPDATE_PGD, step pgd_step)."""
    check_no_train_dropout(model.speaker_encoder)
    if ptb0 is None:
        ptb0 = _draw_ptb(vc_tgt)
    ctx = context_for(model.speaker_encoder, vc_tgt.device)
    out, losses, grad0 = ctx.emb_attack(vc_tgt.detach().float(), adv_tgt.detach().float(), ptb0.detach().float(),
                                        eps, n_iters, precision=precision, reduction=reduction,
                                        want_losses=return_info, want_grad0=return_info, update=update,
                                        pgd_step=pgd_step)
    # the reference returns a graph-attached tensor (requires_grad=True); callers use .data
    out.requires_grad_(True)
    if return_info:
        return out, {"losses": losses, "grad0": grad0}
    return out


def _vc_attack(kind, model, vc_src, vc_tgt, adv_tgt, eps, n_iters, ptb0, reduction, precision, return_info,
               update="adam", pgd_step=1e-3):
    if ptb0 is None:
        ptb0 = _draw_ptb(vc_tgt)
    ctx = vc_context_for(model, vc_tgt.device)
    out, losses, grad0 = ctx.vc_attack(kind, vc_src.detach().float(), vc_tgt.detach().float(),
                                       adv_tgt.detach().float(), ptb0.detach().float(), eps, n_iters,
                                       precision=precision, reduction=reduction,
                                       want_losses=return_info, want_grad0=return_info, update=update,
                                       pgd_step=pgd_step)
    out.requires_grad_(True)
    if return_info:
        return out, {"losses": losses, "grad0": grad0}
    return out


def e2e_attack(model: nn.Module, vc_src: torch.Tensor, vc_tgt: torch.Tensor, adv_tgt: torch.Tensor,
               eps: float, n_iters: int, *, ptb0: Optional[torch.Tensor] = None, reduction: str = "independent",
               precision: str = "fp32", return_info: bool = False, update: str = "adam", pgd_step: float = 1e-3):
    """End-to-end attack (attack_utils.py:7-48): perturb vc_tgt so that
    inference(vc_src, vc_tgt + eps*tanh(ptb)) approaches inference(vc_src, adv_tgt) and
    leaves inference(vc_src, vc_tgt).  Keyword extensions as emb_attack."""
    return _vc_attack("e2e", model, vc_src, vc_tgt, adv_tgt, eps, n_iters, ptb0, reduction, precision, return_info,
                      update, pgd_step)


def fb_attack(model: nn.Module, vc_src: torch.Tensor, vc_tgt: torch.Tensor, adv_tgt: torch.Tensor,
              eps: float, n_iters: int, *, ptb0: Optional[torch.Tensor] = None, reduction: str = "independent",
              precision: str = "fp32", return_info: bool = False, update: str = "adam", pgd_step: float = 1e-3):
    """Feedback attack (attack_utils.py:89-130): perturb vc_tgt so that
    SpeakerEncoder(inference(vc_src, adv)) approaches SpeakerEncoder(adv_tgt) and leaves
    SpeakerEncoder(inference(vc_src, vc_tgt)).  Keyword extensions as emb_attack."""
    return _vc_attack("fb", model, vc_src, vc_tgt, adv_tgt, eps, n_iters, ptb0, reduction, precision, return_info,
                      update, pgd_step)
