"""CPU baseline: the reference's embedding attack restated in functional torch
(ATen CPU kernels, autograd, torch.optim.Adam) — the arithmetic the reference
itself runs on a CPU host.

TEST/BENCH INFRASTRUCTURE ONLY: used by bench.py's cpu_baseline leg (and tests)
as the timed CPU path; the product never imports it.  Pinned bitwise against
the reference's golden vectors in tests/test_oracle_golden.py.

Follows /root/reference/models.py:10-30 (pad_layer), 82-104 (conv_bank),
285-343 (SpeakerEncoder), 181-208 (ContentEncoder), 403-435 (Decoder) and
attack_utils.py:7-130 (e2e_attack, emb_attack, fb_attack).
"""
from typing import Dict

import torch
import torch.nn.functional as F


def _pad_conv(x, w, b, stride=1):
    k = w.shape[2]
    pad = (k // 2, k // 2 - 1) if k % 2 == 0 else (k // 2, k // 2)
    return F.conv1d(F.pad(x, pad, mode="reflect"), w, b, stride=stride)


def se_forward(sd: Dict[str, torch.Tensor], cfg: Dict, x: torch.Tensor, p="speaker_encoder.") -> torch.Tensor:
    act = (lambda t: F.leaky_relu(t)) if cfg["act"] == "lrelu" else F.relu
    nb = len(range(cfg["bank_scale"], cfg["bank_size"] + 1, cfg["bank_scale"]))
    outs = [act(_pad_conv(x, sd[f"{p}conv_bank.{i}.weight"], sd[f"{p}conv_bank.{i}.bias"])) for i in range(nb)]
    out = torch.cat(outs + [x], dim=1)
    out = act(_pad_conv(out, sd[p + "in_conv_layer.weight"], sd[p + "in_conv_layer.bias"]))
    for l in range(cfg["n_conv_blocks"]):
        s = cfg["subsample"][l]
        y = act(_pad_conv(out, sd[f"{p}first_conv_layers.{l}.weight"], sd[f"{p}first_conv_layers.{l}.bias"]))
        y = act(_pad_conv(y, sd[f"{p}second_conv_layers.{l}.weight"], sd[f"{p}second_conv_layers.{l}.bias"],
                          stride=s))
        if s > 1:
            out = F.avg_pool1d(out, kernel_size=s, ceil_mode=True)
        out = y + out
    out = F.adaptive_avg_pool1d(out, 1).squeeze(-1)
    for l in range(cfg["n_dense_blocks"]):
        y = act(F.linear(out, sd[f"{p}first_dense_layers.{l}.weight"], sd[f"{p}first_dense_layers.{l}.bias"]))
        y = act(F.linear(y, sd[f"{p}second_dense_layers.{l}.weight"], sd[f"{p}second_dense_layers.{l}.bias"]))
        out = y + out
    return F.linear(out, sd[p + "output_layer.weight"], sd[p + "output_layer.bias"])


def emb_attack(sd, cfg, vc_tgt, adv_tgt, eps, n_iters, ptb0, iter_hook=None, weight_grads=True):
    """attack_utils.py:51-86 with an explicit ptb0 (B=1 semantics per call).
    weight_grads=True keeps the reference's as-shipped cost: its model
    parameters require grad, so every backward also accumulates weight
    gradients."""
    se = cfg["SpeakerEncoder"] if "SpeakerEncoder" in cfg else cfg
    sd = {k: v.detach().clone().requires_grad_(weight_grads) for k, v in sd.items()}
    ptb = ptb0.clone().requires_grad_(True)
    opt = torch.optim.Adam([ptb])
    with torch.no_grad():
        org = se_forward(sd, se, vc_tgt)
        tgt = se_forward(sd, se, adv_tgt)
    for it in range(n_iters):
        adv = vc_tgt + eps * ptb.tanh()
        emb = se_forward(sd, se, adv)
        loss = F.mse_loss(emb, tgt) - 0.1 * F.mse_loss(emb, org)
        opt.zero_grad()
        loss.backward()
        opt.step()
        if iter_hook is not None:
            iter_hook(it)
    return (vc_tgt + eps * ptb.tanh()).detach()


def ce_forward(sd, cfg, x, p="content_encoder."):
    """ContentEncoder.forward -> mu (models.py:181-208)."""
    act = (lambda t: F.leaky_relu(t)) if cfg["act"] == "lrelu" else F.relu
    nb = len(range(cfg["bank_scale"], cfg["bank_size"] + 1, cfg["bank_scale"]))
    outs = [act(_pad_conv(x, sd[f"{p}conv_bank.{i}.weight"], sd[f"{p}conv_bank.{i}.bias"])) for i in range(nb)]
    out = torch.cat(outs + [x], dim=1)
    out = act(F.instance_norm(_pad_conv(out, sd[p + "in_conv_layer.weight"], sd[p + "in_conv_layer.bias"])))
    for l in range(cfg["n_conv_blocks"]):
        s = cfg["subsample"][l]
        y = act(F.instance_norm(_pad_conv(out, sd[f"{p}first_conv_layers.{l}.weight"],
                                          sd[f"{p}first_conv_layers.{l}.bias"])))
        y = act(F.instance_norm(_pad_conv(y, sd[f"{p}second_conv_layers.{l}.weight"],
                                          sd[f"{p}second_conv_layers.{l}.bias"], stride=s)))
        if s > 1:
            out = F.avg_pool1d(out, kernel_size=s, ceil_mode=True)
        out = y + out
    return _pad_conv(out, sd[p + "mean_layer.weight"], sd[p + "mean_layer.bias"])


def dec_forward(sd, cfg, z, cond, p="decoder."):
    """Decoder.forward (models.py:403-435) with append_cond / pixel_shuffle_1d / upsample."""
    act = (lambda t: F.leaky_relu(t)) if cfg["act"] == "lrelu" else F.relu

    def adain(y, c):
        h = c.shape[1] // 2
        return y * c[:, h:].unsqueeze(2) + c[:, :h].unsqueeze(2)

    out = act(F.instance_norm(_pad_conv(z, sd[p + "in_conv_layer.weight"], sd[p + "in_conv_layer.bias"])))
    for l in range(cfg["n_conv_blocks"]):
        up = cfg["upsample"][l]
        y = F.instance_norm(_pad_conv(out, sd[f"{p}first_conv_layers.{l}.weight"], sd[f"{p}first_conv_layers.{l}.bias"]))
        y = act(adain(y, F.linear(cond, sd[f"{p}conv_affine_layers.{2*l}.weight"],
                                  sd[f"{p}conv_affine_layers.{2*l}.bias"])))
        y = _pad_conv(y, sd[f"{p}second_conv_layers.{l}.weight"], sd[f"{p}second_conv_layers.{l}.bias"])
        if up > 1:
            B, C, W = y.shape
            y = y.contiguous().view(B, C // up, up, W).permute(0, 1, 3, 2).contiguous().view(B, C // up, W * up)
        y = F.instance_norm(y)
        y = act(adain(y, F.linear(cond, sd[f"{p}conv_affine_layers.{2*l+1}.weight"],
                                  sd[f"{p}conv_affine_layers.{2*l+1}.bias"])))
        out = y + (F.interpolate(out, scale_factor=up, mode="nearest") if up > 1 else out)
    return _pad_conv(out, sd[p + "out_conv_layer.weight"], sd[p + "out_conv_layer.bias"])


def inference(sd, cfg, src, tgt):
    """AdaInVC.inference (models.py:472-489)."""
    return dec_forward(sd, cfg["Decoder"], ce_forward(sd, cfg["ContentEncoder"], src),
                       se_forward(sd, cfg["SpeakerEncoder"], tgt))


def vc_attack(kind, sd, cfg, vc_src, vc_tgt, adv_tgt, eps, n_iters, ptb0, iter_hook=None, weight_grads=True):
    """e2e_attack (attack_utils.py:7-48) / fb_attack (89-130) with an explicit ptb0, as the
    reference runs them (the ContentEncoder recomputed inside every inference call)."""
    sd = {k: v.detach().clone().requires_grad_(weight_grads) for k, v in sd.items()}
    ptb = ptb0.clone().requires_grad_(True)
    opt = torch.optim.Adam([ptb])
    se = cfg["SpeakerEncoder"]
    with torch.no_grad():
        if kind == "e2e":
            org, tgt = inference(sd, cfg, vc_src, vc_tgt), inference(sd, cfg, vc_src, adv_tgt)
        else:
            org = se_forward(sd, se, inference(sd, cfg, vc_src, vc_tgt))
            tgt = se_forward(sd, se, adv_tgt)
    for it in range(n_iters):
        adv = vc_tgt + eps * ptb.tanh()
        out = inference(sd, cfg, vc_src, adv)
        if kind == "fb":
            out = se_forward(sd, se, out)
        loss = F.mse_loss(out, tgt) - 0.1 * F.mse_loss(out, org)
        opt.zero_grad()
        loss.backward()
        opt.step()
        if iter_hook is not None:
            iter_hook(it)
    return (vc_tgt + eps * ptb.tanh()).detach()


def pm_forward(sd, x):
    """PredictiveModel.forward (models/predictive_model.py:87-110), eval mode, functional ATen."""
    for i, s in enumerate([(1, 2), (2, 2), (2, 2), (2, 2), (2, 2), (2, 2), (2, 2)]):
        p = f"down_blocks.{i}.conv."
        x = F.conv2d(F.pad(x, (1, 1, 1, 1), mode="reflect"), sd[p + "1.weight"], sd[p + "1.bias"], stride=s)
        x = F.batch_norm(x, sd[p + "2.running_mean"], sd[p + "2.running_var"], sd[p + "2.weight"], sd[p + "2.bias"],
                         training=False, eps=1e-5)
        x = F.prelu(x, sd[p + "3.weight"])
    for i in range(5):
        p = f"up_blocks.{i}.conv_transpose.0."
        x = F.leaky_relu(F.conv_transpose2d(x, sd[p + "weight"], sd[p + "bias"], stride=2), 0.2)
    return torch.tanh(x)
