"""CPU oracle: numpy restatement of the reference AdaIN-VC attack path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product (attack-vc_amd/) imports,
links or executes this module; only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg use it, and only as the checker / the timed CPU
baseline.  It is pinned against golden vectors produced by the real reference
(tests/golden/make_golden.py -> tests/golden/*.npz; tests/test_oracle_golden.py).

Every function restates the reference's arithmetic, citing the file:line of
/root/reference it follows.  Activations are [B, C, T] like the reference.
The backward pass is written out by hand (input-gradient only: the reference
also accumulates weight gradients it never uses, attack_utils.py:83, SURVEY.md
8(a) A13; those do not influence the result).

dtype: float32 reproduces the reference's arithmetic type; float64 is used to
measure fp32 drift.
"""
import numpy as np
from numpy.lib.stride_tricks import sliding_window_view

# ----------------------------------------------------------------------------------
# primitives
# ----------------------------------------------------------------------------------


def bank_pads(k):
    """models.py:23-27 (pad_layer): even k -> (k//2, k//2-1), odd k -> (k//2, k//2)."""
    return (k // 2, k // 2 - 1) if k % 2 == 0 else (k // 2, k // 2)


def reflect_pad(x, pl, pr):
    """models.py:28, F.pad(mode="reflect") (edge sample not repeated)."""
    if pl == 0 and pr == 0:
        return x
    return np.pad(x, ((0, 0), (0, 0), (pl, pr)), mode="reflect")


def reflect_pad_backward(gxp, pl, pr, T):
    """Adjoint of reflect_pad: fold the padded gradient back onto [0,T)."""
    g = gxp[:, :, pl:pl + T].copy()
    for i in range(pl):           # padded[i] = x[pl - i]
        g[:, :, pl - i] += gxp[:, :, i]
    for i in range(pr):           # padded[pl + T + i] = x[T - 2 - i]
        g[:, :, T - 2 - i] += gxp[:, :, pl + T + i]
    return g


def conv1d_valid(xp, W, b, stride=1):
    """nn.Conv1d on an already padded input (models.py:29 layer(inp)).
    xp [B,Ci,Tp], W [Co,Ci,k], b [Co] -> [B,Co,Tout]."""
    Co, Ci, k = W.shape
    win = sliding_window_view(xp, k, axis=2)[:, :, ::stride, :]     # [B,Ci,Tout,k]
    B, _, Tout, _ = win.shape
    cols = np.ascontiguousarray(win.transpose(0, 2, 1, 3)).reshape(B, Tout, Ci * k)
    out = cols @ W.reshape(Co, Ci * k).T                              # [B,Tout,Co]
    out = out.transpose(0, 2, 1)
    if b is not None:
        out = out + b[None, :, None]
    return np.ascontiguousarray(out)


def conv1d_valid_dgrad(gy, W, stride, Tp):
    """Input gradient of conv1d_valid: gy [B,Co,Tout] -> g_xp [B,Ci,Tp]."""
    Co, Ci, k = W.shape
    B, _, Tout = gy.shape
    gcols = gy.transpose(0, 2, 1) @ W.reshape(Co, Ci * k)             # [B,Tout,Ci*k]
    gcols = gcols.reshape(B, Tout, Ci, k)
    gxp = np.zeros((B, Ci, Tp), dtype=gy.dtype)
    for j in range(k):
        gxp[:, :, j:j + stride * (Tout - 1) + 1:stride] += gcols[:, :, :, j].transpose(0, 2, 1)
    return gxp


def pad_conv(x, W, b, stride=1):
    """models.py:10-30 pad_layer: reflect pad by kernel size, then conv."""
    pl, pr = bank_pads(W.shape[2])
    return conv1d_valid(reflect_pad(x, pl, pr), W, b, stride)


def pad_conv_dgrad(gy, W, stride, T):
    pl, pr = bank_pads(W.shape[2])
    gxp = conv1d_valid_dgrad(gy, W, stride, T + pl + pr)
    return reflect_pad_backward(gxp, pl, pr, T)


def relu(x):
    """models.py:107-118 get_act("relu")."""
    return np.maximum(x, 0)


def acts(cfg):
    """models.py:107-118 get_act: "lrelu" -> LeakyReLU(0.01), anything else ReLU.
    Returns (act, act') with act' evaluated on the activation's output (same sign as
    its input, which is what torch's threshold / leaky_relu backward tests)."""
    if cfg.get("act") == "lrelu":
        return (lambda t: np.where(t > 0, t, t * t.dtype.type(0.01)),
                lambda y: np.where(y > 0, y.dtype.type(1), y.dtype.type(0.01)))
    return relu, (lambda y: (y > 0).astype(y.dtype))


def avg_pool_ceil(x, s):
    """F.avg_pool1d(kernel=s, ceil_mode=True) (models.py:206,303): the last
    window of an odd-length input averages the single remaining sample."""
    B, C, T = x.shape
    To = -(-T // s)
    out = np.zeros((B, C, To), dtype=x.dtype)
    for t in range(To):
        lo, hi = s * t, min(s * t + s, T)
        out[:, :, t] = x[:, :, lo:hi].sum(axis=2) / x.dtype.type(hi - lo)
    return out


def avg_pool_ceil_backward(g, s, T):
    B, C, To = g.shape
    gx = np.zeros((B, C, T), dtype=g.dtype)
    for t in range(To):
        lo, hi = s * t, min(s * t + s, T)
        gx[:, :, lo:hi] += (g[:, :, t] / g.dtype.type(hi - lo))[:, :, None]
    return gx


def instance_norm(x, eps=1e-5):
    """nn.InstanceNorm1d(affine=False) (models.py:176,396): biased variance over T."""
    mu = x.mean(axis=2, keepdims=True)
    var = ((x - mu) ** 2).mean(axis=2, keepdims=True)
    return (x - mu) / np.sqrt(var + x.dtype.type(eps))


def linear(x, W, b):
    """nn.Linear (models.py:276-282, 398)."""
    return x @ W.T + b


# ----------------------------------------------------------------------------------
# weights
# ----------------------------------------------------------------------------------


class Weights:
    """state_dict view: w("speaker_encoder.conv_bank.0.weight") -> ndarray."""

    def __init__(self, state, dtype=np.float32):
        self.d = {k: np.asarray(v, dtype=dtype) for k, v in state.items()}

    def __call__(self, key):
        return self.d[key]


# ----------------------------------------------------------------------------------
# SpeakerEncoder (models.py:213-343)
# ----------------------------------------------------------------------------------


def se_forward(w, cfg, x, p="speaker_encoder."):
    """SpeakerEncoder.forward (models.py:327-343). Returns (emb, stash)."""
    ks = list(range(cfg["bank_scale"], cfg["bank_size"] + 1, cfg["bank_scale"]))
    relu, _ = acts(cfg)
    st = {"x": x, "bank": []}
    outs = []
    for i, k in enumerate(ks):                                         # conv_bank 82-104
        o = relu(pad_conv(x, w(f"{p}conv_bank.{i}.weight"), w(f"{p}conv_bank.{i}.bias")))
        outs.append(o)
    st["bank"] = outs
    cat = np.concatenate(outs + [x], axis=1)                           # models.py:103
    h = relu(pad_conv(cat, w(p + "in_conv_layer.weight"), w(p + "in_conv_layer.bias")))  # 337-338
    st["h0"] = h
    st["blocks"] = []
    for l in range(cfg["n_conv_blocks"]):                              # conv_blocks 285-305
        s = cfg["subsample"][l]
        a1 = relu(pad_conv(h, w(f"{p}first_conv_layers.{l}.weight"), w(f"{p}first_conv_layers.{l}.bias")))
        a2 = relu(pad_conv(a1, w(f"{p}second_conv_layers.{l}.weight"),
                           w(f"{p}second_conv_layers.{l}.bias"), stride=s))
        res = avg_pool_ceil(h, s) if s > 1 else h
        st["blocks"].append((h, a1, a2))
        h = a2 + res
    st["hN"] = h
    e = h.mean(axis=2)                                                 # AdaptiveAvgPool1d 275,340
    st["dense"] = []
    for l in range(cfg["n_dense_blocks"]):                             # dense_blocks 307-325
        y1 = relu(linear(e, w(f"{p}first_dense_layers.{l}.weight"), w(f"{p}first_dense_layers.{l}.bias")))
        y2 = relu(linear(y1, w(f"{p}second_dense_layers.{l}.weight"), w(f"{p}second_dense_layers.{l}.bias")))
        st["dense"].append((y1, y2))
        e = y2 + e
    emb = linear(e, w(p + "output_layer.weight"), w(p + "output_layer.bias"))   # 342
    return emb, st


def se_backward(w, cfg, st, g_emb, p="speaker_encoder."):
    """Input gradient d(loss)/dx of se_forward given d(loss)/d(emb)."""
    _, d = acts(cfg)
    g = g_emb @ w(p + "output_layer.weight")
    for l in reversed(range(cfg["n_dense_blocks"])):
        y1, y2 = st["dense"][l]
        gy2 = g * d(y2)
        gy1 = (gy2 @ w(f"{p}second_dense_layers.{l}.weight")) * d(y1)
        g = g + gy1 @ w(f"{p}first_dense_layers.{l}.weight")
    T_N = st["hN"].shape[2]
    gh = np.repeat((g / g.dtype.type(T_N))[:, :, None], T_N, axis=2)
    for l in reversed(range(cfg["n_conv_blocks"])):
        s = cfg["subsample"][l]
        h, a1, a2 = st["blocks"][l]
        T = h.shape[2]
        g2 = gh * d(a2)
        ga1 = pad_conv_dgrad(g2, w(f"{p}second_conv_layers.{l}.weight"), s, T)
        g1 = ga1 * d(a1)
        gx = pad_conv_dgrad(g1, w(f"{p}first_conv_layers.{l}.weight"), 1, T)
        gres = avg_pool_ceil_backward(gh, s, T) if s > 1 else gh
        gh = gx + gres
    T = st["x"].shape[2]
    g0 = gh * d(st["h0"])
    Wi = w(p + "in_conv_layer.weight")
    gcat = np.einsum("oc,bot->bct", Wi[:, :, 0], g0)
    nb = len(st["bank"])
    cb = st["bank"][0].shape[1]
    gx = gcat[:, nb * cb:, :].copy()                                   # cat passthrough
    for i, o in enumerate(st["bank"]):
        gb = gcat[:, i * cb:(i + 1) * cb, :] * d(o)
        gx += pad_conv_dgrad(gb, w(f"{p}conv_bank.{i}.weight"), 1, T)
    return gx


# ----------------------------------------------------------------------------------
# ContentEncoder (models.py:121-210) forward, Decoder (models.py:346-435) forward + backward
# ----------------------------------------------------------------------------------


def ce_forward(w, cfg, x, p="content_encoder.", log_sigma=False):
    """ContentEncoder.forward -> mu (models.py:181-208; log_sigma unused by inference), or
    (mu, log_sigma) (models.py:208-210) with log_sigma=True."""
    relu, _ = acts(cfg)
    ks = list(range(cfg["bank_scale"], cfg["bank_size"] + 1, cfg["bank_scale"]))
    outs = [relu(pad_conv(x, w(f"{p}conv_bank.{i}.weight"), w(f"{p}conv_bank.{i}.bias")))
            for i, _ in enumerate(ks)]
    out = np.concatenate(outs + [x], axis=1)
    out = relu(instance_norm(pad_conv(out, w(p + "in_conv_layer.weight"), w(p + "in_conv_layer.bias"))))
    for l in range(cfg["n_conv_blocks"]):
        s = cfg["subsample"][l]
        y = relu(instance_norm(pad_conv(out, w(f"{p}first_conv_layers.{l}.weight"),
                                        w(f"{p}first_conv_layers.{l}.bias"))))
        y = relu(instance_norm(pad_conv(y, w(f"{p}second_conv_layers.{l}.weight"),
                                        w(f"{p}second_conv_layers.{l}.bias"), stride=s)))
        if s > 1:
            out = avg_pool_ceil(out, s)
        out = y + out
    mu = pad_conv(out, w(p + "mean_layer.weight"), w(p + "mean_layer.bias"))
    if log_sigma:
        return mu, pad_conv(out, w(p + "std_layer.weight"), w(p + "std_layer.bias"))
    return mu


def pixel_shuffle_1d(x, s):
    """models.py:33-49: out[b, c, s*w + r] = in[b, s*c + r, w]."""
    B, C, W = x.shape
    return x.reshape(B, C // s, s, W).transpose(0, 1, 3, 2).reshape(B, C // s, W * s)


def append_cond(x, cond):
    """models.py:66-79: first half of cond is the mean, second half the std."""
    p = cond.shape[1] // 2
    return x * cond[:, p:, None] + cond[:, :p, None]


def instance_norm_st(x, eps=1e-5):
    """instance_norm that also returns (yhat, invstd) for the backward."""
    mu = x.mean(axis=2, keepdims=True)
    var = ((x - mu) ** 2).mean(axis=2, keepdims=True)
    inv = 1 / np.sqrt(var + x.dtype.type(eps))
    return (x - mu) * inv, inv


def instance_norm_backward(g, yhat, inv):
    """d/dx of (x - mean) * invstd (biased variance): invstd (g - mean(g) - yhat mean(g yhat))."""
    return inv * (g - g.mean(axis=2, keepdims=True) - yhat * (g * yhat).mean(axis=2, keepdims=True))


def spectral_norm_step(w, p="decoder."):
    """sn=True (models.py:382): torch.nn.utils.spectral_norm's forward pre-hook in train mode
    (torch/nn/utils/spectral_norm.py compute_weight; the reference never calls .eval()) for every
    Decoder layer that has a weight_orig: one power iteration on W = weight_orig.reshape(out, -1),
        v = normalize(W^T u),  u = normalize(W v)   (normalize: x / max(||x||, 1e-12)),
        sigma = u . (W v),     weight = weight_orig / sigma,
    with u, v updated in place (the module buffers weight_u / weight_v).  No-op for sn=False.
    w.sn_train = False: the eval-mode hook (compute_weight with do_power_iteration=False) --
    sigma = u . (W v) from the stored u / v, which stay unchanged."""
    for k in [k for k in w.d if k.startswith(p) and k.endswith(".weight_orig")]:
        n = k[: -len("weight_orig")]
        W = w.d[k]
        Wm = W.reshape(W.shape[0], -1)
        if not getattr(w, "sn_train", True):
            w.d[n + "weight"] = W / (w.d[n + "weight_u"] @ (Wm @ w.d[n + "weight_v"]))
            continue
        eps = W.dtype.type(1e-12)
        v = Wm.T @ w.d[n + "weight_u"]
        v = v / max(np.sqrt((v * v).sum()), eps)
        t = Wm @ v
        u = t / max(np.sqrt((t * t).sum()), eps)
        w.d[n + "weight_u"], w.d[n + "weight_v"] = u, v
        w.d[n + "weight"] = W / (u @ (Wm @ v))


def dec_forward(w, cfg, z, cond, p="decoder.", st=None):
    """Decoder.forward (models.py:403-435).  st: optional list filled with each block's
    (yhat1, z1, yhat2, z2, inv1, inv2, cond1, cond2) for dec_backward.  sn=True: every call first
    runs spectral_norm_step (the reference's train-mode power iteration), and dec_backward then uses
    the weights of the forward before it."""
    spectral_norm_step(w, p)
    relu, _ = acts(cfg)
    out = relu(instance_norm(pad_conv(z, w(p + "in_conv_layer.weight"), w(p + "in_conv_layer.bias"))))
    for l in range(cfg["n_conv_blocks"]):
        up = cfg["upsample"][l]
        c1 = linear(cond, w(f"{p}conv_affine_layers.{2*l}.weight"), w(f"{p}conv_affine_layers.{2*l}.bias"))
        c2 = linear(cond, w(f"{p}conv_affine_layers.{2*l+1}.weight"), w(f"{p}conv_affine_layers.{2*l+1}.bias"))
        yh1, inv1 = instance_norm_st(pad_conv(out, w(f"{p}first_conv_layers.{l}.weight"),
                                              w(f"{p}first_conv_layers.{l}.bias")))
        z1 = append_cond(yh1, c1)                                       # append_cond 66-79
        y = pad_conv(relu(z1), w(f"{p}second_conv_layers.{l}.weight"), w(f"{p}second_conv_layers.{l}.bias"))
        if up > 1:
            y = pixel_shuffle_1d(y, up)                                 # 33-49
        yh2, inv2 = instance_norm_st(y)
        z2 = append_cond(yh2, c2)
        if st is not None:
            st.append((yh1, z1, yh2, z2, inv1, inv2, c1, c2))
        out = relu(z2) + (np.repeat(out, up, axis=2) if up > 1 else out)   # upsample 52-63 (nearest)
    return pad_conv(out, w(p + "out_conv_layer.weight"), w(p + "out_conv_layer.bias"))


def _adain_backward(g, yhat, zpre, inv, cond, dact):
    """act + append_cond + InstanceNorm backward: returns (d/d conv output, d/d cond)."""
    C = yhat.shape[1]
    gz = g * dact(zpre)
    gcond = np.concatenate([gz.sum(axis=2), (gz * yhat).sum(axis=2)], axis=1)   # [mean | std]
    return instance_norm_backward(gz * cond[:, C:, None], yhat, inv), gcond


def dec_backward(w, cfg, st, g_out, p="decoder."):
    """d loss / d cond of dec_forward given d loss / d out (the content code is constant
    in the attacks, so the chain stops at the first block's AdaIN)."""
    _, dact = acts(cfg)
    Wo = w(p + "out_conv_layer.weight")[:, :, 0]
    gh = np.einsum("oc,bot->bct", Wo, g_out)
    g_cond = np.zeros((g_out.shape[0], w(f"{p}conv_affine_layers.0.weight").shape[1]), dtype=g_out.dtype)
    for l in reversed(range(cfg["n_conv_blocks"])):
        up = cfg["upsample"][l]
        yh1, z1, yh2, z2, inv1, inv2, c1, c2 = st[l]
        B, C, To = gh.shape
        T = To // up
        g2, gc2 = _adain_backward(gh, yh2, z2, inv2, c2, dact)
        if up > 1:   # pixel_shuffle adjoint: pre[b, up*c + s, t] = post[b, c, up*t + s]
            g2 = g2.reshape(B, C, T, up).transpose(0, 1, 3, 2).reshape(B, C * up, T)
        ga1 = pad_conv_dgrad(g2, w(f"{p}second_conv_layers.{l}.weight"), 1, T)
        g1, gc1 = _adain_backward(ga1, yh1, z1, inv1, c1, dact)
        g_cond += gc2 @ w(f"{p}conv_affine_layers.{2*l+1}.weight") + gc1 @ w(f"{p}conv_affine_layers.{2*l}.weight")
        ghl = gh.reshape(B, C, T, up).sum(axis=3) if up > 1 else gh     # nearest-upsample adjoint
        if l > 0:
            ghl = ghl + pad_conv_dgrad(g1, w(f"{p}first_conv_layers.{l}.weight"), 1, T)
        gh = ghl
    return g_cond


def inference(w, cfg, src, tgt):
    """AdaInVC.inference (models.py:472-485)."""
    mu = ce_forward(w, cfg["ContentEncoder"], src)
    emb, _ = se_forward(w, cfg["SpeakerEncoder"], tgt)
    return dec_forward(w, cfg["Decoder"], mu, emb)


# ----------------------------------------------------------------------------------
# loss + optimiser
# ----------------------------------------------------------------------------------


def emb_loss(emb, tgt, org, n_elems):
    """attack_utils.py:81 MSE(adv,tgt) - 0.1*MSE(adv,org), mean over n_elems."""
    d = emb.dtype.type(n_elems)
    return ((emb - tgt) ** 2).sum(axis=-1) / d - 0.1 * ((emb - org) ** 2).sum(axis=-1) / d


def emb_loss_grad(emb, tgt, org, n_elems):
    """Autograd of nn.MSELoss(mean): 2*(x-y)/N * grad_out, grad_out = 1 and -0.1."""
    norm = emb.dtype.type(2.0 / n_elems)
    return norm * (emb - tgt) + norm * (emb - org) * emb.dtype.type(-0.1)


class Adam:
    """torch.optim.Adam defaults (attack_utils.py:69), _single_tensor_adam math:
    m.lerp_(g, 1-b1); v.mul_(b2).addcmul_(g, g, 1-b2);
    p.addcdiv_(m, sqrt(v)/sqrt(1-b2^t) + eps, value=-lr/(1-b1^t))."""

    def __init__(self, p, lr=1e-3, betas=(0.9, 0.999), eps=1e-8):
        self.p = p
        self.m = np.zeros_like(p)
        self.v = np.zeros_like(p)
        self.t = 0
        self.lr, self.b1, self.b2, self.eps = lr, betas[0], betas[1], eps

    def step(self, g):
        ft = self.p.dtype.type
        self.t += 1
        self.m += ft(1 - self.b1) * (g - self.m)
        self.v *= ft(self.b2)
        self.v += ft(1 - self.b2) * g * g
        bc1 = 1 - self.b1 ** self.t
        bc2s = (1 - self.b2 ** self.t) ** 0.5
        denom = np.sqrt(self.v) / ft(bc2s) + ft(self.eps)
        self.p += ft(-self.lr / bc1) * (self.m / denom)


# ----------------------------------------------------------------------------------
# attacks
# ----------------------------------------------------------------------------------


def attack(kind, w, cfg, vc_src, vc_tgt, adv_tgt, eps, n_iters, ptb0, reduction="independent", record=None):
    """emb / e2e / fb attack (attack_utils.py:51-86 / 7-48 / 89-130) with an explicit ptb0.

    reduction="independent": each utterance of the batch is its own attack
    (loss summed over utterances, each an MSE mean over its own output); equals
    B separate reference calls.  reduction="mean": the loss is the reference's
    MSE mean over the whole batch, i.e. the reference called on the batched
    tensor.  record: optional dict filled with "losses" and "grad0".
    The ContentEncoder output of vc_src is computed once (it is constant).
    """
    se = cfg["SpeakerEncoder"] if "SpeakerEncoder" in cfg else cfg
    dt = vc_tgt.dtype.type
    ptb = ptb0.astype(vc_tgt.dtype).copy()
    opt = Adam(ptb)
    if kind != "emb":
        mu = ce_forward(w, cfg["ContentEncoder"], vc_src)
        dec = cfg["Decoder"]

        def infer(x, st_se=None, st_dec=None):
            emb, st1 = se_forward(w, se, x)
            if st_se is not None:
                st_se.append(st1)
            return dec_forward(w, dec, mu, emb, st=st_dec)
    if kind == "emb":                                                  # attack_utils.py:73-75
        org, _ = se_forward(w, se, vc_tgt)
        tgt, _ = se_forward(w, se, adv_tgt)
    elif kind == "e2e":                                                # 35-37
        org, tgt = infer(vc_tgt), infer(adv_tgt)
    else:                                                              # 117-119
        org, _ = se_forward(w, se, infer(vc_tgt))
        tgt, _ = se_forward(w, se, adv_tgt)
    B = org.shape[0]
    per = int(np.prod(org.shape[1:]))
    n_el = per if reduction == "independent" else B * per
    losses = []
    for it in range(n_iters):
        th = np.tanh(ptb)
        adv = vc_tgt + dt(eps) * th                                    # 78 / 40 / 122
        if kind == "emb":
            out, st = se_forward(w, se, adv)
        else:
            st_se, st_dec = [], []
            out = infer(adv, st_se, st_dec)
            if kind == "fb":
                dec_out = out
                out, st_fb = se_forward(w, se, dec_out)
        flat = out.reshape(B, -1)
        if record is not None:
            losses.append(emb_loss(flat, tgt.reshape(B, -1), org.reshape(B, -1), n_el))
        g = emb_loss_grad(out, tgt, org, n_el)
        if kind == "emb":
            g_adv = se_backward(w, se, st, g)
        else:
            if kind == "fb":
                g = se_backward(w, se, st_fb, g)                       # d loss / d decoder output
            g_emb = dec_backward(w, dec, st_dec, g)
            g_adv = se_backward(w, se, st_se[0], g_emb)
        g = (g_adv * dt(eps)) * (dt(1) - th * th)                       # tanh backward
        if record is not None and it == 0:
            record["grad0"] = g.copy()
        opt.step(g)
    if record is not None:
        record["losses"] = np.stack(losses, axis=-1) if losses else None
    return vc_tgt + dt(eps) * np.tanh(ptb)


def emb_attack(w, cfg, vc_tgt, adv_tgt, eps, n_iters, ptb0, reduction="independent", record=None):
    """emb_attack (attack_utils.py:51-86) with an explicit ptb0 (see attack())."""
    return attack("emb", w, cfg, None, vc_tgt, adv_tgt, eps, n_iters, ptb0, reduction, record)


def e2e_attack(w, cfg, vc_src, vc_tgt, adv_tgt, eps, n_iters, ptb0, reduction="independent", record=None):
    """e2e_attack (attack_utils.py:7-48) with an explicit ptb0 (see attack())."""
    return attack("e2e", w, cfg, vc_src, vc_tgt, adv_tgt, eps, n_iters, ptb0, reduction, record)


def fb_attack(w, cfg, vc_src, vc_tgt, adv_tgt, eps, n_iters, ptb0, reduction="independent", record=None):
    """fb_attack (attack_utils.py:89-130) with an explicit ptb0 (see attack())."""
    return attack("fb", w, cfg, vc_src, vc_tgt, adv_tgt, eps, n_iters, ptb0, reduction, record)
