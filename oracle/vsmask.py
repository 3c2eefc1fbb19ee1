"""CPU oracle: numpy restatement of the VSMask mel loop and the perturbation header.

TEST INFRASTRUCTURE ONLY (tests/); the product never imports it.

Follows /root/reference/vsmask.py:177-208 (_protect_waveform between waveform_to_mel and
mel_to_waveform), /root/reference/utils/audio.py:77-116 (apply_weighted_constraint) and
/root/reference/models/header_model.py:70-95 (UniversalPerturbationHeader.apply_header),
statement by statement, in the caller's dtype (float32 reproduces the reference's fp32
tensor arithmetic element for element; float64 for a drift-free check).

The reference as shipped cannot execute this loop (SURVEY.md 2 note A):
  * waveform_to_mel returns a 3-D [1, n_mels, T'] mel, which vsmask.py:183/188/199 index
    with four subscripts; and apply_weighted_constraint (audio.py:94) unpacks three dims
    from the 4-D perturbation vsmask.py:203 hands it;
  * PredictiveModel maps an [.., 80, 100] window to [.., 95, 63] (predictive_model.py), so
    vsmask.py:199's in-place add of 95 rows onto the 80-row mel cannot broadcast.
Settled here (and in libavc) as: the mel is 4-D [B, 1, F, T]; the band clamp sees the
[B*1, F, T] view (so freq_dim = F); the predictor's rows [0, min(F, Ho)) are added and the
rest dropped.  Parity of this loop is therefore against this restatement, not against an
execution of the reference (which fails, and whose torchaudio dependency is absent here):
"parity unpinned" beyond the PredictiveModel itself, which tests/golden/predictive.npz pins.
"""
import numpy as np

from oracle import adain_vc as _av


def n_windows(T, window_size=100, future_step=10):
    """vsmask.py:186: len(range(0, T - window_size, future_step))."""
    return len(range(0, T - window_size, future_step))


def weighted_constraint(pert, epsilon1=0.1, epsilon2=0.05, epsilon3=0.08):
    """utils/audio.py:77-116 on a [N, F, T] perturbation (N = B*1 of the 4-D mel)."""
    _, freq_dim, _ = pert.shape
    low_freq_end = int(freq_dim * 0.3)
    high_freq_start = int(freq_dim * 0.7)
    ft = pert.dtype.type
    low = np.clip(pert[:, :low_freq_end, :], -ft(epsilon1), ft(epsilon1))
    mid = np.clip(pert[:, low_freq_end:high_freq_start, :], -ft(epsilon2), ft(epsilon2))
    high = np.clip(pert[:, high_freq_start:, :], -ft(epsilon3), ft(epsilon3))
    return np.concatenate([low, mid, high], axis=1)


def protect_mel(mel, header, predictor, window_size=100, future_step=10,
                epsilon1=0.1, epsilon2=0.05, epsilon3=0.08):
    """vsmask.py:181-208.  mel [B,1,F,T]; header [1,1,F,Th] or None; predictor maps a
    window batch [n,1,F,W] to [n,1,Ho,Wo] (the PredictiveModel; called once per window,
    in loop order, as the reference does)."""
    mel = np.asarray(mel)
    B, _, F, T = mel.shape
    perturbed = mel.copy()
    if header is not None:
        hl = min(T, header.shape[-1])
        perturbed[:, :, :, :hl] += header[:, :, :, :hl].astype(mel.dtype)
    for start in range(0, T - window_size, future_step):
        window = mel[:, :, :, start:start + window_size]
        pert = np.asarray(predictor(window), dtype=mel.dtype)
        fi = start + window_size
        fe = min(fi + pert.shape[-1], T)
        if fi < T:
            rows = min(F, pert.shape[2])           # settled 95 -> 80 crop (module docstring)
            perturbed[:, :, :rows, fi:fe] += pert[:, :, :rows, :fe - fi]
    w = weighted_constraint((perturbed - mel).reshape(B, F, T), epsilon1, epsilon2, epsilon3)
    return mel + w.reshape(B, 1, F, T)


def apply_header(mel, header):
    """header_model.py:70-95: add the header on the first min(T, Th) frames, clamp to [-1, 1]."""
    mel = np.asarray(mel)
    T = mel.shape[-1]
    h = header[:, :, :, :T] if T < header.shape[-1] else header
    out = mel.copy()
    out[:, :, :, :h.shape[3]] += h.astype(mel.dtype)
    ft = mel.dtype.type
    return np.clip(out, ft(-1.0), ft(1.0))


def header_optimize(w, se_cfg, source, target, header, n_iters, epsilon=0.1, lambda_param=0.5, lr=1e-3,
                    betas=(0.9, 0.999), adam_eps=1e-8):
    """header_model.py:40-65 (+ train_header.py:46: torch Adam on the header) with the
    SpeakerEncoder restatement oracle/adain_vc.py.  source / target [N, F, T] (the settled 3-D
    mels), header [F, T].  Returns (header, per-iteration batch losses)."""
    dt = source.dtype.type
    src_emb, _ = _av.se_forward(w, se_cfg, source)
    tgt_emb, _ = _av.se_forward(w, se_cfg, target)
    n_el = src_emb.size
    opt = _av.Adam(header.astype(source.dtype).copy(), lr, betas, adam_eps)
    losses = []
    for _ in range(n_iters):
        pre = source + opt.p
        x = np.clip(pre, dt(-1), dt(1))
        emb, st = _av.se_forward(w, se_cfg, x)
        losses.append(((emb - tgt_emb) ** 2).mean() - lambda_param * ((emb - src_emb) ** 2).mean())
        norm = dt(2.0 / n_el)
        g_emb = norm * (emb - tgt_emb) + norm * (emb - src_emb) * dt(-lambda_param)
        gx = _av.se_backward(w, se_cfg, st, g_emb)
        g = np.where((pre >= -1) & (pre <= 1), gx, dt(0)).sum(axis=0)
        opt.step(g)
        opt.p = np.clip(opt.p, dt(-epsilon), dt(epsilon))
    return opt.p, np.array(losses)
