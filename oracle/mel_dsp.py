"""CPU oracle: numpy restatement of the reference's mel front / back end.

TEST INFRASTRUCTURE ONLY.  Nothing in the product (attack-vc_amd/) imports,
links or executes this module; only tests/ and bench.py's cpu_baseline leg use
it, as the checker and the timed CPU baseline.

The reference's DSP (data_utils.py:16-197) calls librosa, which is absent from
this image and from /root/reference (no requirements file pins it).  The
reference calls `librosa.filters.mel(sr, n_fft, n_mels)` and
`librosa.istft(X, hop, win, window=...)` positionally (data_utils.py:29,110,
191-192), which librosa >= 0.10 rejects, so the version it ran on is <= 0.9;
this module restates the published algorithms of librosa 0.8.1 (the release
of the reference's era): `filters.mel` (Slaney mel scale, Slaney area
normalisation), `stft` / `istft` (centered frames, periodic Hann window padded
to n_fft, window-sum-square normalisation), `effects.trim` (frame RMS in dB
against the peak).
Pinned against scipy 1.15 (importable here; the reference calls scipy.signal
itself, data_utils.py:163): the Hann window (`scipy.signal.get_window`), the
STFT / ISTFT (`scipy.signal.stft` / `istft` with the even (= reflect) boundary),
the de-emphasis (`scipy.signal.lfilter`) and the reference's Griffin-Lim
composition on those transforms -- to 1e-12 relative (tests/test_dsp_oracle.py).
PARITY UNPINNED for the two pieces only librosa defines: the Slaney mel filter
bank and `effects.trim` (no librosa output exists in the reference); they are
checked by properties (filter areas, trim bounds).

Computation is float64 (numpy's pocketfft computes in double, as librosa's
calls did).
"""
import numpy as np

# ----------------------------------------------------------------------------------
# librosa 0.8.1 primitives
# ----------------------------------------------------------------------------------


def hann_periodic(n):
    """scipy.signal.get_window('hann', n, fftbins=True)."""
    k = np.arange(n, dtype=np.float64)
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * k / n)


def pad_center(w, size):
    """librosa.util.pad_center: zero-pad to `size`, lpad = (size - n) // 2."""
    lpad = (size - len(w)) // 2
    return np.pad(w, (lpad, size - len(w) - lpad))


def stft_window(n_fft, win_length):
    return pad_center(hann_periodic(win_length), n_fft)


def hz_to_mel(f):
    """librosa.core.convert.hz_to_mel, htk=False (Slaney)."""
    f = np.asarray(f, np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    return np.where(f >= min_log_hz, min_log_mel + np.log(np.maximum(f, 1e-30) / min_log_hz) / logstep, mels)


def mel_to_hz(m):
    m = np.asarray(m, np.float64)
    f_sp = 200.0 / 3
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    return np.where(m >= min_log_mel, min_log_hz * np.exp(logstep * (m - min_log_mel)), f_sp * m)


def mel_filters(sr, n_fft, n_mels, fmin=0.0, fmax=None):
    """librosa.filters.mel(sr, n_fft, n_mels) (htk=False, norm='slaney'), float32 like librosa."""
    fmax = sr / 2.0 if fmax is None else fmax
    fftfreqs = np.linspace(0, sr / 2.0, 1 + n_fft // 2)
    mel_f = mel_to_hz(np.linspace(hz_to_mel(fmin), hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = mel_f[:, None] - fftfreqs[None, :]
    w = np.zeros((n_mels, 1 + n_fft // 2), np.float32)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        w[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    w *= enorm[:, None]
    return w


def stft(y, n_fft, hop, win, pad_mode="reflect"):
    """librosa.stft(y, n_fft, hop, win), center=True -> complex [1 + n_fft//2, frames]."""
    y = np.asarray(y, np.float64)
    w = stft_window(n_fft, win)
    yp = np.pad(y, n_fft // 2, mode=pad_mode)
    nfr = 1 + (len(yp) - n_fft) // hop
    idx = np.arange(n_fft)[:, None] + hop * np.arange(nfr)[None, :]
    return np.fft.rfft(w[:, None] * yp[idx], axis=0)


def window_sumsquare(n_frames, hop, win, n_fft):
    """librosa.filters.window_sumsquare(window='hann', norm=None)."""
    n = n_fft + hop * (n_frames - 1)
    x = np.zeros(n)
    wsq = pad_center(hann_periodic(win) ** 2, n_fft)
    for i in range(n_frames):
        s = i * hop
        x[s:min(n, s + n_fft)] += wsq[:max(0, min(n_fft, n - s))]
    return x


def istft(S, hop, win):
    """librosa.istft(S, hop, win, window='hann'), center=True, length=None."""
    n_fft = 2 * (S.shape[0] - 1)
    w = stft_window(n_fft, win)
    nfr = S.shape[1]
    y = np.zeros(n_fft + hop * (nfr - 1))
    fr = w[:, None] * np.fft.irfft(S, n=n_fft, axis=0)
    for t in range(nfr):
        y[t * hop:t * hop + n_fft] += fr[:, t]
    ws = window_sumsquare(nfr, hop, win, n_fft)
    nz = ws > np.finfo(np.float64).tiny
    y[nz] /= ws[nz]
    return y[n_fft // 2:-(n_fft // 2)]


def trim(y, top_db, frame_length=2048, hop_length=512):
    """librosa.effects.trim(y, top_db) (ref=np.max): frame RMS (center, reflect pad)
    in dB against the loudest frame; keep [first, last] non-silent frame."""
    y = np.asarray(y)
    yp = np.pad(y.astype(np.float64), frame_length // 2, mode="reflect")
    nfr = 1 + (len(yp) - frame_length) // hop_length
    idx = np.arange(frame_length)[None, :] + hop_length * np.arange(nfr)[:, None]
    mse = np.mean(np.abs(yp[idx]) ** 2, axis=1)
    db = 10 * np.log10(np.maximum(1e-10, mse)) - 10 * np.log10(np.maximum(1e-10, mse.max()))
    nz = np.flatnonzero(db > -top_db)
    if nz.size == 0:
        return y[0:0], (0, 0)
    start = int(nz[0] * hop_length)
    end = min(len(y), int((nz[-1] + 1) * hop_length))
    return y[start:end], (start, end)


# ----------------------------------------------------------------------------------
# the reference's compositions (data_utils.py)
# ----------------------------------------------------------------------------------


def inv_mel_matrix(sr, n_fft, n_mels):
    """data_utils.py:16-32."""
    m = mel_filters(sr, n_fft, n_mels)
    p = m @ m.T
    d = [1.0 / x if np.abs(x) > 1e-8 else x for x in np.sum(p, axis=0)]
    return m.T @ np.diag(d)


def wav2mel(wav, sample_rate, preemph, n_fft, hop_length, win_length, n_mels, ref_db, max_db,
            pad_mode="reflect"):
    """data_utils.py:99-118 after load + trim: pre-emphasis, |STFT|, mel, dB, clip -> [T, n_mels]."""
    wav = np.asarray(wav, np.float64)
    wav = np.append(wav[0], wav[1:] - preemph * wav[:-1])
    mag = np.abs(stft(wav, n_fft, hop_length, win_length, pad_mode))
    mel = mel_filters(sample_rate, n_fft, n_mels).astype(np.float64) @ mag
    mel = 20 * np.log10(np.maximum(1e-5, mel))
    mel = np.clip((mel - ref_db + max_db) / max_db, 1e-8, 1)
    return mel.T


def griffin_lim(spect, hop_length, win_length, n_fft, n_iter=100):
    """data_utils.py:168-197."""
    X = np.asarray(spect, np.float64).astype(np.complex128)
    for _ in range(n_iter):
        xt = istft(X, hop_length, win_length)
        est = stft(xt, n_fft, hop_length, win_length)
        X = spect * (est / np.maximum(1e-8, np.abs(est)))
    return np.real(istft(X, hop_length, win_length))


def deemphasis(x, preemph):
    """scipy.signal.lfilter([1], [1, -preemph], x) as a plain recurrence."""
    y = np.empty(len(x))
    acc = 0.0
    for i, v in enumerate(np.asarray(x, np.float64)):
        acc = v + preemph * acc
        y[i] = acc
    return y


def mel2mag(mel, sample_rate, n_fft, n_mels, ref_db, max_db):
    """data_utils.py:150-157: mel [T, n_mels] (denormalised) -> linear magnitude [F, T]."""
    m = np.asarray(mel, np.float64).T
    m = (np.clip(m, 0, 1) * max_db) - max_db + ref_db
    m = np.power(10.0, m * 0.05)
    return inv_mel_matrix(sample_rate, n_fft, n_mels) @ m


def mel2wav(mel, sample_rate, preemph, n_fft, hop_length, win_length, n_mels, ref_db, max_db, n_iter=100):
    """data_utils.py:121-165."""
    mag = mel2mag(mel, sample_rate, n_fft, n_mels, ref_db, max_db)
    wav = griffin_lim(mag, hop_length, win_length, n_fft, n_iter)
    return deemphasis(wav, preemph).astype(np.float32)


# ----------------------------------------------------------------------------------
# utils/audio.py's torchaudio converter (VSMask; MelSpectrogramConverter, 8-116)
# ----------------------------------------------------------------------------------
# torchaudio is absent from this image and /root/reference pins no version; restated from
# torchaudio >= 2.1's published functional code: melscale_fbanks (mel_scale="htk", norm=None),
# Spectrogram (center, reflect, power 2), InverseMelScale (torch.linalg.lstsq, then relu),
# griffinlim (momentum, rand_init).  PARITY UNPINNED against torchaudio; the STFT / ISTFT are the
# scipy-pinned ones above (torch.stft / istft with a Hann window and center=True compute the same
# transforms).


def htk_hz_to_mel(f):
    return 2595.0 * np.log10(1.0 + np.asarray(f, np.float64) / 700.0)


def htk_mel_to_hz(m):
    return 700.0 * (10.0 ** (np.asarray(m, np.float64) / 2595.0) - 1.0)


def ta_mel_fbanks(n_freqs, f_min, f_max, n_mels, sample_rate):
    """torchaudio.functional.melscale_fbanks(norm=None, mel_scale='htk') -> [n_freqs, n_mels]."""
    all_freqs = np.linspace(0, sample_rate // 2, n_freqs)
    f_pts = htk_mel_to_hz(np.linspace(htk_hz_to_mel(f_min), htk_hz_to_mel(f_max), n_mels + 2))
    f_diff = f_pts[1:] - f_pts[:-1]
    slopes = f_pts[None, :] - all_freqs[:, None]
    down = -slopes[:, :-2] / f_diff[:-1]
    up = slopes[:, 2:] / f_diff[1:]
    return np.maximum(0.0, np.minimum(down, up))


def ta_fb(sample_rate, n_fft, n_mels):
    """MelSpectrogram's bank: f_min 0, f_max sample_rate // 2."""
    return ta_mel_fbanks(n_fft // 2 + 1, 0.0, float(sample_rate // 2), n_mels, sample_rate)


def ta_wav2mel(wav, sample_rate=16000, n_fft=1024, hop_length=256, n_mels=80):
    """utils/audio.py:44-57: log10(clamp(MelSpectrogram(wav), 1e-5)) for wav [L] -> [n_mels, Tf]."""
    S = np.abs(stft(np.asarray(wav, np.float64), n_fft, hop_length, n_fft)) ** 2
    return np.log10(np.maximum(ta_fb(sample_rate, n_fft, n_mels).T @ S, 1e-5))


def ta_inverse_mel(mel_power, sample_rate=16000, n_fft=1024, n_mels=80):
    """InverseMelScale: relu(lstsq(fb^T, mel)) (minimum-norm solution) -> [n_fft/2+1, T]."""
    fbT = ta_fb(sample_rate, n_fft, n_mels).T
    return np.maximum(np.linalg.lstsq(fbT, np.asarray(mel_power, np.float64), rcond=None)[0], 0.0)


def ta_griffin_lim(spec_power, n_fft=1024, hop_length=256, n_iter=32, momentum=0.99, angles0=None):
    """torchaudio.functional.griffinlim (power 2, center, length None): spec [F, T] -> wav."""
    mag = np.sqrt(np.asarray(spec_power, np.float64))
    angles = np.ones(mag.shape, np.complex128) if angles0 is None else np.asarray(angles0, np.complex128)
    tprev = 0.0
    for _ in range(n_iter):
        inverse = istft(mag * angles, hop_length, n_fft)
        rebuilt = stft(inverse, n_fft, hop_length, n_fft)
        angles = rebuilt - tprev * (momentum / (1.0 + momentum)) if momentum else rebuilt
        angles = angles / (np.abs(angles) + 1e-16)
        tprev = rebuilt
    return istft(mag * angles, hop_length, n_fft)


def ta_mel2wav(logmel, sample_rate=16000, n_fft=1024, hop_length=256, n_mels=80, n_iter=32, momentum=0.99,
               angles0=None):
    """utils/audio.py:59-75 for one channel: log10 mel [n_mels, T] -> wav [hop * (T - 1)]."""
    spec = ta_inverse_mel(10.0 ** np.asarray(logmel, np.float64), sample_rate, n_fft, n_mels)
    return ta_griffin_lim(spec, n_fft, hop_length, n_iter, momentum, angles0)


def band_clamp(p, eps1=0.1, eps2=0.05, eps3=0.08):
    """utils/audio.py:77-116 along the second-to-last axis."""
    p = np.asarray(p)
    F = p.shape[-2]
    lo, hi = int(F * 0.3), int(F * 0.7)
    out = p.copy()
    out[..., :lo, :] = np.clip(p[..., :lo, :], -eps1, eps1)
    out[..., lo:hi, :] = np.clip(p[..., lo:hi, :], -eps2, eps2)
    out[..., hi:, :] = np.clip(p[..., hi:, :], -eps3, eps3)
    return out
