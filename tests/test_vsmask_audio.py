"""CPU: VSMask's torchaudio-flavor mel converter (utils/audio.py:8-146) -- the numpy restatement
(oracle/mel_dsp.py ta_*), libavc's host-side HTK filter bank and its least-squares inverse
(avc_dsp_mel_basis, flavor 1), the float WAV writer and the random shift.  No GPU compute.

PARITY UNPINNED against torchaudio (absent here and unpinned by the reference): the restatement
follows torchaudio >= 2.1's published functional code and is checked by the properties it has
(triangular filters peaking at their HTK centres, the minimum-norm least-squares inverse, the
momentum-free Griffin-Lim equal to the reference's data_utils composition)."""
import numpy as np
import pytest
import torch

import audio
import avc_native
import data_utils
from oracle import mel_dsp

SR, NFFT, HOP, NMEL = 16000, 1024, 256, 80


def _signal(n, seed=0):
    g = np.random.default_rng(seed)
    t = np.arange(n) / SR
    return (0.3 * np.sin(2 * np.pi * 220 * t) + 0.2 * np.sin(2 * np.pi * 1330 * t + 0.5) +
            0.05 * g.standard_normal(n)).astype(np.float32)


def test_htk_filter_bank_shape_and_triangles():
    fb = mel_dsp.ta_fb(SR, NFFT, NMEL)                 # [F, n_mels]
    assert fb.shape == (NFFT // 2 + 1, NMEL)
    assert fb.min() >= 0 and fb.max() <= 1 + 1e-12
    freqs = np.linspace(0, SR // 2, NFFT // 2 + 1)
    f_pts = mel_dsp.htk_mel_to_hz(np.linspace(0, mel_dsp.htk_hz_to_mel(SR // 2), NMEL + 2))
    for m in range(NMEL):
        nz = np.flatnonzero(fb[:, m])
        assert nz.size >= 1, m                          # every filter sees a bin: full row rank
        assert freqs[nz[0]] > f_pts[m] - 1e-9 and freqs[nz[-1]] < f_pts[m + 2] + 1e-9
        # the peak bin is the one nearest the centre frequency
        assert abs(freqs[nz[np.argmax(fb[nz, m])]] - f_pts[m + 1]) <= (SR / NFFT) / 2 + 1e-9
    assert np.linalg.matrix_rank(fb.T) == NMEL


def test_libavc_htk_bank_and_pinv_match_restatement():
    pre = avc_native.ta_preprocess(SR, NFFT, HOP, NMEL)
    W, inv = avc_native.mel_basis(pre)
    fbT = mel_dsp.ta_fb(SR, NFFT, NMEL).T
    assert W.shape == fbT.shape and inv.shape == fbT.T.shape
    assert np.abs(W.numpy() - fbT).max() <= 1e-6
    pinv = np.linalg.pinv(fbT)
    rel = np.abs(inv.numpy() - pinv).max() / np.abs(pinv).max()
    print(f"libavc pinv vs numpy pinv: rel {rel:.2e}")
    assert rel <= 1e-4
    # the minimum-norm least-squares solution of fb^T X = mel (InverseMelScale's lstsq)
    g = np.random.default_rng(1)
    mel = fbT @ np.abs(g.standard_normal((NFFT // 2 + 1, 7)))
    X = inv.numpy().astype(np.float64) @ mel
    assert np.abs(fbT @ X - mel).max() <= 1e-4 * np.abs(mel).max()
    Xl = np.linalg.lstsq(fbT, mel, rcond=None)[0]
    assert np.abs(X - Xl).max() <= 1e-4 * np.abs(Xl).max()


def test_ta_flavor_config_checks():
    pre = avc_native.ta_preprocess()
    pre["preemph"] = 0.97
    with pytest.raises(RuntimeError, match="pre-emphasis"):
        avc_native.mel_basis(pre)
    pre = avc_native.ta_preprocess()
    pre["flavor"] = 2
    with pytest.raises(RuntimeError, match="flavor"):
        avc_native.mel_basis(pre)


def test_ta_wav2mel_restatement():
    """log10(clamp(fb^T |STFT|^2, 1e-5)) on the scipy-pinned STFT; frames 1 + L // hop."""
    x = _signal(HOP * 30 + 17)
    mel = mel_dsp.ta_wav2mel(x, SR, NFFT, HOP, NMEL)
    assert mel.shape == (NMEL, 1 + len(x) // HOP)
    S = np.abs(mel_dsp.stft(x.astype(np.float64), NFFT, HOP, NFFT)) ** 2
    direct = np.log10(np.maximum(np.einsum("fm,ft->mt", mel_dsp.ta_fb(SR, NFFT, NMEL), S), 1e-5))
    assert np.abs(mel - direct).max() <= 1e-12
    assert mel.min() >= -5.0


def test_ta_griffin_lim_without_momentum_is_the_plain_projection():
    """momentum 0, unit initial angles: torchaudio's iteration is the data_utils projection
    X = |S| est / |est| (the two differ only in the 1e-16 / 1e-8 guards)."""
    x = _signal(HOP * 24)
    S = np.abs(mel_dsp.stft(x.astype(np.float64), NFFT, HOP, NFFT))
    a = mel_dsp.ta_griffin_lim(S ** 2, NFFT, HOP, n_iter=4, momentum=0.0)
    b = mel_dsp.griffin_lim(S, HOP, NFFT, NFFT, n_iter=4)
    assert a.shape == b.shape == (HOP * (S.shape[1] - 1),)
    assert np.abs(a - b).max() <= 1e-9 * np.abs(b).max()


def test_ta_griffin_lim_momentum_converges():
    """With a consistent magnitude, 32 momentum iterations from random phases reach a lower
    spectral distance than 32 plain ones (the fast Griffin-Lim property torchaudio relies on)."""
    x = _signal(HOP * 40, seed=3)
    S = np.abs(mel_dsp.stft(x.astype(np.float64), NFFT, HOP, NFFT))
    g = np.random.default_rng(0)
    a0 = g.random(S.shape) + 1j * g.random(S.shape)

    def dist(y):
        return np.linalg.norm(np.abs(mel_dsp.stft(y, NFFT, HOP, NFFT)) - S) / np.linalg.norm(S)
    fast = dist(mel_dsp.ta_griffin_lim(S ** 2, NFFT, HOP, 32, 0.99, a0))
    plain = dist(mel_dsp.ta_griffin_lim(S ** 2, NFFT, HOP, 32, 0.0, a0))
    print(f"spectral distance: momentum {fast:.4f}, plain {plain:.4f}")
    assert fast < plain


def test_band_clamp_edges():
    p = np.full((2, 80, 5), 1.0)
    out = mel_dsp.band_clamp(p, 0.1, 0.05, 0.08)
    assert (out[:, :24] == 0.1).all() and (out[:, 24:56] == 0.05).all() and (out[:, 56:] == 0.08).all()
    out = mel_dsp.band_clamp(-p, 0.1, 0.05, 0.08)
    assert (out[:, :24] == -0.1).all() and (out[:, 24:56] == -0.05).all() and (out[:, 56:] == -0.08).all()


def test_write_wav_float_roundtrip(tmp_path):
    g = np.random.default_rng(2)
    x = (0.5 * g.standard_normal((2, 1000))).astype(np.float32)
    p = str(tmp_path / "f.wav")
    data_utils.write_wav_float(p, x, 16000)
    y, sr = data_utils.read_wav(p)
    assert sr == 16000 and y.shape == (1000,)
    assert np.array_equal(y, x.mean(axis=0).astype(np.float32))
    data_utils.write_wav_float(p, x[0], 8000)
    y, sr = data_utils.read_wav(p)
    assert sr == 8000 and np.array_equal(y, x[0])


def test_apply_random_shift():
    w = torch.arange(1, 11, dtype=torch.float32)[None]
    for seed in range(20):
        g = torch.Generator().manual_seed(seed)
        shift = int(torch.randint(-3, 4, (1,), generator=torch.Generator().manual_seed(seed)).item())
        out = audio.apply_random_shift(w, 3, generator=g)
        assert out.shape == w.shape
        if shift > 0:
            assert (out[0, :shift] == 0).all() and torch.equal(out[0, shift:], w[0, :-shift])
        elif shift < 0:
            assert (out[0, shift:] == 0).all() and torch.equal(out[0, :shift], w[0, -shift:])
        else:
            assert torch.equal(out, w)


def test_converter_defaults_mirror_reference():
    c = audio.MelSpectrogramConverter()
    assert (c.sample_rate, c.n_fft, c.hop_length, c.n_mels) == (16000, 1024, 256, 80)
    assert (c.n_iter, c.momentum, c.rand_init) == (32, 0.99, True)
    assert c.frames(16000) == 63
    with pytest.raises(RuntimeError, match="ROCm"):
        c.waveform_to_mel(torch.zeros(1, 4000))
