"""CPU: the mel front / back end oracle (oracle/mel_dsp.py), libavc's host-side
filter bank, and the host plumbing of the data_utils / attack.py mirrors (wav I/O,
silence trim, load_model, CLI flags).  No GPU compute.

PARITY UNPINNED against librosa itself (absent here, and from the reference): the
oracle restates librosa 0.8.1's published algorithms and is checked here by the
properties the reference relies on."""
import os
import pickle

import numpy as np
import pytest
import torch
import yaml

import avc_native
import data_utils
from oracle import mel_dsp

CFGS = [
    # (sample_rate, n_fft, hop, win, n_mels): the assumed AdaIN-VC preprocess section, the
    # reference's VSMask STFT (train_header.py:102-105) and a small one
    (16000, 2048, 300, 1200, 80),
    (22050, 1024, 256, 1024, 80),
    (8000, 256, 64, 200, 40),
]


def _signal(n, sr, seed=0):
    g = np.random.default_rng(seed)
    t = np.arange(n) / sr
    x = 0.3 * np.sin(2 * np.pi * 220 * t) + 0.2 * np.sin(2 * np.pi * 1330 * t + 0.5) + 0.05 * g.standard_normal(n)
    return x.astype(np.float32)


@pytest.mark.parametrize("sr,n_fft,hop,win,n_mels", CFGS)
def test_stft_istft_reconstructs(sr, n_fft, hop, win, n_mels):
    """librosa's istft(stft(y)) == y (window-sum-square normalisation, center trim)."""
    y = _signal(hop * 40, sr).astype(np.float64)
    S = mel_dsp.stft(y, n_fft, hop, win)
    assert S.shape == (n_fft // 2 + 1, 1 + len(y) // hop)
    r = mel_dsp.istft(S, hop, win)
    assert len(r) == hop * (S.shape[1] - 1)
    assert np.abs(r - y[:len(r)]).max() < 1e-9


def test_stft_matches_direct_dft():
    y = _signal(700, 8000, 3).astype(np.float64)
    n_fft, hop, win = 64, 16, 48
    S = mel_dsp.stft(y, n_fft, hop, win)
    w = mel_dsp.stft_window(n_fft, win)
    yp = np.pad(y, n_fft // 2, mode="reflect")
    t = 5
    fr = w * yp[t * hop:t * hop + n_fft]
    k = np.arange(n_fft // 2 + 1)[:, None]
    n = np.arange(n_fft)[None, :]
    ref = (fr[None, :] * np.exp(-2j * np.pi * k * n / n_fft)).sum(1)
    assert np.abs(S[:, t] - ref).max() < 1e-10


@pytest.mark.parametrize("sr,n_fft,hop,win,n_mels", CFGS)
def test_mel_filters_slaney(sr, n_fft, hop, win, n_mels):
    """Slaney filters: triangles on the Slaney mel scale with unit area in Hz."""
    W = mel_dsp.mel_filters(sr, n_fft, n_mels)
    assert W.dtype == np.float32 and W.shape == (n_mels, n_fft // 2 + 1)
    assert (W >= 0).all()
    df = sr / n_fft
    wide = [m for m in range(n_mels) if (W[m] > 0).sum() >= 12]
    assert wide
    for m in wide:
        assert abs(W[m].sum() * df - 1.0) < 0.05
    assert np.allclose(mel_dsp.mel_to_hz(mel_dsp.hz_to_mel([0, 500, 1000, 4000, 8000])), [0, 500, 1000, 4000, 8000])
    assert abs(float(mel_dsp.hz_to_mel(1000.0)) - 15.0) < 1e-12


@pytest.mark.parametrize("sr,n_fft,hop,win,n_mels", CFGS)
def test_libavc_mel_basis_matches_oracle(sr, n_fft, hop, win, n_mels):
    """libavc's host-side filter bank is the oracle's bit for bit; inv_mel_matrix to fp32."""
    pre = dict(sample_rate=sr, n_fft=n_fft, hop_length=hop, win_length=win, n_mels=n_mels, preemph=0.97,
               ref_db=20, max_db=100)
    W, inv = avc_native.mel_basis(pre)
    assert np.array_equal(W.numpy(), mel_dsp.mel_filters(sr, n_fft, n_mels))
    inv0 = mel_dsp.inv_mel_matrix(sr, n_fft, n_mels)
    assert np.abs(inv.numpy() - inv0).max() <= 1e-6 * np.abs(inv0).max()
    assert np.array_equal(data_utils.inv_mel_matrix(sr, n_fft, n_mels), inv.numpy())


def test_bad_dsp_configs_fail_loudly():
    pre = dict(sample_rate=16000, n_fft=1000, hop_length=256, win_length=800, n_mels=80, preemph=0.97,
               ref_db=20, max_db=100)
    with pytest.raises(RuntimeError, match="power of two"):
        avc_native.mel_basis(pre)
    pre.update(n_fft=1024, win_length=2048)
    with pytest.raises(RuntimeError, match="win_length"):
        avc_native.mel_basis(pre)


def test_griffin_lim_oracle_converges():
    """The reference's Griffin-Lim (data_utils.py:168-197) lowers the spectral distance."""
    sr, n_fft, hop, win = 8000, 256, 64, 200
    y = _signal(hop * 30, sr, 5)
    mag = np.abs(mel_dsp.stft(y, n_fft, hop, win))

    def dist(w):
        return np.linalg.norm(np.abs(mel_dsp.stft(w, n_fft, hop, win)) - mag) / np.linalg.norm(mag)
    d = [dist(mel_dsp.griffin_lim(mag, hop, win, n_fft, n)) for n in (0, 5, 30)]
    assert d[2] < d[1] < d[0]


def test_deemphasis_inverts_preemphasis():
    x = _signal(5000, 16000, 2).astype(np.float64)
    p = np.append(x[0], x[1:] - 0.97 * x[:-1])
    assert np.abs(mel_dsp.deemphasis(p, 0.97) - x).max() < 1e-6


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_trim_matches_oracle(seed):
    g = np.random.default_rng(seed)
    sr = 16000
    n0, n1, n2 = g.integers(0, 20000, 3)
    x = np.concatenate([1e-4 * g.standard_normal(n0), _signal(int(n1) + 3000, sr, seed),
                        1e-4 * g.standard_normal(n2)]).astype(np.float32)
    for top_db in (15, 20, 60):
        a, ia = data_utils.trim(x, top_db)
        b, ib = mel_dsp.trim(x, top_db)
        assert ia == ib and np.array_equal(a, b)


def test_wav_io_roundtrip(tmp_path):
    x = _signal(3000, 16000) * 2.0
    p = str(tmp_path / "a.wav")
    data_utils.write_wav(p, x, 16000)
    y, sr = data_utils.read_wav(p)
    assert sr == 16000 and len(y) == len(x)
    # libsndfile's float -> PCM_16 (lrintf(x * 0x7FFF)), saturated; read back as PCM / 32768
    want = np.clip(np.rint(x.astype(np.float64) * 32767.0), -32768, 32767) / 32768.0
    assert np.array_equal(y, want.astype(np.float32))
    # resampling on load (librosa.load(sr=...))
    z = data_utils.load_wav(p, 8000)
    assert abs(len(z) - 1500) <= 1


def test_wav_reader_formats(tmp_path):
    import struct
    x = np.array([0.0, 0.5, -0.5, 0.25], np.float64)

    def riff(fmt_tag, ch, bits, data):
        fmt = struct.pack("<HHIIHH", fmt_tag, ch, 16000, 16000 * ch * bits // 8, ch * bits // 8, bits)
        body = b"WAVE" + b"fmt " + struct.pack("<I", len(fmt)) + fmt + b"data" + struct.pack("<I", len(data)) + data
        return b"RIFF" + struct.pack("<I", len(body)) + body
    cases = {
        "f32": riff(3, 1, 32, x.astype("<f4").tobytes()),
        "i24": riff(1, 1, 24, b"".join(int(round(v * (1 << 23))).to_bytes(3, "little", signed=True) for v in x)),
        "st16": riff(1, 2, 16, np.repeat(np.round(x * 32768).astype("<i2"), 2).tobytes()),
    }
    for name, blob in cases.items():
        p = tmp_path / f"{name}.wav"
        p.write_bytes(blob)
        y, sr = data_utils.read_wav(str(p))
        assert sr == 16000 and np.abs(y - x).max() < 1e-6, name


def _model_dir(tmp_path, golden):
    import helpers
    z = golden("small_T32")
    m = helpers.model_from_fixture(z)
    d = tmp_path / "model"
    d.mkdir()
    pre = dict(sample_rate=8000, preemph=0.97, n_fft=256, hop_length=64, win_length=200, n_mels=80, ref_db=20,
               max_db=100, top_db=30)
    with open(d / "config.yaml", "w") as f:
        yaml.safe_dump({"model": helpers.cfg_of(z), "preprocess": pre}, f)
    torch.save(m.state_dict(), d / "model.ckpt")
    with open(d / "attr.pkl", "wb") as f:
        pickle.dump({"mean": np.linspace(0.2, 0.6, 80), "std": np.linspace(0.1, 0.3, 80)}, f)
    return d, m


def test_load_model(tmp_path, golden):
    d, m = _model_dir(tmp_path, golden)
    model, config, attr, device = data_utils.load_model(str(d))
    assert device == ("cuda" if torch.cuda.is_available() else "cpu")
    assert config["preprocess"]["n_fft"] == 256 and attr["mean"].shape == (80,)
    for k, v in m.state_dict().items():
        assert torch.equal(model.state_dict()[k].cpu(), v)


def test_attr_loader_refuses_code(tmp_path):
    class Evil:
        def __reduce__(self):
            return (os.system, ("true",))
    p = tmp_path / "attr.pkl"
    with open(p, "wb") as f:
        pickle.dump({"mean": Evil(), "std": 1}, f)
    with pytest.raises(pickle.UnpicklingError):
        data_utils.load_attr(str(p))


def test_attack_cli_flags_match_reference():
    import attack
    a = attack.build_parser().parse_args(["m", "t.wav", "a.wav", "o.wav"])
    assert (a.vc_src, a.eps, a.n_iters, a.attack_type) == (None, 0.1, 1500, "emb")
    a = attack.build_parser().parse_args(["m", "t", "a", "o", "--vc_src", "s", "--eps", "0.05", "--n_iters", "10",
                                          "--attack_type", "fb"])
    assert (a.vc_src, a.eps, a.n_iters, a.attack_type) == ("s", 0.05, 10, "fb")
    with pytest.raises(SystemExit):
        attack.build_parser().parse_args(["m", "t", "a", "o", "--attack_type", "xx"])


# ---- oracle primitives pinned against scipy (the reference's own DSP library besides librosa:
# data_utils.py:163 calls scipy.signal.lfilter; librosa 0.8's get_window / stft / istft are
# scipy.signal.get_window + a centered reflect-padded framing that scipy.signal.stft /
# istft(boundary='even' / True) reproduce).  librosa itself is absent: the mel filter bank and
# trim stay restated (parity of those two unpinned), everything else below is pinned here.

def _scipy_stft(y, n_fft, hop, win):
    import scipy.signal as ss
    w = mel_dsp.stft_window(n_fft, win)
    _, _, Z = ss.stft(y, fs=1.0, window=w, nperseg=n_fft, noverlap=n_fft - hop, nfft=n_fft, detrend=False,
                      return_onesided=True, boundary="even", padded=False, scaling="spectrum")
    return Z * w.sum()            # scaling="spectrum" divides by sum(window); librosa does not


def _scipy_istft(S, n_fft, hop, win):
    import scipy.signal as ss
    w = mel_dsp.stft_window(n_fft, win)
    _, y = ss.istft(S / w.sum(), fs=1.0, window=w, nperseg=n_fft, noverlap=n_fft - hop, nfft=n_fft,
                    input_onesided=True, boundary=True, scaling="spectrum")
    return y


@pytest.mark.parametrize("win", [1200, 2048, 801])
def test_hann_window_is_scipy(win):
    import scipy.signal as ss
    np.testing.assert_allclose(mel_dsp.hann_periodic(win), ss.get_window("hann", win, fftbins=True),
                               rtol=0, atol=1e-15)


def test_deemphasis_is_scipy_lfilter():
    """data_utils.py:163: signal.lfilter([1], [1, -preemph], wav)."""
    import scipy.signal as ss
    x = np.random.default_rng(3).standard_normal(20000)
    for a in (0.97, 0.5):
        np.testing.assert_allclose(mel_dsp.deemphasis(x, a), ss.lfilter([1], [1, -a], x), rtol=0, atol=1e-12)


@pytest.mark.parametrize("n_fft,hop,win,n", [(2048, 300, 1200, 16000), (512, 128, 512, 4000), (1024, 256, 600, 7001)])
def test_stft_istft_are_scipy(n_fft, hop, win, n):
    y = np.random.default_rng(n).standard_normal(n)
    S = mel_dsp.stft(y, n_fft, hop, win)
    Z = _scipy_stft(y, n_fft, hop, win)
    assert S.shape == Z.shape
    assert np.abs(S - Z).max() <= 1e-12 * np.abs(S).max()
    yo = mel_dsp.istft(S, hop, win)
    ys = _scipy_istft(S, n_fft, hop, win)
    assert np.abs(yo - ys[:len(yo)]).max() <= 1e-12 * np.abs(yo).max()


def test_griffin_lim_composition_on_scipy():
    """The reference's griffin_lim (data_utils.py:168-197) composed of scipy's transforms equals
    the oracle's (3 iterations of a random magnitude)."""
    n_fft, hop, win = 512, 128, 400
    mag = np.abs(np.random.default_rng(5).standard_normal((n_fft // 2 + 1, 40)))
    X = mag.astype(np.complex128)
    for _ in range(3):
        xt = _scipy_istft(X, n_fft, hop, win)[:hop * (mag.shape[1] - 1)]
        est = _scipy_stft(xt, n_fft, hop, win)
        X = mag * (est / np.maximum(1e-8, np.abs(est)))
    ref = np.real(_scipy_istft(X, n_fft, hop, win))[:hop * (mag.shape[1] - 1)]
    out = mel_dsp.griffin_lim(mag, hop, win, n_fft, n_iter=3)
    assert out.shape == ref.shape
    np.testing.assert_allclose(out, ref, rtol=0, atol=1e-10 * np.abs(ref).max())
