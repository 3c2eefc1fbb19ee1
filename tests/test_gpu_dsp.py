"""GPU parity of the mel front / back end (csrc/avc_dsp.hip, through the C ABI)
against the float64 oracle (oracle/mel_dsp.py: librosa 0.8.1 restated; parity
unpinned against librosa itself, which is absent).

Tolerances (fp32 radix-2 FFTs against float64 transforms):
  * wav2mel: normalized mel within TOL_MEL absolute (values in [1e-8, 1]);
  * Griffin-Lim of a consistent magnitude at small n_iter, and mel2wav at n_iter=0:
    waveform within TOL_WAV (x (1 + n_iter)) of its peak;
  * 100 iterations: the spectral distance of the result within 2% (relative) of
    the oracle's -- Griffin-Lim is a non-convex fixed-point iteration, so
    bit-level trajectories of fp32 and fp64 separate, the converged quality does
    not.
"""
import numpy as np
import pytest
import torch

import avc_native
import data_utils
from oracle import mel_dsp

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
TOL_MEL = 2e-4
TOL_WAV = 2e-4

CFGS = [
    dict(sample_rate=16000, preemph=0.97, n_fft=2048, hop_length=300, win_length=1200, n_mels=80, ref_db=20,
         max_db=100, top_db=15),
    dict(sample_rate=22050, preemph=0.97, n_fft=1024, hop_length=256, win_length=1024, n_mels=80, ref_db=20,
         max_db=100, top_db=20),
    dict(sample_rate=8000, preemph=0.9, n_fft=256, hop_length=64, win_length=200, n_mels=40, ref_db=16,
         max_db=90, top_db=30),
]


def _signal(n, sr, seed=0):
    g = np.random.default_rng(seed)
    t = np.arange(n) / sr
    env = 0.5 + 0.5 * np.sin(2 * np.pi * 1.3 * t)
    x = env * (0.3 * np.sin(2 * np.pi * 220 * t) + 0.2 * np.sin(2 * np.pi * 1330 * t + 0.5)) + \
        0.02 * g.standard_normal(n)
    return x.astype(np.float32)


def _o(pre):
    return {k: pre[k] for k in ("sample_rate", "preemph", "n_fft", "hop_length", "win_length", "n_mels", "ref_db",
                                "max_db")}


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.fail("no ROCm device visible")


@pytest.mark.parametrize("ci", range(len(CFGS)))
@pytest.mark.parametrize("L", [4000, 20001])
def test_wav2mel_vs_oracle(ci, L):
    pre = CFGS[ci]
    x = _signal(L, pre["sample_rate"], ci)
    d = data_utils.dsp_for(pre, DEV)
    mel = d.wav2mel(torch.from_numpy(x).to(DEV)[None])[0].cpu().numpy()
    ref = mel_dsp.wav2mel(x, **_o(pre))
    assert mel.shape == ref.shape == (1 + L // pre["hop_length"], pre["n_mels"])
    err = np.abs(mel - ref)
    print(f"wav2mel cfg{ci} L={L}: max {err.max():.3g} mean {err.mean():.3g}")
    assert err.max() <= TOL_MEL


def test_wav2mel_batch_layouts_and_normalize():
    pre = CFGS[1]
    g = torch.Generator().manual_seed(3)
    B, L = 5, 9000
    x = torch.stack([torch.from_numpy(_signal(L, pre["sample_rate"], s)) for s in range(B)]) + \
        0.01 * torch.randn(B, L, generator=g)
    d = data_utils.dsp_for(pre, DEV)
    xd = x.to(DEV)
    a = d.wav2mel(xd)
    mean, std = np.linspace(0.3, 0.5, 80), np.linspace(0.1, 0.2, 80)
    b = d.wav2mel(xd, mean, std, transpose=True)
    for i in range(B):
        one = d.wav2mel(xd[i:i + 1])[0]
        assert torch.equal(one, a[i])          # an utterance's result is independent of the batch
    n = (a.cpu().numpy() - mean) / std
    assert np.abs(b.cpu().numpy().transpose(0, 2, 1) - n).max() <= 1e-5 * np.abs(n).max()


@pytest.mark.parametrize("ci", range(len(CFGS)))
def test_short_signals_and_pad_modes(ci):
    """Signals shorter than n_fft/2 (numpy's repeated reflection) and constant padding."""
    pre = CFGS[ci]
    for L in (1, 2, 7, pre["n_fft"] // 2 + 3):
        x = _signal(L, pre["sample_rate"], L)
        for mode in ("reflect", "constant"):
            d = data_utils.dsp_for(pre, DEV, pad_mode=mode)
            mel = d.wav2mel(torch.from_numpy(x).to(DEV)[None])[0].cpu().numpy()
            ref = mel_dsp.wav2mel(x, **_o(pre), pad_mode=mode)
            assert np.abs(mel - ref).max() <= TOL_MEL, (L, mode)


@pytest.mark.parametrize("ci", range(len(CFGS)))
@pytest.mark.parametrize("n_iter", [0, 1, 4])
def test_griffin_lim_vs_oracle(ci, n_iter):
    pre = CFGS[ci]
    n_fft, hop, win = pre["n_fft"], pre["hop_length"], pre["win_length"]
    y = _signal(hop * 37 + 11, pre["sample_rate"], 7)
    mag = np.abs(mel_dsp.stft(y, n_fft, hop, win)).astype(np.float32)
    w = data_utils.griffin_lim(mag, hop, win, n_fft, n_iter)
    ref = mel_dsp.griffin_lim(mag.astype(np.float64), hop, win, n_fft, n_iter)
    assert w.shape == ref.shape == (hop * (mag.shape[1] - 1),)
    err = np.abs(w - ref).max() / np.abs(ref).max()
    print(f"griffin_lim cfg{ci} n_iter={n_iter}: rel max {err:.3g}")
    assert err <= TOL_WAV * (1 + n_iter)


def test_griffin_lim_100_quality():
    pre = CFGS[0]
    n_fft, hop, win = pre["n_fft"], pre["hop_length"], pre["win_length"]
    y = _signal(hop * 60, pre["sample_rate"], 9)
    mag = np.abs(mel_dsp.stft(y, n_fft, hop, win))

    def dist(w):
        return np.linalg.norm(np.abs(mel_dsp.stft(w, n_fft, hop, win)) - mag) / np.linalg.norm(mag)
    w = data_utils.griffin_lim(mag.astype(np.float32), hop, win, n_fft)
    ref = mel_dsp.griffin_lim(mag, hop, win, n_fft, 100)
    dg, dr = dist(w), dist(ref)
    print(f"griffin_lim 100: spectral distance gpu {dg:.4g} oracle {dr:.4g}")
    assert dg <= dr * 1.02 + 1e-4


@pytest.mark.parametrize("ci", range(len(CFGS)))
def test_mel2wav_vs_oracle(ci):
    """n_iter=0 (inverse dB, inv_mel_matrix, zero-phase ISTFT, de-emphasis): element-wise.
    n_iter > 0 from a pseudo-inverse magnitude: the phase of bins where the estimate
    nearly vanishes (est / max(1e-8, |est|)) is ill-conditioned, so fp32 and fp64 runs
    separate element-wise (1e-3..1e-2 after 2 iterations); their spectral distance to the
    target magnitude is compared instead."""
    pre = CFGS[ci]
    n_fft, hop, win = pre["n_fft"], pre["hop_length"], pre["win_length"]
    x = _signal(hop * 50, pre["sample_rate"], 11)
    mel = mel_dsp.wav2mel(x, **_o(pre)).astype(np.float32)
    mag = mel_dsp.mel2mag(mel, pre["sample_rate"], n_fft, pre["n_mels"], pre["ref_db"], pre["max_db"])
    a = pre["preemph"]

    def dist(w):   # undo the de-emphasis, then |STFT| against the target magnitude
        w = np.asarray(w, np.float64)
        y = np.append(w[0], w[1:] - a * w[:-1])
        return np.linalg.norm(np.abs(mel_dsp.stft(y, n_fft, hop, win)) - mag) / np.linalg.norm(mag)
    d = data_utils.dsp_for(pre, DEV)
    for n_iter in (0, 2, 20):
        w = d.mel2wav(torch.from_numpy(mel).to(DEV)[None], n_iter=n_iter)[0].cpu().numpy()
        ref = mel_dsp.mel2wav(mel, **_o(pre), n_iter=n_iter)
        err = np.abs(w - ref).max() / np.abs(ref).max()
        dg, dr = dist(w), dist(ref)
        print(f"mel2wav cfg{ci} n_iter={n_iter}: rel max {err:.3g}, spectral distance gpu {dg:.4g} oracle {dr:.4g}")
        if n_iter == 0:
            assert err <= TOL_WAV
        assert dg <= dr * 1.02 + 1e-4


def test_mel2wav_denormalize_and_layout():
    pre = CFGS[1]
    x = _signal(pre["hop_length"] * 40, pre["sample_rate"], 2)
    mel = mel_dsp.wav2mel(x, **_o(pre)).astype(np.float32)
    mean, std = np.linspace(0.3, 0.5, 80), np.linspace(0.1, 0.2, 80)
    nmel = ((mel - mean) / std).astype(np.float32)
    d = data_utils.dsp_for(pre, DEV)
    a = d.mel2wav(torch.from_numpy(mel).to(DEV)[None], n_iter=0)
    b = d.mel2wav(torch.from_numpy(np.ascontiguousarray(nmel.T)).to(DEV)[None], mean, std, transpose=True, n_iter=0)
    assert torch.allclose(a, b, rtol=0, atol=1e-4 * float(a.abs().max()))


def test_file2mel_mel2wav_roundtrip(tmp_path):
    """data_utils.file2mel / mel2wav (the reference's signatures) on a written wav."""
    pre = CFGS[0]
    x = np.concatenate([np.zeros(4000, np.float32), _signal(24000, 16000, 4), np.zeros(3000, np.float32)])
    p = str(tmp_path / "x.wav")
    data_utils.write_wav(p, x, 16000)
    mel = data_utils.file2mel(p, **pre)
    xr, _ = data_utils.read_wav(p)
    xt, _ = mel_dsp.trim(xr, pre["top_db"])
    ref = mel_dsp.wav2mel(xt, **_o(pre))
    assert mel.shape == ref.shape and np.abs(mel - ref).max() <= TOL_MEL
    w = data_utils.mel2wav(mel, **pre)
    assert w.dtype == np.float32 and w.shape == (pre["hop_length"] * (mel.shape[0] - 1),)
    assert np.isfinite(w).all()


def _model_dir(tmp_path, golden):
    import pickle

    import yaml

    import helpers
    z = golden("full_T128")
    m = helpers.model_from_fixture(z)
    d = tmp_path / "model"
    d.mkdir()
    pre = dict(CFGS[0])
    with open(d / "config.yaml", "w") as f:
        yaml.safe_dump({"model": helpers.cfg_of(z), "preprocess": pre}, f)
    torch.save(m.state_dict(), d / "model.ckpt")
    with open(d / "attr.pkl", "wb") as f:
        pickle.dump({"mean": np.full(80, 0.4), "std": np.full(80, 0.2)}, f)
    return d, pre


@pytest.mark.parametrize("frames", [{"src": 90, "tgt": 110, "adv": 70},        # all within the fused engine
                                    {"src": 213, "tgt": 266, "adv": 160}])    # 4 s / 5 s / 3 s: long engine
def test_attack_cli_end_to_end(tmp_path, golden, frames):
    """attack.py main() (the reference's CLI): wav files in, defended wav out, all on the GPU.
    The three wavs have different lengths, as real utterances do (attack.py:49-56 loads each
    on its own; the reference's attacks never require equal lengths); the second case has a
    5-second vc_tgt (266 frames at hop 300 / 16 kHz)."""
    import attack
    d, pre = _model_dir(tmp_path, golden)
    paths = {}
    for i, k in enumerate(("src", "tgt", "adv")):
        paths[k] = str(tmp_path / f"{k}.wav")
        data_utils.write_wav(paths[k], _signal(300 * frames[k], 16000, 20 + i), 16000)
    n_tgt = data_utils.file2mel(paths["tgt"], **pre).shape[0]
    for kind in ("emb", "e2e", "fb"):
        out = str(tmp_path / f"out_{kind}.wav")
        attack.main(str(d), paths["src"], paths["tgt"], paths["adv"], out, 0.1, 5, kind)
        w, sr = data_utils.read_wav(out)
        # the defended utterance keeps vc_tgt's frames (mel2wav: hop * (T - 1) samples)
        assert sr == 16000 and len(w) == pre["hop_length"] * (n_tgt - 1) and np.isfinite(w).all()


def test_inference_cli(tmp_path, golden):
    """inference.py main() (reference inference.py:9-47): source content in the target's
    voice; source 4 s (long engine), target 2 s; the output has the source's frames."""
    import inference
    d, pre = _model_dir(tmp_path, golden)
    src, tgt, out = (str(tmp_path / f"{k}.wav") for k in ("src", "tgt", "out"))
    data_utils.write_wav(src, _signal(300 * 213, 16000, 31), 16000)
    data_utils.write_wav(tgt, _signal(300 * 107, 16000, 32), 16000)
    inference.main(str(d), src, tgt, out)
    n_src = data_utils.file2mel(src, **pre).shape[0]
    w, sr = data_utils.read_wav(out)
    assert sr == 16000 and np.isfinite(w).all()
    assert len(w) == pre["hop_length"] * (8 * ((n_src + 7) // 8) - 1)     # decoder: 8 * ceil(T / 8) frames


def test_deemphasis_long_signal():
    """dsp_deemph's chunked scan == the sequential recurrence (mel2wav's lfilter)."""
    pre = CFGS[2]
    hop = pre["hop_length"]
    x = _signal(hop * 900, pre["sample_rate"], 5)
    mel = mel_dsp.wav2mel(x, **_o(pre)).astype(np.float32)
    w = data_utils.dsp_for(pre, DEV).mel2wav(torch.from_numpy(mel).to(DEV)[None], n_iter=0)[0].cpu().numpy()
    ref = mel_dsp.mel2wav(mel, **_o(pre), n_iter=0)
    assert np.abs(w - ref).max() <= TOL_WAV * np.abs(ref).max()


def test_bad_arguments_fail_loudly():
    pre = CFGS[2]
    d = data_utils.dsp_for(pre, DEV)
    with pytest.raises(RuntimeError):
        d.wav2mel(torch.zeros(1, 100))                  # host tensor
    with pytest.raises(RuntimeError):
        d.mel2wav(torch.zeros(1, 5, 7, device=DEV))     # wrong n_mels
    with pytest.raises(RuntimeError):
        d.mel2wav(torch.zeros(1, 1, 40, device=DEV))    # Tf < 2
