"""Drop-in replacement for /root/reference/data_utils.py on MI355X.

Same function names, arguments and return types as the reference:

  inv_mel_matrix(sample_rate, n_fft, n_mels)                 data_utils.py:16-32
  normalize(mel, attr) / denormalize(mel, attr)              data_utils.py:35-62
  file2mel(audio_path, sample_rate, preemph, n_fft, hop_length, win_length,
           n_mels, ref_db, max_db, top_db)                   data_utils.py:65-118
  mel2wav(mel, sample_rate, preemph, n_fft, hop_length, win_length, n_mels,
          ref_db, max_db, top_db)                            data_utils.py:121-165
  griffin_lim(spect, hop_length, win_length, n_fft, n_iter=100)  data_utils.py:168-197
  load_model(model_dir)                                      data_utils.py:200-223

The reference computes its DSP with librosa (absent here, and <= 0.9 by its
positional calls).  Here the transforms (pre-emphasis, STFT, mel projection, dB,
the pseudo-inverse mel, the 100 Griffin-Lim iterations, de-emphasis) run in
libavc's HIP kernels (csrc/avc_dsp.hip) through avc_native.Dsp; the host keeps
what is I/O or data-dependent slicing: reading the wav file (stdlib `wave`;
PCM 8/16/24/32-bit and float WAV), resampling when the file's rate differs
(scipy.signal.resample_poly, where librosa 0.8 used resampy), and the silence
trim (librosa.effects.trim: frame RMS in dB against the loudest frame).

Batched GPU entry points for many utterances at once: `wav2mel_batch`,
`mel2wav_batch` (device tensors in, device tensors out).
"""
import os
import pickle
import struct
import wave
from typing import Dict, Optional, Tuple

import numpy as np
import torch
import torch.nn as nn
import yaml

import avc_native
from models import AdaInVC

_DSP: Dict[Tuple, "avc_native.Dsp"] = {}

PRE_KEYS = ("sample_rate", "preemph", "n_fft", "hop_length", "win_length", "n_mels", "ref_db", "max_db")


def _device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("libavc's DSP runs on MI355X (ROCm) devices only; no device is visible")
    return torch.device("cuda", torch.cuda.current_device())


def dsp_for(preprocess: Dict, device: Optional[torch.device] = None, pad_mode: str = "reflect") -> "avc_native.Dsp":
    """Cached libavc DSP context for a config.yaml `preprocess` section."""
    device = device or _device()
    key = tuple(float(preprocess[k]) for k in PRE_KEYS) + (pad_mode, device.index or 0)
    d = _DSP.get(key)
    if d is None:
        d = _DSP[key] = avc_native.Dsp(preprocess, device.index or 0, pad_mode)
    return d


def inv_mel_matrix(sample_rate: int, n_fft: int, n_mels: int) -> np.ndarray:
    """data_utils.py:16-32: pseudo-inverse of the Slaney mel filter bank, [n_fft/2+1, n_mels]."""
    pre = dict(sample_rate=sample_rate, n_fft=n_fft, hop_length=1, win_length=n_fft, n_mels=n_mels,
               preemph=0.0, ref_db=0.0, max_db=1.0)
    return avc_native.mel_basis(pre)[1].numpy()


def normalize(mel: np.ndarray, attr: Dict) -> np.ndarray:
    """data_utils.py:35-47."""
    mean, std = attr["mean"], attr["std"]
    return (mel - mean) / std


def denormalize(mel: np.ndarray, attr: Dict) -> np.ndarray:
    """data_utils.py:50-62."""
    mean, std = attr["mean"], attr["std"]
    return mel * std + mean


# ----------------------------------------------------------------------------------
# host I/O: wav read / write, resample, silence trim
# ----------------------------------------------------------------------------------


def read_wav(path: str) -> Tuple[np.ndarray, int]:
    """Mono float32 samples in [-1, 1) and the file's rate (channels averaged, as
    librosa.load(mono=True) does).  PCM 8/16/24/32-bit and IEEE-float WAV."""
    with open(path, "rb") as f:
        head = f.read(12)
        if head[:4] != b"RIFF" or head[8:12] != b"WAVE":
            raise RuntimeError(f"{path}: not a RIFF/WAVE file")
        fmt = None
        data = None
        while True:
            ck = f.read(8)
            if len(ck) < 8:
                break
            cid, size = ck[:4], struct.unpack("<I", ck[4:])[0]
            body = f.read(size + (size & 1))[:size]
            if cid == b"fmt ":
                tag, ch, rate, _, _, bits = struct.unpack("<HHIIHH", body[:16])
                if tag == 0xFFFE and len(body) >= 26:          # WAVE_FORMAT_EXTENSIBLE
                    tag = struct.unpack("<H", body[24:26])[0]
                fmt = (tag, ch, rate, bits)
            elif cid == b"data":
                data = body
    if fmt is None or data is None:
        raise RuntimeError(f"{path}: missing fmt or data chunk")
    tag, ch, rate, bits = fmt
    if tag == 3 and bits in (32, 64):
        x = np.frombuffer(data, "<f4" if bits == 32 else "<f8").astype(np.float32)
    elif tag == 1 and bits == 8:
        x = (np.frombuffer(data, np.uint8).astype(np.float32) - 128.0) / 128.0
    elif tag == 1 and bits == 16:
        x = np.frombuffer(data, "<i2").astype(np.float32) / 32768.0
    elif tag == 1 and bits == 24:
        b = np.frombuffer(data, np.uint8).reshape(-1, 3).astype(np.int32)
        v = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
        x = (np.where(v >= 1 << 23, v - (1 << 24), v)).astype(np.float32) / float(1 << 23)
    elif tag == 1 and bits == 32:
        x = np.frombuffer(data, "<i4").astype(np.float32) / float(1 << 31)
    else:
        raise RuntimeError(f"{path}: unsupported WAV encoding (format {tag}, {bits} bits)")
    x = x[: len(x) // ch * ch].reshape(-1, ch).mean(axis=1).astype(np.float32)
    return x, rate


def write_wav(path: str, wav: np.ndarray, sample_rate: int) -> None:
    """soundfile.write(path, wav, sr) for a .wav path: 16-bit PCM (soundfile's default
    subtype) with libsndfile's float -> PCM_16 conversion: lrintf(x * 0x7FFF) (round half to
    even).  libsndfile does not clip by default (out-of-range samples overflow the short);
    here they saturate at -32768 / 32767 instead -- the only difference (parity unpinned: no
    soundfile output exists in the reference)."""
    x = np.rint(np.asarray(wav, np.float64) * 32767.0)
    pcm = np.clip(x, -32768, 32767).astype("<i2")
    with wave.open(path, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(2)
        w.setframerate(int(sample_rate))
        w.writeframes(pcm.tobytes())


def write_wav_float(path: str, wav: np.ndarray, sample_rate: int) -> None:
    """torchaudio.save(path, wav [C, L] float32, sr) for a .wav path: 32-bit IEEE-float WAV
    (WAVE_FORMAT_IEEE_FLOAT, torchaudio's encoding for float32 tensors), channels interleaved."""
    x = np.asarray(wav, np.float32)
    if x.ndim == 1:
        x = x[None]
    ch = x.shape[0]
    data = np.ascontiguousarray(x.T).astype("<f4").tobytes()
    fmt = struct.pack("<HHIIHH", 3, ch, int(sample_rate), int(sample_rate) * 4 * ch, 4 * ch, 32)
    fact = struct.pack("<I", x.shape[1])
    body = b"WAVE" + b"fmt " + struct.pack("<I", len(fmt)) + fmt + b"fact" + struct.pack("<I", 4) + fact + \
        b"data" + struct.pack("<I", len(data)) + data
    with open(path, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", len(body)) + body)


def resample(x: np.ndarray, rate: int, sample_rate: int) -> np.ndarray:
    """x at `rate` -> `sample_rate` by scipy's polyphase filter (librosa.load's resampy and
    torchaudio's Resample filter differently: parity unpinned)."""
    if rate == sample_rate:
        return x
    from math import gcd

    from scipy.signal import resample_poly
    g = gcd(int(rate), int(sample_rate))
    return resample_poly(x, int(sample_rate) // g, int(rate) // g).astype(np.float32)


def load_wav(audio_path: str, sample_rate: int) -> np.ndarray:
    """librosa.load(audio_path, sr=sample_rate): mono float32 at sample_rate."""
    x, rate = read_wav(audio_path)
    return resample(x, rate, sample_rate)


def trim(wav: np.ndarray, top_db: float, frame_length: int = 2048, hop_length: int = 512):
    """librosa.effects.trim(wav, top_db=top_db): keep the span from the first to the last
    frame whose RMS is within top_db of the loudest frame (frames centered, reflect pad)."""
    wav = np.asarray(wav)
    if len(wav) == 0:
        return wav, (0, 0)
    pad = frame_length // 2
    y = np.pad(wav.astype(np.float64), pad, mode="reflect") if len(wav) > 1 else np.full(len(wav) + 2 * pad, float(wav[0]))
    n = 1 + (len(y) - frame_length) // hop_length
    c = np.concatenate([[0.0], np.cumsum(y * y)])
    starts = np.arange(n) * hop_length
    power = (c[starts + frame_length] - c[starts]) / frame_length
    db = 10.0 * np.log10(np.maximum(1e-10, power)) - 10.0 * np.log10(max(1e-10, float(power.max())))
    keep = np.flatnonzero(db > -top_db)
    if keep.size == 0:
        return wav[0:0], (0, 0)
    start = int(keep[0] * hop_length)
    end = min(len(wav), int((keep[-1] + 1) * hop_length))
    return wav[start:end], (start, end)


# ----------------------------------------------------------------------------------
# the reference's functions
# ----------------------------------------------------------------------------------


def _pre(sample_rate, preemph, n_fft, hop_length, win_length, n_mels, ref_db, max_db) -> Dict:
    return dict(sample_rate=sample_rate, preemph=preemph, n_fft=n_fft, hop_length=hop_length,
                win_length=win_length, n_mels=n_mels, ref_db=ref_db, max_db=max_db)


def wav2mel_batch(wav: torch.Tensor, preprocess: Dict, attr: Optional[Dict] = None,
                  transpose: bool = True) -> torch.Tensor:
    """Trimmed waveforms [B, L] (device) -> normalized mels [B, n_mels, Tf] (the attacks'
    input layout; [B, Tf, n_mels] if not transpose).  attr=None skips normalize()."""
    d = dsp_for(preprocess, wav.device)
    mean, std = (attr["mean"], attr["std"]) if attr is not None else (None, None)
    return d.wav2mel(wav, mean, std, transpose)


def mel2wav_batch(mel: torch.Tensor, preprocess: Dict, attr: Optional[Dict] = None, transpose: bool = True,
                  n_iter: int = 100) -> torch.Tensor:
    """Normalized mels [B, n_mels, Tf] (device; [B, Tf, n_mels] if not transpose) ->
    waveforms [B, hop * (Tf - 1)]: denormalize + mel2wav for a batch."""
    d = dsp_for(preprocess, mel.device)
    mean, std = (attr["mean"], attr["std"]) if attr is not None else (None, None)
    return d.mel2wav(mel, mean, std, transpose, n_iter)


def file2mel(audio_path: str, sample_rate: int, preemph: float, n_fft: int, hop_length: int, win_length: int,
             n_mels: int, ref_db: float, max_db: float, top_db: float) -> np.ndarray:
    """data_utils.py:65-118 -> float32 [T, n_mels]."""
    wav = load_wav(audio_path, sample_rate)
    wav, _ = trim(wav, top_db=top_db)
    if len(wav) == 0:
        raise RuntimeError(f"{audio_path}: no samples left after trimming silence")
    pre = _pre(sample_rate, preemph, n_fft, hop_length, win_length, n_mels, ref_db, max_db)
    x = torch.from_numpy(np.ascontiguousarray(wav, np.float32)).to(_device()).unsqueeze(0)
    return wav2mel_batch(x, pre, None, transpose=False)[0].cpu().numpy()


def mel2wav(mel: np.ndarray, sample_rate: int, preemph: float, n_fft: int, hop_length: int, win_length: int,
            n_mels: int, ref_db: float, max_db: float, top_db: float) -> np.ndarray:
    """data_utils.py:121-165: [T, n_mels] (denormalized) -> float32 waveform."""
    pre = _pre(sample_rate, preemph, n_fft, hop_length, win_length, n_mels, ref_db, max_db)
    m = torch.as_tensor(np.ascontiguousarray(mel, np.float32)).to(_device()).unsqueeze(0)
    return mel2wav_batch(m, pre, None, transpose=False)[0].cpu().numpy()


def griffin_lim(spect: np.ndarray, hop_length: int, win_length: int, n_fft: int,
                n_iter: Optional[int] = 100) -> np.ndarray:
    """data_utils.py:168-197: magnitude [n_fft/2+1, T] -> waveform."""
    pre = _pre(16000, 0.0, n_fft, hop_length, win_length, 1, 0.0, 1.0)
    d = dsp_for(pre)
    s = torch.as_tensor(np.ascontiguousarray(spect, np.float32)).to(_device()).unsqueeze(0)
    return d.griffin_lim(s, 100 if n_iter is None else n_iter)[0].cpu().numpy()


class _AttrUnpickler(pickle.Unpickler):
    """attr.pkl holds {"mean": ndarray, "std": ndarray}: allow only numpy's array
    reconstruction, nothing else executes."""
    ALLOWED = {("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
               ("numpy", "ndarray"), ("numpy", "dtype"), ("numpy.core.multiarray", "scalar"),
               ("numpy._core.multiarray", "scalar"), ("builtins", "dict")}

    def find_class(self, module, name):
        if (module, name) in self.ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"attr.pkl: refusing to load {module}.{name}")


def load_attr(path: str) -> Dict:
    with open(path, "rb") as f:
        attr = _AttrUnpickler(f).load()
    if not isinstance(attr, dict) or "mean" not in attr or "std" not in attr:
        raise RuntimeError(f"{path}: expected a dict with 'mean' and 'std'")
    return attr


def load_model(model_dir: str) -> Tuple[nn.Module, Dict, Dict, str]:
    """data_utils.py:200-223: (model, config, attr, device) from model_dir/{attr.pkl,
    config.yaml, model.ckpt}.  The checkpoint is read with weights_only=True and mapped
    to the device; shapes are checked against config.yaml by load_state_dict."""
    device = "cuda" if torch.cuda.is_available() else "cpu"
    attr = load_attr(os.path.join(model_dir, "attr.pkl"))
    with open(os.path.join(model_dir, "config.yaml"), "r") as f:
        config = yaml.safe_load(f)
    model = AdaInVC(config["model"]).to(device)
    state = torch.load(os.path.join(model_dir, "model.ckpt"), map_location=device, weights_only=True)
    model.load_state_dict(state)
    nm = int(config["preprocess"]["n_mels"]) if "preprocess" in config else None
    for k in ("mean", "std"):
        if nm is not None and np.asarray(attr[k]).reshape(-1).shape[0] != nm:
            raise RuntimeError(f"attr.pkl {k} has {np.asarray(attr[k]).size} bins, config n_mels = {nm}")
    return model, config, attr, device
