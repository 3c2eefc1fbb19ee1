"""VSMask's mel converter (/root/reference/utils/audio.py) on MI355X.

``MelSpectrogramConverter`` keeps the reference's name, constructor defaults and methods; the
transforms run in libavc's DSP kernels (csrc/avc_dsp.hip, a flavor-1 ``avc_dsp`` context) with
torchaudio's semantics:

  * ``waveform_to_mel`` (utils/audio.py:44-57): ``MelSpectrogram(sample_rate, n_fft, hop_length,
    n_mels)`` -- centred frames (reflect padding), periodic Hann(n_fft), power 2, HTK mel filter
    bank without normalisation over [0, sample_rate // 2] -- then ``log10(clamp(., 1e-5))``.
  * ``mel_to_waveform`` (59-75): ``pow(10, .)``, ``InverseMelScale`` (torch.linalg.lstsq of
    fb^T X = mel: the minimum-norm least-squares solution for the full-rank bank, as one pinv
    matrix; relu), ``GriffinLim(n_fft, hop_length)`` with torchaudio's defaults: power 2, 32
    iterations, momentum 0.99, random initial phases drawn exactly as torchaudio draws them
    (``torch.rand(shape, dtype=complex64)`` on the CPU generator -- the reference's converter modules are
    never moved to a device, so utils/audio.py only runs on CPU and draws there; the draw is then moved
    to the GPU, so a seeded run takes the reference's draw).
  * ``apply_weighted_constraint`` (77-116): the per-band clamp (``avc_vsmask_band_clamp``).

torchaudio is absent here, so these numerics are restated from its published algorithms
(oracle/mel_dsp.py ``ta_*``) and checked against that restatement: parity unpinned against
torchaudio itself.  InverseMelScale follows torchaudio >= 2.1 (least squares); older releases
fitted it by SGD.
"""
from typing import Dict, Optional

import torch

import avc_native


class MelSpectrogramConverter:
    """utils/audio.py:8-116 on libavc."""

    def __init__(self, sample_rate: int = 16000, n_fft: int = 1024, hop_length: int = 256, n_mels: int = 80):
        self.sample_rate = sample_rate
        self.n_fft = n_fft
        self.hop_length = hop_length
        self.n_mels = n_mels
        # torchaudio.transforms.GriffinLim defaults (utils/audio.py:37-40 sets only n_fft / hop)
        self.n_iter = 32
        self.momentum = 0.99
        self.rand_init = True
        self._pre = avc_native.ta_preprocess(sample_rate, n_fft, hop_length, n_mels)
        self._dsp: Dict[int, avc_native.Dsp] = {}

    def _ctx(self, device: torch.device) -> "avc_native.Dsp":
        if device.type != "cuda":
            raise RuntimeError("libavc runs the mel converter on MI355X (ROCm) devices only")
        dev = device.index if device.index is not None else torch.cuda.current_device()
        d = self._dsp.get(dev)
        if d is None:
            d = self._dsp[dev] = avc_native.Dsp(self._pre, dev)
        return d

    def frames(self, n_samples: int) -> int:
        """STFT frames of an n-sample waveform (1 + n // hop_length)."""
        return 1 + int(n_samples) // self.hop_length

    def waveform_to_mel(self, waveform: torch.Tensor) -> torch.Tensor:
        """utils/audio.py:44-57: waveform [C, L] (or [L]) -> log10 mel [C, n_mels, 1 + L // hop]."""
        w = waveform.float()
        squeeze = w.dim() == 1
        if squeeze:
            w = w[None]
        if w.dim() != 2:
            raise RuntimeError(f"expected a waveform [C, L] or [L], got {tuple(waveform.shape)}")
        mel = self._ctx(w.device).wav2mel(w.contiguous(), transpose=True)
        return mel[0] if squeeze else mel

    def mel_to_waveform(self, mel_spec: torch.Tensor) -> torch.Tensor:
        """utils/audio.py:59-75: log10 mel [C, n_mels, T] -> waveform.unsqueeze(0) = [1, C, hop (T-1)].
        A [B, 1, n_mels, T] mel (vsmask.py's 4-D layout) is taken as C = B."""
        m = mel_spec.float()
        if m.dim() == 4 and m.shape[1] == 1:
            m = m[:, 0]
        if m.dim() == 2:
            m = m[None]
        if m.dim() != 3 or m.shape[1] != self.n_mels:
            raise RuntimeError(f"expected a log-mel [C, {self.n_mels}, T], got {tuple(mel_spec.shape)}")
        C, _, T = m.shape
        angles0 = None
        if self.rand_init:   # torchaudio.functional.griffinlim's draw (same shape and dtype, CPU generator)
            angles0 = torch.rand((C, self.n_fft // 2 + 1, T), dtype=torch.complex64).to(m.device)
        wav = self._ctx(m.device).ta_mel2wav(m.contiguous(), self.n_iter, self.momentum, angles0)
        return wav.unsqueeze(0)

    def apply_weighted_constraint(self, perturbation: torch.Tensor, epsilon1: float = 0.1, epsilon2: float = 0.05,
                                  epsilon3: float = 0.08) -> torch.Tensor:
        """utils/audio.py:77-116: clamp rows [0, int(0.3 F)) to +-epsilon1, [.., int(0.7 F)) to
        +-epsilon2, the rest to +-epsilon3 (F = the second-to-last dimension)."""
        return avc_native.vsmask_band_clamp(perturbation, epsilon1, epsilon2, epsilon3).reshape(perturbation.shape)


def apply_random_shift(waveform: torch.Tensor, max_shift: int = 100,
                       generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """utils/audio.py:118-146: shift [1, T] by a uniform integer in [-max_shift, max_shift],
    zero-filling the vacated samples (the same torch.randint draw as the reference)."""
    shift = int(torch.randint(-max_shift, max_shift + 1, (1,), generator=generator).item())
    if shift > 0:
        return torch.cat([torch.zeros(1, shift, device=waveform.device), waveform[:, :-shift]], dim=1)
    if shift < 0:
        return torch.cat([waveform[:, -shift:], torch.zeros(1, -shift, device=waveform.device)], dim=1)
    return waveform
