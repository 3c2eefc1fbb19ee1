"""VSMask mel protection (/root/reference/vsmask.py, models/header_model.py) on MI355X.

Mirrors the reference's classes with the same names, constructor arguments and defaults:

  * ``UniversalPerturbationHeader`` (header_model.py:7-104): the [1, 1, 80, 100] header,
    ``optimize`` (libavc ``avc_header_optimize``), ``load``/``save`` and ``apply_header``
    (libavc ``avc_vsmask_apply_header``).
  * ``VSMask`` (vsmask.py:14-213): loads a PredictiveModel state_dict and a header, and
    ``protect_mel`` runs the sliding-window loop of ``_protect_waveform`` (vsmask.py:177-208)
    in libavc: window gather -> ONE batched PredictiveModel forward over every window ->
    per-element combine in the reference's add order -> per-band clamp
    (``avc_vsmask_protect``).

The waveform entry points run utils/audio.py's converter on libavc's DSP kernels
(audio.MelSpectrogramConverter: torchaudio MelSpectrogram / InverseMelScale / GriffinLim
semantics, flavor 1 of avc_dsp): ``protect_file`` (vsmask.py:41-80) and ``_protect_waveform``
(160-213) are waveform -> log-mel -> ``protect_mel`` -> waveform; ``protect_stream`` (82-158)
replays the reference's chunk loop.  The reference as shipped cannot run (3-D mel indexed as
4-D; 95 predicted rows added to an 80-row mel; a [1, 1, L] waveform handed to
torchaudio.save); the settlement -- 4-D [B, 1, F, T] mel, predicted rows cropped to F, [C, L]
waveforms -- is documented in include/avc.h and oracle/vsmask.py.

CLI (the reference's arguments: audio in, audio out; a .npy input / output is a log-mel):

  python vsmask.py --predictive_model PM.pt --header HEADER.pt --input in.wav --output out.wav
"""
import argparse
from typing import Optional

import numpy as np
import torch

import avc_native
import data_utils
from audio import MelSpectrogramConverter
from predictive_model import PredictiveModel


class UniversalPerturbationHeader:
    """header_model.py:7-104 on libavc."""

    def __init__(self, mel_bins: int = 80, time_length: int = 100, device: str = "cuda"):
        self.mel_bins = mel_bins
        self.time_length = time_length
        self.device = device
        self.header = torch.zeros((1, 1, mel_bins, time_length), device=device)
        self.header.requires_grad = True

    def optimize(self, source_mel: torch.Tensor, target_mel: torch.Tensor, speaker_encoder, optimizer,
                 num_iterations: int = 1000, epsilon: float = 0.1, lambda_param: float = 0.5,
                 precision: str = "fp32") -> None:
        """header_model.py:25-68 on the MI355X (avc_header_optimize): the whole loop -- clamp
        (source + header), SpeakerEncoder forward, the loss MSE(., SE(target)) - lambda MSE(.,
        SE(source)), its input-gradient, torch Adam on the header with `optimizer`'s lr /
        betas / eps, clamp to +-epsilon -- runs in libavc, one captured graph per iteration.

        source_mel / target_mel: [N, 1, F, T] as train_header.py builds them (or [N, F, T]; the
        reference's SpeakerEncoder cannot take the 4-D form, SURVEY.md 2 note A).  The header
        is updated in place, and `optimizer` advances exactly as torch's Adam would: its
        hyper-parameters come from param_groups[0], its state for the header (exp_avg,
        exp_avg_sq, step) is continued and written back, so repeated calls with one optimizer
        follow the reference's trajectory.  Prints the batch loss every 100 iterations like the
        reference."""
        def mel3(x):
            return x[:, 0] if x.dim() == 4 else x
        src, tgt = mel3(source_mel).float(), mel3(target_mel).float()
        g = optimizer.param_groups[0]
        if g.get("amsgrad") or g.get("weight_decay", 0) or g.get("maximize"):
            raise RuntimeError("libavc implements plain Adam (no amsgrad / weight_decay / maximize)")
        if g.get("differentiable"):
            raise RuntimeError("libavc's header optimiser does not record an autograd graph (differentiable=True)")
        ctx = avc_native.context_for(speaker_encoder, src.device)
        hdr0 = self.header.detach()[0, 0]
        # torch Adam's per-parameter state for the header (created on its first step)
        st = optimizer.state[self.header] if self.header in optimizer.state else {}
        if st:
            m = st["exp_avg"].detach()[0, 0].float().contiguous().clone()
            v = st["exp_avg_sq"].detach()[0, 0].float().contiguous().clone()
            step0 = int(st["step"])
        else:
            m = torch.zeros_like(hdr0, dtype=torch.float32)
            v = torch.zeros_like(hdr0, dtype=torch.float32)
            step0 = 0
        new, losses = ctx.header_optimize(src, tgt, hdr0, int(num_iterations), epsilon, lambda_param, g["lr"],
                                          g["betas"], g["eps"], precision, adam_state=(m, v, step0))
        with torch.no_grad():
            self.header.data.copy_(new.reshape(self.header.shape))
        if int(num_iterations) > 0:
            shape = self.header.shape
            # torch keeps `step` as a float32 scalar tensor, on the parameter's device when the
            # optimizer is capturable / fused (torch.optim.adam's _get_scalar_dtype / device rule)
            on_dev = bool(g.get("capturable") or g.get("fused"))
            optimizer.state[self.header] = {
                "step": torch.tensor(float(step0 + int(num_iterations)), dtype=torch.float32,
                                     device=self.header.device if on_dev else "cpu"),
                "exp_avg": m.reshape(shape).to(self.header.dtype),
                "exp_avg_sq": v.reshape(shape).to(self.header.dtype)}
        batch = losses.mean(dim=1).cpu()
        for i in range(99, int(num_iterations), 100):
            print(f"Iteration {i+1}/{num_iterations}, Loss: {batch[i].item():.6f}")
        self.losses = batch

    def apply_header(self, source_mel: torch.Tensor) -> torch.Tensor:
        """header_model.py:70-95: mel [B,1,F,T] + header on frames [0, min(T, 100)), clamped to [-1, 1]."""
        return avc_native.vsmask_apply_header(source_mel, self.header)

    def save(self, path: str) -> None:
        torch.save(self.header.detach(), path)

    def load(self, path: str) -> None:
        h = torch.load(path, map_location=self.device, weights_only=True)
        if not isinstance(h, torch.Tensor) or h.dim() != 4 or h.shape[:2] != (1, 1):
            raise RuntimeError(f"{path}: expected a [1, 1, F, T] header tensor")
        self.header = h.float()
        self.mel_bins, self.time_length = int(h.shape[2]), int(h.shape[3])
        self.header.requires_grad = True


class VSMask:
    """vsmask.py:14-39 constructor; protect_mel = the mel loop of _protect_waveform."""

    def __init__(self, predictive_model_path: Optional[str], header_path: Optional[str],
                 device: str = "cuda"):
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("libavc runs VSMask on MI355X (ROCm) devices only")
        self.predictive_model = PredictiveModel().to(self.device)
        if predictive_model_path is not None:
            sd = torch.load(predictive_model_path, map_location=self.device, weights_only=True)
            self.predictive_model.load_state_dict(sd)
        self.predictive_model.eval()
        self.header = UniversalPerturbationHeader(device=self.device)
        if header_path is not None:
            self.header.load(header_path)
        self.converter = MelSpectrogramConverter()

    def protect_mel(self, mel_spec: torch.Tensor, window_size: int = 100, future_step: int = 10,
                    epsilon1: float = 0.1, epsilon2: float = 0.05, epsilon3: float = 0.08) -> torch.Tensor:
        """vsmask.py:181-208 on a log-mel [B,1,F,T] (or [1,F,T] / [F,T]); returns the same shape."""
        shape = mel_spec.shape
        if mel_spec.dim() == 2:
            mel4 = mel_spec[None, None]
        elif mel_spec.dim() == 3:
            mel4 = mel_spec.unsqueeze(1)          # [B, F, T] -> [B, 1, F, T] (SURVEY 2 note A)
        else:
            mel4 = mel_spec
        ctx = avc_native.pm_context_for(self.predictive_model, mel4.device)
        out = ctx.protect(mel4.float(), self.header.header, window_size, future_step,
                          epsilon1, epsilon2, epsilon3)
        return out.reshape(shape)

    def protect_file(self, input_path: str, output_path: str, window_size: int = 100, future_step: int = 10,
                     epsilon1: float = 0.1, epsilon2: float = 0.05, epsilon3: float = 0.08) -> None:
        """vsmask.py:41-80: load (channels averaged), resample to the converter's rate, protect,
        save as a 32-bit float WAV at that rate (torchaudio.save's encoding of a float tensor)."""
        x, rate = data_utils.read_wav(input_path)
        sr = self.converter.sample_rate
        x = data_utils.resample(x, rate, sr)
        waveform = torch.from_numpy(np.ascontiguousarray(x, np.float32))[None].to(self.device)
        protected = self._protect_waveform(waveform, window_size, future_step, epsilon1, epsilon2, epsilon3)
        data_utils.write_wav_float(output_path, protected.cpu().numpy(), sr)
        print(f"protected audio saved to {output_path}")

    def _protect_waveform(self, waveform: torch.Tensor, window_size: int = 100, future_step: int = 10,
                          epsilon1: float = 0.1, epsilon2: float = 0.05, epsilon3: float = 0.08) -> torch.Tensor:
        """vsmask.py:160-213: waveform [1, L] -> log-mel -> header + sliding-window predictions +
        per-band clamp (protect_mel) -> Griffin-Lim waveform [1, hop * (Tf - 1)]."""
        mel = self.converter.waveform_to_mel(waveform)            # [1, F, Tf]
        protected = self.protect_mel(mel.unsqueeze(1), window_size, future_step, epsilon1, epsilon2, epsilon3)
        return self.converter.mel_to_waveform(protected[:, 0])[0]

    def protect_stream(self, input_stream, output_stream, window_size: int = 100, future_step: int = 10,
                       epsilon1: float = 0.1, epsilon2: float = 0.05, epsilon3: float = 0.08) -> None:
        """vsmask.py:82-158: `input_stream.read(window_size)` yields sample chunks until an empty
        one.  The first chunk gets the header added to its log-mel (frames [0, min(T, Th)), no
        clamp) and is resynthesised; every later chunk joins a buffer of at most
        window_size // len(chunk) chunks (oldest dropped first), whose log-mel the PredictiveModel
        predicts on (so a chunk must span a window the model takes: 25344 samples = 100 frames),
        the prediction added from frame future_step, the difference band-clamped, and the last
        len(chunk) samples of the resynthesis are written: `output_stream.write([1, n] array)`."""
        buffer = []
        header_applied = False
        hdr = self.header.header.detach().float()
        while True:
            audio_chunk = input_stream.read(window_size)
            if audio_chunk is None or len(audio_chunk) == 0:
                break
            chunk = torch.as_tensor(np.asarray(audio_chunk, np.float32)).reshape(1, -1).to(self.device)
            if not header_applied:
                chunk_mel = self.converter.waveform_to_mel(chunk)   # [1, F, Tc]
                hl = min(chunk_mel.shape[-1], hdr.shape[-1])
                rows = min(chunk_mel.shape[1], hdr.shape[-2])
                chunk_mel[:, :rows, :hl] += hdr[0, 0, :rows, :hl]
                protected_chunk = self.converter.mel_to_waveform(chunk_mel)[0]
                header_applied = True
            else:
                buffer.append(chunk)
                if len(buffer) > window_size // chunk.shape[1]:
                    buffer.pop(0)
                window = torch.cat(buffer, dim=1)
                window_mel = self.converter.waveform_to_mel(window)  # [1, F, Tw]
                with torch.no_grad():
                    perturbation = self.predictive_model(window_mel.unsqueeze(1))
                future_mel = window_mel.clone()
                future_end = min(future_step + perturbation.shape[-1], future_mel.shape[-1])
                rows = min(future_mel.shape[1], perturbation.shape[-2])
                if future_end > future_step:
                    future_mel[:, :rows, future_step:future_end] += perturbation[:, 0, :rows, :future_end - future_step]
                weighted = self.converter.apply_weighted_constraint(future_mel - window_mel, epsilon1, epsilon2,
                                                                    epsilon3)
                future_wave = self.converter.mel_to_waveform(window_mel + weighted)[0]
                protected_chunk = future_wave[:, -chunk.shape[1]:]
            output_stream.write(protected_chunk.cpu().numpy())


def main(argv=None):
    """vsmask.py:215-264 arguments: --input / --output audio files (protect_file); .npy paths
    are log-mels [F,T], [1,F,T] or [B,1,F,T] (protect_mel)."""
    p = argparse.ArgumentParser(description="VSMask protection on MI355X")
    p.add_argument("--predictive_model", type=str, required=True)
    p.add_argument("--header", type=str, required=True)
    p.add_argument("--input", type=str, required=True, help="audio file (.wav), or a log-mel .npy")
    p.add_argument("--output", type=str, required=True)
    p.add_argument("--window_size", type=int, default=100)
    p.add_argument("--future_step", type=int, default=10)
    p.add_argument("--epsilon1", type=float, default=0.1)
    p.add_argument("--epsilon2", type=float, default=0.05)
    p.add_argument("--epsilon3", type=float, default=0.08)
    p.add_argument("--device", type=str, default="cuda")
    a = p.parse_args(argv)
    vs = VSMask(a.predictive_model, a.header, device=a.device)
    if a.input.endswith(".npy"):
        mel = torch.from_numpy(np.load(a.input).astype(np.float32)).to(vs.device)
        out = vs.protect_mel(mel, a.window_size, a.future_step, a.epsilon1, a.epsilon2, a.epsilon3)
        np.save(a.output, out.cpu().numpy())
    else:
        vs.protect_file(a.input, a.output, a.window_size, a.future_step, a.epsilon1, a.epsilon2, a.epsilon3)


if __name__ == "__main__":
    main()
