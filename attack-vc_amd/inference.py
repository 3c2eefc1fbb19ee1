"""Drop-in replacement for /root/reference/inference.py (inference.py:9-60) on MI355X.

Same positional arguments as the reference:

  python inference.py MODEL_DIR SOURCE TARGET OUTPUT

Plain voice conversion: the content of SOURCE in the voice of TARGET.  The wav -> mel
front end, AdaInVC.inference (ContentEncoder -> SpeakerEncoder -> AdaIN Decoder,
models.py:472-489) and the Griffin-Lim back end all run in libavc's HIP kernels; SOURCE
and TARGET may have any (different) lengths -- the output has SOURCE's frames, as in the
reference.  The output is written as 16-bit PCM WAV like soundfile's default.
"""
import argparse

import torch

from data_utils import denormalize, file2mel, load_model, mel2wav, normalize, write_wav


def main(model_dir: str, source: str, target: str, output: str):
    """inference.py:9-47."""
    model, config, attr, device = load_model(model_dir)

    src_mel = file2mel(source, **config["preprocess"])
    tgt_mel = file2mel(target, **config["preprocess"])
    src_mel = normalize(src_mel, attr)
    tgt_mel = normalize(tgt_mel, attr)
    src_mel = torch.from_numpy(src_mel).float().T.unsqueeze(0).to(device)
    tgt_mel = torch.from_numpy(tgt_mel).float().T.unsqueeze(0).to(device)

    with torch.no_grad():
        out_mel = model.inference(src_mel, tgt_mel)
        out_mel = out_mel.squeeze(0).T

    out_mel = denormalize(out_mel.data.cpu().numpy(), attr)
    out_wav = mel2wav(out_mel, **config["preprocess"])
    write_wav(output, out_wav, config["preprocess"]["sample_rate"])


def build_parser() -> argparse.ArgumentParser:
    """inference.py:50-59."""
    p = argparse.ArgumentParser()
    p.add_argument("model_dir", type=str, help="The directory of model files.")
    p.add_argument("source", type=str, help="The source utterance providing linguistic content.")
    p.add_argument("target", type=str, help="The target utterance providing vocal timbre.")
    p.add_argument("output", type=str, help="The output converted utterance.")
    return p


if __name__ == "__main__":
    main(**vars(build_parser().parse_args()))
