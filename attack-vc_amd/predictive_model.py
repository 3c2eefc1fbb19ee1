"""VSMask PredictiveModel (/root/reference/models/predictive_model.py:6-110) with the
reference's module tree -- identical parameter names, shapes and registration order, so
a reference state_dict loads unchanged and ``torch.manual_seed(s); PredictiveModel()``
draws the reference's default-init weights -- whose forward runs on the MI355X through
libavc's HIP kernels (csrc/avc_pm.hip), eval-mode semantics (BatchNorm running
statistics), no autograd.
"""
import weakref
from typing import Tuple

import torch
import torch.nn as nn


class _Block:
    """A block's forward runs on libavc through the PredictiveModel it belongs to (its weights are
    uploaded with the whole network's): weak back-reference + its layer index."""

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        ref = self.__dict__.get("_avc_parent")
        m = ref() if ref is not None else None
        if m is None:
            raise RuntimeError(f"{type(self).__name__}.forward runs on libavc through the PredictiveModel it belongs "
                               "to; build it inside PredictiveModel")
        from avc_native import pm_context_for
        return pm_context_for(m, x.device).block_forward(self.__dict__["_avc_layer"], x.float())

    def __getstate__(self):
        st = self.__dict__.copy()
        st.pop("_avc_parent", None)
        return st


class DownSamplingBlock(_Block, nn.Module):
    """predictive_model.py:6-29: ReflectionPad2d -> Conv2d -> BatchNorm2d -> PReLU (eval semantics)."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: Tuple[int, int], stride: Tuple[int, int]):
        super().__init__()
        self.conv = nn.Sequential(
            nn.ReflectionPad2d((kernel_size[0] // 2, kernel_size[0] // 2, kernel_size[1] // 2, kernel_size[1] // 2)),
            nn.Conv2d(in_channels, out_channels, kernel_size, stride),
            nn.BatchNorm2d(out_channels),
            nn.PReLU())


class UpSamplingBlock(_Block, nn.Module):
    """predictive_model.py:31-51: ConvTranspose2d -> LeakyReLU(0.2)."""

    def __init__(self, in_channels: int, out_channels: int, kernel_size: Tuple[int, int], stride: Tuple[int, int]):
        super().__init__()
        self.conv_transpose = nn.Sequential(nn.ConvTranspose2d(in_channels, out_channels, kernel_size, stride),
                                            nn.LeakyReLU(0.2))


class PredictiveModel(nn.Module):
    """predictive_model.py:53-110.  forward(x [B,1,F,T]) -> [B,1,F',T'] on libavc."""

    def __init__(self, mel_bins: int = 80, time_dim: int = 100):
        super().__init__()
        self.down_blocks = nn.ModuleList([
            DownSamplingBlock(1, 32, (3, 3), (1, 2)),
            DownSamplingBlock(32, 64, (3, 3), (2, 2)),
            DownSamplingBlock(64, 128, (3, 3), (2, 2)),
            DownSamplingBlock(128, 256, (3, 3), (2, 2)),
            DownSamplingBlock(256, 256, (3, 3), (2, 2)),
            DownSamplingBlock(256, 512, (3, 3), (2, 2)),
            DownSamplingBlock(512, 512, (3, 3), (2, 2))])
        self.up_blocks = nn.ModuleList([
            UpSamplingBlock(512, 256, (3, 3), (2, 2)),
            UpSamplingBlock(256, 128, (3, 3), (2, 2)),
            UpSamplingBlock(128, 64, (3, 3), (2, 2)),
            UpSamplingBlock(64, 32, (3, 3), (2, 2)),
            UpSamplingBlock(32, 1, (3, 3), (2, 2))])
        self.tanh = nn.Tanh()
        self._avc_link()

    def _avc_link(self):
        for i, blk in enumerate(list(self.down_blocks) + list(self.up_blocks)):
            object.__setattr__(blk, "_avc_parent", weakref.ref(self))
            object.__setattr__(blk, "_avc_layer", i)

    def __setstate__(self, state):
        super().__setstate__(state)
        self._avc_link()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        from avc_native import predictive_forward
        return predictive_forward(self, x)
