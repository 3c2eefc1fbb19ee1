"""CPU oracle: numpy restatement of the VSMask PredictiveModel forward (eval mode).

TEST INFRASTRUCTURE ONLY (tests/, bench.py's cpu_baseline leg); the product never
imports it.  Pinned against tests/golden/predictive.npz, made by the real reference
(tests/golden/make_predictive.py).

Follows /root/reference/models/predictive_model.py: DownSamplingBlock 6-29
(ReflectionPad2d(1) -> Conv2d 3x3 stride s -> BatchNorm2d (eval: running stats,
eps 1e-5) -> PReLU), UpSamplingBlock 31-51 (ConvTranspose2d 3x3 stride 2 ->
LeakyReLU(0.2)), PredictiveModel.forward 87-110 (7 down, 5 up, tanh).
"""
import numpy as np
from numpy.lib.stride_tricks import sliding_window_view

DOWN = [(1, 32, (1, 2)), (32, 64, (2, 2)), (64, 128, (2, 2)), (128, 256, (2, 2)), (256, 256, (2, 2)),
        (256, 512, (2, 2)), (512, 512, (2, 2))]
UP = [(512, 256), (256, 128), (128, 64), (64, 32), (32, 1)]


def conv2d_reflect(x, W, b, stride):
    """ReflectionPad2d(1) + Conv2d(3x3, stride): x [B,Ci,H,W], W [Co,Ci,3,3]."""
    xp = np.pad(x, ((0, 0), (0, 0), (1, 1), (1, 1)), mode="reflect")
    win = sliding_window_view(xp, (3, 3), axis=(2, 3))[:, :, ::stride[0], ::stride[1]]   # [B,Ci,Ho,Wo,3,3]
    B, Ci, Ho, Wo = win.shape[:4]
    cols = win.transpose(0, 2, 3, 1, 4, 5).reshape(B, Ho, Wo, Ci * 9)
    y = cols @ W.reshape(W.shape[0], -1).T                                                 # [B,Ho,Wo,Co]
    return y.transpose(0, 3, 1, 2) + b[None, :, None, None]


def conv_transpose2d(x, W, b):
    """ConvTranspose2d(3x3, stride 2, no padding): x [B,Ci,H,W], W [Ci,Co,3,3]."""
    B, Ci, H, Wd = x.shape
    Co = W.shape[1]
    y = np.zeros((B, Co, 2 * (H - 1) + 3, 2 * (Wd - 1) + 3), dtype=x.dtype)
    for ky in range(3):
        for kx in range(3):
            contrib = np.einsum("bchw,co->bohw", x, W[:, :, ky, kx])
            y[:, :, ky:ky + 2 * H - 1:2, kx:kx + 2 * Wd - 1:2] += contrib
    return y + b[None, :, None, None]


def forward(sd, x, eps=1e-5):
    """PredictiveModel.forward (predictive_model.py:87-110), eval mode; sd = state_dict (numpy)."""
    x = np.asarray(x)
    ft = x.dtype.type
    for i, (_, _, s) in enumerate(DOWN):
        p = f"down_blocks.{i}.conv."
        y = conv2d_reflect(x, sd[p + "1.weight"], sd[p + "1.bias"], s)
        scale = sd[p + "2.weight"] / np.sqrt(sd[p + "2.running_var"] + ft(eps))
        y = (y - sd[p + "2.running_mean"][None, :, None, None]) * scale[None, :, None, None] \
            + sd[p + "2.bias"][None, :, None, None]
        a = sd[p + "3.weight"][0]
        x = np.where(y >= 0, y, a * y)                                  # PReLU (one parameter)
    for i in range(len(UP)):
        p = f"up_blocks.{i}.conv_transpose.0."
        y = conv_transpose2d(x, sd[p + "weight"], sd[p + "bias"])
        x = np.where(y >= 0, y, ft(0.2) * y)                            # LeakyReLU(0.2)
    return np.tanh(x)
