"""ctypes binding of libavc (include/avc.h) — the only way this package computes.

There is deliberately no CPU or ATen fallback: if libavc.so is missing, or the
tensors are not on a ROCm device, every entry point raises.  The reference
(/root/reference/attack_utils.py, models.py) has no FFI of its own; this is the
binding INTEGRATION.md shows a maintainer adding to it.
"""
import ctypes
import os
import threading
import weakref
from typing import Dict, Optional, Tuple

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
# (AVC_LIB_PATH: another libavc build, for A/B timing of kernel variants)
LIB_PATH = os.environ.get("AVC_LIB_PATH") or os.path.join(_HERE, "libavc.so")
MAX_BLOCKS = 16

PREC = {"fp32": 0, "bf16": 1}
REDUCE = {"independent": 0, "mean": 1}
ENGINE = {"auto": 0, "layered": 1, "fused": 2, "long": 3}


class SECfg(ctypes.Structure):
    _fields_ = [("c_in", ctypes.c_int32), ("c_h", ctypes.c_int32), ("c_out", ctypes.c_int32),
                ("kernel_size", ctypes.c_int32), ("bank_size", ctypes.c_int32),
                ("bank_scale", ctypes.c_int32), ("c_bank", ctypes.c_int32),
                ("n_conv_blocks", ctypes.c_int32), ("n_dense_blocks", ctypes.c_int32),
                ("subsample", ctypes.c_int32 * MAX_BLOCKS), ("act", ctypes.c_int32)]


class VCCfg(ctypes.Structure):
    _fields_ = [("ce_c_in", ctypes.c_int32), ("ce_c_h", ctypes.c_int32), ("ce_c_out", ctypes.c_int32),
                ("ce_kernel_size", ctypes.c_int32), ("ce_bank_size", ctypes.c_int32),
                ("ce_bank_scale", ctypes.c_int32), ("ce_c_bank", ctypes.c_int32),
                ("ce_n_conv_blocks", ctypes.c_int32), ("ce_subsample", ctypes.c_int32 * MAX_BLOCKS),
                ("ce_act", ctypes.c_int32),
                ("dec_c_in", ctypes.c_int32), ("dec_c_cond", ctypes.c_int32), ("dec_c_h", ctypes.c_int32),
                ("dec_c_out", ctypes.c_int32), ("dec_kernel_size", ctypes.c_int32),
                ("dec_n_conv_blocks", ctypes.c_int32), ("dec_upsample", ctypes.c_int32 * MAX_BLOCKS),
                ("dec_act", ctypes.c_int32), ("dec_sn", ctypes.c_int32)]


class AttackOpts(ctypes.Structure):
    _fields_ = [("precision", ctypes.c_int32), ("reduction", ctypes.c_int32),
                ("use_graph", ctypes.c_int32), ("losses", ctypes.c_void_p),
                ("grad0", ctypes.c_void_p), ("update", ctypes.c_int32), ("pgd_step", ctypes.c_float)]


UPDATE = {"adam": 0, "pgd": 1}


class DspCfg(ctypes.Structure):
    _fields_ = [("sample_rate", ctypes.c_int32), ("n_fft", ctypes.c_int32), ("hop_length", ctypes.c_int32),
                ("win_length", ctypes.c_int32), ("n_mels", ctypes.c_int32), ("preemph", ctypes.c_float),
                ("ref_db", ctypes.c_float), ("max_db", ctypes.c_float), ("pad_mode", ctypes.c_int32),
                ("flavor", ctypes.c_int32)]


PAD_MODE = {"reflect": 0, "constant": 1}

_lib = None
_lib_lock = threading.Lock()

# (name, restype, argtypes) of every symbol include/avc.h declares
SIGNATURES = [
    ("avc_se_weight_count", ctypes.c_size_t, [ctypes.POINTER(SECfg)]),
    ("avc_create", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(SECfg), ctypes.c_void_p, ctypes.c_size_t,
                                  ctypes.POINTER(ctypes.c_void_p)]),
    ("avc_destroy", None, [ctypes.c_void_p]),
    ("avc_se_forward", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.c_void_p]),
    ("avc_emb_attack", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.POINTER(AttackOpts), ctypes.c_void_p]),
    ("avc_emb_attack_emb", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int,
                                          ctypes.c_void_p, ctypes.POINTER(AttackOpts), ctypes.c_void_p]),
    ("avc_emb_attack_ragged", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                             ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_float,
                                             ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(AttackOpts),
                                             ctypes.c_void_p]),
    ("avc_header_optimize", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_void_p, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                           ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_void_p, ctypes.c_void_p]),
    ("avc_header_optimize_state", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                                 ctypes.c_int, ctypes.c_void_p, ctypes.c_float, ctypes.c_float,
                                                 ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                                 ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    ("avc_vc_weight_count", ctypes.c_size_t, [ctypes.POINTER(VCCfg)]),
    ("avc_attach_vc", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(VCCfg), ctypes.c_void_p, ctypes.c_size_t]),
    ("avc_vc_out_frames", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    ("avc_sn_state_count", ctypes.c_size_t, [ctypes.c_void_p]),
    ("avc_set_sn_state", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
    ("avc_get_sn_state", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
    ("avc_sn_state_dev", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int,
                                         ctypes.c_void_p]),
    ("avc_set_sn_train", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]),
    ("avc_content_encoder", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("avc_content_frames", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    ("avc_decoder", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                   ctypes.c_void_p, ctypes.c_void_p]),
    ("avc_inference", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_void_p, ctypes.c_void_p]),
    ("avc_inference_emb", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("avc_e2e_attack_emb", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                          ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(AttackOpts), ctypes.c_void_p]),
    ("avc_fb_attack_emb", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                         ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                         ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(AttackOpts), ctypes.c_void_p]),
    ("avc_e2e_attack", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                      ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.POINTER(AttackOpts), ctypes.c_void_p]),
    ("avc_fb_attack", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_int,
                                     ctypes.c_void_p, ctypes.POINTER(AttackOpts), ctypes.c_void_p]),
    ("avc_pm_weight_count", ctypes.c_size_t, []),
    ("avc_pm_create", ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]),
    ("avc_pm_destroy", None, [ctypes.c_void_p]),
    ("avc_pm_out_shape", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                        ctypes.POINTER(ctypes.c_int)]),
    ("avc_pm_forward", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                      ctypes.c_void_p, ctypes.c_void_p]),
    ("avc_pm_block_shape", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                          ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    ("avc_pm_block_forward", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    ("avc_vsmask_windows", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
    ("avc_vsmask_protect", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                          ctypes.c_float, ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p]),
    ("avc_vsmask_apply_header", ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                               ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    ("avc_dsp_create", ctypes.c_int, [ctypes.c_int, ctypes.POINTER(DspCfg), ctypes.POINTER(ctypes.c_void_p)]),
    ("avc_dsp_destroy", None, [ctypes.c_void_p]),
    ("avc_dsp_frames", ctypes.c_int, [ctypes.POINTER(DspCfg), ctypes.c_int]),
    ("avc_dsp_mel_basis", ctypes.c_int, [ctypes.POINTER(DspCfg), ctypes.c_void_p, ctypes.c_void_p]),
    ("avc_dsp_wav2mel", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                       ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]),
    ("avc_dsp_mel2wav", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                       ctypes.c_void_p]),
    ("avc_dsp_griffin_lim", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                           ctypes.c_void_p, ctypes.c_void_p]),
    ("avc_dsp_ta_mel2wav", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.c_float, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("avc_vsmask_band_clamp", ctypes.c_int, [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_void_p,
                                             ctypes.c_void_p]),
    ("avc_dsp_set_profiling", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    ("avc_dsp_profile_count", ctypes.c_int, [ctypes.c_void_p]),
    ("avc_dsp_profile_kernel", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                              ctypes.POINTER(ctypes.c_long), ctypes.POINTER(ctypes.c_double)]),
    ("avc_set_engine", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    ("avc_get_engine", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    ("avc_set_profiling", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    ("avc_get_profile", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                       ctypes.POINTER(ctypes.c_double)]),
    ("avc_profile_kernel_count", ctypes.c_int, [ctypes.c_void_p]),
    ("avc_profile_kernel", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_long), ctypes.POINTER(ctypes.c_double),
                                          ctypes.POINTER(ctypes.c_double)]),
    ("avc_ktime", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                 ctypes.POINTER(ctypes.c_int64)]),
    ("avc_ws_stats", ctypes.c_int, [ctypes.c_void_p] + [ctypes.POINTER(ctypes.c_int64)] * 5),
    ("avc_set_ws_cache", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]),
    ("avc_last_error", ctypes.c_char_p, []),
    ("avc_version", ctypes.c_char_p, []),
]


def lib():
    """Load libavc.so (built in-tree by __graft_entry__.build()); raise if absent."""
    global _lib
    with _lib_lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(f"libavc.so not found at {LIB_PATH}; build it with "
                                   "`python -c 'import __graft_entry__ as g; g.build()'`")
            L = ctypes.CDLL(LIB_PATH)
            for name, res, args in SIGNATURES:
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


def _check(rc: int):
    if rc != 0:
        raise RuntimeError(lib().avc_last_error().decode(errors="replace"))


def _require_gpu(*ts: torch.Tensor):
    for t in ts:
        if not t.is_cuda:
            raise RuntimeError("libavc runs on MI355X (ROCm) devices only; got a tensor on " + str(t.device))
        if t.dtype != torch.float32:
            raise RuntimeError(f"libavc expects float32 tensors, got {t.dtype}")


def se_cfg_struct(cfg: Dict) -> SECfg:
    s = SECfg()
    for k in ("c_in", "c_h", "c_out", "kernel_size", "bank_size", "bank_scale", "c_bank",
              "n_conv_blocks", "n_dense_blocks", "act"):
        setattr(s, k, int(cfg[k]))
    sub = list(cfg["subsample"])[: int(cfg["n_conv_blocks"])]
    if len(sub) > MAX_BLOCKS:
        raise RuntimeError(f"at most {MAX_BLOCKS} conv blocks supported")
    for i, v in enumerate(sub):
        s.subsample[i] = int(v)
    return s


class Context:
    """One libavc context (packed weights + workspace) per (module, device)."""

    def __init__(self, cfg: Dict, flat_weights: torch.Tensor, device: int):
        self.cfg = dict(cfg)
        self._cs = se_cfg_struct(cfg)
        w = flat_weights.detach().to("cpu", torch.float32).contiguous()
        need = lib().avc_se_weight_count(ctypes.byref(self._cs))
        if w.numel() != need:
            raise RuntimeError(f"weights: got {w.numel()} values, config needs {need}")
        h = ctypes.c_void_p()
        _check(lib().avc_create(int(device), ctypes.byref(self._cs), ctypes.c_void_p(w.data_ptr()),
                                w.numel(), ctypes.byref(h)))
        self.h = h
        self.device = device
        self._lock = threading.Lock()

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value and _lib is not None:
            _lib.avc_destroy(h)
            self.h = None

    def se_forward(self, x: torch.Tensor) -> torch.Tensor:
        _require_gpu(x)
        x = x.contiguous()
        B, C, T = x.shape
        emb = torch.empty(B, self.cfg["c_out"], device=x.device, dtype=torch.float32)
        stream = torch.cuda.current_stream(x.device).cuda_stream
        with self._lock:
            _check(lib().avc_se_forward(self.h, ctypes.c_void_p(x.data_ptr()), B, T,
                                        ctypes.c_void_p(emb.data_ptr()), ctypes.c_void_p(stream)))
        return emb

    @staticmethod
    def _check_mel(name: str, t: torch.Tensor, c_in: int, B: int = None):
        if t.dim() != 3 or t.shape[1] != c_in:
            raise RuntimeError(f"{name}: expected [B, {c_in}, T], got {tuple(t.shape)}")
        if B is not None and t.shape[0] != B:
            raise RuntimeError(f"{name}: batch {t.shape[0]} != {B}")

    def _opts(self, precision, reduction, use_graph, n_iters, like, want_losses, want_grad0, update="adam",
              pgd_step=1e-3):
        B = like.shape[0]
        if update not in UPDATE:
            raise RuntimeError(f"update must be one of {sorted(UPDATE)}")
        losses = torch.empty(n_iters, B, device=like.device) if want_losses and n_iters > 0 else None
        grad0 = torch.empty_like(like) if want_grad0 and n_iters > 0 else None
        o = AttackOpts(PREC[precision], REDUCE[reduction], 1 if use_graph else 0,
                       losses.data_ptr() if losses is not None else None,
                       grad0.data_ptr() if grad0 is not None else None, UPDATE[update], float(pgd_step))
        return o, losses, grad0

    def _tgt_emb(self, tgt_emb, B):
        _require_gpu(tgt_emb)
        if tuple(tgt_emb.shape) != (B, self.cfg["c_out"]):
            raise RuntimeError(f"tgt_emb: expected [{B}, {self.cfg['c_out']}], got {tuple(tgt_emb.shape)}")
        return tgt_emb.contiguous()

    def emb_attack(self, vc_tgt, adv_tgt, ptb0, eps: float, n_iters: int, precision="fp32",
                   reduction="independent", use_graph=True, want_losses=False, want_grad0=False, update="adam",
                   pgd_step=1e-3, tgt_emb=None):
        """avc_emb_attack; an adv_tgt of another length than vc_tgt is embedded on its own first
        (the reference embeds it separately, attack_utils.py:74-75) -> avc_emb_attack_emb.
        tgt_emb [B, c_out] (= SpeakerEncoder(adv_tgt), computed by the caller) replaces adv_tgt."""
        _require_gpu(vc_tgt, ptb0)
        vc_tgt, ptb0 = vc_tgt.contiguous(), ptb0.contiguous()
        c_in = self.cfg["c_in"]
        self._check_mel("vc_tgt", vc_tgt, c_in)
        B, C, T = vc_tgt.shape
        if tgt_emb is None:
            _require_gpu(adv_tgt)
            adv_tgt = adv_tgt.contiguous()
            self._check_mel("adv_tgt", adv_tgt, c_in, B)
        if ptb0.shape != vc_tgt.shape:
            raise RuntimeError(f"shape mismatch: vc_tgt {tuple(vc_tgt.shape)}, ptb0 {tuple(ptb0.shape)}")
        out = torch.empty_like(vc_tgt)
        o, losses, grad0 = self._opts(precision, reduction, use_graph, n_iters, vc_tgt, want_losses, want_grad0,
                                      update, pgd_step)
        stream = torch.cuda.current_stream(vc_tgt.device).cuda_stream
        if tgt_emb is not None:
            tgt_emb = self._tgt_emb(tgt_emb, B)
        elif adv_tgt.shape != vc_tgt.shape:
            tgt_emb = self.se_forward(adv_tgt)
        with self._lock:
            if tgt_emb is None:
                _check(lib().avc_emb_attack(self.h, ctypes.c_void_p(vc_tgt.data_ptr()),
                                            ctypes.c_void_p(adv_tgt.data_ptr()), ctypes.c_void_p(ptb0.data_ptr()),
                                            B, T, float(eps), int(n_iters), ctypes.c_void_p(out.data_ptr()),
                                            ctypes.byref(o), ctypes.c_void_p(stream)))
            else:
                _check(lib().avc_emb_attack_emb(self.h, ctypes.c_void_p(vc_tgt.data_ptr()),
                                                ctypes.c_void_p(tgt_emb.data_ptr()), ctypes.c_void_p(ptb0.data_ptr()),
                                                B, T, float(eps), int(n_iters), ctypes.c_void_p(out.data_ptr()),
                                                ctypes.byref(o), ctypes.c_void_p(stream)))
        return out, losses, grad0

    def emb_attack_ragged(self, vc_tgts, tgt_emb, ptb0s, eps: float, n_iters: int, precision="fp32",
                          use_graph=True, want_losses=False, want_grad0=False, update="adam", pgd_step=1e-3):
        """avc_emb_attack_ragged: ONE batch of utterances of different lengths (vc_tgts[b] [80, T_b], ptb0s[b]
        likewise; tgt_emb [B, c_out] = SpeakerEncoder(adv_tgt_b), each embedded at its own length) -- every
        pass is one launch over all of them (the long engine with per-workgroup lengths).  Returns
        (adv list [80, T_b], losses [n_iters, B] or None, grad0 list or None)."""
        B = len(vc_tgts)
        if B == 0 or len(ptb0s) != B:
            raise RuntimeError("emb_attack_ragged: one ptb0 per utterance, at least one utterance")
        c_in = self.cfg["c_in"]
        for name, ts in (("vc_tgt", vc_tgts), ("ptb0", ptb0s)):
            for b, t in enumerate(ts):
                _require_gpu(t)
                if t.dim() != 2 or t.shape[0] != c_in:
                    raise RuntimeError(f"{name}[{b}]: expected [{c_in}, T], got {tuple(t.shape)}")
        lens = [int(t.shape[1]) for t in vc_tgts]
        if [int(t.shape[1]) for t in ptb0s] != lens:
            raise RuntimeError("emb_attack_ragged: ptb0 lengths differ from vc_tgt lengths")
        dev = vc_tgts[0].device
        vc = torch.cat([t.reshape(-1).float() for t in vc_tgts]).contiguous()
        p0 = torch.cat([t.reshape(-1).float() for t in ptb0s]).to(dev).contiguous()
        tgt_emb = self._tgt_emb(tgt_emb, B)
        out = torch.empty_like(vc)
        o, losses, g0 = self._opts(precision, "independent", use_graph, n_iters, torch.empty(B, 1, device=dev),
                                   want_losses, False, update, pgd_step)
        grad0 = torch.empty_like(vc) if want_grad0 and n_iters > 0 else None
        if grad0 is not None:
            o.grad0 = grad0.data_ptr()
        arr = (ctypes.c_int * B)(*lens)
        stream = torch.cuda.current_stream(dev).cuda_stream
        with self._lock:
            _check(lib().avc_emb_attack_ragged(self.h, ctypes.c_void_p(vc.data_ptr()), arr, B,
                                               ctypes.c_void_p(tgt_emb.data_ptr()), ctypes.c_void_p(p0.data_ptr()),
                                               float(eps), int(n_iters), ctypes.c_void_p(out.data_ptr()),
                                               ctypes.byref(o), ctypes.c_void_p(stream)))
        def split(x):
            res, off = [], 0
            for T in lens:
                res.append(x[off:off + c_in * T].view(c_in, T))
                off += c_in * T
            return res
        return split(out), losses, (split(grad0) if grad0 is not None else None)

    def header_optimize(self, source, target, header, n_iters: int, epsilon=0.1, lambda_param=0.5, lr=1e-3,
                        betas=(0.9, 0.999), adam_eps=1e-8, precision="fp32", adam_state=None):
        """avc_header_optimize (UniversalPerturbationHeader.optimize, header_model.py:25-68):
        source / target [N, 80, T], header [80, T] -> (new header [80, T], losses [n_iters, N]).
        adam_state = (exp_avg [80, T], exp_avg_sq [80, T], step) continues an optimiser: the two
        moment tensors are updated in place and the caller advances its step by n_iters
        (avc_header_optimize_state)."""
        _require_gpu(source, target, header)
        source, target = source.contiguous(), target.contiguous()
        c_in = self.cfg["c_in"]
        self._check_mel("source", source, c_in)
        N, _, T = source.shape
        self._check_mel("target", target, c_in, N)
        if target.shape != source.shape:
            raise RuntimeError(f"shape mismatch: source {tuple(source.shape)}, target {tuple(target.shape)}")
        if tuple(header.shape) != (c_in, T):
            raise RuntimeError(f"header {tuple(header.shape)} does not broadcast onto mels {tuple(source.shape)}")
        if precision not in PREC:
            raise RuntimeError(f"precision must be one of {list(PREC)}")
        hdr = header.detach().clone().contiguous()
        losses = torch.empty(max(int(n_iters), 1), N, device=source.device, dtype=torch.float32)
        stream = torch.cuda.current_stream(source.device).cuda_stream
        m = v = None
        step0 = 0
        if adam_state is not None:
            m, v, step0 = adam_state
            _require_gpu(m, v)
            if tuple(m.shape) != (c_in, T) or tuple(v.shape) != (c_in, T) or not (m.is_contiguous() and v.is_contiguous()):
                raise RuntimeError(f"Adam state must be contiguous [{c_in}, {T}] tensors")
        with self._lock:
            _check(lib().avc_header_optimize_state(
                self.h, ctypes.c_void_p(source.data_ptr()), ctypes.c_void_p(target.data_ptr()), N, T,
                ctypes.c_void_p(hdr.data_ptr()), float(epsilon), float(lambda_param), float(lr), float(betas[0]),
                float(betas[1]), float(adam_eps), int(n_iters), PREC[precision], ctypes.c_void_p(losses.data_ptr()),
                ctypes.c_void_p(m.data_ptr() if m is not None else 0), ctypes.c_void_p(v.data_ptr() if v is not None else 0),
                int(step0), ctypes.c_void_p(stream)))
        return hdr, losses[:n_iters]

    # --- voice-conversion path (ContentEncoder + Decoder) ----------------------------
    def attach_vc(self, ce_cfg: Dict, dec_cfg: Dict, flat: torch.Tensor):
        """Hand the ContentEncoder / Decoder weights (content_encoder.* then decoder.*,
        state_dict order) to libavc (avc_attach_vc)."""
        self._vcs = vc_cfg_struct(ce_cfg, dec_cfg)
        w = flat.detach().to("cpu", torch.float32).contiguous()
        need = lib().avc_vc_weight_count(ctypes.byref(self._vcs))
        if w.numel() != need:
            raise RuntimeError(f"ContentEncoder/Decoder weights: got {w.numel()} values, config needs {need}")
        _check(lib().avc_attach_vc(self.h, ctypes.byref(self._vcs), ctypes.c_void_p(w.data_ptr()), w.numel()))

    _sn_dec = None

    def _sn_call(self, fn):
        """Run fn() (a call that runs Decoder forwards) with a spectral-norm Decoder's u / v loaded
        from its module buffers, under the hook mode the module's .training selects (torch's
        spectral_norm compute_weight, models.py:382):
          train: one power iteration per Decoder forward, the buffers written back afterwards (the
                 reference never calls .eval(), so its attacks run this mode);
          eval : sigma = u . (W v) from the stored u / v, the buffers left as they are.
        Device buffers are copied device-to-device on the caller's stream (no host round trip)."""
        dec = self._sn_dec() if self._sn_dec is not None else None
        if dec is None:
            return fn()
        bufs = _sn_buffers(dec)
        n = lib().avc_sn_state_count(self.h)
        train = bool(dec.training)
        on_dev = all(b.is_cuda for b in bufs)
        dev = bufs[0].device if on_dev else torch.device("cuda", torch.cuda.current_device())
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        with torch.no_grad():
            uv = torch.cat([b.detach().reshape(-1).to(dev, torch.float32) for b in bufs]).contiguous()
        if uv.numel() != n:
            raise RuntimeError(f"spectral-norm state: module holds {uv.numel()} u / v values, libavc expects {n}")
        _check(lib().avc_set_sn_train(self.h, int(train), stream))
        _check(lib().avc_sn_state_dev(self.h, ctypes.c_void_p(uv.data_ptr()), n, 1, stream))
        out = fn()
        if train:
            _check(lib().avc_sn_state_dev(self.h, ctypes.c_void_p(uv.data_ptr()), n, 0, stream))
            with torch.no_grad():
                o = 0
                for b in bufs:
                    b.copy_(uv[o:o + b.numel()].view_as(b))
                    o += b.numel()
        return out

    def vc_out_frames(self, T: int) -> int:
        n = lib().avc_vc_out_frames(self.h, int(T))
        if n < 0:
            raise RuntimeError(lib().avc_last_error().decode(errors="replace"))
        return n

    def content_encoder(self, x: torch.Tensor):
        """ContentEncoder.forward (models.py:181-210): x [B, 80, T] -> (mu, log_sigma) [B, c_out, Tce]."""
        _require_gpu(x)
        x = x.contiguous()
        self._check_mel("x", x, self.cfg["c_in"])
        B, _, T = x.shape
        n = lib().avc_content_frames(self.h, int(T))
        if n < 0:
            _check(1)
        mu = torch.empty(B, self._vcs.ce_c_out, n, device=x.device)
        ls = torch.empty_like(mu)
        stream = torch.cuda.current_stream(x.device).cuda_stream
        with self._lock:
            _check(lib().avc_content_encoder(self.h, ctypes.c_void_p(x.data_ptr()), B, T, ctypes.c_void_p(mu.data_ptr()),
                                             ctypes.c_void_p(ls.data_ptr()), ctypes.c_void_p(stream)))
        return mu, ls

    def decoder(self, z: torch.Tensor, cond: torch.Tensor) -> torch.Tensor:
        """Decoder.forward (models.py:403-435): z [B, 128, Tz], cond [B, 128] -> [B, 80, Tz * prod(upsample)]."""
        _require_gpu(z, cond)
        z, cond = z.contiguous(), cond.contiguous()
        if z.dim() != 3 or z.shape[1] != self._vcs.dec_c_in:
            raise RuntimeError(f"z: expected [B, {self._vcs.dec_c_in}, T], got {tuple(z.shape)}")
        B, _, Tz = z.shape
        if tuple(cond.shape) != (B, self._vcs.dec_c_cond):
            raise RuntimeError(f"cond: expected [{B}, {self._vcs.dec_c_cond}], got {tuple(cond.shape)}")
        up = 1
        for i in range(self._vcs.dec_n_conv_blocks):
            up *= int(self._vcs.dec_upsample[i])
        out = torch.empty(B, self._vcs.dec_c_out, Tz * up, device=z.device)
        stream = torch.cuda.current_stream(z.device).cuda_stream
        with self._lock:
            self._sn_call(lambda: _check(lib().avc_decoder(
                self.h, ctypes.c_void_p(z.data_ptr()), B, Tz, ctypes.c_void_p(cond.data_ptr()),
                ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(stream))))
        return out

    def inference(self, src: torch.Tensor, tgt: torch.Tensor) -> torch.Tensor:
        """AdaInVC.inference: the output takes src's length (models.py:472-489); a tgt of another
        length is embedded on its own first (avc_inference_emb)."""
        _require_gpu(src, tgt)
        src, tgt = src.contiguous(), tgt.contiguous()
        c_in = self.cfg["c_in"]
        self._check_mel("src", src, c_in)
        B, C, T = src.shape
        self._check_mel("tgt", tgt, c_in, B)
        out = torch.empty(B, 80, self.vc_out_frames(T), device=src.device, dtype=torch.float32)
        stream = torch.cuda.current_stream(src.device).cuda_stream
        emb = self.se_forward(tgt) if tgt.shape != src.shape else None
        def run():
            if emb is None:
                _check(lib().avc_inference(self.h, ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(tgt.data_ptr()),
                                           B, T, ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(stream)))
            else:
                _check(lib().avc_inference_emb(self.h, ctypes.c_void_p(src.data_ptr()), B, T,
                                               ctypes.c_void_p(emb.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                               ctypes.c_void_p(stream)))
        with self._lock:
            self._sn_call(run)
        return out

    def vc_attack(self, kind: str, vc_src, vc_tgt, adv_tgt, ptb0, eps: float, n_iters: int, precision="fp32",
                  reduction="independent", use_graph=True, want_losses=False, want_grad0=False, update="adam",
                  pgd_step=1e-3, tgt_emb=None):
        """kind "e2e" (avc_e2e_attack) or "fb" (avc_fb_attack).  vc_src, vc_tgt and adv_tgt may have
        different lengths (each is loaded from its own wav by attack.py:49-56): then adv_tgt is
        embedded on its own and the *_attack_emb entry points run.  tgt_emb [B, c_out] (=
        SpeakerEncoder(adv_tgt), computed by the caller) replaces adv_tgt."""
        _require_gpu(vc_src, vc_tgt, ptb0)
        vc_src, vc_tgt, ptb0 = (t.contiguous() for t in (vc_src, vc_tgt, ptb0))
        c_in = self.cfg["c_in"]
        self._check_mel("vc_tgt", vc_tgt, c_in)
        B, C, T = vc_tgt.shape
        self._check_mel("vc_src", vc_src, c_in, B)
        if tgt_emb is None:
            _require_gpu(adv_tgt)
            adv_tgt = adv_tgt.contiguous()
            self._check_mel("adv_tgt", adv_tgt, c_in, B)
        if ptb0.shape != vc_tgt.shape:
            raise RuntimeError(f"shape mismatch: vc_tgt {tuple(vc_tgt.shape)}, ptb0 {tuple(ptb0.shape)}")
        Ts = vc_src.shape[2]
        out = torch.empty_like(vc_tgt)
        o, losses, grad0 = self._opts(precision, reduction, use_graph, n_iters, vc_tgt, want_losses, want_grad0,
                                      update, pgd_step)
        stream = torch.cuda.current_stream(vc_tgt.device).cuda_stream
        if tgt_emb is not None:
            same = False
            tgt_emb = self._tgt_emb(tgt_emb, B)
        else:
            same = vc_src.shape == vc_tgt.shape == adv_tgt.shape
            tgt_emb = None if same else self.se_forward(adv_tgt)
        def run():
            if same:
                fn = {"e2e": lib().avc_e2e_attack, "fb": lib().avc_fb_attack}[kind]
                _check(fn(self.h, ctypes.c_void_p(vc_src.data_ptr()), ctypes.c_void_p(vc_tgt.data_ptr()),
                          ctypes.c_void_p(adv_tgt.data_ptr()), ctypes.c_void_p(ptb0.data_ptr()), B, T, float(eps),
                          int(n_iters), ctypes.c_void_p(out.data_ptr()), ctypes.byref(o), ctypes.c_void_p(stream)))
            else:
                fn = {"e2e": lib().avc_e2e_attack_emb, "fb": lib().avc_fb_attack_emb}[kind]
                _check(fn(self.h, ctypes.c_void_p(vc_src.data_ptr()), Ts, ctypes.c_void_p(vc_tgt.data_ptr()),
                          ctypes.c_void_p(tgt_emb.data_ptr()), ctypes.c_void_p(ptb0.data_ptr()), B, T, float(eps),
                          int(n_iters), ctypes.c_void_p(out.data_ptr()), ctypes.byref(o), ctypes.c_void_p(stream)))
        with self._lock:
            self._sn_call(run)
        return out, losses, grad0

    def ws_stats(self) -> Dict[str, int]:
        """avc_ws_stats: workspace builds / replans / hits, graph captures, evictions."""
        v = [ctypes.c_int64() for _ in range(5)]
        _check(lib().avc_ws_stats(self.h, *[ctypes.byref(x) for x in v]))
        return dict(zip(("builds", "replans", "hits", "captures", "evictions"), (x.value for x in v)))

    def set_ws_cache(self, n_shapes: int):
        _check(lib().avc_set_ws_cache(self.h, int(n_shapes)))

    def set_engine(self, engine: str = "auto"):
        """"auto" | "layered" | "fused" | "long" (include/avc.h AVC_ENGINE_*)."""
        _check(lib().avc_set_engine(self.h, ENGINE[engine]))

    def engine_for(self, T: int) -> str:
        return {v: k for k, v in ENGINE.items()}[lib().avc_get_engine(self.h, int(T))]

    # --- profiling (bench.py roofline) ---------------------------------------------
    KTIME_KERNELS = tuple(f"{k}<{p}>" for k in ("se_fwd_fused", "se_bwd_fused", "lz_se_fwd", "lz_se_bwd", "lz_dec_fwd",
                                                 "lz_dec_bwd", "dec_fwd_fused", "dec_bwd_fused", "se_attack_fused")
                         for p in ("f32", "bf16"))

    def ktime_start(self):
        """Start in-graph kernel timing (avc_ktime): device wall-clock stamps in the hot kernels."""
        _check(lib().avc_ktime(self.h, 1, None, None))

    def ktime_stop(self) -> Dict[str, Tuple[int, float]]:
        """Stop in-graph kernel timing: {kernel: (launches, average launch microseconds)} for the
        kernels that ran."""
        us = (ctypes.c_double * 18)()
        n = (ctypes.c_int64 * 18)()
        _check(lib().avc_ktime(self.h, 0, us, n))
        return {k: (int(n[i]), float(us[i])) for i, k in enumerate(self.KTIME_KERNELS) if n[i] > 0}

    def set_profiling(self, on: bool):
        _check(lib().avc_set_profiling(self.h, 1 if on else 0))

    def profile(self) -> Tuple[float, Dict[str, Tuple[int, float, float]]]:
        ms, fl = ctypes.c_double(), ctypes.c_double()
        _check(lib().avc_get_profile(self.h, ctypes.byref(ms), ctypes.byref(fl)))
        self.prof_flop_per_iter = fl.value      # algorithmic FLOPs of one whole-batch iteration
        stats = {}
        for i in range(lib().avc_profile_kernel_count(self.h)):
            name = ctypes.create_string_buffer(128)
            n, t, f = ctypes.c_long(), ctypes.c_double(), ctypes.c_double()
            _check(lib().avc_profile_kernel(self.h, i, name, 128, ctypes.byref(n), ctypes.byref(t),
                                            ctypes.byref(f)))
            stats[name.value.decode()] = (n.value, t.value, f.value)
        return ms.value, stats


_ctx_cache: "weakref.WeakKeyDictionary" = weakref.WeakKeyDictionary()


def flat_weights(se: torch.nn.Module) -> torch.Tensor:
    """Speaker-encoder parameters in state_dict order (the layout avc_create expects)."""
    return torch.cat([v.detach().reshape(-1).to("cpu", torch.float32) for v in se.state_dict().values()])


def se_config(se: torch.nn.Module) -> Dict:
    """Hyper-parameters of a SpeakerEncoder module (ours or the reference's, models.py:213-283)."""
    if hasattr(se, "avc_config"):
        return se.avc_config()
    ks = [m.kernel_size[0] for m in se.conv_bank]
    bank_scale = ks[1] - ks[0] if len(ks) > 1 else ks[0]
    act = 1 if isinstance(se.act, torch.nn.LeakyReLU) else 0
    return dict(c_in=se.conv_bank[0].in_channels, c_h=se.c_h, c_out=se.c_out, kernel_size=se.kernel_size,
                bank_size=ks[-1], bank_scale=bank_scale, c_bank=se.conv_bank[0].out_channels,
                n_conv_blocks=se.n_conv_blocks, n_dense_blocks=se.n_dense_blocks,
                subsample=list(se.subsample), act=act)


def vc_cfg_struct(ce: Dict, dec: Dict) -> VCCfg:
    s = VCCfg()
    for k in ("c_in", "c_h", "c_out", "kernel_size", "bank_size", "bank_scale", "c_bank", "n_conv_blocks", "act"):
        setattr(s, "ce_" + k, int(ce[k]))
    for k in ("c_in", "c_cond", "c_h", "c_out", "kernel_size", "n_conv_blocks", "act"):
        setattr(s, "dec_" + k, int(dec[k]))
    s.dec_sn = int(dec.get("sn", 0))
    sub = list(ce["subsample"])[: int(ce["n_conv_blocks"])]
    ups = list(dec["upsample"])[: int(dec["n_conv_blocks"])]
    if len(sub) > MAX_BLOCKS or len(ups) > MAX_BLOCKS:
        raise RuntimeError(f"at most {MAX_BLOCKS} conv blocks supported")
    for i, v in enumerate(sub):
        s.ce_subsample[i] = int(v)
    for i, v in enumerate(ups):
        s.dec_upsample[i] = int(v)
    return s


def _act_of(mod) -> int:
    return 1 if isinstance(getattr(mod, "act", None), torch.nn.LeakyReLU) else 0


def ce_config(ce: torch.nn.Module) -> Dict:
    """Hyper-parameters of a ContentEncoder (ours or the reference's, models.py:121-179)."""
    if hasattr(ce, "avc_config"):
        return ce.avc_config()
    ks = [m.kernel_size[0] for m in ce.conv_bank]
    return dict(c_in=ce.conv_bank[0].in_channels, c_h=ce.in_conv_layer.out_channels,
                c_out=ce.mean_layer.out_channels, kernel_size=ce.first_conv_layers[0].kernel_size[0],
                bank_size=ks[-1], bank_scale=ks[1] - ks[0] if len(ks) > 1 else ks[0],
                c_bank=ce.conv_bank[0].out_channels, n_conv_blocks=ce.n_conv_blocks,
                subsample=list(ce.subsample), act=_act_of(ce))


def dec_config(dec: torch.nn.Module) -> Dict:
    """Hyper-parameters of a Decoder (ours or the reference's, models.py:346-401)."""
    if hasattr(dec, "avc_config"):
        return dec.avc_config()
    return dict(c_in=dec.in_conv_layer.in_channels, c_cond=dec.conv_affine_layers[0].in_features,
                c_h=dec.in_conv_layer.out_channels, c_out=dec.out_conv_layer.out_channels,
                kernel_size=dec.first_conv_layers[0].kernel_size[0], n_conv_blocks=dec.n_conv_blocks,
                upsample=list(dec.upsample), act=_act_of(dec), sn=int(_dec_has_sn(dec)))


def _dec_layers(dec: torch.nn.Module):
    """The Decoder's Conv1d / Linear layers in module (= state_dict) order (models.py:383-399)."""
    return [dec.in_conv_layer, *dec.first_conv_layers, *dec.second_conv_layers, *dec.conv_affine_layers,
            dec.out_conv_layer]


def _dec_has_sn(dec: torch.nn.Module) -> bool:
    """sn=True (models.py:382): every layer carries torch's spectral_norm (weight_orig / weight_u / weight_v)."""
    return hasattr(dec.in_conv_layer, "weight_orig")


def _dec_flat(dec: torch.nn.Module) -> torch.Tensor:
    """Decoder weights for avc_attach_vc: (weight, bias) per layer in module order -- weight_orig for a
    spectral-normed layer (libavc divides it by the layer's sigma before every Decoder forward)."""
    parts = []
    for m in _dec_layers(dec):
        W = m.weight_orig if hasattr(m, "weight_orig") else m.weight
        parts += [W.detach().reshape(-1).to("cpu", torch.float32), m.bias.detach().reshape(-1).to("cpu", torch.float32)]
    return torch.cat(parts)


def _sn_buffers(dec: torch.nn.Module):
    """weight_u then weight_v of every spectral-normed Decoder layer (avc_set_sn_state's order)."""
    out = []
    for m in _dec_layers(dec):
        out += [m.weight_u, m.weight_v]
    return out


def context_for(se: torch.nn.Module, device: torch.device) -> Context:
    """Cached libavc context for this speaker encoder's current weights on `device`."""
    if device.type != "cuda":
        raise RuntimeError("libavc runs on MI355X (ROCm) devices only; got " + str(device))
    dev = device.index if device.index is not None else torch.cuda.current_device()
    version = tuple((p.data_ptr(), p._version) for p in se.parameters())
    per = _ctx_cache.setdefault(se, {})
    hit = per.get(dev)
    if hit is not None and hit[0] == version:
        return hit[1]
    ctx = Context(se_config(se), flat_weights(se), dev)
    per[dev] = (version, ctx)
    return ctx


def check_no_train_dropout(*mods: torch.nn.Module):
    """The reference never calls .eval() (data_utils.py:219-222, attack.py:38), so a module with
    dropout_rate > 0 applies random dropout on every forward of its attack loop
    (models.py:195-204, 298-323, 416-429).  libavc computes the deterministic (eval / p = 0)
    network only: refuse such a module loudly instead of silently diverging."""
    for m in mods:
        d = getattr(m, "dropout_layer", None)
        if d is not None and float(getattr(d, "p", 0.0)) > 0.0 and m.training:
            raise NotImplementedError(
                f"{type(m).__name__} has dropout_rate={d.p} and is in training mode: the reference then applies "
                "random dropout inside the attack loop (models.py:298-323), which libavc does not reproduce; "
                "call model.eval() or use dropout_rate=0")


def speaker_encoder_forward(se: torch.nn.Module, x: torch.Tensor) -> torch.Tensor:
    """SpeakerEncoder.forward (models.py:327-343) on the MI355X; no autograd."""
    _require_gpu(x)
    check_no_train_dropout(se)
    return context_for(se, x.device).se_forward(x)


def vc_context_for(model: torch.nn.Module, device: torch.device) -> Context:
    """Context of model.speaker_encoder with model.content_encoder / model.decoder attached
    (re-attached whenever their parameters change)."""
    check_no_train_dropout(model.speaker_encoder, model.content_encoder, model.decoder)
    ctx = context_for(model.speaker_encoder, device)
    mods = (model.content_encoder, model.decoder)
    version = tuple((p.data_ptr(), p._version) for m in mods for p in m.parameters())
    if getattr(ctx, "_vc_version", None) != version:
        flat = torch.cat([v.detach().reshape(-1).to("cpu", torch.float32)
                          for v in model.content_encoder.state_dict().values()] + [_dec_flat(model.decoder)])
        ctx.attach_vc(ce_config(model.content_encoder), dec_config(model.decoder), flat)
        ctx._vc_version = version
    # spectral norm: the module's weight_u / weight_v are the state every Decoder forward advances
    ctx._sn_dec = weakref.ref(model.decoder) if _dec_has_sn(model.decoder) else None
    return ctx


class PMContext:
    """libavc PredictiveModel (VSMask predictor) weights on one device (avc_pm_*)."""

    def __init__(self, flat: torch.Tensor, device: int):
        w = flat.detach().to("cpu", torch.float32).contiguous()
        need = lib().avc_pm_weight_count()
        if w.numel() != need:
            raise RuntimeError(f"PredictiveModel weights: got {w.numel()} values, need {need}")
        h = ctypes.c_void_p()
        _check(lib().avc_pm_create(int(device), ctypes.c_void_p(w.data_ptr()), w.numel(), ctypes.byref(h)))
        self.h = h
        self._lock = threading.Lock()

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value and _lib is not None:
            _lib.avc_pm_destroy(h)
            self.h = None

    @staticmethod
    def out_shape(H: int, W: int) -> Tuple[int, int]:
        ho, wo = ctypes.c_int(), ctypes.c_int()
        _check(lib().avc_pm_out_shape(int(H), int(W), ctypes.byref(ho), ctypes.byref(wo)))
        return ho.value, wo.value

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        _require_gpu(x)
        x = x.contiguous()
        if x.dim() != 4 or x.shape[1] != 1:
            raise RuntimeError(f"PredictiveModel expects [B, 1, F, T], got {tuple(x.shape)}")
        B, _, H, W = x.shape
        ho, wo = self.out_shape(H, W)
        y = torch.empty(B, 1, ho, wo, device=x.device, dtype=torch.float32)
        stream = torch.cuda.current_stream(x.device).cuda_stream
        with self._lock:
            _check(lib().avc_pm_forward(self.h, ctypes.c_void_p(x.data_ptr()), B, H, W,
                                        ctypes.c_void_p(y.data_ptr()), ctypes.c_void_p(stream)))
        return y

    def block_forward(self, layer: int, x: torch.Tensor) -> torch.Tensor:
        """One block: layer 0..6 = down_blocks.i, 7..11 = up_blocks.(i-7) (avc_pm_block_forward)."""
        _require_gpu(x)
        x = x.contiguous()
        if x.dim() != 4:
            raise RuntimeError(f"expected [B, C, H, W], got {tuple(x.shape)}")
        B, C, H, W = x.shape
        c, ho, wo, cin = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _check(lib().avc_pm_block_shape(self.h, int(layer), int(H), int(W), ctypes.byref(c), ctypes.byref(ho),
                                        ctypes.byref(wo), ctypes.byref(cin)))
        if C != cin.value:   # torch's Conv2d / ConvTranspose2d shape error (the C ABI refuses it too)
            raise RuntimeError(f"PredictiveModel block {layer}: expected input[{B}, {cin.value}, {H}, {W}], "
                               f"got {C} channels")
        y = torch.empty(B, c.value, ho.value, wo.value, device=x.device, dtype=torch.float32)
        stream = torch.cuda.current_stream(x.device).cuda_stream
        with self._lock:
            _check(lib().avc_pm_block_forward(self.h, int(layer), ctypes.c_void_p(x.data_ptr()), B, C, H, W,
                                              ctypes.c_void_p(y.data_ptr()), ctypes.c_void_p(stream)))
        return y

    def protect(self, mel: torch.Tensor, header: Optional[torch.Tensor], window_size: int = 100,
                future_step: int = 10, epsilon1: float = 0.1, epsilon2: float = 0.05,
                epsilon3: float = 0.08) -> torch.Tensor:
        """VSMask mel loop (vsmask.py:177-208) on mel [B,1,F,T] -> protected mel [B,1,F,T]."""
        hdr = _vsm_header(header, mel)
        _require_gpu(mel, *([hdr] if hdr is not None else []))
        mel = mel.contiguous()
        B, _, F, T = mel.shape
        out = torch.empty_like(mel)
        stream = torch.cuda.current_stream(mel.device).cuda_stream
        with self._lock:
            _check(lib().avc_vsmask_protect(
                self.h, ctypes.c_void_p(mel.data_ptr()), B, F, T,
                ctypes.c_void_p(hdr.data_ptr() if hdr is not None else 0), hdr.shape[-1] if hdr is not None else 0,
                int(window_size), int(future_step), float(epsilon1), float(epsilon2), float(epsilon3),
                ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(stream)))
        return out


def _vsm_header(header: Optional[torch.Tensor], mel: torch.Tensor) -> Optional[torch.Tensor]:
    """[1,1,F,Th] (header_model.py:22) or [F,Th] header -> contiguous [F,Th] on mel's device."""
    if mel.dim() != 4 or mel.shape[1] != 1:
        raise RuntimeError(f"VSMask expects a mel of shape [B, 1, F, T], got {tuple(mel.shape)}")
    if header is None:
        return None
    h = header.detach()
    if h.dim() == 4 and h.shape[:2] == (1, 1):
        h = h[0, 0]
    if h.dim() != 2 or h.shape[0] != mel.shape[2]:
        raise RuntimeError(f"header of shape {tuple(header.shape)} does not match mel bins {mel.shape[2]}")
    if h.device != mel.device:
        raise RuntimeError(f"header on {h.device}, mel on {mel.device}")
    return h.contiguous()


def vsmask_apply_header(mel: torch.Tensor, header: torch.Tensor) -> torch.Tensor:
    """UniversalPerturbationHeader.apply_header (header_model.py:70-95) on the MI355X."""
    hdr = _vsm_header(header, mel)
    _require_gpu(mel, hdr)
    mel = mel.contiguous()
    B, _, F, T = mel.shape
    out = torch.empty_like(mel)
    dev = mel.device.index if mel.device.index is not None else torch.cuda.current_device()
    stream = torch.cuda.current_stream(mel.device).cuda_stream
    _check(lib().avc_vsmask_apply_header(dev, ctypes.c_void_p(mel.data_ptr()), B, F, T,
                                         ctypes.c_void_p(hdr.data_ptr()), hdr.shape[-1],
                                         ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(stream)))
    return out


def vsmask_band_clamp(x: torch.Tensor, eps1: float, eps2: float, eps3: float) -> torch.Tensor:
    """MelSpectrogramConverter.apply_weighted_constraint (utils/audio.py:77-116): x [..., F, T]
    clamped to +-eps1 / eps2 / eps3 on rows [0, int(0.3 F)) / [.., int(0.7 F)) / the rest."""
    _require_gpu(x)
    if x.dim() < 2:
        raise RuntimeError(f"expected [..., F, T], got {tuple(x.shape)}")
    xc = x.float().contiguous()
    F, T = xc.shape[-2], xc.shape[-1]
    B = xc.numel() // max(F * T, 1)
    out = torch.empty_like(xc)
    dev = xc.device.index if xc.device.index is not None else torch.cuda.current_device()
    _check(lib().avc_vsmask_band_clamp(dev, ctypes.c_void_p(xc.data_ptr()), B, F, T, float(eps1), float(eps2),
                                       float(eps3), ctypes.c_void_p(out.data_ptr()),
                                       ctypes.c_void_p(torch.cuda.current_stream(xc.device).cuda_stream)))
    return out


def vsmask_windows(T: int, window_size: int = 100, future_step: int = 10) -> int:
    """Number of predictor windows of the reference loop, len(range(0, T - W, S))."""
    n = ctypes.c_int()
    _check(lib().avc_vsmask_windows(int(T), int(window_size), int(future_step), ctypes.byref(n)))
    return n.value


def pm_flat_weights(model: torch.nn.Module) -> torch.Tensor:
    """Floating tensors of a PredictiveModel state_dict in order (num_batches_tracked excluded)."""
    return torch.cat([v.detach().reshape(-1).to("cpu", torch.float32) for v in model.state_dict().values()
                      if v.is_floating_point()])


def predictive_forward(model: torch.nn.Module, x: torch.Tensor) -> torch.Tensor:
    """PredictiveModel.forward (models/predictive_model.py:87-110), eval semantics, on the MI355X."""
    _require_gpu(x)
    return pm_context_for(model, x.device).forward(x)


def pm_context_for(model: torch.nn.Module, device: torch.device) -> "PMContext":
    """The libavc PredictiveModel handle of `model` on `device` (re-uploaded when weights change)."""
    device = torch.device(device)
    if model.training:
        raise RuntimeError("libavc implements PredictiveModel inference (eval mode: BatchNorm running "
                           "statistics); call model.eval() first")
    dev = device.index if device.index is not None else torch.cuda.current_device()
    version = tuple((t.data_ptr(), t._version) for t in model.state_dict().values())
    per = _ctx_cache.setdefault(model, {})
    hit = per.get(("pm", dev))
    if hit is None or hit[0] != version:
        hit = (version, PMContext(pm_flat_weights(model), dev))
        per[("pm", dev)] = hit
    return hit[1]


# --- mel front / back end (data_utils.py:16-197) ------------------------------------

def dsp_cfg_struct(preprocess: Dict, pad_mode: str = "reflect") -> DspCfg:
    """config.yaml `preprocess` section -> avc_dsp_cfg (top_db is host-side: trim).  A
    `flavor: 1` entry selects utils/audio.py's torchaudio converter (TA_PREPROCESS below)."""
    c = DspCfg()
    for k in ("sample_rate", "n_fft", "hop_length", "win_length", "n_mels"):
        setattr(c, k, int(preprocess[k]))
    for k in ("preemph", "ref_db", "max_db"):
        setattr(c, k, float(preprocess[k]))
    if pad_mode not in PAD_MODE:
        raise RuntimeError(f"pad_mode must be one of {sorted(PAD_MODE)}")
    c.pad_mode = PAD_MODE[pad_mode]
    c.flavor = int(preprocess.get("flavor", 0))
    return c


def ta_preprocess(sample_rate: int = 16000, n_fft: int = 1024, hop_length: int = 256, n_mels: int = 80) -> Dict:
    """utils/audio.py:9-42's MelSpectrogram / InverseMelScale / GriffinLim parameters as an
    avc_dsp_cfg source (win_length = n_fft, no pre-emphasis, reflect padding, flavor 1)."""
    return dict(sample_rate=int(sample_rate), n_fft=int(n_fft), hop_length=int(hop_length), win_length=int(n_fft),
                n_mels=int(n_mels), preemph=0.0, ref_db=0.0, max_db=0.0, flavor=1)


def mel_basis(preprocess: Dict):
    """(librosa.filters.mel(sr, n_fft, n_mels), inv_mel_matrix) as float32 tensors, computed by
    libavc's host code (no device needed)."""
    c = dsp_cfg_struct(preprocess)
    F = int(preprocess["n_fft"]) // 2 + 1
    nm = int(preprocess["n_mels"])
    W = torch.empty(nm, F)
    inv = torch.empty(F, nm)
    _check(lib().avc_dsp_mel_basis(ctypes.byref(c), ctypes.c_void_p(W.data_ptr()), ctypes.c_void_p(inv.data_ptr())))
    return W, inv


class Dsp:
    """One libavc DSP context (window / twiddle / mel tables + workspace) per (config, device)."""

    def __init__(self, preprocess: Dict, device: int, pad_mode: str = "reflect"):
        self.pre = dict(preprocess)
        self._c = dsp_cfg_struct(preprocess, pad_mode)
        h = ctypes.c_void_p()
        _check(lib().avc_dsp_create(int(device), ctypes.byref(self._c), ctypes.byref(h)))
        self.h = h
        self.device = device
        self._lock = threading.Lock()

    def __del__(self):
        h = getattr(self, "h", None)
        if h is not None and h.value and _lib is not None:
            _lib.avc_dsp_destroy(h)

    def frames(self, n_samples: int) -> int:
        n = lib().avc_dsp_frames(ctypes.byref(self._c), int(n_samples))
        if n < 0:
            _check(1)
        return n

    @staticmethod
    def _stats(mean, std, like):
        if (mean is None) != (std is None):
            raise RuntimeError("give both mean and std, or neither")
        if mean is None:
            return None, None
        m = torch.as_tensor(mean, dtype=torch.float32).reshape(-1).to(like.device).contiguous()
        s = torch.as_tensor(std, dtype=torch.float32).reshape(-1).to(like.device).contiguous()
        return m, s

    def wav2mel(self, wav: torch.Tensor, mean=None, std=None, transpose: bool = False) -> torch.Tensor:
        """wav [B, L] (trimmed) -> mel [B, Tf, n_mels] ([B, n_mels, Tf] if transpose)."""
        _require_gpu(wav)
        wav = wav.contiguous()
        if wav.dim() != 2:
            raise RuntimeError(f"expected [B, L] waveforms, got {tuple(wav.shape)}")
        B, L = wav.shape
        Tf = self.frames(L)
        nm = int(self.pre["n_mels"])
        m, s = self._stats(mean, std, wav)
        out = torch.empty((B, nm, Tf) if transpose else (B, Tf, nm), device=wav.device)
        with self._lock:
            _check(lib().avc_dsp_wav2mel(self.h, ctypes.c_void_p(wav.data_ptr()), B, L,
                                         ctypes.c_void_p(m.data_ptr()) if m is not None else None,
                                         ctypes.c_void_p(s.data_ptr()) if s is not None else None,
                                         1 if transpose else 0, ctypes.c_void_p(out.data_ptr()),
                                         ctypes.c_void_p(torch.cuda.current_stream(wav.device).cuda_stream)))
        return out

    def mel2wav(self, mel: torch.Tensor, mean=None, std=None, transpose: bool = False,
                n_iter: int = 100) -> torch.Tensor:
        """mel [B, Tf, n_mels] ([B, n_mels, Tf] if transpose) -> wav [B, hop * (Tf - 1)]."""
        _require_gpu(mel)
        mel = mel.contiguous()
        nm = int(self.pre["n_mels"])
        if mel.dim() != 3 or mel.shape[1 if transpose else 2] != nm:
            raise RuntimeError(f"expected mel with {nm} bins, got {tuple(mel.shape)}")
        B, Tf = mel.shape[0], mel.shape[2 if transpose else 1]
        m, s = self._stats(mean, std, mel)
        out = torch.empty(B, int(self.pre["hop_length"]) * (Tf - 1), device=mel.device)
        with self._lock:
            _check(lib().avc_dsp_mel2wav(self.h, ctypes.c_void_p(mel.data_ptr()), B, Tf, 1 if transpose else 0,
                                         ctypes.c_void_p(m.data_ptr()) if m is not None else None,
                                         ctypes.c_void_p(s.data_ptr()) if s is not None else None,
                                         int(n_iter), ctypes.c_void_p(out.data_ptr()),
                                         ctypes.c_void_p(torch.cuda.current_stream(mel.device).cuda_stream)))
        return out

    def griffin_lim(self, spect: torch.Tensor, n_iter: int = 100) -> torch.Tensor:
        """spect [B, n_fft/2+1, Tf] (magnitude, the reference's layout) -> wav [B, hop * (Tf - 1)]."""
        _require_gpu(spect)
        spect = spect.contiguous()
        F = int(self.pre["n_fft"]) // 2 + 1
        if spect.dim() != 3 or spect.shape[1] != F:
            raise RuntimeError(f"expected [B, {F}, Tf] magnitudes, got {tuple(spect.shape)}")
        B, _, Tf = spect.shape
        out = torch.empty(B, int(self.pre["hop_length"]) * (Tf - 1), device=spect.device)
        with self._lock:
            _check(lib().avc_dsp_griffin_lim(self.h, ctypes.c_void_p(spect.data_ptr()), B, Tf, int(n_iter),
                                             ctypes.c_void_p(out.data_ptr()),
                                             ctypes.c_void_p(torch.cuda.current_stream(spect.device).cuda_stream)))
        return out

    def ta_mel2wav(self, mel: torch.Tensor, n_iter: int = 32, momentum: float = 0.99,
                   angles0: Optional[torch.Tensor] = None) -> torch.Tensor:
        """flavor-1 context: log10 mel [B, n_mels, Tf] -> wav [B, hop * (Tf - 1)] (InverseMelScale +
        GriffinLim; angles0 [B, n_fft/2+1, Tf] complex64 initial phases or None for all ones)."""
        _require_gpu(mel)
        mel = mel.float().contiguous()
        nm, F = int(self.pre["n_mels"]), int(self.pre["n_fft"]) // 2 + 1
        if mel.dim() != 3 or mel.shape[1] != nm:
            raise RuntimeError(f"expected log-mel [B, {nm}, Tf], got {tuple(mel.shape)}")
        B, _, Tf = mel.shape
        if angles0 is not None:
            if angles0.dtype != torch.complex64 or tuple(angles0.shape) != (B, F, Tf):
                raise RuntimeError(f"angles0 must be complex64 [{B}, {F}, {Tf}], got {angles0.dtype} "
                                   f"{tuple(angles0.shape)}")
            if angles0.device != mel.device:
                raise RuntimeError("angles0 must be on the mel's device")
            angles0 = angles0.contiguous()
        out = torch.empty(B, int(self.pre["hop_length"]) * (Tf - 1), device=mel.device)
        with self._lock:
            _check(lib().avc_dsp_ta_mel2wav(self.h, ctypes.c_void_p(mel.data_ptr()), B, Tf, int(n_iter),
                                            float(momentum),
                                            ctypes.c_void_p(angles0.data_ptr()) if angles0 is not None else None,
                                            ctypes.c_void_p(out.data_ptr()),
                                            ctypes.c_void_p(torch.cuda.current_stream(mel.device).cuda_stream)))
        return out

    def set_profiling(self, on: bool):
        _check(lib().avc_dsp_set_profiling(self.h, 1 if on else 0))

    def profile(self) -> Dict[str, Tuple[int, float]]:
        """{kernel name: (launches, total device ms)} since set_profiling(True)."""
        out = {}
        for i in range(lib().avc_dsp_profile_count(self.h)):
            name = ctypes.create_string_buffer(128)
            n, ms = ctypes.c_long(), ctypes.c_double()
            _check(lib().avc_dsp_profile_kernel(self.h, i, name, 128, ctypes.byref(n), ctypes.byref(ms)))
            out[name.value.decode()] = (n.value, ms.value)
        return out
