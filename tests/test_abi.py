"""CPU: libavc.so builds/loads and exports every symbol include/avc.h declares;
the Python mirror of the config struct agrees with the library.  No compute
calls (there is no GPU here)."""
import ctypes
import os
import re

import pytest

import avc_native
from conftest import ROOT


def header_functions():
    src = open(os.path.join(ROOT, "include", "avc.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(avc_\w+)\s*\(", src)))


def test_library_loads_and_exports_header():
    L = avc_native.lib()
    names = header_functions()
    assert "avc_emb_attack" in names and "avc_se_forward" in names
    for n in names:
        assert hasattr(L, n), n
    bound = {n for n, _, _ in avc_native.SIGNATURES}
    assert set(names) <= bound, set(names) - bound
    assert b"gfx950" in L.avc_version()


def test_weight_count_matches_state_dict(golden):
    import helpers
    for name in ("small_T32", "full_T128"):
        z = golden(name)
        m = helpers.model_from_fixture(z)
        cfg = avc_native.se_config(m.speaker_encoder)
        cs = avc_native.se_cfg_struct(cfg)
        n = avc_native.lib().avc_se_weight_count(ctypes.byref(cs))
        assert n == avc_native.flat_weights(m.speaker_encoder).numel()


def test_se_config_of_reference_style_module(golden):
    """se_config derives the same hyper-parameters from a module without
    avc_config() (the reference's SpeakerEncoder exposes only attributes)."""
    import helpers
    z = golden("full_T128")
    se = helpers.model_from_fixture(z).speaker_encoder
    ours = se.avc_config()

    class Bare:   # attribute-only view, like /root/reference/models.py:249-283
        pass
    b = Bare()
    for k in ("conv_bank", "c_h", "c_out", "kernel_size", "n_conv_blocks", "n_dense_blocks", "subsample"):
        setattr(b, k, getattr(se, k))
    import torch
    b.act = torch.nn.ReLU()
    assert avc_native.se_config(b) == ours


def test_cpu_tensors_fail_loudly():
    import torch
    with pytest.raises(RuntimeError, match="MI355X"):
        avc_native._require_gpu(torch.zeros(1))


def test_header_struct_layout():
    # SECfg mirrors avc_se_cfg: 9 int32 + subsample[16] + act
    assert ctypes.sizeof(avc_native.SECfg) == 4 * (9 + avc_native.MAX_BLOCKS + 1)
    assert ctypes.sizeof(avc_native.AttackOpts) == 8 + 8 + 8 + 8 + 8   # ... update, pgd_step
