"""CPU checks of the VSMask loop restatement (oracle/vsmask.py) -- the checker the GPU
tests use -- against hand-computed cases of /root/reference/vsmask.py:177-208 and
utils/audio.py:77-116."""
import numpy as np
import pytest

from oracle import vsmask as vo


def test_band_edges_and_window_count():
    # utils/audio.py:97-98 with freq_dim = 80: int(24.0) / int(56.0) (0.7 * 80 rounds to 56.0)
    assert (int(80 * 0.3), int(80 * 0.7)) == (24, 56)
    assert vo.n_windows(100) == 0 and vo.n_windows(101) == 1 and vo.n_windows(110) == 1
    assert vo.n_windows(111) == 2 and vo.n_windows(400) == 30
    assert vo.n_windows(50, 100, 10) == 0


def test_constant_predictor_hand_case():
    """T = 125, W = 100, S = 10: windows at 0, 10, 20 add at 100.., 110.., 120..."""
    F, T = 80, 125
    mel = np.zeros((1, 1, F, T), np.float32)
    hdr = np.full((1, 1, F, 100), 0.01, np.float32)

    def pred(w):
        return np.full((w.shape[0], 1, 95, 63), 0.02, np.float32)
    out = vo.protect_mel(mel, hdr, pred, 100, 10, 0.1, 0.05, 0.08)
    assert out.shape == mel.shape
    exp = np.zeros(T, np.float64)
    exp[:100] += 0.01
    for s in (0, 10, 20):
        exp[s + 100:] += 0.02
    for f, cap in ((0, 0.1), (23, 0.1), (24, 0.05), (55, 0.05), (56, 0.08), (79, 0.08)):
        np.testing.assert_allclose(out[0, 0, f], np.minimum(exp, cap), rtol=1e-6)


def test_windows_read_unperturbed_mel_and_crop_rows():
    F, T = 80, 140
    rng = np.random.default_rng(0)
    mel = rng.standard_normal((2, 1, F, T)).astype(np.float32)
    seen = []

    def pred(w):
        seen.append(w.copy())
        return np.ones((w.shape[0], 1, 95, 63), np.float32) * 1e-3
    hdr = rng.standard_normal((1, 1, F, 100)).astype(np.float32)
    vo.protect_mel(mel, hdr, pred)
    assert len(seen) == vo.n_windows(T)
    for k, w in enumerate(seen):
        assert np.array_equal(w, mel[:, :, :, 10 * k:10 * k + 100])


def test_apply_header():
    rng = np.random.default_rng(1)
    hdr = rng.uniform(-0.5, 0.5, (1, 1, 80, 100)).astype(np.float32)
    for T in (37, 100, 180):
        mel = rng.uniform(-1, 1, (3, 1, 80, T)).astype(np.float32)
        out = vo.apply_header(mel, hdr)
        n = min(T, 100)
        exp = mel.copy()
        exp[..., :n] += hdr[..., :n]
        assert np.array_equal(out, np.clip(exp, -1, 1))


@pytest.mark.parametrize("T", [100, 101, 173])
def test_float32_loop_equals_reordered_sum(T):
    """The per-element ascending-window sum libavc's combine kernel performs equals the
    reference loop's in-place adds bit for bit (same fp32 operations, same order)."""
    rng = np.random.default_rng(T)
    F, W, S = 80, 100, 10
    mel = rng.standard_normal((1, 1, F, T)).astype(np.float32)
    hdr = (rng.standard_normal((1, 1, F, 100)) * 0.05).astype(np.float32)
    nw = vo.n_windows(T, W, S)
    ys = (rng.standard_normal((max(nw, 1), 1, 95, 63)) * 0.05).astype(np.float32)
    it = iter(range(nw))
    ref = vo.protect_mel(mel, hdr, lambda w: ys[next(it)][None], W, S)
    acc = mel[0, 0].copy()
    acc[:, :min(T, 100)] += hdr[0, 0, :, :min(T, 100)]
    out = np.empty_like(acc)
    for f in range(F):
        for t in range(T):
            a = acc[f, t]
            for k in range(nw):
                if 10 * k + W <= t < 10 * k + W + 63:
                    a = np.float32(a + ys[k, 0, f, t - 10 * k - W])
            e = np.float32(0.1 if f < 24 else (0.05 if f < 56 else 0.08))
            p = np.float32(min(max(np.float32(a - mel[0, 0, f, t]), -e), e))
            out[f, t] = np.float32(mel[0, 0, f, t] + p)
    assert np.array_equal(out, ref[0, 0])


def test_header_optimize_restatement_properties(golden):
    """The header-optimisation restatement (header_model.py:40-65) keeps the header inside
    +-epsilon, lowers its objective and matches a hand-computed first Adam step's size."""
    from helpers import cfg_of, model_from_fixture, oracle_weights
    z = golden("small_T32")
    w = oracle_weights(model_from_fixture(z))
    se = cfg_of(z)["SpeakerEncoder"]
    rng = np.random.default_rng(5)
    src = rng.uniform(-0.95, 0.95, (3, 80, 32))
    tgt = rng.uniform(-0.95, 0.95, (3, 80, 32))
    hdr, losses = vo.header_optimize(w, se, src, tgt, np.zeros((80, 32)), 25, epsilon=0.05, lr=2e-3)
    assert np.abs(hdr).max() <= 0.05 + 1e-12
    assert losses[-1] < losses[0]
    h1, _ = vo.header_optimize(w, se, src, tgt, np.zeros((80, 32)), 1, epsilon=0.05, lr=2e-3)
    # Adam's first step is lr * g / (|g| + eps): at most lr, ~lr wherever |g| >> eps
    moved = np.abs(h1[np.abs(h1) > 0])
    assert moved.max() <= 2e-3 * (1 + 1e-9) and abs(np.median(moved) - 2e-3) <= 2e-5
