"""GPU parity of the waveform preprocessing (autovc_preprocess_f64: make_spect.py:74-76
filtfilt + RandomState dither) against scipy / numpy, the reference's own host code.

Bar: bit-exact (np.array_equal) — the kernel runs scipy's recurrence in scipy's operation
order and numpy's MT19937 word for word (oracle/frontend.py restates both; pinned in
tests/test_oracle_frontend.py)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import frontend as fe

pytestmark = pytest.mark.gpu


def _filtfilt(x):
    from scipy import signal
    b, a = fe.butter_highpass()
    return signal.filtfilt(b, a, x)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_filtfilt_ragged_batch_bit_exact(cuda, dtype):
    """Edge lengths: 19 (shortest scipy accepts), lengths that are not multiples of the
    kernel's 8-sample groups, and a 4 s utterance, in one ragged batch."""
    from autovc_amd import dsp
    rs = np.random.RandomState(3)
    lens = [19, 20, 25, 26, 27, 100, 1001, 64000]
    wavs = [rs.uniform(-0.9, 0.9, n).astype(dtype) for n in lens]
    wav, got_lens = dsp.preprocess_gpu(wavs, seeds=None, device=cuda)
    assert got_lens == lens and wav.dtype.is_floating_point and wav.element_size() == 8
    got = np.split(wav.cpu().numpy(), np.cumsum(lens)[:-1])
    for w, g in zip(wavs, got):
        assert np.array_equal(g, _filtfilt(w)), len(w)


def test_dither_streams_bit_exact(cuda):
    """Two speakers' files share one RandomState each, consumed in file order
    (make_spect.py:68-76); odd file lengths put stream boundaries mid-twist."""
    from autovc_amd import dsp
    rs = np.random.RandomState(4)
    groups = [3, 2, 1]
    seeds = [225, 226, 2**32 - 1]
    lens = [3001, 777, 20011, 19, 5000, 1313]
    wavs = [rs.uniform(-0.5, 0.5, n).astype(np.float32) for n in lens]
    wav, _ = dsp.preprocess_gpu(wavs, seeds=seeds, groups=groups, device=cuda)
    got = np.split(wav.cpu().numpy(), np.cumsum(lens)[:-1])
    i = 0
    for seed, g in zip(seeds, groups):
        prng = np.random.RandomState(seed)
        for _ in range(g):
            assert np.array_equal(got[i], fe.preprocess(wavs[i], prng)), (seed, i)
            i += 1


def test_spect_speaker_on_golden_wavs(cuda, tmp_path):
    """Spect.speaker (GPU preprocess -> GPU STFT+mel) on the reference's own bundled wavs
    against the reference's npy outputs (1e-4 abs, the STFT's bound); p225_003 is the
    speaker's first file, so its dither stream starts fresh as in make_spect.py."""
    from types import SimpleNamespace
    from autovc_amd.make_spect import Spect
    for name in ["p225_003", "p226_003"]:
        sp = Spect(SimpleNamespace(model_type="spmel", main_dir=str(tmp_path), device=cuda))
        out = sp.speaker([os.path.join(GOLDEN, "frontend", name + ".wav")], name[:4])
        ref = np.load(os.path.join(GOLDEN, "frontend", name + ".npy"))
        assert out[name].shape == ref.shape
        assert np.abs(out[name] - ref).max() <= 1e-4


def test_preprocess_errors(cuda):
    from autovc_amd import dsp
    w, lens = dsp.preprocess_gpu([], device=cuda)
    assert lens == [] and w.numel() == 0
    with pytest.raises(ValueError, match="padlen"):
        dsp.preprocess_gpu([np.zeros(18, np.float32)], device=cuda)
    with pytest.raises(ValueError, match="mix"):
        dsp.preprocess_gpu([np.zeros(30, np.float32), np.zeros(30)], device=cuda)
    with pytest.raises(ValueError, match="groups"):
        dsp.preprocess_gpu([np.zeros(30), np.zeros(30)], seeds=[1], groups=[1], device=cuda)
