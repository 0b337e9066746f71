"""Oracle pinning for the front end: the numpy restatement (oracle/frontend.py) against
the reference's own bundled pairs wavs/*.wav -> spmel/*.npy (make_spect.py output)."""
import glob
import os

import numpy as np
import pytest

from conftest import GOLDEN, REFERENCE, reference_available
from oracle import frontend as fe

FILES = ["p225_003", "p226_003", "p001_003"]  # first file of each speaker: fresh dither RNG


@pytest.mark.parametrize("name", FILES)
def test_oracle_matches_bundled_golden_bit_exact(name):
    wav = fe.load_wav(os.path.join(GOLDEN, "frontend", name + ".wav"))
    prng = np.random.RandomState(int(name[1:4]))
    got = fe.spmel_from_wav(fe.preprocess(wav, prng))
    ref = np.load(os.path.join(GOLDEN, "frontend", name + ".npy"))
    assert got.shape == ref.shape and got.dtype == ref.dtype
    assert np.array_equal(got, ref)


@pytest.mark.skipif(not reference_available(), reason="/root/reference not mounted")
def test_oracle_all_71_bundled_pairs():
    n = 0
    for spk in sorted(os.listdir(os.path.join(REFERENCE, "wavs"))):
        out = fe.speaker_spmels(glob.glob(os.path.join(REFERENCE, "wavs", spk, "*.wav")), spk)
        for k, v in out.items():
            g = os.path.join(REFERENCE, "spmel", spk, k + ".npy")
            if os.path.exists(g):
                assert np.array_equal(np.load(g), v), k
                n += 1
    assert n == 71


def test_product_mel_basis_matches_oracle():
    from autovc_amd import dsp
    assert np.array_equal(dsp.mel_basis(), fe.librosa_mel())
    assert dsp.mel_basis().shape == (80, 513)


def test_sparse_mel_roundtrip():
    from autovc_amd import dsp
    B = dsp.mel_basis()
    lo, ln, off, w = dsp.sparse_mel(B)
    dense = np.zeros_like(B)
    for m in range(B.shape[0]):
        dense[m, lo[m]:lo[m] + ln[m]] = w[off[m]:off[m] + ln[m]]
    assert np.array_equal(dense, B)
    assert int((B != 0).sum()) == 941


def test_frame_count_matches_reference():
    from autovc_amd import dsp
    for n in [600, 1000, 16000, 48000, 48001, 48255, 48256]:
        assert dsp.n_frames(n) == fe.py_stft(np.random.RandomState(0).rand(n)).shape[1] == n // 256 + 1


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_filtfilt_restatement_is_scipy_bit_exact(dtype):
    """The operation order the GPU filtfilt follows (make_spect.py:74) equals scipy's."""
    from scipy import signal
    rs = np.random.RandomState(7)
    b, a = fe.butter_highpass()
    for n in (19, 20, 333, 3000):
        x = rs.uniform(-0.6, 0.6, n).astype(dtype)
        assert np.array_equal(fe.filtfilt_restated(x), signal.filtfilt(b, a, x)), n


@pytest.mark.parametrize("seed", [0, 1, 225, 2**32 - 1])
def test_mt19937_restatement_is_numpy_bit_exact(seed):
    """make_spect.py:76's prng.rand(n), restated as the GPU dither computes it; 700 draws
    cross two 624-word twists."""
    assert np.array_equal(fe.mt19937_rand(seed, 700), np.random.RandomState(seed).rand(700))
