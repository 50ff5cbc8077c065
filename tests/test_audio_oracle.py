"""The audio-feature oracle (oracle/audio.py, a numpy restatement of librosa 0.10.0 as
preprocessing/audio_preprocessing.py calls it) against what can be checked without librosa:
the reference's own tests (tests/test_preprocessing.py:30-66: shapes 40 / 12 / 4 and finite
values on np.random.randn audio), scipy's window and DCT, and closed-form properties."""
import numpy as np
import scipy.fftpack
import scipy.signal

from oracle import audio as oa


def test_reference_shapes_and_finiteness_on_random_audio():
    rng = np.random.default_rng(0)
    audio = rng.standard_normal(oa.SR * oa.DURATION)
    f, tidx = oa.features(audio)
    assert f.shape == (56,) and f.dtype == np.float32
    mfcc, chroma, spectral = f[:40], f[40:52], f[52:]
    assert mfcc.shape == (oa.N_MFCC,) and chroma.shape == (12,) and spectral.shape == (4,)
    assert np.all(np.isfinite(f))
    assert 0 <= tidx < 100


def test_stft_matches_direct_dft():
    y = oa.synthetic_clips(1, seed=3, n=4096)[0]
    X = oa.stft(y)
    assert X.shape == (1025, 1 + 4096 // 512) and X.dtype == np.complex64
    w = scipy.signal.get_window('hann', 2048, fftbins=True)
    yp = np.pad(y.astype(np.float64), 1024)
    t = 3
    seg = w * yp[t * 512:t * 512 + 2048]
    k = np.arange(1025)[:, None]
    direct = (seg[None, :] * np.exp(-2j * np.pi * k * np.arange(2048)[None, :] / 2048)).sum(1)
    assert np.abs(X[:, t] - direct).max() <= 1e-5 * np.abs(direct).max()


def test_mel_filterbank_properties():
    fb = oa.mel_filters()
    assert fb.shape == (128, 1025) and fb.dtype == np.float32
    assert (fb >= 0).all()
    # Slaney area norm: each triangle integrates (in Hz) to about 1 -> sum(w) * bin_hz ~ 1
    area = fb.sum(1) * (oa.SR / oa.N_FFT)
    assert np.all(np.abs(area[10:] - 1) < 0.05)
    assert (np.count_nonzero(fb, axis=0) <= 2).all()  # each bin in at most two triangles


def test_chroma_filterbank_properties():
    for t in (-0.5, 0.0, 0.37):
        fb = oa.chroma_filters(t)
        assert fb.shape == (12, 1025) and fb.dtype == np.float32 and (fb >= 0).all()


def test_sine_features_are_consistent():
    """A 440 Hz sine: chroma peaks at A (index 9, base C), tuning 0, centroid near 440 Hz,
    rms 0.5 / sqrt(2), zero-crossing rate 2 * 440 / sr."""
    t = np.arange(oa.SR * oa.DURATION) / oa.SR
    y = (0.5 * np.sin(2 * np.pi * 440.0 * t)).astype(np.float32)
    f, tidx = oa.features(y)
    chroma = f[40:52]
    assert int(np.argmax(chroma)) == 9
    assert abs(oa.TUNING_EDGES[tidx]) < 0.03  # parabolic peak bias on the power spectrum
    zcr, centroid, rolloff, rms = f[52:]
    assert abs(rms - 0.5 / np.sqrt(2)) < 0.01
    assert abs(zcr - 2 * 440 / oa.SR) < 2e-3
    assert 400 < centroid < 600 and 400 < rolloff < 500


def test_dct_is_scipy_ortho():
    x = np.random.default_rng(1).standard_normal(128).astype(np.float32)
    D = np.array([[np.sqrt((1 if k == 0 else 2) / 128) * np.cos(np.pi * k * (2 * m + 1) / 256) for m in range(128)]
                  for k in range(40)])
    assert np.abs(D @ x - scipy.fftpack.dct(x, type=2, norm='ortho')[:40]).max() < 1e-5
