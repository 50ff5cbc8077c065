"""GPU speech features (csrc/audio.hip, mec_audio_fwd) against the oracle restatement of
preprocess_audio (oracle/audio.py; librosa is absent, so the oracle is parity-unpinned
beyond scipy/numpy pieces — tests/test_audio_oracle.py).

The STFT is computed in float64 and rounded to complex64 as librosa stores it, so the
power spectrogram matches the oracle's to float32 rounding; the discrete steps (peak
picking, the median gate, the tuning histogram, the rolloff bin) then agree exactly, and the
continuous outputs agree to float32 reassociation:
  MFCC within 5e-4 dB absolute (values ~ 1e2), chroma within 1e-6, zcr exact,
  centroid / rolloff / rms within 1e-6 relative, tuning identical.
"""
import numpy as np
import pytest
import torch

from mec import engine, synthetic as syn
from oracle import audio as oa
from oracle import speech as o_s

pytestmark = pytest.mark.gpu

MFCC_ATOL, CHROMA_ATOL, SPEC_RTOL = 5e-4, 1e-6, 1e-6


@pytest.fixture(scope='module')
def fx(dev):
    return engine.AudioFeaturizer(device=dev)


def _run(fx, dev, wave):
    feat, tun = fx.forward(engine.to_device(np.ascontiguousarray(wave, np.float32), dev), return_tuning=True)
    torch.cuda.synchronize()
    return feat.cpu().numpy(), tun.cpu().numpy()


def _compare(name, got, gt, ref, rt):
    tidx = np.rint((gt + 0.5) * 100).astype(int)
    d_mfcc = np.abs(got[:, :40] - ref[:, :40]).max()
    d_chroma = np.abs(got[:, 40:52] - ref[:, 40:52]).max()
    rel = np.abs(got[:, 52:] - ref[:, 52:]) / np.maximum(np.abs(ref[:, 52:]), 1e-12)
    print(f'{name}: tuning {list(tidx)} vs {list(rt)}; mfcc max|d| {d_mfcc:.3g}, chroma {d_chroma:.3g}, '
          f'spectral rel {rel.max(0)}')
    assert (tidx == rt).all()
    assert d_mfcc <= MFCC_ATOL
    assert d_chroma <= CHROMA_ATOL
    assert (got[:, 52] == ref[:, 52]).all() or rel[:, 0].max() <= 1e-6  # zcr: exact count / 2048
    assert rel[:, 1:].max() <= SPEC_RTOL


@pytest.mark.parametrize('kind', ['tonal', 'noise'])
def test_audio_features_vs_oracle(fx, dev, kind):
    wave = oa.synthetic_clips(6, seed=11, kind=kind)
    got, gt = _run(fx, dev, wave)
    ref, rt = oa.features_batch(wave)
    _compare(kind, got, gt, ref, rt)


def test_audio_reference_random_audio(fx, dev):
    """The reference's own test input: np.random.randn(SAMPLE_RATE * AUDIO_DURATION)
    (tests/test_preprocessing.py:36), shapes 40 / 12 / 4 and finite."""
    wave = np.random.default_rng(7).standard_normal((3, oa.SR * oa.DURATION)).astype(np.float32)
    got, gt = _run(fx, dev, wave)
    assert got.shape == (3, 56) and np.isfinite(got).all()
    ref, rt = oa.features_batch(wave)
    _compare('randn', got, gt, ref, rt)


def test_audio_edge_cases(fx, dev):
    """Silence (empty peak set: tuning 0.0; log floor; zero chroma), a clip with a leading
    silence, and a short clip (1 s: 44 frames)."""
    n = oa.SR * oa.DURATION
    wave = np.zeros((2, n), np.float32)
    wave[1] = oa.synthetic_clips(1, seed=5, kind='tonal')[0]
    wave[1, :n // 2] = 0
    got, gt = _run(fx, dev, wave)
    ref, rt = oa.features_batch(wave)
    _compare('silence/half', got, gt, ref, rt)
    short = oa.synthetic_clips(2, seed=6, n=oa.SR)
    got, gt = _run(fx, dev, short)
    ref, rt = oa.features_batch(short)
    _compare('1 s clips', got, gt, ref, rt)


def test_audio_batch_invariance(fx, dev):
    wave = oa.synthetic_clips(5, seed=21)
    big, _ = _run(fx, dev, wave)
    for i in (0, 3):
        one, _ = _run(fx, dev, wave[i:i + 1])
        assert np.array_equal(one[0], big[i])


def test_waveform_to_speech_prediction(fx, dev):
    """Waveform -> GPU features -> GPU speech DNN against the oracle chain (oracle features ->
    oracle DNN): the SpeechInference.predict arithmetic from the waveform on
    (inference/speech_inference.py:65-69)."""
    wave = oa.synthetic_clips(8, seed=31)
    x = fx.forward(engine.to_device(wave, dev))
    sp = engine.SpeechEncoder(device=dev)
    _, _, probs = sp.forward(x)
    probs = probs.cpu().numpy()
    ref_feat, _ = oa.features_batch(wave)
    _, _, ref_probs = o_s.forward(syn.weights('speech'), ref_feat)
    print(f'speech from waveform: probs max|d| {np.abs(probs - ref_probs).max():.3g}')
    assert (probs.argmax(1) == ref_probs.argmax(1)).all()
    assert np.abs(probs - ref_probs).max() <= 1e-4


def test_audio_long_clip_median_from_hbm(fx, dev):
    """A 30 s clip: more peaks than the clip kernel keeps in LDS (24576), so the median's
    radix select reads the per-frame peak lists from HBM."""
    wave = oa.synthetic_clips(1, seed=9, n=30 * oa.SR, kind='noise')
    got, gt = _run(fx, dev, wave)
    ref, rt = oa.features_batch(wave)
    _compare('30 s noise', got, gt, ref, rt)


def test_audio_features_at_44100_hz(dev):
    """A handle at another sample rate (AudioModel::create takes 8-96 kHz): every sr-dependent
    table and piptrack's pitch = (bin + shift) * sr / n_fft follow the handle's rate."""
    fx44 = engine.AudioFeaturizer(sample_rate=44100, device=dev)
    wave = oa.synthetic_clips(3, seed=17, n=44100 * 2, kind='mixed')
    got, gt = _run(fx44, dev, wave)
    ref, rt = oa.features_batch(wave, sr=44100)
    _compare('44.1 kHz', got, gt, ref, rt)


def test_audio_rate_too_low_for_the_peak_list_is_rejected(dev):
    """Below ~21.6 kHz the 150-4000 Hz piptrack band holds more local maxima per frame than the
    per-frame peak list: the handle refuses the rate instead of dropping peaks."""
    from mec._lib import MecError
    with pytest.raises(MecError, match='sample_rate too low'):
        engine.AudioFeaturizer(sample_rate=16000, device=dev)
