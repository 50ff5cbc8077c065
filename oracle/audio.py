"""ORACLE (test infrastructure only): the 56-d speech features, numpy restatement.

Restates preprocessing/audio_preprocessing.py:
  load_audio        :12-19  pad/trim to sr * duration (22050 * 3 = 66150 samples; the file
                            decode + resample is host I/O and stays out of the path)
  extract_mfcc      :22-24  mean over frames of librosa.feature.mfcc(y, sr, n_mfcc=40)
  extract_chroma    :27-29  mean over frames of librosa.feature.chroma_stft(y, sr)
  extract_spectral  :32-37  means of zero_crossing_rate, spectral_centroid,
                            spectral_rolloff, rms
  preprocess_audio  :40-46  concat [40 mfcc | 12 chroma | 4 spectral] -> f32[56]
with librosa==0.10.0 (requirements.txt:10) defaults, which the reference never overrides:
n_fft 2048, hop 512, periodic Hann window, center=True with pad_mode='constant' (zeros),
power 2 mel spectrogram on 128 Slaney mel bands (fmax = sr/2, 'slaney' area norm),
power_to_db(ref=1, amin=1e-10, top_db=80), DCT-II ortho (scipy.fftpack, librosa's DCT);
chroma: estimate_tuning (piptrack on the power spectrogram, fmin 150, fmax 4000,
threshold 0.1; median magnitude gate; 100-bin residual histogram) -> chroma filterbank
(ctroct 5, octwidth 2, L2 column norm, base C) -> per-frame max normalisation.
dtypes follow librosa's: the windowed frames and the FFT in float64, the STFT rounded to
complex64, the spectrogram and filterbanks float32.

librosa is absent here, so this restatement is PARITY UNPINNED beyond the
pieces checked against what IS present: scipy.signal.get_window('hann', fftbins=True) (the
window librosa requests), scipy.fftpack.dct (the DCT librosa calls), numpy.fft.rfft /
rfftfreq (librosa's default FFT library and fft_frequencies), numpy.histogram (pitch_tuning).
The reference's own tests (tests/test_preprocessing.py:30-66) check only shapes (40, 12, 4)
and finiteness on np.random.randn audio; tests/test_audio_oracle.py repeats those checks.
"""
import numpy as np
import scipy.fftpack
import scipy.signal

SR, DURATION, N_MFCC = 22050, 3, 40  # config.py:57-59
N_FFT, HOP, N_MELS = 2048, 512, 128
N_CHROMA = 12
FEATURES = N_MFCC + N_CHROMA + 4


def frames_count(n_samples: int) -> int:
    return 1 + n_samples // HOP


def pad_trim(y: np.ndarray, sr: int = SR, duration: int = DURATION) -> np.ndarray:
    """load_audio's fixed length (audio_preprocessing.py:14-18), after decoding."""
    y = np.asarray(y, np.float32)
    target = sr * duration
    return np.pad(y, (0, target - len(y))) if len(y) < target else y[:target]


# ---------------------------------------------------------------- librosa.convert / filters
def fft_frequencies(sr=SR, n_fft=N_FFT):
    return np.fft.rfftfreq(n=n_fft, d=1.0 / sr)


def hz_to_mel(f):  # Slaney (htk=False)
    f = np.asanyarray(f, dtype=np.float64)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    if mels.ndim:
        t = f >= min_log_hz
        mels[t] = min_log_mel + np.log(f[t] / min_log_hz) / logstep
    elif f >= min_log_hz:
        mels = min_log_mel + np.log(f / min_log_hz) / logstep
    return mels


def mel_to_hz(m):
    m = np.asanyarray(m, dtype=np.float64)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz, min_log_mel, logstep = 1000.0, 1000.0 / f_sp, np.log(6.4) / 27.0
    t = m >= min_log_mel
    freqs[t] = min_log_hz * np.exp(logstep * (m[t] - min_log_mel))
    return freqs


def mel_filters(sr=SR, n_fft=N_FFT, n_mels=N_MELS):
    """librosa.filters.mel(sr, n_fft, n_mels, fmin=0, fmax=sr/2, htk=False, norm='slaney',
    dtype=float32): triangles rounded to float32, then the float64 Slaney area factor applied
    in place (float32 *= float64)."""
    weights = np.zeros((n_mels, 1 + n_fft // 2), dtype=np.float32)
    fftfreqs = fft_frequencies(sr, n_fft)
    mel_f = mel_to_hz(np.linspace(hz_to_mel(0.0), hz_to_mel(float(sr) / 2), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    for i in range(n_mels):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    enorm = 2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels])
    weights *= enorm[:, np.newaxis]
    return weights


def hz_to_octs(f, tuning=0.0, bins_per_octave=12):
    a440 = 440.0 * 2.0 ** (tuning / bins_per_octave)
    return np.log2(f / (float(a440) / 16))


def normalize(S, norm, axis=0):
    """librosa.util.normalize(fill=None, threshold=tiny(S)) for norm in {inf, 1, 2}."""
    mag = np.abs(S).astype(float)
    if norm == np.inf:
        length = np.max(mag, axis=axis, keepdims=True)
    else:
        length = np.sum(mag ** norm, axis=axis, keepdims=True) ** (1.0 / norm)
    length[length < np.finfo(S.dtype).tiny] = 1.0
    out = np.empty_like(S)
    out[:] = S / length
    return out


def chroma_filters(tuning: float, sr=SR, n_fft=N_FFT, n_chroma=N_CHROMA):
    """librosa.filters.chroma(sr, n_fft, tuning, n_chroma=12, ctroct=5, octwidth=2, norm=2,
    base_c=True, dtype=float32)."""
    frequencies = np.linspace(0, sr, n_fft, endpoint=False)[1:]
    frqbins = n_chroma * hz_to_octs(frequencies, tuning=tuning, bins_per_octave=n_chroma)
    frqbins = np.concatenate(([frqbins[0] - 1.5 * n_chroma], frqbins))
    binwidthbins = np.concatenate((np.maximum(frqbins[1:] - frqbins[:-1], 1.0), [1]))
    D = np.subtract.outer(frqbins, np.arange(0, n_chroma, dtype='d')).T
    n_chroma2 = np.round(float(n_chroma) / 2)
    D = np.remainder(D + n_chroma2 + 10 * n_chroma, n_chroma) - n_chroma2
    wts = np.exp(-0.5 * (2 * D / np.tile(binwidthbins, (n_chroma, 1))) ** 2)
    wts = normalize(wts, norm=2, axis=0)
    wts *= np.tile(np.exp(-0.5 * (((frqbins / n_chroma - 5.0) / 2) ** 2)), (n_chroma, 1))
    wts = np.roll(wts, -3 * (n_chroma // 12), axis=0)
    return np.ascontiguousarray(wts[:, :int(1 + n_fft / 2)], dtype=np.float32)


TUNING_EDGES = np.linspace(-0.5, 0.5, 101)  # pitch_tuning(resolution=0.01) histogram bins


# ---------------------------------------------------------------- librosa.core.spectrum
def frame(y, frame_length, hop_length):
    n = 1 + (len(y) - frame_length) // hop_length
    idx = np.arange(frame_length)[:, None] + hop_length * np.arange(n)[None, :]
    return y[idx]  # [frame_length, n_frames]


def stft(y):
    """librosa.stft(y, n_fft=2048, hop=512, window='hann', center=True, pad_mode='constant'):
    float64 window x frames, numpy rfft, result stored as complex64 [1025, n_frames]."""
    y = np.asarray(y, np.float32)
    window = scipy.signal.get_window('hann', N_FFT, fftbins=True)
    yp = np.pad(y, (N_FFT // 2, N_FFT // 2), mode='constant')
    fr = frame(yp, N_FFT, HOP)
    return np.fft.rfft(window[:, None] * fr, axis=0).astype(np.complex64)


def power_to_db(S, amin=1e-10, top_db=80.0):
    log_spec = 10.0 * np.log10(np.maximum(amin, S))
    log_spec -= 10.0 * np.log10(np.maximum(amin, 1.0))
    return np.maximum(log_spec, log_spec.max() - top_db)


def piptrack(S, sr=SR, n_fft=N_FFT, fmin=150.0, fmax=4000.0, threshold=0.1):
    """librosa.piptrack(S=S) (0.10.0): np.gradient slope, vectorised parabolic interpolation
    (shift = -b/a, zero where |b| >= |a| and at the edges), peaks = freq-masked local maxima of
    S * (S > threshold * max(S)); float32 throughout like S."""
    S = np.abs(S)
    fft_freqs = fft_frequencies(sr, n_fft)
    avg = np.gradient(S, axis=-2)
    a = S[2:] + S[:-2] - 2 * S[1:-1]
    b = (S[2:] - S[:-2]) / 2
    shift = np.zeros_like(S)
    with np.errstate(divide='ignore', invalid='ignore'):
        sh = np.where(np.abs(b) >= np.abs(a), np.float32(0), -b / a)
    shift[1:-1] = sh
    dskew = 0.5 * avg * shift
    pitches = np.zeros_like(S)
    mags = np.zeros_like(S)
    freq_mask = ((fmin <= fft_freqs) & (fft_freqs < fmax))[:, None]
    ref_value = threshold * np.max(S, axis=-2, keepdims=True)
    Sx = S * (S > ref_value)
    xp = np.pad(Sx, [(1, 1), (0, 0)], mode='edge')
    localmax = (Sx > xp[:-2]) & (Sx >= xp[2:])
    idx = np.nonzero(freq_mask & localmax)
    pitches[idx] = (idx[-2] + shift[idx]) * float(sr) / n_fft
    mags[idx] = (S + dskew)[idx]
    return pitches, mags


def estimate_tuning_index(S, sr=SR):
    """librosa.estimate_tuning(S=S, sr=sr, bins_per_octave=12) -> index into TUNING_EDGES
    (estimate_tuning passes sr on to piptrack: the pitch of a bin is (bin + shift) * sr / n_fft)."""
    pitch, mag = piptrack(S, sr=sr)
    mask = pitch > 0
    thr = np.median(mag[mask]) if mask.any() else 0.0
    freqs = pitch[(mag >= thr) & mask]
    freqs = freqs[freqs > 0]
    if not np.any(freqs):
        return 50  # pitch_tuning's empty set -> 0.0 == TUNING_EDGES[50]
    residual = np.mod(N_CHROMA * hz_to_octs(freqs), 1.0)
    residual[residual >= 0.5] -= 1.0
    counts, _ = np.histogram(residual, TUNING_EDGES)
    return int(np.argmax(counts))


# ---------------------------------------------------------------- features
def features(y, sr=SR, tuning_index=None):
    """preprocess_audio after load_audio: y f32[66150] -> (f32[56], tuning index).
    tuning_index overrides the estimate (to compare chroma at a given tuning)."""
    y = np.asarray(y, np.float32)
    X = stft(y)
    mag = np.abs(X)                        # float32 (|complex64|)
    P = mag ** 2                           # power 2 spectrogram
    mel = np.einsum('ft,mf->mt', P, mel_filters(sr), optimize=True)
    mfcc = scipy.fftpack.dct(power_to_db(mel), axis=0, type=2, norm='ortho')[:N_MFCC]
    f_mfcc = np.mean(mfcc.T, axis=0)
    tidx = estimate_tuning_index(P, sr) if tuning_index is None else tuning_index
    fb = chroma_filters(float(TUNING_EDGES[tidx]), sr)
    chroma = normalize(np.einsum('cf,ft->ct', fb, P, optimize=True), norm=np.inf, axis=0)
    f_chroma = np.mean(chroma.T, axis=0)
    # zero_crossing_rate: edge-padded frames, |y| <= 1e-10 -> 0, sign-bit changes, pad=False
    ye = np.pad(y, (N_FFT // 2, N_FFT // 2), mode='edge')
    fr = frame(ye, N_FFT, HOP).copy()
    fr[np.abs(fr) <= 1e-10] = 0
    sb = np.signbit(fr)
    crossings = np.concatenate([np.zeros((1, fr.shape[1]), bool), sb[1:] != sb[:-1]], axis=0)
    zcr = float(np.mean(np.mean(crossings, axis=0)))
    freq = fft_frequencies(sr)[:, None]
    centroid = float(np.mean(np.sum(freq * normalize(mag, norm=1, axis=0), axis=0)))
    total = np.cumsum(mag, axis=0)
    thr = 0.85 * total[-1]
    ind = np.where(total < thr, np.nan, 1)
    rolloff = float(np.mean(np.nanmin(ind * freq, axis=0)))
    yz = np.pad(y, (N_FFT // 2, N_FFT // 2), mode='constant')
    rms = float(np.mean(np.sqrt(np.mean(frame(yz, N_FFT, HOP) ** 2, axis=0))))
    spectral = np.array([zcr, centroid, rolloff, rms], dtype=np.float32)
    return np.concatenate([f_mfcc, f_chroma, spectral]).astype(np.float32), tidx


def features_batch(wave, sr=SR):
    """wave f32[B, n] -> (f32[B,56], tuning indices [B])."""
    out = [features(w, sr) for w in np.asarray(wave, np.float32)]
    return np.stack([o[0] for o in out]), np.array([o[1] for o in out])


def synthetic_clips(B: int, seed: int = 0, n: int = SR * DURATION, kind: str = 'mixed'):
    """Seeded test waveforms [B, n] f32: 'tonal' = harmonic tones with vibrato-free pitch
    and a noise floor (a peaked tuning histogram), 'noise' = np.random.randn like the
    reference's own tests, 'mixed' = alternating."""
    rng = np.random.default_rng(seed)
    t = np.arange(n) / SR
    out = np.empty((B, n), np.float32)
    for b in range(B):
        k = kind if kind != 'mixed' else ('tonal' if b % 2 == 0 else 'noise')
        if k == 'noise':
            out[b] = rng.standard_normal(n)
        else:
            f0 = 110.0 * 2 ** (rng.integers(0, 36) / 12 + rng.uniform(-0.3, 0.3) / 12)
            y = sum((0.8 ** h) * np.sin(2 * np.pi * f0 * (h + 1) * t + rng.uniform(0, 6.28)) for h in range(6))
            env = np.minimum(1.0, np.minimum(t / 0.05, (t[-1] - t) / 0.05))
            out[b] = (0.3 * y * env + 0.003 * rng.standard_normal(n)).astype(np.float32)
    return out
