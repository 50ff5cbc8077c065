"""
Speech inference on the MI355X HIP path — drop-in for the reference's
inference/speech_inference.py (same class, methods, result dicts).

The model arithmetic (StandardScaler -> 5 x [Dense, BN, ReLU] -> Dense7 -> softmax) runs in
one fused HIP kernel (csrc/speech_fusion.hip) through libmec_hip.so, and the 56-d
MFCC / chroma / spectral features of preprocess_audio (preprocessing/audio_preprocessing.py:
22-46) run on the GPU too (csrc/audio.hip). Only audio decoding and resampling stay in the
reference's untouched preprocessing/ package (load_audio, imported lazily from the tree this
module is dropped into, as the reference does at inference/speech_inference.py:9).

Added beyond the reference: predict_features(features) for an already-extracted 56-d
vector, predict_batch(x) for a device-resident [B,56] batch, and features_from_waveforms /
predict_waveforms for device-resident [B, n] waveforms.
"""

from typing import Dict

import numpy as np

from config import Config
from mec import checkpoints, engine


def _preprocessing():
    # reference: from preprocessing.audio_preprocessing import preprocess_audio, ...
    from preprocessing import audio_preprocessing  # noqa: WPS433 (lazy, needs librosa)
    return audio_preprocessing


class SpeechInference:
    def __init__(self, weights=None, seed=None, device=None):
        self.emotions = Config.EMOTIONS
        self.model = None
        self.scaler = None  # the scaler is part of the device model (applied in-kernel)
        w = checkpoints.resolve('speech', weights, seed)
        if w is not None:
            # No silent CPU fallback: a missing libmec_hip.so or GPU raises MecError here.
            self.model = engine.SpeechEncoder(w, device=device)
        self.device = self.model.device if self.model is not None else None
        self._audio = None

    def _featurizer(self):
        if self._audio is None:
            self._audio = engine.AudioFeaturizer(Config.SAMPLE_RATE, Config.N_MFCC, device=self.device)
        return self._audio

    def _file_features(self, audio_file_path: str) -> np.ndarray:
        # preprocess_audio (audio_preprocessing.py:40-46): load_audio on the host (decode,
        # resample, pad/trim), the feature arithmetic on the GPU
        audio, sr = _preprocessing().load_audio(audio_file_path)
        if int(sr) != Config.SAMPLE_RATE:
            return _preprocessing().preprocess_audio(audio_file_path)
        wave = engine.to_device(np.asarray(audio, np.float32).reshape(1, -1), self.device)
        return self._featurizer().forward(wave).cpu().numpy()[0]

    def features_from_waveforms(self, wave):
        """wave: device f32 [B, n] (load_audio's fixed length) -> raw 56-d features [B, 56]."""
        return self._featurizer().forward(wave)

    def predict_waveforms(self, wave):
        """wave: device f32 [B, n] -> (feat [B,64], logits [B,7], probs [B,7])."""
        return self.predict_batch(self.features_from_waveforms(wave))

    def _heuristic_predict(self, audio_path: str) -> Dict:
        # reference :36-58 — RMS energy / spectral centroid rule
        ap = _preprocessing()
        audio, sr = ap.load_audio(audio_path)
        zcr, centroid, rolloff, rms = ap.extract_spectral_features(audio, sr)
        if rms > 0.06 and centroid > 2000:
            label = 'angry'
        elif rms < 0.02 and centroid < 1500:
            label = 'sad'
        else:
            label = 'neutral'
        probs = np.ones(len(self.emotions)) * (0.1 / (len(self.emotions) - 1))
        idx = self.emotions.index(label)
        probs[idx] = 0.9
        return {'emotion': label, 'confidence': float(probs[idx]), 'all_probabilities': probs.tolist()}

    def _forward(self, features: np.ndarray):
        x = np.asarray(features, dtype=np.float32).reshape(1, 56)
        feat, logits, probs = self.model.forward(engine.to_device(x, self.device))
        feat, probs = feat.cpu().numpy()[0], probs.cpu().numpy()[0]  # synchronizes the stream
        self.model.check()  # an expired in-kernel wait raises MecError instead of NaN probs
        return feat, probs

    @staticmethod
    def _as_dict(emotions, probs: np.ndarray) -> Dict:
        idx = int(np.argmax(probs))
        return {'emotion': emotions[idx], 'confidence': float(probs[idx]), 'all_probabilities': probs.tolist()}

    def predict_features(self, features) -> Dict:
        """Per-sample prediction from a raw (pre-scaler) 56-d feature vector."""
        return self._as_dict(self.emotions, self._forward(features)[1])

    def predict(self, audio_file_path: str) -> Dict:
        if self.model is None:
            return self._heuristic_predict(audio_file_path)
        return self.predict_features(self._file_features(audio_file_path))

    def extract_features(self, audio_file_path: str):
        """(64-d block-5 ReLU feature, 7 probs) — one forward instead of the reference's three."""
        if self.model is None:
            return None, None
        return self._forward(self._file_features(audio_file_path))

    def predict_batch(self, x):
        """x: device f32 [B,56] raw features -> (feat [B,64], logits [B,7], probs [B,7])."""
        if self.model is None:
            raise RuntimeError('speech model not loaded')
        return self.model.forward(x)
