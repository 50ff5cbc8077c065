"""
Multimodal fusion on the MI355X HIP path — drop-in for the reference's
inference/multimodal_fusion.py (same class, methods, result dicts).

fuse_with_attention runs the attention-MLP fusion model in one HIP kernel
(csrc/speech_fusion.hip: fusion_kernel); fuse_predictions runs the 0.3/0.35/0.35 weighted
average in float64 on the GPU, bit-identical to the reference's numpy arithmetic.
predict_multimodal follows the reference's control flow (:244-287) but runs each encoder
once: features and probabilities come out of the same forward.

Added beyond the reference: predict_batch(x, ids, mask, gray) -> the whole batched path
(mec.engine.FusedPipeline semantics) on device tensors.
"""

from typing import Dict, Optional

import numpy as np
import torch

from config import Config
from mec import checkpoints, engine
from mec._lib import MecError

from inference.speech_inference import SpeechInference
from inference.text_inference import TextInference
from inference.image_inference import ImageInference

_MODS = ('speech', 'text', 'image')


class MultimodalFusion:
    def __init__(self, weights=None, seed=None, device=None, precision=None):
        weights = weights or {}
        self.emotions = Config.EMOTIONS
        self.weights = [0.3, 0.35, 0.35]  # speech, text, image (reference :23)
        self.fusion_model = None
        self.speech_inference = SpeechInference(weights.get('speech'), seed, device)
        self.text_inference = TextInference(weights.get('text'), seed, device, precision=precision)
        self.image_inference = ImageInference(weights.get('image'), seed, device, precision=precision)
        w = checkpoints.resolve('fusion', weights.get('fusion'), seed)
        if w is not None:
            self.fusion_model = engine.FusionHead(w, device=device)  # raises MecError without HIP/GPU
        self.device = (self.fusion_model.device if self.fusion_model is not None
                       else engine.require_gpu(device))

    def fuse_predictions(self, speech_probs, text_probs, image_probs) -> Dict:
        """Weighted average (fallback), float64 like the reference's numpy (:184-199)."""
        def t(p):
            return None if p is None else torch.tensor(np.asarray(p, np.float64).reshape(1, 7), device=self.device)
        weighted = engine.fuse_weighted_f64(t(speech_probs), t(text_probs), t(image_probs),
                                            device=self.device).cpu().numpy()[0]
        idx = int(np.argmax(weighted))
        return {'emotion': self.emotions[idx], 'confidence': float(weighted[idx]),
                'all_probabilities': weighted.tolist()}

    def _fusion_tensors(self, speech_feat, text_feat, image_feat, speech_pred, text_pred, image_pred):
        f = lambda a, d: engine.to_device(np.asarray(a, np.float32).reshape(1, d), self.device)  # noqa: E731
        return (f(speech_feat, 64), f(text_feat, 768), f(image_feat, 512),
                f(speech_pred, 7), f(text_pred, 7), f(image_pred, 7))

    def fuse_with_attention(self, speech_feat, text_feat, image_feat,
                            speech_pred, text_pred, image_pred) -> Dict:
        """Attention-MLP fusion (:201-242)."""
        if self.fusion_model is None:
            return self.fuse_predictions(speech_pred, text_pred, image_pred)
        try:
            logits, probs, aw, dw = self.fusion_model.forward(
                *self._fusion_tensors(speech_feat, text_feat, image_feat, speech_pred, text_pred, image_pred))
            preds, aw, dw = probs.cpu().numpy()[0], aw.cpu().numpy()[0], dw.cpu().numpy()[0]
            idx = int(np.argmax(preds))
            return {
                'emotion': self.emotions[idx],
                'confidence': float(preds[idx]),
                'all_probabilities': preds.tolist(),
                'attention_weights': {m: float(aw[j]) for j, m in enumerate(_MODS)},
                'decision_weights': {m: float(dw[j]) for j, m in enumerate(_MODS)},
            }
        except MecError:
            raise
        except Exception as e:
            print(f"Fusion model error: {e}")
            return self.fuse_predictions(speech_pred, text_pred, image_pred)

    def predict_multimodal(self, audio_path: Optional[str] = None,
                           text: Optional[str] = None,
                           image_path: Optional[str] = None):
        """Any combination of modalities (:244-287)."""
        results = {}
        if audio_path:
            results['speech'] = self.speech_inference.predict(audio_path)
        if text:
            results['text'] = self.text_inference.predict(text)
        if image_path:
            results['image'] = self.image_inference.predict(image_path)

        if len(results) > 1:
            s_probs = results['speech']['all_probabilities'] if 'speech' in results else None
            t_probs = results['text']['all_probabilities'] if 'text' in results else None
            i_probs = results['image']['all_probabilities'] if 'image' in results else None
            if self.fusion_model is not None and audio_path and text and image_path:
                try:
                    s_feat, s_pred = self.speech_inference.extract_features(audio_path)
                    t_feat, t_pred = self.text_inference.extract_features(text)
                    i_feat, i_pred = self.image_inference.extract_features(image_path)
                    if all(x is not None for x in (s_feat, t_feat, i_feat)):
                        results['fusion'] = self.fuse_with_attention(s_feat, t_feat, i_feat, s_pred, t_pred, i_pred)
                    else:
                        results['fusion'] = self.fuse_predictions(s_probs, t_probs, i_probs)
                except MecError:
                    raise
                except Exception as e:
                    print(f"Feature extraction failed: {e}")
                    results['fusion'] = self.fuse_predictions(s_probs, t_probs, i_probs)
            else:
                results['fusion'] = self.fuse_predictions(s_probs, t_probs, i_probs)
        return results

    def predict_batch(self, x_speech, ids, mask, gray):
        """Whole tri-modal batch on device tensors -> dict of (feat, logits, probs) per
        modality and (logits, probs, attn_w, dec_w) for the fusion."""
        for m, obj in (('speech', self.speech_inference), ('text', self.text_inference),
                       ('image', self.image_inference)):
            if obj.model is None:
                raise RuntimeError(f'{m} model not loaded')
        if self.fusion_model is None:
            raise RuntimeError('fusion model not loaded')
        sf, sl, sp = self.speech_inference.model.forward(x_speech)
        # fp32x3 text / image handles: synchronized and checked (a batch outside the planes' range is
        # answered by the fp32 engine before the fusion reads it; TextInference / ImageInference.predict_batch)
        tf, tl, tp = self.text_inference.predict_batch(ids, mask)
        imf, il, ip = self.image_inference.predict_batch(gray)
        fl, fp, aw, dw = self.fusion_model.forward(sf, tf, imf, sp, tp, ip)
        return {'speech': (sf, sl, sp), 'text': (tf, tl, tp), 'image': (imf, il, ip), 'fusion': (fl, fp, aw, dw)}

    def check(self):
        """After predict_batch: synchronize the device and raise MecError if a kernel flagged an
        after-the-fact error (the speech DNN's expired wait; an fp32x3 activation outside the f16 range)."""
        torch.cuda.synchronize(self.device)
        for obj in (self.speech_inference.model, self.text_inference.model, self.image_inference.model,
                    self.fusion_model):
            if obj is not None:
                obj.check()
