"""
Text inference (BERT-base sequence classification) on the MI355X HIP path — drop-in for the
reference's inference/text_inference.py (same class, methods, result dicts, keyword fallback).

The 12-layer encoder, pooler and classifier run as hand-written HIP kernels (csrc/bert.hip,
csrc/gemm_glds.hip). Tokenisation stays on the host: a local BertTokenizer directory at
Config.BERT_MODEL_PATH (never a hub download), exactly the reference's call at :78-85.

Added beyond the reference: predict_ids(ids, mask) for pre-tokenised input and
predict_batch(ids, mask) for a device-resident [B,128] batch.
"""

import os
import re
from typing import Dict, List

import numpy as np

from config import Config
from mec import checkpoints, engine
from mec._lib import MecError

# Keyword fallback vocabulary (reference :13-21).
KEYWORD_MAP = {
    'happy': ['happy', 'joy', 'glad', 'pleased', 'delighted', 'cheerful', 'love', 'excited'],
    'sad': ['sad', 'down', 'unhappy', 'depressed', 'blue', 'disappointed', 'heartbroken'],
    'angry': ['angry', 'mad', 'furious', 'rage', 'annoyed', 'irritated', 'frustrated'],
    'fear': ['scared', 'afraid', 'fear', 'terrified', 'anxious', 'nervous', 'worried'],
    'disgust': ['disgust', 'gross', 'nasty', 'revolting', 'sick'],
    'surprise': ['surprised', 'amazed', 'astonished', 'wow', 'shocked'],
    'neutral': [],
}


class _Cleaner:
    """TextPreprocessor.clean_text (preprocessing/text_preprocessing.py:28-33) — the only
    part of the preprocessor the keyword fallback uses; constructing the reference class
    would trigger a by-name tokenizer download (:24)."""

    @staticmethod
    def clean_text(text: str) -> str:
        text = text.lower()
        text = re.sub(r'http\S+|www\S+|https\S+', '', text)
        text = re.sub(r'[^a-zA-Z\s]', '', text)
        return text.strip()


def _local_tokenizer(fast: bool = False):
    """The reference's tokenizer (text_inference.py:39 -> preprocessing/text_preprocessing.py:24)
    from the local BERT_MODEL_PATH only (never a by-name hub fetch). fast=True builds the
    Rust WordPiece (BertTokenizerFast) from the same vocab, for batched encoding."""
    if not os.path.isdir(Config.BERT_MODEL_PATH):
        return None
    try:
        from transformers import BertTokenizer, BertTokenizerFast
        cls = BertTokenizerFast if fast else BertTokenizer
        return cls.from_pretrained(Config.BERT_MODEL_PATH, local_files_only=True)
    except Exception as e:
        print(f"Warning: Could not load BERT tokenizer: {e}")
        return None


def encode_batch(tokenizer, texts):
    """Batched form of the reference's per-text call (text_inference.py:78-85): raw text (no
    clean_text), [CLS]/[SEP], pad to / truncate at MAX_TEXT_LENGTH. -> int32 ids, mask [B,128]."""
    enc = tokenizer(list(texts), add_special_tokens=True, max_length=Config.MAX_TEXT_LENGTH,
                    padding='max_length', truncation=True, return_tensors='np')
    return enc['input_ids'].astype(np.int32), enc['attention_mask'].astype(np.int32)


class TextInference:
    def __init__(self, weights=None, seed=None, device=None, tokenizer=None, precision=None):
        self.emotions = Config.EMOTIONS
        self.model = None
        self.preprocessor = _Cleaner()
        w = checkpoints.resolve('text', weights, seed)
        if w is not None:  # raises MecError without HIP/GPU
            self.model = engine.TextEncoder(w, device=device, precision=checkpoints.precision(precision))
        self.tokenizer = tokenizer if tokenizer is not None else (_local_tokenizer() if self.model else None)
        self._fast = None  # built on first batched call
        self.device = self.model.device if self.model is not None else None

    def _keyword_heuristic(self, text: str) -> Dict:
        cleaned = self.preprocessor.clean_text(text)
        selected = 'neutral'
        for label, keywords in KEYWORD_MAP.items():
            if any(f" {kw} " in f" {cleaned} " for kw in keywords):
                selected = label
                break
        probs = np.ones(len(self.emotions)) * (0.1 / (len(self.emotions) - 1))
        idx = self.emotions.index(selected)
        probs[idx] = 0.9
        return {'emotion': selected, 'confidence': float(probs[idx]), 'all_probabilities': probs.tolist()}

    def _encode(self, text: str):
        # reference :78-85 (raw text, no clean_text; pad/truncate to MAX_TEXT_LENGTH)
        enc = self.tokenizer(text, add_special_tokens=True, max_length=Config.MAX_TEXT_LENGTH,
                             padding='max_length', truncation=True, return_tensors='np')
        return enc['input_ids'].astype(np.int32), enc['attention_mask'].astype(np.int32)

    def _forward(self, ids: np.ndarray, mask: np.ndarray):
        ids = np.asarray(ids, np.int32).reshape(1, -1)
        mask = np.asarray(mask, np.int32).reshape(1, -1)
        if ids.size and (ids.min() < 0 or ids.max() >= engine.TextEncoder.VOCAB):
            # the reference's nn.Embedding raises IndexError for such ids
            raise ValueError(f'token id out of range [0, {engine.TextEncoder.VOCAB})')
        # synchronized and checked: an fp32x3 batch whose activations leave the planes' range is re-run on
        # the fp32 engine (engine.HipModel.recover), never answered with NaN probs
        cls, logits, probs = self.model.checked('forward', engine.to_device(ids, self.device),
                                                engine.to_device(mask, self.device))
        return cls.cpu().numpy()[0], probs.cpu().numpy()[0]

    @staticmethod
    def _as_dict(emotions, probs: np.ndarray) -> Dict:
        idx = int(np.argmax(probs))
        return {'emotion': emotions[idx], 'confidence': float(probs[idx]), 'all_probabilities': probs.tolist()}

    def predict_ids(self, ids, mask) -> Dict:
        """Per-sample prediction from token ids / attention mask of length 128."""
        return self._as_dict(self.emotions, self._forward(ids, mask)[1])

    def predict(self, text: str) -> Dict:
        if self.model is None or self.tokenizer is None:
            return self._keyword_heuristic(text)
        try:
            return self.predict_ids(*self._encode(text))
        except MecError:
            raise  # a failing HIP kernel is never hidden behind the heuristic
        except Exception as e:
            print(f"Text inference error: {e}")
            return self._keyword_heuristic(text)

    def extract_features(self, text: str):
        """(768-d pre-pooler CLS feature, 7 probs) — one forward instead of three."""
        if self.model is None or self.tokenizer is None:
            return None, None
        return self._forward(*self._encode(text))

    def encode_batch(self, texts):
        """int32 ids / mask [B,128] for a list of strings (the fast tokenizer from the same
        vocab when available: same ids as the reference's BertTokenizer, tests/test_tokenizer.py)."""
        if self._fast is None and self.tokenizer is not None and not getattr(self.tokenizer, 'is_fast', False):
            self._fast = _local_tokenizer(fast=True) or self.tokenizer
        return encode_batch(self._fast or self.tokenizer, texts)

    def predict_texts(self, texts) -> List[Dict]:
        """Batched `predict`: one tokenizer call and one BERT forward for all texts."""
        texts = list(texts)
        if self.model is None or self.tokenizer is None:
            return [self._keyword_heuristic(t) for t in texts]
        if not texts:
            return []
        ids, mask = self.encode_batch(texts)
        _, _, probs = self.model.checked('forward', engine.to_device(ids, self.device),
                                         engine.to_device(mask, self.device))
        probs = probs.cpu().numpy()
        return [self._as_dict(self.emotions, p) for p in probs]

    def predict_batch(self, ids, mask):
        """ids/mask: device int32 [B,128] -> (cls [B,768], logits [B,7], probs [B,7]). Asynchronous on the
        current stream, except on an fp32x3 handle: there it synchronizes and checks, so a batch outside
        the planes' range is answered by the fp32 engine (engine.HipModel.checked)."""
        if self.model is None:
            raise RuntimeError('text model not loaded')
        if self.model.precision == 'fp32x3':
            return self.model.checked('forward', ids, mask, True)
        return self.model.forward(ids, mask, check_ids=True)
