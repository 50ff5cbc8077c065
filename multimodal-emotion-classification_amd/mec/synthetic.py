"""Deterministic synthetic weights and inputs (the reference ships no trained weights).

The reference loads trained checkpoints (inference/speech_inference.py:21-28,
inference/text_inference.py:40-41, inference/image_inference.py:35-38,
inference/multimodal_fusion.py:41-54) but none are in the repo (.gitignore:25-30),
so parity is defined on seeded synthetic weights.

Every tensor is drawn from numpy's PCG64 *raw* uint64 stream (version-stable,
unlike numpy's distribution samplers), seeded by SeedSequence([seed, crc32(name)]),
so any tensor can be regenerated independently and identically on any host.

Tensor names/shapes follow the reference's own layouts:
  speech  Keras Sequential of model_training/train_speech_model.py:55-90
          (Dense kernel [in,out]) + StandardScaler (speech_inference.py:66-67)
  text    HF BertForSequenceClassification state_dict (text_inference.py:41)
  image   ImageEmotionModel state_dict: torchvision resnet50 under `base.` with the
          2048->512->7 head (image_inference.py:55-65)
  image_mbv2  the same model on torchvision mobilenet_v2 (README.md:13): `base.features`
          + a 1280->512->7 `base.classifier` head (no reference code: parity unpinned)
  fusion  MultiModalFusionModel state_dict (multimodal_fusion.py:108-154)
"""
from __future__ import annotations

import functools
import zlib
from collections import OrderedDict

import numpy as np

NUM_CLASSES = 7

# ----------------------------------------------------------------------------- RNG


def _u01(seed: int, name: str, n: int) -> np.ndarray:
    ss = np.random.SeedSequence([int(seed) & 0xFFFFFFFF, zlib.crc32(name.encode())])
    raw = np.random.PCG64(ss).random_raw(n)
    return (raw >> np.uint64(40)).astype(np.float64) * (1.0 / 16777216.0)


def uniform(seed: int, name: str, shape, lo: float, hi: float) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    return (lo + (hi - lo) * _u01(seed, name, n)).astype(np.float32).reshape(shape)


def randint(seed: int, name: str, shape, lo: int, hi: int) -> np.ndarray:
    """Integers in [lo, hi) from the raw stream."""
    n = int(np.prod(shape))
    ss = np.random.SeedSequence([int(seed) & 0xFFFFFFFF, zlib.crc32(name.encode())])
    raw = np.random.PCG64(ss).random_raw(n)
    return (lo + (raw % np.uint64(hi - lo)).astype(np.int64)).reshape(shape)


# ----------------------------------------------------------------------------- specs
# Each spec entry: (name, shape, kind, arg)  kind in {'u' (±a), 'r' (lo,hi)}

SPEECH_DIMS = [56, 512, 512, 256, 128, 64]


def speech_spec():
    s = [('scaler/mean_', (56,), 'r', (-1.0, 1.0)),
         ('scaler/scale_', (56,), 'r', (0.5, 2.0))]
    for i in range(5):
        fi, fo = SPEECH_DIMS[i], SPEECH_DIMS[i + 1]
        a = float(np.sqrt(6.0 / (fi + fo)))  # glorot_uniform (Keras Dense default)
        s += [(f'dense_{i}/kernel', (fi, fo), 'u', a),
              (f'dense_{i}/bias', (fo,), 'u', 0.05),
              (f'batch_normalization_{i}/gamma', (fo,), 'r', (0.8, 1.2)),
              (f'batch_normalization_{i}/beta', (fo,), 'r', (-0.1, 0.1)),
              (f'batch_normalization_{i}/moving_mean', (fo,), 'r', (-0.1, 0.1)),
              (f'batch_normalization_{i}/moving_variance', (fo,), 'r', (0.5, 1.5))]
    a = 3.0 * float(np.sqrt(6.0 / (64 + 7)))  # scaled up: clear top-2 margins
    s += [('dense_5/kernel', (64, 7), 'u', a), ('dense_5/bias', (7,), 'u', 0.05)]
    return s


BERT_VOCAB, BERT_H, BERT_I, BERT_LAYERS, BERT_HEADS, BERT_MAXPOS = 30522, 768, 3072, 12, 12, 512


def text_spec():
    a = 0.02 * float(np.sqrt(3.0))  # uniform with std 0.02 (HF initializer_range)
    ln = lambda p: [(p + '.weight', (BERT_H,), 'r', (0.9, 1.1)), (p + '.bias', (BERT_H,), 'u', 0.05)]
    s = [('bert.embeddings.word_embeddings.weight', (BERT_VOCAB, BERT_H), 'u', a),
         ('bert.embeddings.position_embeddings.weight', (BERT_MAXPOS, BERT_H), 'u', a),
         ('bert.embeddings.token_type_embeddings.weight', (2, BERT_H), 'u', a)]
    s += ln('bert.embeddings.LayerNorm')
    for i in range(BERT_LAYERS):
        p = f'bert.encoder.layer.{i}.'
        for n in ('query', 'key', 'value'):
            s += [(p + f'attention.self.{n}.weight', (BERT_H, BERT_H), 'u', a),
                  (p + f'attention.self.{n}.bias', (BERT_H,), 'u', 0.02)]
        s += [(p + 'attention.output.dense.weight', (BERT_H, BERT_H), 'u', a),
              (p + 'attention.output.dense.bias', (BERT_H,), 'u', 0.02)]
        s += ln(p + 'attention.output.LayerNorm')
        s += [(p + 'intermediate.dense.weight', (BERT_I, BERT_H), 'u', a),
              (p + 'intermediate.dense.bias', (BERT_I,), 'u', 0.02),
              (p + 'output.dense.weight', (BERT_H, BERT_I), 'u', a),
              (p + 'output.dense.bias', (BERT_H,), 'u', 0.02)]
        s += ln(p + 'output.LayerNorm')
    s += [('bert.pooler.dense.weight', (BERT_H, BERT_H), 'u', a),
          ('bert.pooler.dense.bias', (BERT_H,), 'u', 0.02),
          ('classifier.weight', (NUM_CLASSES, BERT_H), 'u', 0.35),  # std 0.2: clear margins
          ('classifier.bias', (NUM_CLASSES,), 'u', 0.02)]
    return s


RESNET_LAYERS = [(64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)]  # (width, blocks, stride)


def image_spec():
    s = []

    def conv(name, co, ci, k):
        s.append((name, (co, ci, k, k), 'u', float(np.sqrt(6.0 / (ci * k * k)))))  # He-uniform

    def bn(name, c, gamma=(0.8, 1.2)):
        s.extend([(name + '.weight', (c,), 'r', gamma),
                  (name + '.bias', (c,), 'r', (-0.1, 0.1)),
                  (name + '.running_mean', (c,), 'r', (-0.1, 0.1)),
                  (name + '.running_var', (c,), 'r', (0.8, 1.2))])

    conv('base.conv1.weight', 64, 3, 7)
    bn('base.bn1', 64)
    cin = 64
    for li, (w, nb, st) in enumerate(RESNET_LAYERS):
        for b in range(nb):
            p = f'base.layer{li + 1}.{b}.'
            conv(p + 'conv1.weight', w, cin, 1); bn(p + 'bn1', w)
            conv(p + 'conv2.weight', w, w, 3); bn(p + 'bn2', w)
            conv(p + 'conv3.weight', 4 * w, w, 1); bn(p + 'bn3', 4 * w, gamma=(0.2, 0.4))
            if b == 0:
                conv(p + 'downsample.0.weight', 4 * w, cin, 1); bn(p + 'downsample.1', 4 * w)
            cin = 4 * w
    a1 = 1.0 / np.sqrt(2048.0)
    a2 = 3.0 / np.sqrt(512.0)
    s += [('base.fc.1.weight', (512, 2048), 'u', a1), ('base.fc.1.bias', (512,), 'u', a1),
          ('base.fc.4.weight', (NUM_CLASSES, 512), 'u', a2), ('base.fc.4.bias', (NUM_CLASSES,), 'u', 0.05)]
    return s


# MobileNetV2 (torchvision mobilenet_v2(weights=None), width 1.0): inverted-residual
# settings (t, c, n, s) and the same Dropout/Linear(.,512)/ReLU/Dropout/Linear(512,7) head the
# reference puts on ResNet50 (image_inference.py:59-65), here as base.classifier (README.md:13
# names MobileNetV2 as the image model; the reference ships no MobileNetV2 code).
MBV2_SETTINGS = [(1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1), (6, 160, 3, 2),
                 (6, 320, 1, 1)]
MBV2_LAST = 1280
MBV2_GAMMA = ((4.0, 8.0), (0.8, 1.2), (0.4, 0.8))  # BN gamma ranges: stem, expand / depthwise, projections


def mbv2_blocks():
    """[(t, cin, hidden, cout, stride)] for features[1..17]."""
    out, cin = [], 32
    for t, c, n, s in MBV2_SETTINGS:
        for i in range(n):
            out.append((t, cin, cin * t, c, s if i == 0 else 1))
            cin = c
    return out


def image_mbv2_spec():
    s = []

    def conv(name, co, ci, k, groups=1):
        s.append((name, (co, ci // groups, k, k), 'u', float(np.sqrt(6.0 / (ci // groups * k * k)))))

    def bn(name, c, gamma=(0.8, 1.2)):
        s.extend([(name + '.weight', (c,), 'r', gamma),
                  (name + '.bias', (c,), 'r', (-0.1, 0.1)),
                  (name + '.running_mean', (c,), 'r', (-0.1, 0.1)),
                  (name + '.running_var', (c,), 'r', (0.8, 1.2))])

    # BN scales (MBV2_GAMMA): every ReLU6 zeroes and saturates part of its inputs, yet the
    # net stays well conditioned (an f16 storage of every activation moves the probs by
    # < 1e-4 in fp32 emulation; larger gammas make the random net chaotic)
    stem, act, proj = MBV2_GAMMA
    conv('base.features.0.0.weight', 32, 3, 3); bn('base.features.0.1', 32, gamma=stem)
    for i, (t, cin, hid, cout, st) in enumerate(mbv2_blocks()):
        p = f'base.features.{i + 1}.conv.'
        if t == 1:
            conv(p + '0.0.weight', hid, hid, 3, groups=hid); bn(p + '0.1', hid, gamma=act)
            conv(p + '1.weight', cout, hid, 1); bn(p + '2', cout, gamma=proj)
        else:
            conv(p + '0.0.weight', hid, cin, 1); bn(p + '0.1', hid, gamma=act)
            conv(p + '1.0.weight', hid, hid, 3, groups=hid); bn(p + '1.1', hid, gamma=act)
            conv(p + '2.weight', cout, hid, 1); bn(p + '3', cout, gamma=proj)
    conv('base.features.18.0.weight', MBV2_LAST, 320, 1); bn('base.features.18.1', MBV2_LAST, gamma=act)
    a1 = 1.0 / np.sqrt(float(MBV2_LAST))
    a2 = 1.0 / np.sqrt(512.0)
    s += [('base.classifier.1.weight', (512, MBV2_LAST), 'u', a1), ('base.classifier.1.bias', (512,), 'u', a1),
          ('base.classifier.4.weight', (NUM_CLASSES, 512), 'u', a2),
          ('base.classifier.4.bias', (NUM_CLASSES,), 'u', 0.05)]
    return s


FUSION_HIDDEN = 256
FUSION_DIMS = {'speech': 64, 'text': 768, 'image': 512}


def fusion_spec():
    H, C = FUSION_HIDDEN, NUM_CLASSES
    s = []

    def lin(name, o, i, scale=1.0):
        a = 1.0 / np.sqrt(i)
        s.extend([(name + '.weight', (o, i), 'u', float(scale * a)), (name + '.bias', (o,), 'u', float(a))])

    def ln(name, c):
        s.extend([(name + '.weight', (c,), 'r', (0.9, 1.1)), (name + '.bias', (c,), 'u', 0.05)])

    for m in ('speech', 'text', 'image'):
        lin(f'{m}_proj.0', H, FUSION_DIMS[m]); ln(f'{m}_proj.1', H)
    for m in ('speech', 'text', 'image'):
        p = f'cross_attn_{m}.'
        s.append((p + 'attention.in_proj_weight', (3 * H, H), 'u', float(np.sqrt(6.0 / (4 * H)))))
        s.append((p + 'attention.in_proj_bias', (3 * H,), 'u', 0.02))
        s.append((p + 'attention.out_proj.weight', (H, H), 'u', float(1.0 / np.sqrt(H))))
        s.append((p + 'attention.out_proj.bias', (H,), 'u', 0.02))
        ln(p + 'norm', H)
    for j in range(3):
        lin(f'attention_fusion.projections.{j}.0', H, H); ln(f'attention_fusion.projections.{j}.1', H)
    lin('attention_fusion.attention.0', H, 3 * H)
    lin('attention_fusion.attention.2', 3, H)
    lin('decision_weights.0', 64, 3 * C)
    lin('decision_weights.2', 3, 64)
    lin('classifier.0', H, H + C); ln('classifier.1', H)
    lin('classifier.4', H // 2, H)
    lin('classifier.7', C, H // 2, scale=3.0)  # clear top-2 margins
    return s


SPECS = {'speech': speech_spec, 'text': text_spec, 'image': image_spec, 'fusion': fusion_spec,
         'image_mbv2': image_mbv2_spec}
KIND_IDS = {'speech': 0, 'text': 1, 'image': 2, 'fusion': 3, 'image_mbv2': 4}


def spec(kind: str):
    return SPECS[kind]()


@functools.lru_cache(maxsize=8)
def _weights_cached(kind: str, seed: int):
    out = OrderedDict()
    for name, shape, k, arg in spec(kind):
        if k == 'u':
            out[name] = uniform(seed, f'{kind}/{name}', shape, -arg, arg)
        else:
            out[name] = uniform(seed, f'{kind}/{name}', shape, arg[0], arg[1])
    return out


def weights(kind: str, seed: int = 1234) -> "OrderedDict[str, np.ndarray]":
    """Seeded weights for `kind` as an ordered name -> float32 array dict (read-only views)."""
    return _weights_cached(kind, int(seed))


def pack(kind: str, w) -> np.ndarray:
    """Flatten a weight dict into the canonical host blob consumed by mec_create()."""
    parts = []
    for name, shape, _, _ in spec(kind):
        a = np.asarray(w[name], dtype=np.float32)
        if tuple(a.shape) != tuple(shape):
            raise ValueError(f'{kind}: tensor {name} has shape {a.shape}, expected {shape}')
        parts.append(a.reshape(-1))
    return np.ascontiguousarray(np.concatenate(parts))


def blob_size(kind: str) -> int:
    return int(sum(int(np.prod(sh)) for _, sh, _, _ in spec(kind)))


# ----------------------------------------------------------------------------- inputs


def speech_inputs(B: int, seed: int = 0, wseed: int = 1234) -> np.ndarray:
    """Raw (pre-scaler) 56-d feature vectors: mean_ + scale_ * U(-1.7, 1.7)."""
    w = weights('speech', wseed)
    z = uniform(seed, 'in/speech', (B, 56), -1.7, 1.7)
    return (w['scaler/mean_'][None] + w['scaler/scale_'][None] * z).astype(np.float32)


def text_inputs(B: int, L: int = 128, seed: int = 0, ragged: bool = False):
    """Token ids [B,L] int32 + attention mask [B,L] int32.

    [CLS]=101 at 0, [SEP]=102 at len-1, ids U{1000..30521} between, 0 padding
    (padding='max_length', text_inference.py:78-85). ragged=False: every row full.
    """
    ids = randint(seed, 'in/text/ids', (B, L), 1000, BERT_VOCAB).astype(np.int32)
    if ragged:
        lens = randint(seed, 'in/text/len', (B,), 8, L + 1).astype(np.int64)
        if B > 0:
            lens[0] = L
        if B > 1:
            lens[1] = 8
    else:
        lens = np.full((B,), L, dtype=np.int64)
    mask = (np.arange(L)[None, :] < lens[:, None]).astype(np.int32)
    ids[:, 0] = 101
    ids[np.arange(B), lens - 1] = 102
    ids[mask == 0] = 0
    return ids, mask


def image_inputs(B: int, seed: int = 0) -> np.ndarray:
    """u8 grayscale FER2013-shaped faces [B,48,48] ~ U{0..255}."""
    return randint(seed, 'in/image', (B, 48, 48), 0, 256).astype(np.uint8)
