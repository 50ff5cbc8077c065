"""Where a model's weights come from (the reference loads trained checkpoints per request).

resolve(kind, weights, seed) returns a name -> float32 array dict in the canonical order of
mec.synthetic.spec(kind), or None when nothing is available (the reference then runs its
heuristic fallback: inference/speech_inference.py:61-62, text_inference.py:73-74,
image_inference.py:105-106, multimodal_fusion.py:204-205). Order of precedence:
  1. an explicit `weights` dict;
  2. a synthetic seed (argument, or MEC_SYNTHETIC_SEED in the environment);
  3. the trained checkpoint at the reference's Config path (config.py:39-44):
       text    BERT_MODEL_PATH/ (HF save_pretrained: model.safetensors | pytorch_model.bin),
               text_inference.py:40-41, train_text_model.py:221-222
       image   IMAGE_MODEL_PATH with .h5 -> .pt (state_dict), image_inference.py:35-38,
               train_image_model.py:273 (image_mbv2: the same file holding a mobilenet_v2
               `base.features.*` / `base.classifier.*` state_dict)
       fusion  FUSION_MODEL_PATH with .pkl -> .pt ({'model_state_dict','config'}),
               multimodal_fusion.py:41-54, train_fusion_model.py:609-618
       speech  a Keras .h5 needs h5py/TensorFlow (absent): use speech_weights.npz, written by
               an offline converter (names = synthetic.speech_spec()), see INTEGRATION.md.
Checkpoints are read only with loaders that execute nothing from the file
(safetensors, torch.load(weights_only=True), numpy without pickles).
"""
from __future__ import annotations

import os

import numpy as np

from config import Config

from . import synthetic


def _conform(kind, sd):
    out = {}
    for name, shape, _, _ in synthetic.spec(kind):
        if name not in sd:
            raise KeyError(f'{kind} checkpoint is missing {name}')
        a = np.asarray(sd[name], dtype=np.float32)
        if tuple(a.shape) != tuple(shape):
            raise ValueError(f'{kind} checkpoint: {name} has shape {a.shape}, expected {shape}')
        out[name] = a
    return out


def _torch_load(path):
    import torch
    obj = torch.load(path, map_location='cpu', weights_only=True)
    return obj


def _to_np(d):
    return {k: (v.detach().cpu().float().numpy() if hasattr(v, 'detach') else np.asarray(v)) for k, v in d.items()}


def load_checkpoint(kind: str):
    if kind == 'text':
        d = Config.BERT_MODEL_PATH
        st = os.path.join(d, 'model.safetensors')
        if os.path.exists(st):
            from safetensors.numpy import load_file
            return _conform(kind, load_file(st))
        pt = os.path.join(d, 'pytorch_model.bin')
        return _conform(kind, _to_np(_torch_load(pt)))
    if kind in ('image', 'image_mbv2'):  # same file; the backbone is told by the state_dict keys
        return _conform(kind, _to_np(_torch_load(Config.IMAGE_MODEL_PATH.replace('.h5', '.pt'))))
    if kind == 'fusion':
        ck = _torch_load(Config.FUSION_MODEL_PATH.replace('.pkl', '.pt'))
        cfg = ck['config']
        want = {'speech_dim': 64, 'text_dim': 768, 'image_dim': 512, 'num_classes': 7, 'hidden_dim': 256}
        for k, v in want.items():
            if int(cfg.get(k, v)) != v:
                raise ValueError(f'fusion checkpoint config {k}={cfg.get(k)} unsupported (expected {v})')
        return _conform(kind, _to_np(ck['model_state_dict']))
    if kind == 'speech':
        p = os.path.join(os.path.dirname(Config.SPEECH_MODEL_PATH), 'speech_weights.npz')
        with np.load(p, allow_pickle=False) as z:
            return _conform(kind, {k: z[k] for k in z.files})
    raise ValueError(kind)


def precision(value=None) -> str:
    """The drop-in classes' arithmetic: an explicit argument, else Config.PRECISION / MEC_PRECISION,
    else 'fp32' (the reference's own; its config.py has no PRECISION)."""
    if value is not None:
        return value
    return getattr(Config, 'PRECISION', None) or os.environ.get('MEC_PRECISION') or 'fp32'


def resolve(kind: str, weights=None, seed=None):
    if weights is not None:
        return weights
    if seed is None:
        # the reference's own config.py (INTEGRATION.md path A) has no SYNTHETIC_SEED
        env = getattr(Config, 'SYNTHETIC_SEED', None) or os.environ.get('MEC_SYNTHETIC_SEED')
        if env not in (None, ''):
            seed = int(env)
    if seed is not None:
        return synthetic.weights(kind, int(seed))
    try:
        return load_checkpoint(kind)
    except Exception as e:  # reference: print a warning, model = None -> heuristic fallback
        print(f'Warning: Could not load {kind} model: {e}')
        return None
