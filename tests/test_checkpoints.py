"""Real-checkpoint loaders: every format the reference's training scripts
write, read back through mec.checkpoints with non-executing loaders only, into the exact
arrays the C-ABI packer expects. CPU only."""
import os
import subprocess

import numpy as np
import pytest
import torch

from config import Config
from mec import checkpoints, synthetic as syn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY39 = '/opt/conda/bin/python3.9'


def _has_h5py39():
    if not os.path.exists(PY39):
        return False
    return subprocess.run([PY39, '-c', 'import h5py'], capture_output=True).returncode == 0


# Writes the Keras-2 legacy HDF5 layout of train_speech_model.py:55-90 (as TF 2.13's
# model.save does): auto-numbered layer names, weightless Activation/Dropout layers between.
_MAKE_H5 = r'''
import sys, numpy as np, h5py
src, dst = sys.argv[1], sys.argv[2]
w = dict(np.load(src))
names = []
with h5py.File(dst, 'w') as f:
    f.attrs['keras_version'] = b'2.13.1'
    g = f.create_group('model_weights')
    def layer(name, weights):
        names.append(name.encode())
        lg = g.create_group(name)
        lg.attrs['weight_names'] = [f'{name}/{k}:0'.encode() for k, _ in weights]
        for k, a in weights:
            lg.create_dataset(f'{name}/{k}:0', data=a)
    for i in range(5):
        dn = 'dense' if i == 0 else f'dense_{i + 3}'       # deliberately offset numbering
        bn = 'batch_normalization' if i == 0 else f'batch_normalization_{i + 3}'
        layer(dn, [('kernel', w[f'dense_{i}/kernel']), ('bias', w[f'dense_{i}/bias'])])
        layer(bn, [(k, w[f'batch_normalization_{i}/{k}']) for k in ('gamma', 'beta', 'moving_mean', 'moving_variance')])
        layer(f'activation_{i}', [])
        layer(f'dropout_{i}', [])
    layer('dense_99', [('kernel', w['dense_5/kernel']), ('bias', w['dense_5/bias'])])
    g.attrs['layer_names'] = names
'''


@pytest.mark.skipif(not _has_h5py39(), reason='needs /opt/conda/bin/python3.9 with h5py')
def test_speech_h5_converter_roundtrip(tmp_path):
    ref = syn.weights('speech', seed=77)
    src = tmp_path / 'w.npz'
    np.savez(src, **{k: v for k, v in ref.items() if not k.startswith('scaler/')})
    h5 = tmp_path / 'speech_model.h5'
    subprocess.run([PY39, '-c', _MAKE_H5, str(src), str(h5)], check=True)
    sc = tmp_path / 'speech_scaler.npz'
    np.savez(sc, mean_=ref['scaler/mean_'].astype(np.float64), scale_=ref['scaler/scale_'].astype(np.float64))
    out = tmp_path / 'speech_weights.npz'
    subprocess.run([PY39, os.path.join(ROOT, 'tools', 'convert_speech_h5.py'), str(h5), '--scaler', str(sc),
                    '-o', str(out)], check=True, capture_output=True)
    with np.load(out, allow_pickle=False) as z:
        got = {k: z[k] for k in z.files}
    assert set(got) == set(ref)
    for k in ref:
        assert np.array_equal(got[k], ref[k]), k


def test_resolve_precedence(monkeypatch):
    w = {'x': 1}
    assert checkpoints.resolve('speech', weights=w) is w
    monkeypatch.setattr(Config, 'SYNTHETIC_SEED', '5')
    a = checkpoints.resolve('speech')
    assert all(np.array_equal(a[k], syn.weights('speech', 5)[k]) for k in a)
    monkeypatch.setattr(Config, 'SYNTHETIC_SEED', None)
    monkeypatch.setattr(Config, 'SPEECH_MODEL_PATH', '/nonexistent/speech_model.h5')
    assert checkpoints.resolve('speech') is None  # reference: warning, model = None


def test_speech_npz_loader(tmp_path, monkeypatch):
    ref = syn.weights('speech', seed=3)
    np.savez(tmp_path / 'speech_weights.npz', **ref)
    monkeypatch.setattr(Config, 'SYNTHETIC_SEED', None)
    monkeypatch.setattr(Config, 'SPEECH_MODEL_PATH', str(tmp_path / 'speech_model.h5'))
    got = checkpoints.resolve('speech')
    assert list(got) == [n for n, *_ in syn.speech_spec()]
    assert all(np.array_equal(got[k], ref[k]) for k in ref)


def test_image_state_dict_loader(tmp_path, monkeypatch):
    """train_image_model.py:273 saves model.state_dict() to IMAGE_MODEL_PATH with .h5 -> .pt."""
    ref = syn.weights('image', seed=4)
    torch.save({k: torch.from_numpy(v) for k, v in ref.items()}, tmp_path / 'image_model.pt')
    monkeypatch.setattr(Config, 'SYNTHETIC_SEED', None)
    monkeypatch.setattr(Config, 'IMAGE_MODEL_PATH', str(tmp_path / 'image_model.h5'))
    got = checkpoints.resolve('image')
    assert all(np.array_equal(got[k], ref[k]) for k in ref)


def test_fusion_checkpoint_loader(tmp_path, monkeypatch):
    """train_fusion_model.py:609-618 saves {'model_state_dict', 'config', ...} to FUSION_MODEL_PATH
    with .pkl -> .pt; a config with other dimensions is rejected, not silently misread."""
    ref = syn.weights('fusion', seed=5)
    cfg = {'speech_dim': 64, 'text_dim': 768, 'image_dim': 512, 'num_classes': 7, 'hidden_dim': 256}
    sd = {k: torch.from_numpy(v) for k, v in ref.items()}
    torch.save({'model_state_dict': sd, 'config': cfg, 'epoch': 3}, tmp_path / 'fusion_model.pt')
    monkeypatch.setattr(Config, 'SYNTHETIC_SEED', None)
    monkeypatch.setattr(Config, 'FUSION_MODEL_PATH', str(tmp_path / 'fusion_model.pkl'))
    got = checkpoints.resolve('fusion')
    assert all(np.array_equal(got[k], ref[k]) for k in ref)
    torch.save({'model_state_dict': sd, 'config': dict(cfg, hidden_dim=128)}, tmp_path / 'fusion_model.pt')
    assert checkpoints.resolve('fusion') is None


def test_checkpoint_shape_mismatch_is_rejected(tmp_path, monkeypatch):
    ref = dict(syn.weights('speech', seed=3))
    ref['dense_0/kernel'] = ref['dense_0/kernel'][:, :100]
    np.savez(tmp_path / 'speech_weights.npz', **ref)
    monkeypatch.setattr(Config, 'SYNTHETIC_SEED', None)
    monkeypatch.setattr(Config, 'SPEECH_MODEL_PATH', str(tmp_path / 'speech_model.h5'))
    with pytest.raises(ValueError):
        checkpoints.load_checkpoint('speech')
    assert checkpoints.resolve('speech') is None


def test_text_save_pretrained_loaders(tmp_path, monkeypatch):
    """text_inference.py:40-41 loads BERT_MODEL_PATH/ as written by save_pretrained
    (train_text_model.py:221-222): model.safetensors (current HF default) or pytorch_model.bin."""
    from safetensors.numpy import save_file
    ref = syn.weights('text', seed=1234)
    monkeypatch.setattr(Config, 'SYNTHETIC_SEED', None)
    monkeypatch.setattr(Config, 'BERT_MODEL_PATH', str(tmp_path))
    save_file(dict(ref), str(tmp_path / 'model.safetensors'))
    got = checkpoints.resolve('text')
    assert list(got) == list(ref) and all(np.array_equal(got[k], ref[k]) for k in ref)
    os.remove(tmp_path / 'model.safetensors')
    small = {k: torch.from_numpy(v) for k, v in ref.items()}
    torch.save(small, tmp_path / 'pytorch_model.bin')
    got = checkpoints.resolve('text')
    assert all(np.array_equal(got[k], ref[k]) for k in ref)


class _RefConfig:
    """The reference's config.py attribute set for the hot path (config.py:39-65): no
    SYNTHETIC_SEED (INTEGRATION.md path A keeps the reference's own Config)."""
    SPEECH_MODEL_PATH = '/nonexistent/models/speech_model.h5'
    SPEECH_SCALER_PATH = '/nonexistent/models/speech_scaler.pkl'
    TEXT_MODEL_PATH = '/nonexistent/models/text_model.h5'
    IMAGE_MODEL_PATH = '/nonexistent/models/image_model.h5'
    FUSION_MODEL_PATH = '/nonexistent/models/fusion_model.pkl'
    BERT_MODEL_PATH = '/nonexistent/models/bert_model'
    EMOTIONS = ['happy', 'sad', 'angry', 'fear', 'disgust', 'surprise', 'neutral']
    NUM_EMOTIONS = 7
    SAMPLE_RATE = 22050
    AUDIO_DURATION = 3
    N_MFCC = 40
    MAX_TEXT_LENGTH = 128
    IMAGE_SIZE = (224, 224)


def test_inference_classes_under_reference_config(monkeypatch):
    """Every drop-in class constructs with the reference's Config (no SYNTHETIC_SEED) and no
    checkpoints: model = None and the heuristic fallbacks answer, as in the reference."""
    import importlib
    monkeypatch.delenv('MEC_SYNTHETIC_SEED', raising=False)
    mods = {n: importlib.import_module(f'inference.{n}') for n in
            ('speech_inference', 'text_inference', 'image_inference', 'multimodal_fusion')}
    monkeypatch.setattr(checkpoints, 'Config', _RefConfig)
    for m in mods.values():
        monkeypatch.setattr(m, 'Config', _RefConfig)
    s = mods['speech_inference'].SpeechInference()
    t = mods['text_inference'].TextInference()
    i = mods['image_inference'].ImageInference()
    assert s.model is None and t.model is None and i.model is None
    r = t.predict('I am so happy today')
    assert r['emotion'] in _RefConfig.EMOTIONS and len(r['all_probabilities']) == 7
    if torch.cuda.is_available():
        f = mods['multimodal_fusion'].MultimodalFusion()
        assert f.fuse_predictions(None, None, None)['emotion'] in _RefConfig.EMOTIONS
    else:  # its weighted average runs on the GPU: no GPU is a MecError, never an AttributeError
        from mec._lib import MecError
        with pytest.raises(MecError):
            mods['multimodal_fusion'].MultimodalFusion()
