"""GPU: the drop-in classes end to end, as app.py drives them.

1. MultimodalFusion.predict_multimodal(audio_path, text, image_path) with all three
   modalities: the attention-fusion branch (inference/multimodal_fusion.py:244-287 -> :269-278
   extract_features x3 -> fuse_with_attention :201-242), with a real WordPiece tokenizer on
   TextInference (text_inference.py:78-85; a synthetic vocab, no BERT vocab exists offline),
   load_audio stubbed with seeded waveforms (librosa is absent; the features run on the GPU),
   and a PNG face. Every dict ('speech', 'text', 'image', 'fusion' with attention_weights and
   decision_weights) against the oracle chain; TextInference.predict(str) against o_t on the
   ids the reference's own tokenizer class (4.30's pure-Python BertTokenizer) produces.
2. The same flow with every model read from checkpoint FILES in the reference's formats at the
   Config paths (image_inference.py:35-40, text_inference.py:40-43,
   multimodal_fusion.py:41-56, speech_inference.py:21-28): seeded weights written as HF
   model.safetensors + vocab.txt, the image_model.pt state_dict, the fusion
   {'model_state_dict', 'config'} .pt and speech_weights.npz (the .h5 converter's output).
"""
import types

import numpy as np
import pytest
import torch

from config import Config
from mec import synthetic as syn
from oracle import audio as oa, fusion as o_f, image as o_i, speech as o_s, text as o_t
from test_tokenizer import PUNCT, SUB, WORDS

pytestmark = pytest.mark.gpu
EMO = Config.EMOTIONS
TEXTS = ['I am so happy today!', 'This is the WORST day ever... not sure how I feel about it']
# per precision: text / image probs bar against the oracle (north_star 1e-3; fp32 path 1e-5).
# Speech and the fused output carry the GPU audio features' float32 reassociation (MFCC within
# 5e-4 dB of the librosa restatement, tests/test_gpu_audio.py): 1e-4.
TOL = {'fp32': 1e-5, 'f16': 1e-3}
SPEECH_TOL = 1e-4


def _write_vocab(d):
    letters = [chr(c) for c in range(ord('a'), ord('z') + 1)]
    toks = ['[PAD]'] + [f'[unused{i}]' for i in range(5)] + ['[UNK]', '[CLS]', '[SEP]', '[MASK]']
    toks += PUNCT + letters + ['##' + c for c in letters] + WORDS + SUB + ['0', '1', '2', '##0', '##1']
    (d / 'vocab.txt').write_text('\n'.join(dict.fromkeys(toks)) + '\n')
    return d / 'vocab.txt'


def _legacy_tokenizer(vocab_file):
    from transformers.models.bert.tokenization_bert_legacy import BertTokenizerLegacy
    return BertTokenizerLegacy(str(vocab_file))  # transformers 4.30's BertTokenizer


def _encode(tok, text):
    enc = tok(text, add_special_tokens=True, max_length=Config.MAX_TEXT_LENGTH, padding='max_length',
              truncation=True, return_tensors='np')
    return enc['input_ids'].astype(np.int32), enc['attention_mask'].astype(np.int32)


def _check_dict(name, d, probs_ref, tol):
    assert set(d) >= {'emotion', 'confidence', 'all_probabilities'}, name
    assert isinstance(d['emotion'], str) and isinstance(d['confidence'], float)
    assert isinstance(d['all_probabilities'], list) and len(d['all_probabilities']) == 7
    assert all(isinstance(v, float) for v in d['all_probabilities'])
    err = float(np.abs(np.array(d['all_probabilities']) - probs_ref).max())
    print(f'{name}: probs max|d| {err:.3g}')
    assert d['emotion'] == EMO[int(np.argmax(probs_ref))], name
    assert err <= tol, f'{name}: {err}'
    assert d['confidence'] == max(d['all_probabilities'])


def _stub_audio(monkeypatch, waves):
    from inference import speech_inference as si
    stub = types.SimpleNamespace(load_audio=lambda path, sr=oa.SR, duration=oa.DURATION: (waves[path], oa.SR))
    monkeypatch.setattr(si, '_preprocessing', lambda: stub)


def _run_three(fusion, tmp_path, monkeypatch, wseed, precision, vocab_file):
    """predict_multimodal on two (audio, text, face) requests vs the oracle chain with the
    weights of seed `wseed`."""
    from PIL import Image
    waves = {f'clip{i}.wav': w for i, w in enumerate(oa.synthetic_clips(2, seed=51))}
    _stub_audio(monkeypatch, waves)
    faces = syn.image_inputs(2, seed=52)
    tok = _legacy_tokenizer(vocab_file)  # the expected ids: the reference's tokenizer class
    w = {k: syn.weights(k, wseed) for k in ('speech', 'text', 'image', 'fusion')}
    ref_feat, _ = oa.features_batch(np.stack(list(waves.values())))
    tol = TOL[precision]
    for i, (clip, text) in enumerate(zip(waves, TEXTS)):
        p = tmp_path / f'face{i}.png'
        Image.fromarray(faces[i], 'L').save(p)
        res = fusion.predict_multimodal(audio_path=clip, text=text, image_path=str(p))
        assert set(res) == {'speech', 'text', 'image', 'fusion'}
        sf, _, sp = o_s.forward(w['speech'], ref_feat[i:i + 1])
        ids, mask = _encode(tok, text)
        tf, _, tp = o_t.forward(w['text'], ids, mask)
        imf, _, ip = o_i.forward(w['image'], faces[i:i + 1])
        _, fp, aw, dw = o_f.forward(w['fusion'], sf, tf, imf, sp, tp, ip)
        _check_dict(f'{precision} request {i} speech', res['speech'], sp[0], SPEECH_TOL)
        _check_dict(f'{precision} request {i} text', res['text'], tp[0], tol)
        _check_dict(f'{precision} request {i} image', res['image'], ip[0], tol)
        _check_dict(f'{precision} request {i} fusion (attention branch)', res['fusion'], fp[0], max(tol, SPEECH_TOL))
        for key, ref in (('attention_weights', aw[0]), ('decision_weights', dw[0])):
            d = res['fusion'][key]
            assert list(d) == ['speech', 'text', 'image'] and all(isinstance(v, float) for v in d.values())
            assert np.abs(np.array(list(d.values())) - ref).max() <= max(tol, SPEECH_TOL), key
        # TextInference.predict(str) alone (text_inference.py:72-104)
        _check_dict(f'{precision} TextInference.predict #{i}', fusion.text_inference.predict(text), tp[0], tol)
        cls, p7 = fusion.text_inference.extract_features(text)
        assert cls.shape == (768,) and np.abs(cls - tf[0]).max() <= (1e-4 if precision == 'fp32' else 1e-2)
        assert np.abs(p7 - tp[0]).max() <= tol
    # the batched text front-end over both texts
    got = fusion.text_inference.predict_texts(TEXTS)
    ids, mask = zip(*(_encode(tok, t) for t in TEXTS))
    _, _, tpb = o_t.forward(w['text'], np.concatenate(ids), np.concatenate(mask))
    for i, d in enumerate(got):
        _check_dict(f'{precision} predict_texts #{i}', d, tpb[i], tol)


@pytest.mark.parametrize('precision', ['fp32', 'f16'])
def test_predict_multimodal_three_modalities(dev, tmp_path, monkeypatch, precision):
    from inference.multimodal_fusion import MultimodalFusion
    fusion = MultimodalFusion(seed=1234, device=dev, precision=precision)
    assert fusion.text_inference.model.precision == precision
    vocab = _write_vocab(tmp_path)
    fusion.text_inference.tokenizer = _legacy_tokenizer(vocab)
    _run_three(fusion, tmp_path, monkeypatch, 1234, precision, vocab)


def test_predict_multimodal_from_checkpoint_files(dev, tmp_path, monkeypatch):
    """Every model from files in the reference's checkpoint formats at the Config paths (no
    seed anywhere): the loaders feed the HIP path, whose outputs match the oracle run on the
    weights that were written."""
    from safetensors.numpy import save_file
    from inference import multimodal_fusion as mf
    wseed = 77
    models = tmp_path / 'models'
    bert = models / 'bert_model'
    bert.mkdir(parents=True)
    vocab = _write_vocab(bert)  # save_pretrained writes the tokenizer beside the weights
    save_file(dict(syn.weights('text', wseed)), str(bert / 'model.safetensors'))
    torch.save({k: torch.from_numpy(v) for k, v in syn.weights('image', wseed).items()}, models / 'image_model.pt')
    cfg = {'speech_dim': 64, 'text_dim': 768, 'image_dim': 512, 'num_classes': 7, 'hidden_dim': 256}
    torch.save({'model_state_dict': {k: torch.from_numpy(v) for k, v in syn.weights('fusion', wseed).items()},
                'config': cfg, 'epoch': 1}, models / 'fusion_model.pt')
    np.savez(models / 'speech_weights.npz', **syn.weights('speech', wseed))
    monkeypatch.delenv('MEC_SYNTHETIC_SEED', raising=False)
    monkeypatch.setattr(Config, 'SYNTHETIC_SEED', None)
    monkeypatch.setattr(Config, 'BERT_MODEL_PATH', str(bert))
    monkeypatch.setattr(Config, 'IMAGE_MODEL_PATH', str(models / 'image_model.h5'))
    monkeypatch.setattr(Config, 'FUSION_MODEL_PATH', str(models / 'fusion_model.pkl'))
    monkeypatch.setattr(Config, 'SPEECH_MODEL_PATH', str(models / 'speech_model.h5'))
    fusion = mf.MultimodalFusion(device=dev)
    assert fusion.fusion_model is not None and fusion.text_inference.tokenizer is not None
    assert all(o.model is not None for o in (fusion.speech_inference, fusion.text_inference, fusion.image_inference))
    _run_three(fusion, tmp_path, monkeypatch, wseed, 'fp32', vocab)
