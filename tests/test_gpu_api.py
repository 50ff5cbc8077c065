"""GPU: the drop-in boundary — the reference's classes/methods/result dicts, run through
the HIP path, against the oracle and the golden dict from the reference's own
fuse_with_attention."""
import numpy as np
import pytest

from mec import synthetic as syn
from oracle import fusion as o_f, image as o_i, speech as o_s, text as o_t

pytestmark = pytest.mark.gpu
EMO = ['happy', 'sad', 'angry', 'fear', 'disgust', 'surprise', 'neutral']


def _check_dict(d, probs_ref, tol):
    assert set(d) >= {'emotion', 'confidence', 'all_probabilities'}
    assert isinstance(d['emotion'], str) and isinstance(d['confidence'], float)
    assert isinstance(d['all_probabilities'], list) and len(d['all_probabilities']) == 7
    assert all(isinstance(v, float) for v in d['all_probabilities'])
    assert d['emotion'] == EMO[int(np.argmax(probs_ref))]
    assert np.abs(np.array(d['all_probabilities']) - probs_ref).max() < tol


@pytest.fixture(scope='module')
def fusion(dev):
    from inference.multimodal_fusion import MultimodalFusion
    return MultimodalFusion(seed=1234, device=dev)


def test_speech_dict(fusion):
    x = syn.speech_inputs(3, seed=9)
    _, _, rp = o_s.forward(syn.weights('speech'), x)
    for i in range(3):
        _check_dict(fusion.speech_inference.predict_features(x[i]), rp[i], 1e-5)


def test_text_dict_from_ids(fusion):
    ids, mask = syn.text_inputs(2, 128, seed=9, ragged=True)
    _, _, rp = o_t.forward(syn.weights('text'), ids, mask)
    for i in range(2):
        _check_dict(fusion.text_inference.predict_ids(ids[i], mask[i]), rp[i], 1e-3)


def test_text_without_tokenizer_uses_keyword_fallback(fusion):
    r = fusion.text_inference.predict('what a wonderful, happy day')
    assert r['emotion'] == 'happy' and r['confidence'] == 0.9


def test_image_file_paths(fusion, tmp_path):
    from PIL import Image
    w = syn.weights('image')
    gray = syn.image_inputs(1, seed=21)[0]
    p = tmp_path / 'face.png'
    Image.fromarray(gray, 'L').save(p)
    _, _, rp = o_i.forward(w, gray[None])
    _check_dict(fusion.image_inference.predict(str(p)), rp[0], 1e-3)
    # non-48x48 grayscale: PIL resize on host, gray stem on GPU
    g2 = syn.image_inputs(1, seed=22)[0].repeat(2, axis=0)[:80, :].repeat(2, axis=1)[:, :64]
    p2 = tmp_path / 'gray.png'
    Image.fromarray(np.ascontiguousarray(g2), 'L').save(p2)
    r2 = np.asarray(Image.open(p2).convert('RGB').resize((224, 224), Image.BILINEAR))[..., 0]
    _, _, rp2 = o_i.forward_resized(w, r2[None])
    _check_dict(fusion.image_inference.predict(str(p2)), rp2[0], 1e-3)
    # colour image: RGB stem (K = 256)
    rgb = np.stack([syn.image_inputs(1, seed=30 + c)[0] for c in range(3)], -1)
    p3 = tmp_path / 'rgb.png'
    Image.fromarray(rgb, 'RGB').save(p3)
    r3 = np.asarray(Image.open(p3).convert('RGB').resize((224, 224), Image.BILINEAR))
    _, _, rp3 = o_i.forward_resized(w, r3[None])
    _check_dict(fusion.image_inference.predict(str(p3)), rp3[0], 1e-3)
    feat, probs = fusion.image_inference.extract_features(str(p3))
    assert feat.shape == (512,) and probs.shape == (7,)


def test_fuse_with_attention_matches_reference_dict(fusion, golden):
    g = golden('fusion.npz')
    d = fusion.fuse_with_attention(g['s_feat'][0], g['t_feat'][0], g['i_feat'][0],
                                   g['s_pred'][0], g['t_pred'][0], g['i_pred'][0])
    assert d['emotion'] == str(g['dict0_emotion'])
    assert abs(d['confidence'] - float(g['dict0_conf'])) < 1e-5
    np.testing.assert_allclose(d['all_probabilities'], g['dict0_probs'], atol=1e-5)
    assert list(d['attention_weights']) == ['speech', 'text', 'image']
    np.testing.assert_allclose([d['attention_weights'][k] for k in ('speech', 'text', 'image')],
                               g['dict0_attn'], atol=1e-5)
    np.testing.assert_allclose([d['decision_weights'][k] for k in ('speech', 'text', 'image')],
                               g['dict0_dec'], atol=1e-5)


def test_fuse_predictions_heuristic_floats_bit_exact(fusion):
    heur = (np.ones(7) * (0.1 / 6))
    heur[6] = 0.9
    s = heur.tolist()
    t = syn.uniform(3, 'api/t', (7,), 0, 1).astype(np.float64).tolist()
    for args in ((s, t, None), (s, None, None), (None, t, s), (None, None, None)):
        d = fusion.fuse_predictions(*args)
        ref = o_f.fuse_predictions(*args)
        assert d['all_probabilities'] == ref.tolist()
        assert d['emotion'] == EMO[int(np.argmax(ref))]


def test_predict_multimodal_image_and_text(fusion, tmp_path):
    from PIL import Image
    gray = syn.image_inputs(1, seed=23)[0]
    p = tmp_path / 'f.png'
    Image.fromarray(gray, 'L').save(p)
    res = fusion.predict_multimodal(text='I am so angry', image_path=str(p))
    assert set(res) == {'text', 'image', 'fusion'}
    ref = o_f.fuse_predictions(None, res['text']['all_probabilities'], res['image']['all_probabilities'])
    assert res['fusion']['all_probabilities'] == ref.tolist()


def test_predict_batch_matches_pipeline(fusion, dev):
    from mec import engine
    B = 4
    x = engine.to_device(syn.speech_inputs(B, seed=5), dev)
    ids, mask = syn.text_inputs(B, 128, seed=5, ragged=True)
    gray = engine.to_device(syn.image_inputs(B, seed=5), dev)
    out = fusion.predict_batch(x, engine.to_device(ids, dev), engine.to_device(mask, dev), gray)
    fl, fp, aw, dw = [t.cpu().numpy() for t in out['fusion']]
    s, t_, i = [[a.cpu().numpy() for a in out[m]] for m in ('speech', 'text', 'image')]
    ref = o_f.forward(syn.weights('fusion'), s[0], t_[0], i[0], s[2], t_[2], i[2])
    assert np.abs(fp - ref[1]).max() < 1e-5


def test_speech_predict_from_file_runs_gpu_features(fusion, monkeypatch):
    """SpeechInference.predict(path): load_audio (the reference's preprocessing/, stubbed here:
    librosa is absent) -> GPU features (csrc/audio.hip) -> GPU DNN, against the oracle chain
    (preprocess_audio restated -> DNN restated); inference/speech_inference.py:60-77."""
    import types
    from inference import speech_inference as si
    from oracle import audio as oa
    wave = oa.synthetic_clips(2, seed=44)
    stub = types.SimpleNamespace(load_audio=lambda path, sr=oa.SR, duration=oa.DURATION: (wave[int(path)], oa.SR))
    monkeypatch.setattr(si, '_preprocessing', lambda: stub)
    ref_feat, _ = oa.features_batch(wave)
    _, _, rp = o_s.forward(syn.weights('speech'), ref_feat)
    for i in range(2):
        _check_dict(fusion.speech_inference.predict(str(i)), rp[i], 1e-4)
        f64, p7 = fusion.speech_inference.extract_features(str(i))
        assert f64.shape == (64,) and np.abs(p7 - rp[i]).max() < 1e-4


def test_text_out_of_range_ids_raise(fusion, dev):
    """nn.Embedding raises for ids outside the vocabulary; so do the drop-in's id entry points
    (the batched hot path skips the check and the kernel clamps)."""
    import torch
    ids, mask = syn.text_inputs(1, 128, seed=3)
    bad = ids.copy()
    bad[0, 5] = 30522
    with pytest.raises(ValueError):
        fusion.text_inference.predict_ids(bad[0], mask[0])
    neg = ids.copy()
    neg[0, 7] = -1
    with pytest.raises(ValueError):
        fusion.text_inference.predict_batch(torch.from_numpy(neg).to(dev), torch.from_numpy(mask).to(dev))
