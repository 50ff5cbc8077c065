"""CPU: the oracle against the golden fixtures made from the reference's own code / the
third-party classes it calls (tests/golden/make_golden.py). Pins the oracle before it is
trusted as the checker of the HIP path."""
import numpy as np

from mec import synthetic as syn
from oracle import fusion as o_f, image as o_i, resize as o_r, speech as o_s, text as o_t


def test_resize_bit_exact_vs_pil(golden):
    g = golden('image_resize.npz')
    out = o_r.resize_bilinear_u8(g['gray'])
    assert out.dtype == np.uint8 and out.shape == g['resized'].shape
    assert np.array_equal(out, g['resized'])


def test_resize_taps_are_pillow_fixed_point():
    xmin, n, kk = o_r.coeffs(48, 224)
    assert (n >= 1).all() and (n <= 3).all()
    # every output pixel's taps sum to 2^22 within the per-tap rounding (Pillow normalize_coeffs_8bpc)
    s = kk.sum(1)
    assert np.all(np.abs(s - (1 << 22)) <= 2)


def test_fusion_oracle_vs_reference_class(golden):
    g = golden('fusion.npz')
    w = syn.weights('fusion', int(g['wseed']))
    out = o_f.forward(w, g['s_feat'], g['t_feat'], g['i_feat'], g['s_pred'], g['t_pred'], g['i_pred'])
    for name, got in zip(('logits', 'probs', 'attn_w', 'dec_w'), out):
        assert np.abs(got - g[name]).max() < 1e-6, name


def test_weighted_average_vs_reference(golden):
    g = golden('fusion.npz')
    for row, (idx, hs, ht, hi) in enumerate(g['wavg_cases']):
        got = o_f.fuse_predictions(g['s_pred'][idx].tolist() if hs else None,
                                   g['t_pred'][idx].tolist() if ht else None,
                                   g['i_pred'][idx].tolist() if hi else None)
        np.testing.assert_array_equal(got, g['wavg'][row])
    np.testing.assert_array_equal(o_f.fuse_predictions(None, None, None), g['wavg_zero'])


def test_fusion_dict_golden_shape(golden):
    g = golden('fusion.npz')
    assert str(g['dict0_emotion']) in ['happy', 'sad', 'angry', 'fear', 'disgust', 'surprise', 'neutral']
    assert g['dict0_probs'].shape == (7,) and g['dict0_attn'].shape == (3,) and g['dict0_dec'].shape == (3,)
    np.testing.assert_allclose(g['dict0_probs'], g['probs'][0], atol=1e-7)


def test_text_oracle_vs_hf_bert(golden):
    g = golden('text_bert.npz')
    cls, logits, probs = o_t.forward(syn.weights('text', int(g['wseed'])), g['ids'], g['mask'])
    assert np.abs(cls - g['cls']).max() < 1e-4
    assert np.abs(logits - g['logits']).max() < 1e-4
    assert np.abs(probs - g['probs']).max() < 1e-5


def test_speech_oracle_fixture(golden):
    g = golden('speech.npz')
    f, l, p = o_s.forward(syn.weights('speech', int(g['wseed'])), g['x'])
    assert np.abs(f - g['feat']).max() < 1e-5
    assert np.abs(p - g['probs']).max() < 1e-6


def test_image_oracle_fixture(golden):
    g = golden('image_full.npz')
    f, l, p = o_i.forward(syn.weights('image', int(g['wseed'])), g['gray'])
    assert np.abs(p - g['probs']).max() < 1e-5
    assert np.array_equal(p.argmax(1), g['probs'].argmax(1))


def test_image_oracle_rgb_equals_gray_when_channels_equal():
    w = syn.weights('image')
    gray = syn.image_inputs(1, seed=4)
    resized = o_r.resize_bilinear_u8(gray)
    a = o_i.forward_resized(w, resized)
    b = o_i.forward_resized(w, np.repeat(resized[..., None], 3, axis=-1))
    assert np.abs(a[2] - b[2]).max() < 1e-6
