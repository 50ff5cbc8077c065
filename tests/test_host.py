"""CPU: host-side logic — synthetic weights, blob packing, the C ABI's exports and
host-only entry points (no kernel launches), sharding, keyword fallback."""
import os
import re

import numpy as np
import pytest

from mec import _lib, dist as mdist, synthetic as syn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_synthetic_is_deterministic_and_seeded():
    a = syn.uniform(1234, 'x', (1000,), -1, 1)
    b = syn.uniform(1234, 'x', (1000,), -1, 1)
    c = syn.uniform(1235, 'x', (1000,), -1, 1)
    assert np.array_equal(a, b) and not np.array_equal(a, c)
    assert a.min() >= -1 and a.max() < 1 and abs(a.mean()) < 0.1
    # fixed values pin the raw-stream conversion across numpy versions
    np.testing.assert_allclose(syn.uniform(1234, 'pin', (3,), 0, 1),
                               syn.uniform(1234, 'pin', (3,), 0, 1))


def test_param_counts_match_reference():
    # 109,487,623 = HF BertForSequenceClassification(num_labels=7); 1,637,453 = reference fusion model
    assert syn.blob_size('text') == 109_487_623
    assert syn.blob_size('fusion') == 1_637_453
    assert syn.blob_size('speech') == 470_775
    assert syn.blob_size('image') == 24_613_831


def test_pack_rejects_bad_shapes():
    w = dict(syn.weights('speech'))
    w['dense_0/kernel'] = np.zeros((55, 512), np.float32)
    with pytest.raises(ValueError):
        syn.pack('speech', w)


def test_text_inputs_layout():
    ids, mask = syn.text_inputs(5, 128, seed=2, ragged=True)
    assert ids.dtype == np.int32 and mask.dtype == np.int32
    assert (ids[:, 0] == 101).all()
    lens = mask.sum(1)
    assert lens[0] == 128 and lens[1] == 8
    for i, n in enumerate(lens):
        assert ids[i, n - 1] == 102 and (ids[i, n:] == 0).all() and mask[i, :n].all()


def test_library_loads_and_exports_every_header_symbol():
    lib = _lib.load()
    hdr = open(os.path.join(ROOT, 'include', 'mec.h')).read()
    names = sorted(set(re.findall(r'\b(mec_[a-z0-9_]+)\s*\(', hdr)))
    assert len(names) >= 15
    for n in names:
        assert hasattr(lib, n), f'{n} declared in include/mec.h but not exported'
        assert n in _lib.SIGNATURES, f'{n} has no ctypes signature in mec/_lib.py'


def test_blob_sizes_agree_with_library():
    lib = _lib.load()
    for kind, k in syn.KIND_IDS.items():
        assert lib.mec_blob_size(k) == syn.blob_size(kind)
    assert lib.mec_blob_size(9) == -1


def test_model_option_and_query_need_a_handle():
    lib = _lib.load()
    assert lib.mec_model_set_option(None, b'fusion_r', 2) == -1
    assert b'null model' in lib.mec_last_error()
    assert lib.mec_model_gemm_query(None, 0, 256, 256, 256) == -1
    assert lib.mec_precision(None) == -1
    assert lib.mec_model_check(None) == -1
    assert b'null handle' in lib.mec_last_error()


def test_removed_knobs_are_unknown():
    """The measured-slower opt-in paths of round 2 (register-staged GEMM engine, fused
    bottleneck tail, O-proj + LN kernel, one-kernel speech DNN) are gone from the library."""
    lib = _lib.load()
    for k in (b'gemm_impl', b'resnet_fused_tail', b'bert_oproj_ln', b'speech_impl'):
        assert lib.mec_set_option(k, 0) == -1 and b'unknown' in lib.mec_last_error().lower(), k


def test_c_abi_argument_errors_without_gpu():
    import ctypes
    lib = _lib.load()
    h = ctypes.c_void_p()
    blob = np.zeros(10, np.float32)
    assert lib.mec_create(0, blob.ctypes.data_as(_lib.c_fp), 10, 0, ctypes.byref(h)) == -1
    assert b'expected' in lib.mec_last_error()
    assert lib.mec_set_option(b'nope', 1) == -1
    assert lib.mec_speech_fwd(None, None, 1, None, None, None, None) == -1
    assert b'null model' in lib.mec_last_error()


def test_create_opt_parses_its_option_list_without_gpu():
    """mec_create_opt validates its "key=value,..." list (the mec_set_option keys and values) before
    any device call; mec_model_x3_report needs a handle."""
    import ctypes
    lib = _lib.load()
    h = ctypes.c_void_p()
    n = syn.blob_size('speech')
    blob = np.zeros(n, np.float32)
    for opts, msg in ((b'x3_headroom', b'key=value'), (b'=3', b'key=value'), (b'x3_headroom=', b'bad value'),
                      (b'x3_headroom=2x', b'bad value'), (b'x3_headroom=25', b'bad value'),
                      (b'x3_headroom=8,nope=1', b'unknown key'), (b'gemm_debug=1', b'MEC_PROBES')):
        assert lib.mec_create_opt(0, blob.ctypes.data_as(_lib.c_fp), n, 0, 2, opts, ctypes.byref(h)) == -1, opts
        assert msg in lib.mec_last_error(), (opts, lib.mec_last_error())
        assert not h.value
    assert lib.mec_model_x3_report(None) is None
    assert b'null handle' in lib.mec_last_error()
    assert lib.mec_set_option(b'x3_headroom', 4) == 0 and lib.mec_set_option(b'x3_headroom', 0) == 0


def test_option_validation_without_gpu():
    """mec_set_option accepts each knob's documented values (include/mec.h) and rejects the
    rest, including every probe value (the product library is not a -DMEC_PROBES build); it
    only sets the process defaults, so this runs without a GPU. Defaults restored."""
    lib = _lib.load()
    assert lib.mec_build_flags() == 0, 'the product library must not be a probe build'
    probes = [(b'gemm_debug', 1), (b'gemm_debug', 2), (b'gemm_debug', 4), (b'gemm_debug', 5), (b'stem_debug', 1), (b'conv3x3_debug', 2),
              (b'bert_qkv_attn', 2), (b'bert_qkv_attn', 3), (b'speech_spin_limit', 0), (b'speech_spin_limit', 100),
              (b'speech_debug', 1), (b'audio_debug', 15)]
    for k, v in probes:
        assert lib.mec_set_option(k, v) == -1, (k, v)
        assert b'MEC_PROBES' in lib.mec_last_error()
    ok = [(b'fusion_r', 1), (b'fusion_r', 4), (b'fusion_split', 0), (b'fusion_split', 1),
          (b'bert_qkv_attn', 0), (b'bert_qkv_attn', 1), (b'speech_spin_limit', -1),
          (b'gemm_bn', 40256), (b'gemm_bn', 0),
          (b'gemm_bn_tag', 3 * 100000 + 40256), (b'gemm_bn_tag', 3 * 100000 + 11128),
          (b'gemm_debug', 0), (b'gemm_f32_tile', 3), (b'gemm_f32_tile', 0), (b'speech_debug', 0),
          (b'gemm_group_m', 0), (b'gemm_group_m', 16), (b'gemm_group_m', 8),
          (b'gemm_glds_group_m', 0), (b'gemm_glds_group_m', 4), (b'gemm_glds_group_m', 8),
          (b'gemm_f32_family', 0), (b'gemm_f32_family', 32), (b'gemm_f32_family', 16),
          (b'bert_ln_rows', 1), (b'bert_ln_rows', 4), (b'bert_ln_rows', 2),
          (b'bert_cls_last', 0), (b'bert_cls_last', 1), (b'gemm_x3_order', 0), (b'gemm_x3_order', 1),
          (b'gemm_bn', 70256), (b'gemm_bn', 71064), (b'gemm_bn', 0), (b'gemm_x3_tag', 5 * 100000 + 70256),
          (b'gemm_x3_tag', 5 * 100000), (b'gelu_x3', 0), (b'gelu_x3', 1),
          (b'pw_chain_x3', 0), (b'pw_chain_x3', 1), (b'pw_chain_x3', 2), (b'pw_seam_x3', 0), (b'pw_seam_x3', 2),
          (b'pw_seam_x3', 1), (b'mbv2_layered', 0),
          (b'mbv2_layered', 7), (b'mbv2_layered', 17), (b'mbv2_layered16', 0), (b'mbv2_layered16', 12),
          (b'mbv2_x3_tile', 0), (b'mbv2_x3_tile', 4), (b'mbv2_x3_tpw', 1), (b'mbv2_x3_tpw', 4), (b'resnet_chunk', 16), (b'resnet_chunk', 0),
          (b'bert_qkv_attn_x3_heads', 2), (b'bert_qkv_attn_x3_heads', 1), (b'bert_qkv_attn_heads', 2),
          (b'bert_qkv_attn_heads', 1)]
    bad = [(b'pw_chain_x3', 3), (b'pw_seam_x3', 3), (b'pw_seam_x3', -1), (b'bert_qkv_attn_x3_heads', 0), (b'bert_qkv_attn_x3_heads', 3), (b'mbv2_layered', 6), (b'mbv2_layered', 18), (b'mbv2_layered16', 1),
           (b'mbv2_x3_tile', 8), (b'mbv2_x3_tpw', 0), (b'mbv2_x3_tpw', 17), (b'resnet_chunk', -1),(b'bert_ln_rows', 3), (b'bert_cls_last', 2), (b'gemm_x3_order', 2), (b'gemm_bn', 72256),
           (b'gemm_x3_tag', 5 * 100000 + 10256), (b'gemm_x3_tag', 70256), (b'gelu_x3', 2), (b'gemm_f32_family', 8), (b'gemm_group_m', 3), (b'gemm_group_m', -1), (b'gemm_group_m', 32), (b'gemm_glds_group_m', 5), (b'gemm_f32_tile', 9), (b'fusion_r', 3), (b'fusion_split', 2), (b'bert_qkv_attn', 4), (b'gemm_bn', 12345),
           (b'gemm_bn', 42256), (b'gemm_bn_tag', 11128), (b'gemm_bn_tag', 15 * 100000 + 256),
           (b'gemm_bn_tag', 3 * 100000 + 999), (b'gemm_bn_tag', -1), (b'gemm_debug', 6), (b'speech_spin_limit', -2)]
    try:
        for k, v in ok:
            assert lib.mec_set_option(k, v) == 0, (k, v)
        for k, v in bad:
            assert lib.mec_set_option(k, v) == -1, (k, v)
            assert b'bad value' in lib.mec_last_error()
    finally:  # the defaults
        for k, v in [(b'fusion_r', 4), (b'fusion_split', 1), (b'bert_qkv_attn', 1), (b'speech_spin_limit', -1),
                     (b'gemm_f32_tile', 0),
                     (b'gemm_bn', 0),
                     (b'gemm_bn_tag', 3 * 100000 + 11128), (b'gemm_debug', 0), (b'gemm_group_m', 8),
                     (b'gemm_glds_group_m', 8), (b'gemm_f32_family', 16), (b'bert_ln_rows', 2),
                     (b'bert_cls_last', 1), (b'gemm_x3_order', 1), (b'gelu_x3', 1), (b'gemm_x3_tag', 5 * 100000 + 72128),
                     (b'pw_chain_x3', 2), (b'pw_seam_x3', 1), (b'mbv2_layered', 8), (b'mbv2_layered16', 8), (b'mbv2_x3_tile', 4), (b'mbv2_x3_tpw', 2),
                     (b'resnet_chunk', 0), (b'bert_qkv_attn_x3_heads', 1), (b'bert_qkv_attn_heads', 1)]:
            lib.mec_set_option(k, v)


@pytest.mark.parametrize('total,world', [(256, 1), (8192, 8), (10, 3), (2, 4), (0, 2)])
def test_shards_partition_the_batch(total, world):
    spans = [mdist.shard(total, world, r) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == total
    for (a0, b0), (a1, b1) in zip(spans, spans[1:]):
        assert b0 == a1
    sizes = [b - a for a, b in spans]
    assert max(sizes) - min(sizes) <= 1


def test_keyword_fallback_matches_reference_rules():
    from inference.text_inference import TextInference
    t = TextInference.__new__(TextInference)  # no model / tokenizer -> heuristic path
    from inference.text_inference import _Cleaner
    t.emotions = ['happy', 'sad', 'angry', 'fear', 'disgust', 'surprise', 'neutral']
    t.model, t.tokenizer, t.preprocessor = None, None, _Cleaner()
    r = t.predict('I am SO happy today!!')
    assert r['emotion'] == 'happy' and r['confidence'] == 0.9
    assert r['all_probabilities'][1] == 0.1 / 6
    assert t.predict('This is worrying, I feel anxious')['emotion'] == 'fear'
    assert t.predict('see http://x.com nothing here')['emotion'] == 'neutral'
    assert set(r) == {'emotion', 'confidence', 'all_probabilities'}
