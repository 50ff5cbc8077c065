"""Batched text front-end vs the reference's tokenizer call.

The reference encodes one string at a time with transformers' BertTokenizer
(text_inference.py:78-85), transformers==4.30.0 (requirements.txt:16): the pure-Python
BasicTokenizer + WordpieceTokenizer. transformers 5.15 (installed) keeps that
implementation as BertTokenizerLegacy, while its BertTokenizer is Rust-backed. No BERT
vocab exists offline, so both are built from a synthetic WordPiece vocab written here: the
pure-Python tokenizer per text (the oracle), and our `encode_batch` with
BertTokenizerFast over the whole batch. Parity of the ids/mask is exact. CPU only."""
import numpy as np
import pytest

from config import Config
from inference.text_inference import TextInference, encode_batch

WORDS = ['i', 'am', 'so', 'happy', 'sad', 'today', 'this', 'is', 'the', 'worst', 'day', 'ever', 'what', 'a',
         'wonderful', 'surprise', 'angry', 'fear', 'of', 'dark', 'not', 'sure', 'how', 'feel', 'about', 'it', 'un',
         'believ', 'able', 'love', 'hate', 'you', 'we', 'they', 'run', 'running']
SUB = ['##s', '##ing', '##ed', '##able', '##ly', '##er', '##est', '##y', '##n', '##d', '##e', '##a']
PUNCT = list('.,!?\'"-:;()')


@pytest.fixture(scope='module')
def vocab_dir(tmp_path_factory):
    d = tmp_path_factory.mktemp('bert_vocab')
    letters = [chr(c) for c in range(ord('a'), ord('z') + 1)]
    toks = ['[PAD]'] + [f'[unused{i}]' for i in range(5)] + ['[UNK]', '[CLS]', '[SEP]', '[MASK]']
    toks += PUNCT + letters + ['##' + c for c in letters] + WORDS + SUB + ['0', '1', '2', '##0', '##1']
    (d / 'vocab.txt').write_text('\n'.join(dict.fromkeys(toks)) + '\n')
    return d


TEXTS = [
    'I am so happy today!',
    'This is the WORST day ever...',
    'what a wonderful surprise',
    '',
    'unbelievable!!! running, runs, ran?',
    'Fear of the dark; not sure how I feel about it.',
    'émotions naïve café — ünïcödé',
    'http://example.com/x?y=1 lol 2024',
    ' '.join(['love'] * 200),                       # truncation at 128
    'a ' * 126 + 'b',                               # exactly at the limit after [CLS]/[SEP]
]


def test_batched_fast_encoding_matches_reference_tokenizer(vocab_dir):
    from transformers import BertTokenizerFast
    from transformers.models.bert.tokenization_bert_legacy import BertTokenizerLegacy
    slow = BertTokenizerLegacy(str(vocab_dir / 'vocab.txt'))    # 4.30's pure-Python BertTokenizer
    fast = BertTokenizerFast.from_pretrained(str(vocab_dir))
    ids, mask = encode_batch(fast, TEXTS)
    assert ids.shape == (len(TEXTS), Config.MAX_TEXT_LENGTH) and ids.dtype == np.int32
    for i, t in enumerate(TEXTS):
        enc = slow(t, add_special_tokens=True, max_length=Config.MAX_TEXT_LENGTH, padding='max_length',
                   truncation=True, return_tensors='np')
        assert np.array_equal(ids[i], enc['input_ids'][0]), t
        assert np.array_equal(mask[i], enc['attention_mask'][0]), t
    assert mask[3].sum() == 2 and mask[8].sum() == Config.MAX_TEXT_LENGTH


def test_predict_texts_without_model_uses_keyword_fallback():
    ti = TextInference.__new__(TextInference)  # no GPU here: model/tokenizer absent
    ti.emotions, ti.model, ti.tokenizer = Config.EMOTIONS, None, None
    from inference.text_inference import _Cleaner
    ti.preprocessor = _Cleaner()
    out = ti.predict_texts(['what a wonderful, happy day', 'nothing here'])
    assert [o['emotion'] for o in out] == ['happy', 'neutral']
