"""GPU: BERT's last layer on the [CLS] rows only (option bert_cls_last, the default) gives the
full layer's bits. The reference's outputs read nothing of the last layer but the [CLS] row
(inference/text_inference.py:125-128: last_hidden_state[:, 0, :] and the pooler's logits), so
the pruned layer computes K / V for every token and Q, attention, O-projection, LayerNorms and
FFN for the B [CLS] rows only; every kernel on that path is row-independent and the [CLS]-only
attention runs the full kernel's instruction sequence for the [CLS] query."""
import numpy as np
import pytest
import torch

from mec import engine, synthetic as syn
from oracle import text as o_t

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('precision', ['f16', 'fp32', 'fp32x3'])
@pytest.mark.parametrize('B,ragged', [(3, True), (64, True), (256, False)])
def test_cls_last_bit_identical_to_full_layer(dev, precision, B, ragged):
    ids, mask = syn.text_inputs(B, 128, seed=900 + B, ragged=ragged)
    args = (engine.to_device(ids, dev), engine.to_device(mask, dev))
    m = engine.TextEncoder(device=dev, precision=precision)
    m.set_option('bert_cls_last', 0)
    full = [t.cpu() for t in m.forward(*args)]
    m.set_option('bert_cls_last', 1)
    cls = [t.cpu() for t in m.forward(*args)]
    torch.cuda.synchronize()
    for name, a, b in zip(('cls', 'logits', 'probs'), full, cls):
        assert torch.equal(a, b), f'{precision} B={B} {name}: max|d| {(a - b).abs().max().item():.3g}'
    m.close()


def test_cls_last_vs_oracle_fp32x3(dev):
    """The pruned path against the oracle at the fp32 bars (probs 1e-5, CLS 1e-4 relative)."""
    B = 16
    ids, mask = syn.text_inputs(B, 128, seed=77, ragged=True)
    m = engine.TextEncoder(device=dev, precision='fp32x3')
    cls, logits, probs = [t.cpu().numpy() for t in m.forward(engine.to_device(ids, dev), engine.to_device(mask, dev))]
    rc, rl, rp = o_t.forward(syn.weights('text'), ids, mask)
    assert (probs.argmax(1) == rp.argmax(1)).all()
    assert np.abs(probs - rp).max() <= 1e-5
    assert np.abs(cls - rc).max() / np.abs(rc).max() <= 1e-4
    m.close()
