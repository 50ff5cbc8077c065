"""ORACLE (test infrastructure only): BERT-base sequence classifier, fp32, torch-CPU.

Restates the forward the reference runs through transformers'
BertForSequenceClassification (inference/text_inference.py:41, :92-93, :124-128;
transformers==4.30.0 pinned at requirements.txt:16, eager attention):
  embeddings  word[ids] + token_type[0] + position[0:L] -> LayerNorm(eps=1e-12)
  x12 layer   Q,K,V = xW^T+b; scores = QK^T/sqrt(64) + (1-mask)*finfo(f32).min;
              softmax; ctx = P V; LN(ctx Wo^T + bo + x); GELU(erf) FFN; LN(. + residual)
  feature     last_hidden_state[:, 0, :]  (pre-pooler CLS, text_inference.py:125)
  head        tanh(cls Wp^T + bp) -> classifier -> softmax (text_inference.py:93, :128)
Pinned against transformers 5.15 BertForSequenceClassification(attn_implementation=
"eager") on the same seeded weights: tests/golden/text_bert.npz.
"""
import numpy as np
import torch
import torch.nn.functional as F

H, HEADS, DH, LAYERS = 768, 12, 64, 12


def _t(a):
    return torch.from_numpy(np.asarray(a, np.float32))


@torch.no_grad()
def forward(w, ids: np.ndarray, mask: np.ndarray):
    """ids/mask int [B,L] -> (cls [B,768], logits [B,7], probs [B,7]) as float32 numpy."""
    ids_t = torch.from_numpy(np.asarray(ids, np.int64))
    m = torch.from_numpy(np.asarray(mask, np.float32))
    B, L = ids_t.shape
    g = lambda n: _t(w[n])
    p = 'bert.embeddings.'
    x = F.embedding(ids_t, g(p + 'word_embeddings.weight')) + g(p + 'token_type_embeddings.weight')[0]
    x = x + g(p + 'position_embeddings.weight')[:L][None]
    x = F.layer_norm(x, (H,), g(p + 'LayerNorm.weight'), g(p + 'LayerNorm.bias'), 1e-12)
    ext = (1.0 - m[:, None, None, :]) * torch.finfo(torch.float32).min
    for i in range(LAYERS):
        p = f'bert.encoder.layer.{i}.'
        def heads(t):
            return t.view(B, L, HEADS, DH).transpose(1, 2)
        q = heads(F.linear(x, g(p + 'attention.self.query.weight'), g(p + 'attention.self.query.bias')))
        k = heads(F.linear(x, g(p + 'attention.self.key.weight'), g(p + 'attention.self.key.bias')))
        v = heads(F.linear(x, g(p + 'attention.self.value.weight'), g(p + 'attention.self.value.bias')))
        s = torch.matmul(q, k.transpose(-1, -2)) / np.sqrt(DH) + ext
        ctx = torch.matmul(torch.softmax(s, dim=-1), v).transpose(1, 2).reshape(B, L, H)
        a = F.linear(ctx, g(p + 'attention.output.dense.weight'), g(p + 'attention.output.dense.bias'))
        x = F.layer_norm(a + x, (H,), g(p + 'attention.output.LayerNorm.weight'),
                         g(p + 'attention.output.LayerNorm.bias'), 1e-12)
        inter = F.gelu(F.linear(x, g(p + 'intermediate.dense.weight'), g(p + 'intermediate.dense.bias')))
        o = F.linear(inter, g(p + 'output.dense.weight'), g(p + 'output.dense.bias'))
        x = F.layer_norm(o + x, (H,), g(p + 'output.LayerNorm.weight'), g(p + 'output.LayerNorm.bias'), 1e-12)
    cls = x[:, 0]
    pooled = torch.tanh(F.linear(cls, g('bert.pooler.dense.weight'), g('bert.pooler.dense.bias')))
    logits = F.linear(pooled, g('classifier.weight'), g('classifier.bias'))
    probs = torch.softmax(logits, dim=-1)
    return cls.numpy().copy(), logits.numpy().copy(), probs.numpy().copy()
