"""ORACLE (test infrastructure only): fusion step, fp32 (attention model) / fp64 (average).

Restates inference/multimodal_fusion.py:
  MultiModalFusionModel.forward  :156-180 (proj :113-130 Linear+LN(1e-5)+ReLU;
      CrossModalAttention :68-77 = nn.MultiheadAttention(256, 4, batch_first) + residual
      + LN; AttentionFusion :79-106; decision_weights :138-143; classifier :145-154)
  fuse_with_attention            :201-242 (softmax over logits :221)
  fuse_predictions               :184-199 (numpy float64 weighted average 0.3/0.35/0.35,
      renormalised when the sum is > 0; a missing modality counts as zeros)
Pinned against the reference's own class, imported here: tests/golden/fusion.npz.
"""
import numpy as np
import torch
import torch.nn.functional as F

HID, NH = 256, 4
WEIGHTS = [0.3, 0.35, 0.35]  # multimodal_fusion.py:23


@torch.no_grad()
def forward(w, s_feat, t_feat, i_feat, s_pred, t_pred, i_pred):
    """-> (logits [B,7], probs [B,7], attn_w [B,3], dec_w [B,3]) float32 numpy."""
    g = lambda n: torch.from_numpy(np.asarray(w[n], np.float32))
    f = lambda a: torch.from_numpy(np.asarray(a, np.float32))
    s_feat, t_feat, i_feat, s_pred, t_pred, i_pred = map(f, (s_feat, t_feat, i_feat, s_pred, t_pred, i_pred))

    def proj(p, x):
        y = F.linear(x, g(p + '.0.weight'), g(p + '.0.bias'))
        return F.relu(F.layer_norm(y, (y.shape[-1],), g(p + '.1.weight'), g(p + '.1.bias'), 1e-5))

    sp, tp, ip = proj('speech_proj', s_feat), proj('text_proj', t_feat), proj('image_proj', i_feat)

    def cross(p, q, kv0, kv1):
        W, bias = g(p + 'attention.in_proj_weight'), g(p + 'attention.in_proj_bias')
        qq = F.linear(q, W[:HID], bias[:HID])
        kv = torch.stack([kv0, kv1], dim=1)                       # [B,2,H]
        kk = F.linear(kv, W[HID:2 * HID], bias[HID:2 * HID])
        vv = F.linear(kv, W[2 * HID:], bias[2 * HID:])
        B = q.shape[0]
        dh = HID // NH
        qh = qq.view(B, NH, 1, dh)
        kh = kk.view(B, 2, NH, dh).transpose(1, 2)
        vh = vv.view(B, 2, NH, dh).transpose(1, 2)
        a = torch.softmax(torch.matmul(qh / np.sqrt(dh), kh.transpose(-1, -2)), dim=-1)
        o = torch.matmul(a, vh).reshape(B, HID)
        o = F.linear(o, g(p + 'attention.out_proj.weight'), g(p + 'attention.out_proj.bias'))
        return F.layer_norm(q + o, (HID,), g(p + 'norm.weight'), g(p + 'norm.bias'), 1e-5)

    se = cross('cross_attn_speech.', sp, tp, ip)
    te = cross('cross_attn_text.', tp, sp, ip)
    ie = cross('cross_attn_image.', ip, sp, tp)
    projd = [proj(f'attention_fusion.projections.{j}', x) for j, x in enumerate((se, te, ie))]
    a = torch.tanh(F.linear(torch.cat(projd, -1), g('attention_fusion.attention.0.weight'),
                            g('attention_fusion.attention.0.bias')))
    attn_w = torch.softmax(F.linear(a, g('attention_fusion.attention.2.weight'),
                                    g('attention_fusion.attention.2.bias')), -1)
    fused = (torch.stack(projd, 1) * attn_w[..., None]).sum(1)
    d = F.relu(F.linear(torch.cat([s_pred, t_pred, i_pred], -1), g('decision_weights.0.weight'),
                        g('decision_weights.0.bias')))
    dec_w = torch.softmax(F.linear(d, g('decision_weights.2.weight'), g('decision_weights.2.bias')), -1)
    wpred = (torch.stack([s_pred, t_pred, i_pred], 1) * dec_w[..., None]).sum(1)
    c = F.linear(torch.cat([fused, wpred], -1), g('classifier.0.weight'), g('classifier.0.bias'))
    c = F.relu(F.layer_norm(c, (HID,), g('classifier.1.weight'), g('classifier.1.bias'), 1e-5))
    c = F.relu(F.linear(c, g('classifier.4.weight'), g('classifier.4.bias')))
    logits = F.linear(c, g('classifier.7.weight'), g('classifier.7.bias'))
    probs = torch.softmax(logits, -1)
    return tuple(t.numpy().copy() for t in (logits, probs, attn_w, dec_w))


def fuse_predictions(s, t, i, n=7):
    """Weighted-average fallback (multimodal_fusion.py:184-199) -> float64 [7]."""
    s = np.array(s) if s is not None else np.zeros(n)
    t = np.array(t) if t is not None else np.zeros(n)
    i = np.array(i) if i is not None else np.zeros(n)
    weighted = WEIGHTS[0] * s + WEIGHTS[1] * t + WEIGHTS[2] * i
    if weighted.sum() > 0:
        weighted = weighted / weighted.sum()
    return weighted
