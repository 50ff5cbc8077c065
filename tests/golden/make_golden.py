"""Generate the golden fixtures under tests/golden/ (run HERE only; needs /root/reference).

    python tests/golden/make_golden.py

What each fixture is pinned to:
  fusion.npz        the reference's own MultiModalFusionModel (built by
                    MultimodalFusion._build_fusion_model, inference/multimodal_fusion.py:63-182)
                    and its fuse_predictions / fuse_with_attention (:184-242), imported from
                    /root/reference with a stub `librosa` module (librosa is absent; it is only
                    needed by preprocessing/audio_preprocessing.py:8, never called here).
                    MultimodalFusion() itself is never constructed (it would construct
                    TextInference -> a by-name hub fetch, preprocessing/text_preprocessing.py:24).
  text_bert.npz     transformers BertForSequenceClassification(BertConfig(num_labels=7,
                    attn_implementation="eager")) — the third-party class the reference
                    loads (inference/text_inference.py:34, :41) — on the seeded weights.
  image_resize.npz  PIL Image.fromarray(L).convert('RGB').resize((224,224), BILINEAR), the
                    call torchvision's Resize makes (inference/image_inference.py:29, :112).
  speech.npz        oracle/speech.py restatement (TensorFlow absent: restatement-pinned).
  image_full.npz    oracle/image.py restatement (torchvision absent: restatement-pinned).
  image_mbv2.npz    oracle/image_mbv2.py restatement (MobileNetV2 backbone; no reference code
                    and torchvision absent: restatement-pinned). `--only mbv2` writes just it.
Only inputs (seeded), seeds and outputs are stored; weights are regenerated from seeds.
"""
import importlib.util
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = '/root/reference'
WSEED = 1234


def load_synthetic():
    p = os.path.join(REPO, 'multimodal-emotion-classification_amd', 'mec', 'synthetic.py')
    spec = importlib.util.spec_from_file_location('mec_synthetic_golden', p)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def import_reference_fusion():
    import transformers  # noqa: F401  (import first, as SURVEY §8c notes)
    stub = types.ModuleType('librosa')
    stub.__spec__ = importlib.machinery.ModuleSpec('librosa', None)
    sys.modules.setdefault('librosa', stub)
    sys.path.insert(0, REF)
    from inference.multimodal_fusion import MultimodalFusion  # reference class
    return MultimodalFusion


def main():
    import torch
    syn = load_synthetic()
    sys.path.insert(0, REPO)
    from oracle import speech as o_speech, image as o_image

    # ------------------------------------------------------------------ fusion
    MF = import_reference_fusion()
    obj = MF.__new__(MF)  # bare object: no encoders, no hub fetch
    obj.emotions = ['happy', 'sad', 'angry', 'fear', 'disgust', 'surprise', 'neutral']
    obj.weights = [0.3, 0.35, 0.35]
    model = obj._build_fusion_model(64, 768, 512, 7, 256)
    w = syn.weights('fusion', WSEED)
    sd = model.state_dict()
    assert list(sd.keys()) == list(w.keys()), 'fusion spec order != reference state_dict order'
    model.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in w.items()})
    model.eval()
    B = 16
    feats = {m: syn.uniform(7, f'golden/fusion/{m}', (B, d), -1.0, 1.0)
             for m, d in (('speech', 64), ('text', 768), ('image', 512))}
    feats['speech'] = np.maximum(feats['speech'], 0) * 2.0   # ReLU features like the encoders'
    feats['image'] = np.maximum(feats['image'], 0) * 2.0
    preds = {}
    for m in ('speech', 'text', 'image'):
        z = syn.uniform(8, f'golden/fusion/pred/{m}', (B, 7), -3.0, 3.0)
        e = np.exp(z - z.max(-1, keepdims=True))
        preds[m] = (e / e.sum(-1, keepdims=True)).astype(np.float32)
    with torch.no_grad():
        t = lambda a: torch.from_numpy(a)
        logits, aw, dw = model(t(feats['speech']), t(feats['text']), t(feats['image']),
                               t(preds['speech']), t(preds['text']), t(preds['image']))
        probs = torch.softmax(logits, -1)
    # dict-level API on two samples through the reference's own method
    obj.fusion_model = model
    obj.torch = torch
    obj.device = torch.device('cpu')
    d0 = obj.fuse_with_attention(feats['speech'][0], feats['text'][0], feats['image'][0],
                                 preds['speech'][0], preds['text'][0], preds['image'][0])
    # weighted-average fallback, incl. missing modalities (multimodal_fusion.py:184-199)
    cases = [(0, 1, 1, 1), (1, 1, 0, 1), (2, 0, 1, 1), (3, 1, 1, 0), (4, 1, 0, 0)]
    wavg = []
    for idx, hs, ht, hi in cases:
        r = obj.fuse_predictions(preds['speech'][idx].tolist() if hs else None,
                                 preds['text'][idx].tolist() if ht else None,
                                 preds['image'][idx].tolist() if hi else None)
        wavg.append(r['all_probabilities'])
    zero = obj.fuse_predictions(None, None, None)['all_probabilities']
    np.savez_compressed(os.path.join(HERE, 'fusion.npz'), wseed=WSEED,
                        s_feat=feats['speech'], t_feat=feats['text'], i_feat=feats['image'],
                        s_pred=preds['speech'], t_pred=preds['text'], i_pred=preds['image'],
                        logits=logits.numpy(), probs=probs.numpy(), attn_w=aw.numpy(), dec_w=dw.numpy(),
                        dict0_emotion=np.array(d0['emotion']), dict0_conf=np.float64(d0['confidence']),
                        dict0_probs=np.array(d0['all_probabilities'], np.float64),
                        dict0_attn=np.array([d0['attention_weights'][k] for k in ('speech', 'text', 'image')]),
                        dict0_dec=np.array([d0['decision_weights'][k] for k in ('speech', 'text', 'image')]),
                        wavg_cases=np.array(cases, np.int32), wavg=np.array(wavg, np.float64),
                        wavg_zero=np.array(zero, np.float64))
    print('fusion.npz written')

    # ------------------------------------------------------------------ text (HF BERT)
    from transformers import BertConfig, BertForSequenceClassification
    cfg = BertConfig(num_labels=7, attn_implementation='eager')
    bert = BertForSequenceClassification(cfg)
    wt = syn.weights('text', WSEED)
    sd = bert.state_dict()
    missing = [k for k in sd if k not in wt]
    assert all('position_ids' in k for k in missing), missing
    assert all(k in sd for k in wt)
    bert.load_state_dict({k: torch.from_numpy(np.array(v)) for k, v in wt.items()}, strict=False)
    bert.eval()
    ids, mask = syn.text_inputs(6, 128, seed=3, ragged=True)
    with torch.no_grad():
        it, mt = torch.from_numpy(ids.astype(np.int64)), torch.from_numpy(mask.astype(np.int64))
        cls = bert.bert(it, attention_mask=mt).last_hidden_state[:, 0, :]   # text_inference.py:124-125
        lg = bert(it, attention_mask=mt).logits                              # :127
        pr = torch.softmax(lg, -1)
    np.savez_compressed(os.path.join(HERE, 'text_bert.npz'), wseed=WSEED, ids=ids, mask=mask,
                        cls=cls.numpy(), logits=lg.numpy(), probs=pr.numpy())
    print('text_bert.npz written')

    # ------------------------------------------------------------------ image resize (PIL)
    from PIL import Image
    gray = syn.image_inputs(4, seed=11)
    gray[0] = 0
    gray[1] = 255
    res = np.stack([np.array(Image.fromarray(g, 'L').convert('RGB').resize((224, 224), Image.BILINEAR))
                    for g in gray])
    assert (res[..., 0] == res[..., 1]).all() and (res[..., 0] == res[..., 2]).all()
    np.savez_compressed(os.path.join(HERE, 'image_resize.npz'), gray=gray, resized=res[..., 0])
    print('image_resize.npz written')

    # ------------------------------------------------------------------ restatement-pinned
    ws = syn.weights('speech', WSEED)
    x = syn.speech_inputs(32, seed=5, wseed=WSEED)
    f, l, p = o_speech.forward(ws, x)
    np.savez_compressed(os.path.join(HERE, 'speech.npz'), wseed=WSEED, x=x, feat=f, logits=l, probs=p)
    wi = syn.weights('image', WSEED)
    g2 = syn.image_inputs(2, seed=13)
    f, l, p = o_image.forward(wi, g2)
    np.savez_compressed(os.path.join(HERE, 'image_full.npz'), wseed=WSEED, gray=g2, feat=f, logits=l, probs=p)
    print('speech.npz, image_full.npz written')
    write_mbv2(syn)


def write_mbv2(syn):
    sys.path.insert(0, REPO)
    from oracle import image_mbv2 as o_mbv2
    w = syn.weights('image_mbv2', WSEED)
    g = syn.image_inputs(2, seed=17)
    f, l, p = o_mbv2.forward(w, g)
    np.savez_compressed(os.path.join(HERE, 'image_mbv2.npz'), wseed=WSEED, gray=g, feat=f, logits=l, probs=p)
    print('image_mbv2.npz written')


if __name__ == '__main__':
    if sys.argv[1:] == ['--only', 'mbv2']:
        write_mbv2(load_synthetic())
    else:
        main()
