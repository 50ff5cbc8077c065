"""Which fp32x3 image forward raises the range flag (diagnostic): B x option sweeps, one fresh
handle each, check() after a synchronized forward."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'multimodal-emotion-classification_amd'))
import torch  # noqa: E402

from mec import engine, synthetic as syn  # noqa: E402
from mec._lib import MecError  # noqa: E402

dev = torch.device('cuda', 0)
cases = [(2, {}), (8, {}), (3, {}), (2, {'gemm_autotune': 0}), (2, {'gemm_prefetch_r': 0}), (2, {'stem_gray_f32': 0}),
         (2, {'gemm_x3_order': 0}), (16, {}), (64, {})]
for B, opts in cases:
    enc = engine.ImageEncoder(device=dev, precision='fp32x3')
    for k, v in opts.items():
        enc.set_option(k, v)
    g = engine.to_device(syn.image_inputs(B, seed=5), dev)
    feat, logits, probs = enc.forward(g)
    torch.cuda.synchronize()
    try:
        enc.check()
        r = 'clean'
    except MecError:
        r = 'FLAG'
    print(f'B={B} {opts}: {r}; probs finite {bool(torch.isfinite(probs).all())}', flush=True)
    enc.close()
for B in (2, 8):
    t = engine.TextEncoder(device=dev, precision='fp32x3')
    ids, mask = syn.text_inputs(B, 128, seed=3, ragged=True)
    t.forward(engine.to_device(ids, dev), engine.to_device(mask, dev))
    torch.cuda.synchronize()
    try:
        t.check()
        print(f'text B={B}: clean', flush=True)
    except MecError:
        print(f'text B={B}: FLAG', flush=True)
