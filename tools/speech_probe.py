"""Stage timeline of speech_flow_kernel (probe build, option speech_debug=1): every block's
s_memrealtime stamps (100 MHz) at entry, weights issued, wait done, A landed, outputs drained,
arrival; printed per stage as min / median / max microseconds after the first block's entry."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'multimodal-emotion-classification_amd'))
os.environ.setdefault('MEC_LIB', os.path.join(ROOT, 'multimodal-emotion-classification_amd', 'mec',
                                              'libmec_hip_probes.so'))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mec import engine, synthetic as syn  # noqa: E402

dev = torch.device('cuda', 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
enc = engine.SpeechEncoder(device=dev)
x = engine.to_device(syn.speech_inputs(B, seed=0), dev)
for _ in range(3):
    enc.forward(x)
enc.set_option('speech_debug', 1)
nch = (B + 15) // 16
groups = [8, 32, 16, 8, 1]
names = ['entry', 'weights', 'waited', 'A landed', 'drained', 'exit']
for rep in range(3):
    feat, _, _ = enc.forward(x)
    torch.cuda.synchronize()
    tr = feat.cpu().numpy().view(np.uint64).reshape(-1)[:nch * 65 * 6].reshape(nch * 65, 6).astype(np.int64)
    t0 = tr[:, 0].min()
    us = (tr - t0) / 100.0
    print(f'--- B={B} launch {rep}: span {us.max():.2f} us')
    b = 0
    for st, g in enumerate(groups):
        blk = us[b:b + g * nch]
        b += g * nch
        cols = ' '.join(f'{names[i]} {blk[:, i].min():5.2f}/{np.median(blk[:, i]):5.2f}/{blk[:, i].max():5.2f}'
                        for i in range(6))
        print(f'stage {st} ({g * nch:3d} blocks): {cols}')
enc.set_option('speech_debug', 0)
