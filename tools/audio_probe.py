"""Time the audio frame kernel's probe builds (libmec_hip_probes.so, option audio_debug):
1 no FFT stages, 2 no rolloff cumsum, 4 no mel / peak search, 8 no spectrum split, 15 all;
32 / 64 / 96 / 128: the clip kernel stops after MFCC / median / tuning histogram / chroma.
    python tools/audio_probe.py B [values...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'multimodal-emotion-classification_amd'))
os.environ.setdefault('MEC_LIB', os.path.join(ROOT, 'multimodal-emotion-classification_amd', 'mec',
                                              'libmec_hip_probes.so'))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mec import engine  # noqa: E402

dev = torch.device('cuda', 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
fx = engine.AudioFeaturizer(device=dev)
wv = torch.from_numpy(np.random.default_rng(0).standard_normal((B, 66150)).astype(np.float32)).to(dev)
for dbg in [int(v) for v in sys.argv[2:]] or (0, 1, 2, 4, 8, 15, 0):
    fx.set_option('audio_debug', dbg)
    fx.forward(wv)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        fx.forward(wv)
    e1.record()
    torch.cuda.synchronize()
    print(f'audio_debug {dbg:2d}: {e0.elapsed_time(e1) / 5 * 1e3:8.1f} us per forward (B={B})')
