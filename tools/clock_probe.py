"""Shader clock under load: a one-wave probe kernel (tools/clock_probe.hip) samples s_memtime /
s_memrealtime on a low-priority stream while the fused pipeline, BERT alone or the ResNet
alone runs back to back; prints the median clock (GHz) per phase.
    python tools/clock_probe.py [--iters 40]"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'multimodal-emotion-classification_amd'))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mec import engine, synthetic as syn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=40)
    a = ap.parse_args()
    so = ctypes.CDLL(os.path.join(ROOT, 'build', 'clock_probe.so'))
    dev = torch.device('cuda', 0)
    B = 256
    pipe = engine.FusedPipeline(seed=1234, device=dev)
    x = engine.to_device(syn.speech_inputs(B, seed=0), dev)
    ids, mask = (engine.to_device(v, dev) for v in syn.text_inputs(B, 128, seed=0))
    gray = engine.to_device(syn.image_inputs(B, seed=0), dev)
    for _ in range(2):
        pipe.forward(x, ids, mask, gray)
    pipe.wait()
    torch.cuda.synchronize()
    probe_stream = torch.cuda.Stream(device=dev, priority=0)
    phases = {'fused': lambda: pipe.forward(x, ids, mask, gray), 'text alone': lambda: pipe.text.forward(ids, mask),
              'image alone': lambda: pipe.image.forward(gray)}
    for name, fn in phases.items():
        n = 200000
        buf = torch.zeros(2 * n + 4, dtype=torch.int64, device=dev)
        stop = torch.zeros(1, dtype=torch.int32, device=dev)
        so.clock_probe_launch(ctypes.c_void_p(buf.data_ptr()), n, ctypes.c_void_p(stop.data_ptr()),
                              ctypes.c_void_p(probe_stream.cuda_stream))
        for _ in range(a.iters):
            fn()
        pipe.wait()
        torch.cuda.current_stream().synchronize()
        stop.fill_(1)
        torch.cuda.synchronize()
        v = buf.cpu().numpy().reshape(-1)[:2 * n].reshape(n, 2)
        v = v[(v[:, 0] > 0) & (v[:, 1] > 0)]
        if len(v) < 10:
            print(name, 'too few samples'); continue
        dc, dr = np.diff(v[:, 0].astype(np.float64)), np.diff(v[:, 1].astype(np.float64))
        ghz = dc / dr * 0.1
        q = np.percentile(ghz[len(ghz) // 10: -len(ghz) // 10 or None], [10, 50, 90])
        print(f'{name:12s} samples {len(ghz):5d}  shader clock GHz p10 {q[0]:.2f}  median {q[1]:.2f}  p90 {q[2]:.2f}',
              flush=True)


if __name__ == '__main__':
    main()
