"""Run ONE encoder of the hot path alone at B=256 (for rocprofv3 per-kernel isolation).

    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_text -o run -- \
        python3 tools/encoder_profile.py --enc text --iters 5
    python3 tools/prof_summary.py gpurun_out/prof_text/run_results.db --window spin --steps 5 --by-grid

Warm-up (autotuning included) happens before the opening marker kernel; the timed
iterations sit between two torch.cuda._sleep marker dispatches.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'multimodal-emotion-classification_amd'))

import torch  # noqa: E402

from mec import engine, synthetic as syn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--enc', choices=['text', 'image', 'image_mbv2', 'speech', 'fusion', 'pipeline', 'audio'], required=True)
    ap.add_argument('--iters', type=int, default=5)
    ap.add_argument('--batch', type=int, default=256)
    ap.add_argument('--opt', action='append', default=[], help='library option NAME=VALUE (mec_set_option)')
    ap.add_argument('--precision', default='f16', choices=['f16', 'fp32', 'fp32x3'])
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    B = a.batch
    if a.opt:
        from mec import _lib
        for kv in a.opt:
            k, v = kv.split('=')
            _lib.check(_lib.load().mec_set_option(k.encode(), int(v)), f'mec_set_option({kv})')
    if a.enc == 'text':
        m = engine.TextEncoder(device=dev, precision=a.precision)
        ids, mask = syn.text_inputs(B, 128, seed=0)
        args = (engine.to_device(ids, dev), engine.to_device(mask, dev))
        fn = lambda: m.forward(*args)  # noqa: E731
    elif a.enc == 'image':
        m = engine.ImageEncoder(device=dev, precision=a.precision)
        g = engine.to_device(syn.image_inputs(B, seed=0), dev)
        fn = lambda: m.forward(g)  # noqa: E731
    elif a.enc == 'image_mbv2':
        m = engine.MobileNetImageEncoder(device=dev, precision=a.precision)
        g = engine.to_device(syn.image_inputs(B, seed=0), dev)
        fn = lambda: m.forward(g)  # noqa: E731
    elif a.enc == 'speech':
        m = engine.SpeechEncoder(device=dev)
        x = engine.to_device(syn.speech_inputs(B, seed=0), dev)
        fn = lambda: m.forward(x)  # noqa: E731
    elif a.enc == 'audio':  # waveform -> 56-d features (csrc/audio.hip), 3 s clips at 22050 Hz
        import numpy as np
        m = engine.AudioFeaturizer(device=dev)
        wv = torch.from_numpy(np.random.default_rng(0).standard_normal((B, 66150)).astype(np.float32)).to(dev)
        fn = lambda: m.forward(wv)  # noqa: E731
    elif a.enc == 'fusion':
        m = engine.FusionHead(device=dev)
        args = [torch.rand(B, d, device=dev) for d in (64, 768, 512)]
        args += [torch.softmax(torch.rand(B, 7, device=dev), 1) for _ in range(3)]
        fn = lambda: m.forward(*args)  # noqa: E731
    else:
        m = engine.FusedPipeline(seed=1234, device=dev, precision=a.precision)
        x = engine.to_device(syn.speech_inputs(B, seed=0), dev)
        ids, mask = syn.text_inputs(B, 128, seed=0)
        ids, mask = engine.to_device(ids, dev), engine.to_device(mask, dev)
        g = engine.to_device(syn.image_inputs(B, seed=0), dev)
        fn = lambda: m.forward(x, ids, mask, g)  # noqa: E731
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    torch.cuda._sleep(1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        fn()
    e1.record()
    torch.cuda._sleep(1)
    torch.cuda.synchronize()
    print(json.dumps({'enc': a.enc, 'batch': B, 'precision': a.precision, 'ms_per_iter': e0.elapsed_time(e1) / a.iters}))


if __name__ == '__main__':
    main()
