"""Interleaved A/B of a library option (mec_model_set_option) on one encoder at B=256.

    python tools/ab_option.py --enc image --opt pw_chain --values 0 2

Each round times every value back to back (hipEvents, --iters calls), median of rounds; the
encoder's outputs under each value are compared with the first value's."""
import argparse
import json
import os
import time
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'multimodal-emotion-classification_amd'))

if '--probes' in sys.argv:  # probe option values: the -DMEC_PROBES build (csrc: make probes)
    os.environ.setdefault('MEC_LIB', os.path.join(ROOT, 'multimodal-emotion-classification_amd', 'mec',
                                                  'libmec_hip_probes.so'))

import torch  # noqa: E402

from mec import _lib, engine, synthetic as syn  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--enc', choices=['text', 'image', 'image_mbv2', 'pipeline', 'fusion'], required=True)
    ap.add_argument('--opt', required=True)
    ap.add_argument('--values', type=int, nargs='+', required=True)
    ap.add_argument('--iters', type=int, default=5)
    ap.add_argument('--batch', type=int, default=256, help='text / image / image_mbv2 batch (BASELINE configs[2]: text 128)')
    ap.add_argument('--rounds', type=int, default=5)
    ap.add_argument('--probes', action='store_true', help='load libmec_hip_probes.so (probe option values)')
    ap.add_argument('--precision', default='f16', choices=['f16', 'fp32', 'fp32x3'])
    ap.add_argument('--save', help='write the first value\'s outputs to this .npz (cross-build bit comparisons, '
                                   'with MEC_LIB naming the other build)')
    ap.add_argument('--handles', default='', help="pipeline only: the handles that get --opt, e.g. 'text' "
                                                  "(default: every handle)")
    ap.add_argument('--set', action='append', default=[], metavar='KEY=VALUE',
                    help='process-default option set before the handles are created (creation-time knobs such '
                         'as x3_plane_scale)')
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    lib = _lib.load()
    for kv in a.set:
        k, v = kv.split('=')
        _lib.check(lib.mec_set_option(k.encode(), int(v)), f'mec_set_option {kv}')
    if a.enc == 'pipeline':  # the bench step: speech + text + image + fusion on three streams
        m = engine.FusedPipeline(seed=1234, device=dev, precision=a.precision)
        ids, mask = syn.text_inputs(256, 128, seed=0)
        args = tuple(engine.to_device(v, dev) for v in (syn.speech_inputs(256, seed=0), ids, mask,
                                                        syn.image_inputs(256, seed=0)))
    elif a.enc == 'fusion':  # the attention-fusion head alone on B = 256 feature rows
        m = engine.FusionHead(device=dev)
        g = torch.Generator().manual_seed(0)
        args = tuple(torch.randn(256, d, generator=g).to(dev) for d in (64, 768, 512))
        args += tuple(torch.softmax(torch.randn(256, 7, generator=g), 1).to(dev) for _ in range(3))
    elif a.enc == 'text':
        m = engine.TextEncoder(device=dev, precision=a.precision)
        ids, mask = syn.text_inputs(a.batch, 128, seed=0)
        args = (engine.to_device(ids, dev), engine.to_device(mask, dev))
    else:
        m = (engine.ImageEncoder(device=dev, precision=a.precision) if a.enc == 'image'
             else engine.MobileNetImageEncoder(device=dev, precision=a.precision))
        args = (engine.to_device(syn.image_inputs(a.batch, seed=0), dev),)
    outs, times = {}, {v: [] for v in a.values}
    def fwd():
        r = m.forward(*args)
        if isinstance(r, dict):
            return [v for v in r.values() if torch.is_tensor(v)]
        return r if isinstance(r, (tuple, list)) else (r,)

    def setopt(v):
        if a.enc == 'pipeline' and a.handles:
            for h in a.handles.split(','):
                getattr(m, h).set_option(a.opt, v)
        else:
            m.set_option(a.opt, v)  # this handle's knob (the pipeline: every handle's)

    for v in a.values:
        setopt(v)
        outs[v] = [t.clone() for t in fwd()]
        torch.cuda.synchronize()
        fwd()
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for v in a.values:
            setopt(v)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                fwd()
            torch.cuda.synchronize()
            times[v].append((time.perf_counter() - t0) * 1e3 / a.iters)
    base = outs[a.values[0]]
    if a.save:
        import numpy as np
        np.savez(a.save, *[t.cpu().numpy() for t in base])
    for v in a.values:
        d = [float((x - y).abs().max()) for x, y in zip(outs[v], base)]
        print(json.dumps({'enc': a.enc, 'precision': a.precision, a.opt: v, 'ms': round(sorted(times[v])[len(times[v]) // 2], 4),
                          'max_abs_diff_vs_first': d}))


if __name__ == '__main__':
    main()
