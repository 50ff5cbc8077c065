"""Interleaved A/B of two builds of libmec_hip.so in one process (same GPU, same clock
state): the in-tree library against a saved copy, on one encoder at B = 256.

    cp multimodal-emotion-classification_amd/mec/libmec_hip.so build/ab/libmec_prev.so   # before a change
    python tools/ab_lib.py --enc image --other build/ab/libmec_prev.so

Outputs of both builds are compared (max abs diff) and each build is timed over --rounds
rounds of --iters forwards (median)."""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'multimodal-emotion-classification_amd'))

import torch  # noqa: E402

from mec import _lib, engine, synthetic as syn  # noqa: E402


def make(lib, kind, dev):
    blob = syn.pack(kind, syn.weights(kind, 1234))
    h = ctypes.c_void_p()
    rc = lib.mec_create(engine.KINDS[kind], blob.ctypes.data_as(_lib.c_fp), blob.size, dev.index, ctypes.byref(h))
    if rc:
        raise RuntimeError(lib.mec_last_error().decode())
    return h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--enc', choices=['image', 'text'], default='image')
    ap.add_argument('--other', required=True)
    ap.add_argument('--iters', type=int, default=10)
    ap.add_argument('--rounds', type=int, default=7)
    a = ap.parse_args()
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    libs = {'tree': _lib.load(), 'other': _lib.load(os.path.abspath(a.other))}
    B = 256
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    outs = {k: [torch.empty(B, 512 if a.enc == 'image' else 768, device=dev), torch.empty(B, 7, device=dev),
                torch.empty(B, 7, device=dev)] for k in libs}
    if a.enc == 'image':
        x = engine.to_device(syn.image_inputs(B, seed=0), dev)
        hs = {k: make(lib, 'image', dev) for k, lib in libs.items()}
        run = lambda k: libs[k].mec_image_fwd(hs[k], p(x), B, *[p(t) for t in outs[k]], st)  # noqa: E731
    else:
        ids, mask = (engine.to_device(v, dev) for v in syn.text_inputs(B, 128, seed=0))
        hs = {k: make(lib, 'text', dev) for k, lib in libs.items()}
        run = lambda k: libs[k].mec_text_fwd(hs[k], p(ids), p(mask), B, 128, *[p(t) for t in outs[k]], st)  # noqa: E731
    for k in libs:
        for _ in range(3):
            assert run(k) == 0, libs[k].mec_last_error()
    torch.cuda.synchronize()
    times = {k: [] for k in libs}
    for _ in range(a.rounds):
        for k in libs:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                run(k)
            torch.cuda.synchronize()
            times[k].append((time.perf_counter() - t0) * 1e3 / a.iters)
    diff = [float((u - v).abs().max()) for u, v in zip(outs['tree'], outs['other'])]
    for k in libs:
        print(json.dumps({'enc': a.enc, 'lib': k, 'ms': round(sorted(times[k])[len(times[k]) // 2], 4),
                          'max_abs_diff_tree_vs_other': diff}))


if __name__ == '__main__':
    main()
