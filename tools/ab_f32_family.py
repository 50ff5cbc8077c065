"""fp32 engine MFMA family (gemm_f32_family 0 / 16 / 32): one fresh handle per value (the knob
acts when a shape is first tuned, so it must be set before the handle's first call), timed
interleaved at B = 256; then each handle's rows at B = 256 vs the same rows run as B = 16."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'multimodal-emotion-classification_amd'))
import torch  # noqa: E402

from mec import _lib, engine, synthetic as syn  # noqa: E402

dev = torch.device('cuda', 0)
lib = _lib.load()
vals = [int(v) for v in sys.argv[1:]] or [0, 16]
for enc in ('image', 'text'):
    hs = {}
    for v in vals:
        _lib.check(lib.mec_set_option(b'gemm_f32_family', v), 'family')
        hs[v] = engine.ImageEncoder(device=dev, precision='fp32') if enc == 'image' else \
            engine.TextEncoder(device=dev, precision='fp32')
    lib.mec_set_option(b'gemm_f32_family', 16)  # the default
    if enc == 'image':
        args = (engine.to_device(syn.image_inputs(256, seed=0), dev),)
        small = (args[0][:16],)
    else:
        ids, mask = syn.text_inputs(256, 128, seed=0)
        args = (engine.to_device(ids, dev), engine.to_device(mask, dev))
        small = (args[0][:16], args[1][:16])
    for h in hs.values():
        h.forward(*args)
        h.forward(*small)
    torch.cuda.synchronize()
    times = {v: [] for v in vals}
    for _ in range(5):
        for v, h in hs.items():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                h.forward(*args)
            torch.cuda.synchronize()
            times[v].append((time.perf_counter() - t0) / 3 * 1e3)
    for v, h in hs.items():
        big = [t[:16].clone() for t in h.forward(*args)]
        sm = h.forward(*small)
        torch.cuda.synchronize()
        inv = all(torch.equal(a, b) for a, b in zip(big, sm))
        print(f'{enc} fp32 family {v}: {sorted(times[v])[2]:.3f} ms at B=256; rows of B=256 == B=16 run: {inv}')
