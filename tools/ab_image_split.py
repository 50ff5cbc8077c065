"""Image encoder at B = 256: one launch sequence vs the batch split over two handles on two
streams (the halves' kernels overlap: one half's HBM-bound 1x1 convs beside the other's MFMA-bound
3x3 convs, and each other's wave-quantization tails). Rows are batch-invariant, so both give the
same bits; printed per round, interleaved."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'multimodal-emotion-classification_amd'))
import torch  # noqa: E402

from mec import engine, synthetic as syn  # noqa: E402

dev = torch.device('cuda', 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
prec = sys.argv[2] if len(sys.argv) > 2 else 'f16'
a = engine.ImageEncoder(device=dev, precision=prec)
b = engine.ImageEncoder(device=dev, precision=prec)
g = engine.to_device(syn.image_inputs(B, seed=0), dev)
h = B // 2
s1, s2 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)


def one():
    return a.forward(g)


def split():
    main = torch.cuda.current_stream(dev)
    s1.wait_stream(main)
    s2.wait_stream(main)
    with torch.cuda.stream(s1):
        r1 = a.forward(g[:h])
    with torch.cuda.stream(s2):
        r2 = b.forward(g[h:])
    main.wait_stream(s1)
    main.wait_stream(s2)
    return [torch.cat([x, y]) for x, y in zip(r1, r2)]


r0 = [t.clone() for t in one()]
a.forward(g[:h]); b.forward(g[h:])  # noqa: E702  (autotune the half shapes serially)
torch.cuda.synchronize()
r1 = split()
torch.cuda.synchronize()
print('bit-identical:', all(torch.equal(x, y) for x, y in zip(r0, r1)))
times = {'one': [], 'split': []}
for _ in range(7):
    for name, fn in (('one', one), ('split', split)):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        times[name].append((time.perf_counter() - t0) * 100)
for k, v in times.items():
    print(f'{prec} B={B} {k}: {sorted(v)[3]:.3f} ms per batch')
