"""Time ResNet layer1's 3x3 conv (B x 56 x 56 x 64 -> 64) through the C ABI: the halo-tile
kernel (conv3x3.hip, with its probe variants) against the implicit-GEMM path.
    python tools/bench_conv3x3.py [--batch 256] [--reps 20]"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'multimodal-emotion-classification_amd'))
# probe option values (*_debug) exist only in the -DMEC_PROBES build (csrc: make probes)
os.environ.setdefault('MEC_LIB', os.path.join(ROOT, 'multimodal-emotion-classification_amd', 'mec',
                                              'libmec_hip_probes.so'))
import torch  # noqa: E402

from mec import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=256)
    ap.add_argument('--reps', type=int, default=20)
    a = ap.parse_args()
    lib = _lib.load()
    dev = torch.device('cuda', 0)
    n = a.batch
    x = torch.rand(n, 56, 56, 64, device=dev).half()
    w = ((torch.rand(64, 3, 3, 64, device=dev) * 2 - 1) / 24).half()
    bias = torch.rand(64, device=dev)
    y = torch.empty(n, 56, 56, 64, device=dev, dtype=torch.float16)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    flops = 2.0 * n * 56 * 56 * 64 * 576

    def run():
        _lib.check(lib.mec_conv_f16(p(x), p(w), p(bias), None, p(y), n, 56, 56, 64, 64, 3, 1, 1, 1, s), 'conv')

    for label, direct, dbg in [('gemm', 0, 0), ('halo', 1, 0), ('halo no-next-dma', 1, 1), ('halo no-stores', 1, 2),
                               ('halo no-lds-reads', 1, 4), ('halo mfma-only', 1, 7), ('halo', 1, 0)]:
        _lib.check(lib.mec_set_option(b'conv3x3_direct', direct), 'opt')
        _lib.check(lib.mec_set_option(b'conv3x3_debug', dbg), 'opt')
        for _ in range(3):
            run()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.reps + 1)]
        ev[0].record()
        for i in range(a.reps):
            run()
            ev[i + 1].record()
        torch.cuda.synchronize()
        ts = sorted(ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(a.reps))
        med = ts[len(ts) // 2]
        print(f'{label:20s} median {med:7.1f} us  min {ts[0]:7.1f} us  {flops / med / 1e6:7.1f} TFLOP/s', flush=True)
    lib.mec_set_option(b'conv3x3_debug', 0)
    lib.mec_set_option(b'conv3x3_direct', 1)


if __name__ == '__main__':
    main()
