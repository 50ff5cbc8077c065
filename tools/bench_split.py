"""Time every tile of the split-f16 (fp32x3) GEMM engine on the BERT shapes at B=256
(mec_gemm_f16x3, gemm_bn forced), interleaved rounds, median; one JSON line per (shape, tile).

    python tools/bench_split.py [--rounds 5] [--iters 10] [--shapes ffn1 ffn2 qkv oproj] [--order 0|1]

--order 1 (the default term order, K-interleaved) times the 7xxxx tiles; --order 0 the pass-major ones.
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'multimodal-emotion-classification_amd'))

import torch  # noqa: E402

from mec import _lib  # noqa: E402

SHAPES = {'qkv': (32768, 2304, 768, 0, False), 'oproj': (32768, 768, 768, 0, True),
          'ffn1': (32768, 3072, 768, 4, False), 'ffn2': (32768, 768, 3072, 0, True)}
TILES = [128, 256, 1128, 10128, 10256, 11128, 20256, 30256, 20128, 50128, 60128, 50256, 40256, 41256]
TILES_X3I = [70256, 70128, 71128, 71064, 70064]


def width(t):
    if 70000 <= t < 80000:  # interleaved split tiles (gemm_x3_order 1): 7 | shape | width
        return t % 1000
    if t >= 40000:
        return 256
    t %= 10000
    return t if t < 1000 else t - 1000


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--rounds', type=int, default=5)
    ap.add_argument('--iters', type=int, default=10)
    ap.add_argument('--shapes', nargs='+', default=list(SHAPES))
    ap.add_argument('--tiles', type=int, nargs='+', default=None)
    ap.add_argument('--order', type=int, default=1, choices=[0, 1])
    a = ap.parse_args()
    lib = _lib.load()
    _lib.check(lib.mec_set_option(b'gemm_x3_order', a.order), 'gemm_x3_order')
    if a.tiles is None:
        a.tiles = TILES_X3I if a.order == 1 else TILES
    dev = torch.device('cuda', 0)
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)  # noqa: E731
    for name in a.shapes:
        M, N, K, act, res = SHAPES[name]
        A = (torch.randn(2, M, K, device=dev) * 0.5).half()
        B = (torch.randn(2, N, K, device=dev) * 0.5).half()
        bias = torch.randn(N, device=dev)
        R = torch.randn(M, N, device=dev) if res else None
        out16 = torch.empty(2, M, N, device=dev, dtype=torch.float16) if not res else None
        out32 = torch.empty(M, N, device=dev) if res else None

        def run():
            _lib.check(lib.mec_gemm_f16x3(p(A), M * K, p(B), N * K, ctypes.c_float(1.0), p(bias), p(R), p(out16),
                                          M * N if out16 is not None else 0, p(out32), M, N, K, act, st), name)

        tiles = [t for t in a.tiles if N % width(t) == 0]
        for t in tiles:  # warm
            lib.mec_set_option(b'gemm_bn', t)
            run()
        times = {t: [] for t in tiles}
        for _ in range(a.rounds):
            for t in tiles:
                lib.mec_set_option(b'gemm_bn', t)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    run()
                e1.record()
                torch.cuda.synchronize()
                times[t].append(e0.elapsed_time(e1) / a.iters)
        lib.mec_set_option(b'gemm_bn', 0)
        flop = 2.0 * M * N * K * 3
        for t in tiles:
            ms = sorted(times[t])[len(times[t]) // 2]
            print(json.dumps({'shape': name, 'tile': t, 'us': round(ms * 1e3, 1),
                              'mfma_tflops': round(flop / ms / 1e9, 1)}), flush=True)


if __name__ == '__main__':
    main()
