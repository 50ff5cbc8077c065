"""Microbenchmark of the GEMM / implicit-GEMM conv engines on the hot path's real shapes.

    python tools/bench_gemm.py [--bn 0 64 128 256] [--iters 20]

Interleaves variants in one process (guide rule 24), random operands (rule 25).
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'multimodal-emotion-classification_amd'))
# probe option values (*_debug) exist only in the -DMEC_PROBES build (csrc: make probes)
os.environ.setdefault('MEC_LIB', os.path.join(ROOT, 'multimodal-emotion-classification_amd', 'mec',
                                              'libmec_hip_probes.so'))

import torch  # noqa: E402

from mec import _lib  # noqa: E402

B = 256
# (name, kind, dims...) plain: (M, N, K, act, resid) ; conv: (n, H, C, Cout, ks, stride, pad)
SHAPES = [
    ('bert_qkv', 'gemm', B * 128, 2304, 768, 0, 0),
    ('bert_oproj', 'gemm', B * 128, 768, 768, 0, 1),
    ('bert_ffn1', 'gemm', B * 128, 3072, 768, 2, 0),
    ('bert_ffn2', 'gemm', B * 128, 768, 3072, 0, 1),
    ('bert_ffn1_noact', 'gemm', B * 128, 3072, 768, 0, 0),
    ('l1_c1', 'gemm', B * 56 * 56, 64, 256, 1, 0),
    ('l1_c3', 'gemm', B * 56 * 56, 256, 64, 1, 2),
    ('l2_c1', 'gemm', B * 28 * 28, 128, 512, 1, 0),
    ('l3_c3', 'gemm', B * 14 * 14, 1024, 256, 1, 2),
    ('l4_c3', 'gemm', B * 7 * 7, 2048, 512, 1, 2),
    ('l1_c2', 'conv', B, 56, 64, 64, 3, 1, 1),
    ('l2_c2', 'conv', B, 28, 128, 128, 3, 1, 1),
    ('l3_c2', 'conv', B, 14, 256, 256, 3, 1, 1),
    ('l4_c2', 'conv', B, 7, 512, 512, 3, 1, 1),
    ('l2_c2s', 'conv', B, 56, 128, 128, 3, 2, 1),
    ('l2_ds', 'conv', B, 56, 256, 512, 1, 2, 0),
]


def p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--impl", type=int, nargs="+", default=[2], help="ignored: one engine (glds)")
    ap.add_argument('--bn', type=int, nargs='+', default=[0])
    ap.add_argument('--iters', type=int, default=10)
    ap.add_argument('--rounds', type=int, default=5)
    ap.add_argument('--only', nargs='*')
    ap.add_argument('--debug', type=int, nargs='+', default=[0])
    ap.add_argument('--prefetch', type=int, nargs='+', default=[1], help='gemm_prefetch_r values to A/B')
    ap.add_argument('--torch', action='store_true', help='also time torch.mm (hipBLASLt) on plain shapes')
    a = ap.parse_args()
    lib = _lib.load()
    dev = torch.device('cuda', 0)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    res = []
    for sh in SHAPES:
        name, kind = sh[0], sh[1]
        if a.only and name not in a.only:
            continue
        if kind == 'gemm':
            M, N, K, act, resid = sh[2:]
            A = (torch.rand(M, K, device=dev) * 2 - 1).half()
            Bw = ((torch.rand(N, K, device=dev) * 2 - 1) * K ** -0.5).half()
            bias = torch.rand(N, device=dev)
            R = (torch.rand(M, N, device=dev) if resid == 1 else (torch.rand(M, N, device=dev).half() if resid == 2 else None))
            C16 = torch.empty(M, N, device=dev, dtype=torch.float16) if resid != 1 else None
            C32 = torch.empty(M, N, device=dev) if resid == 1 else None
            flop = 2.0 * M * N * K

            def run():
                _lib.check(lib.mec_gemm_f16(p(A), p(Bw), p(bias), p(R), 1 if resid == 1 else 0, p(C16), p(C32),
                                            M, N, K, act, st), name)
            ref = lambda: (A[:512].float() @ Bw.float().t() + bias)  # noqa: E731
            out = lambda: (C16 if C16 is not None else C32)[:512].float()  # noqa: E731
        else:
            n, H, C, Co, ks, s, pd = sh[2:]
            x = torch.rand(n, H, H, C, device=dev).half()
            w = ((torch.rand(Co, ks, ks, C, device=dev) * 2 - 1) * (C * ks * ks) ** -0.5).half()
            bias = torch.rand(Co, device=dev)
            OH = (H + 2 * pd - ks) // s + 1
            y = torch.empty(n, OH, OH, Co, device=dev, dtype=torch.float16)
            flop = 2.0 * n * OH * OH * Co * C * ks * ks

            def run():
                _lib.check(lib.mec_conv_f16(p(x), p(w), p(bias), None, p(y), n, H, H, C, Co, ks, s, pd, 1, st), name)
            ref = None
        if a.torch and kind == 'gemm':
            Bt = Bw.t()
            torch.mm(A, Bt)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                torch.mm(A, Bt)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.iters
            r = {'shape': name, 'impl': 'torch.mm', 'us': round(ms * 1e3, 1), 'tflops': round(flop / ms / 1e9, 1)}
            print(json.dumps(r), flush=True)
        variants = [(2, b, d, f) for b in a.bn for d in a.debug
                    for f in a.prefetch]

        def setv(impl, bn, dbg, pf=1):
            lib.mec_set_option(b'gemm_prefetch_r', pf)
            lib.mec_set_option(b'gemm_debug', dbg)
            lib.mec_set_option(b'gemm_bn', bn)

        ok = []
        for v in variants:  # validate + warm (and autotune for bn=0) each variant once
            setv(*v)
            try:
                run()
            except _lib.MecError as e:
                print(json.dumps({'shape': name, 'impl': v[0], 'bn': v[1], 'error': str(e)}), flush=True)
                setv(2, 0, 0, 1)
                continue
            ok.append(v)
        torch.cuda.synchronize()
        # interleaved rounds (guide rule 24): clocks drift over a sweep, so every variant is
        # timed in every round and the median round is reported
        times = {v: [] for v in ok}
        for _ in range(a.rounds):
            for v in ok:
                setv(*v)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    run()
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / a.iters)
        for v in ok:
            impl, bn, dbg, pf = v
            ms = sorted(times[v])[len(times[v]) // 2]
            r = {'shape': name, 'impl': impl, 'bn': bn, 'dbg': dbg, 'prefetch_r': pf, 'us': round(ms * 1e3, 1),
                 'tflops': round(flop / ms / 1e9, 1)}
            if ref is not None and dbg == 0:
                setv(*v)
                run()
                torch.cuda.synchronize()
                rr = ref()
                if act == 1:
                    rr = torch.relu(rr + (R[:512].float() if R is not None else 0))
                elif act == 2:
                    rr = torch.nn.functional.gelu(rr)
                elif R is not None:
                    rr = rr + R[:512].float()
                r['relerr'] = float((out() - rr).abs().max() / rr.abs().max())
            if bn == 0 and kind == 'gemm':
                r['tuned'] = lib.mec_gemm_query(0, M, N, K)
            res.append(r)
            print(json.dumps(r), flush=True)
    lib.mec_set_option(b'gemm_debug', 0)
    lib.mec_set_option(b'gemm_bn', 0)


if __name__ == '__main__':
    main()
