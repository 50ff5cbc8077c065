"""Phase timeline of one block of the ping-pong GEMM (probe build gemm_debug 4): per wave,
s_memtime at phase start / reads + DMA issue retired / past barrier 1 / MFMAs issued, for
the first 12 K tiles of BERT FFN1 (M=32768 N=3072 K=768). Prints per-wave mean cycles of
each section (s_memtime ticks = shader cycles).

    python tools/pp_trace.py [tile id, default 40256]"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'multimodal-emotion-classification_amd'))
# probe option values (*_debug) exist only in the -DMEC_PROBES build (csrc: make probes)
os.environ.setdefault('MEC_LIB', os.path.join(ROOT, 'multimodal-emotion-classification_amd', 'mec',
                                              'libmec_hip_probes.so'))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mec import _lib  # noqa: E402


def p(t):
    return ctypes.c_void_p(t.data_ptr())


def main():
    lib = _lib.load()
    dev = torch.device('cuda', 0)
    tile = int(sys.argv[1]) if len(sys.argv) > 1 else 40256
    M, N, K = 32768, 3072, 768
    A = (torch.rand(M, K, device=dev) * 2 - 1).half()
    B = ((torch.rand(N, K, device=dev) * 2 - 1) * K ** -0.5).half()
    bias = torch.rand(N, device=dev)
    C32 = torch.zeros(M, N, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    _lib.check(lib.mec_set_option(b'gemm_bn', tile), 'opt')
    _lib.check(lib.mec_set_option(b'gemm_debug', 4), 'opt')
    for _ in range(3):
        _lib.check(lib.mec_gemm_f16(p(A), p(B), p(bias), None, 0, None, p(C32), M, N, K, 0, st), 'gemm')
    torch.cuda.synchronize()
    lib.mec_set_option(b'gemm_debug', 0)
    lib.mec_set_option(b'gemm_bn', 0)
    tr = C32.view(torch.int64).flatten()[:8 * 192].cpu().numpy().reshape(8, 12 * 4, 4).astype(np.float64)
    t0 = tr.min()
    names = ['pre', 'barrier1', 'mfma_issue', 'post+barrier2']
    for w in range(8):
        x = tr[w]
        nxt = np.concatenate([x[1:, 0], [np.nan]])
        sec = np.stack([x[:, 1] - x[:, 0], x[:, 2] - x[:, 1], x[:, 3] - x[:, 2], nxt - x[:, 3]], 1)
        m = np.nanmean(sec[4:], 0)  # skip the first K tile
        print(f'tile {tile} wave {w} (row {w // 4}) start {x[0, 0] - t0:8.0f}  per-phase mean cycles: ' +
              '  '.join(f'{n} {v:6.0f}' for n, v in zip(names, m)) + f'  phase total {np.nansum(m):6.0f}')
    ph = np.nanmean(np.diff(tr[0, 4:, 0]))
    print(f'phase period (wave 0): {ph:.0f} cycles; ideal MFMA time per phase per SIMD: 2 waves x 16 x 16 = 512')


if __name__ == '__main__':
    main()
