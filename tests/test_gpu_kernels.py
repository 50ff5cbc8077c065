"""Kernel-level parity on the GPU, through the C ABI: MFMA GEMM / implicit-GEMM conv vs a
torch fp32 reference of the same op, PIL-exact resize bit-exact vs the golden fixture."""
import ctypes

import numpy as np
import pytest
import torch

from mec import _lib

pytestmark = pytest.mark.gpu


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _s():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _rel_err(got, ref):
    return float((got - ref).abs().max() / ref.abs().max().clamp_min(1e-6))


@pytest.mark.parametrize('M,N,K,act', [(256, 128, 64, 0), (300, 192, 128, 1), (1000, 768, 768, 2),
                                       (77, 64, 3072, 0), (4096, 2304, 768, 0)])
def test_gemm_f16(dev, M, N, K, act):
    lib = _lib.load()
    g = torch.Generator().manual_seed(M * 7 + N)
    A = (torch.rand(M, K, generator=g) * 2 - 1).half().to(dev)
    B = (torch.rand(N, K, generator=g) * 2 - 1).mul(K ** -0.5).half().to(dev)
    bias = torch.rand(N, generator=g).to(dev)
    R = torch.rand(M, N, generator=g).to(dev)
    C16 = torch.empty(M, N, dtype=torch.float16, device=dev)
    C32 = torch.empty(M, N, dtype=torch.float32, device=dev)
    _lib.check(lib.mec_gemm_f16(_p(A), _p(B), _p(bias), _p(R), 1, _p(C16), _p(C32), M, N, K, act, _s()), 'gemm')
    torch.cuda.synchronize()
    ref = A.float() @ B.float().t() + bias + R
    ref = torch.relu(ref) if act == 1 else (torch.nn.functional.gelu(ref) if act == 2 else ref)
    assert _rel_err(C32, ref) < 1e-5
    assert _rel_err(C16.float(), ref) < 2e-3


TILE_IDS = [64, 128, 256, 1064, 1128, 10064, 10128, 10256, 11064, 11128, 20256, 30256, 20128, 50128, 60128, 50256]


def _forced(lib, tid, fn):
    assert lib.mec_set_option(b'gemm_bn', tid) == 0, f'tile id {tid} rejected'
    try:
        fn()
    finally:
        lib.mec_set_option(b'gemm_bn', 0)


@pytest.mark.parametrize('amode', ['gemm', 'conv', 'conv1x1'])
def test_every_tile_bit_identical(dev, amode):
    """Every tile id (width, wave layout, MFMA shape, K-stage depth) accumulates each output
    along the same k order, so the autotuner's choice must not change a single bit."""
    lib = _lib.load()
    g = torch.Generator().manual_seed(7)
    outs = {}
    if amode == 'gemm':
        M, N, K = 1000, 768, 768
        A = (torch.rand(M, K, generator=g) * 2 - 1).half().to(dev)
        B = (torch.rand(N, K, generator=g) * 2 - 1).mul(K ** -0.5).half().to(dev)
        bias = torch.rand(N, generator=g).to(dev)
        R = torch.rand(M, N, generator=g).to(dev)
        ref = torch.nn.functional.gelu(A.float() @ B.float().t() + bias + R)
        for tid in TILE_IDS + [40256, 41256]:
            C16 = torch.empty(M, N, dtype=torch.float16, device=dev)
            C32 = torch.empty(M, N, device=dev)
            _forced(lib, tid, lambda: _lib.check(lib.mec_gemm_f16(_p(A), _p(B), _p(bias), _p(R), 1, _p(C16), _p(C32),
                                                                  M, N, K, 2, _s()), f'gemm {tid}'))
            torch.cuda.synchronize()
            assert _rel_err(C32, ref) < 1e-5, tid
            outs[tid] = (C16.cpu(), C32.cpu())
    else:
        n, H, C, Co = 3, 15, 64, 256
        ks, st, pd = (3, 2, 1) if amode == 'conv' else (1, 1, 0)
        x = torch.rand(n, H, H, C, generator=g).half().to(dev)
        w = ((torch.rand(Co, ks, ks, C, generator=g) * 2 - 1) * (C * ks * ks) ** -0.5).half().to(dev)
        bias = torch.rand(Co, generator=g).to(dev)
        OH = (H + 2 * pd - ks) // st + 1
        ref = torch.relu(torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(),
                                                    bias, stride=st, padding=pd)).permute(0, 2, 3, 1)
        for tid in TILE_IDS:
            y = torch.empty(n, OH, OH, Co, dtype=torch.float16, device=dev)
            _forced(lib, tid, lambda: _lib.check(lib.mec_conv_f16(_p(x), _p(w), _p(bias), None, _p(y), n, H, H, C, Co,
                                                                  ks, st, pd, 1, _s()), f'conv {tid}'))
            torch.cuda.synchronize()
            assert _rel_err(y.float(), ref) < 2e-3, tid
            outs[tid] = (y.cpu(),)
    first = outs[TILE_IDS[0]]
    for tid, o in outs.items():
        for a, b in zip(o, first):
            assert torch.equal(a, b), f'tile {tid} differs from tile {TILE_IDS[0]}'


@pytest.mark.parametrize('M,K', [(256, 64), (300, 128), (513, 192), (1000, 3072), (4096, 768)])
def test_pingpong_tile_k_tails(dev, M, K):
    """The ping-pong tiles (40256, 41256) at 1, 2, 3, 48 and 12 K tiles: their prologue /
    restage / vmcnt tails, against torch and bit-identical to the 10256 tile."""
    lib = _lib.load()
    N = 512
    g = torch.Generator().manual_seed(M + K)
    A = (torch.rand(M, K, generator=g) * 2 - 1).half().to(dev)
    B = (torch.rand(N, K, generator=g) * 2 - 1).mul(K ** -0.5).half().to(dev)
    bias = torch.rand(N, generator=g).to(dev)
    ref = A.float() @ B.float().t() + bias
    outs = []
    for tid in (40256, 41256, 10256):
        C32 = torch.empty(M, N, device=dev)
        _forced(lib, tid, lambda: _lib.check(lib.mec_gemm_f16(_p(A), _p(B), _p(bias), None, 0, None, _p(C32),
                                                              M, N, K, 0, _s()), f'gemm {tid}'))
        torch.cuda.synchronize()
        assert _rel_err(C32, ref) < 1e-5, tid
        outs.append(C32.cpu())
    assert all(torch.equal(o, outs[-1]) for o in outs[:-1])


@pytest.mark.parametrize('M,N', [(300, 512), (2304 + 100, 768), (8192, 3072)])
def test_pingpong_group_order_bit_identical(dev, M, N):
    """Tile order inside an XCD's range (gemm_group_m 0 / 2 / 4 / 8 / 16), short last groups
    and partial M tiles included: every order writes the same bits (each output keeps its k
    chain; only which workgroup computes which tile changes)."""
    lib = _lib.load()
    K = 768
    g = torch.Generator().manual_seed(M + N)
    A = (torch.rand(M, K, generator=g) * 2 - 1).half().to(dev)
    B = (torch.rand(N, K, generator=g) * 2 - 1).mul(K ** -0.5).half().to(dev)
    bias = torch.rand(N, generator=g).to(dev)
    ref = A.float() @ B.float().t() + bias
    outs = []
    try:
        for gm in (0, 2, 4, 8, 16):
            _lib.check(lib.mec_set_option(b'gemm_group_m', gm), 'gemm_group_m')
            C32 = torch.empty(M, N, device=dev)
            _forced(lib, 40256, lambda: _lib.check(lib.mec_gemm_f16(_p(A), _p(B), _p(bias), None, 0, None, _p(C32),
                                                                    M, N, K, 0, _s()), f'gemm gm={gm}'))
            torch.cuda.synchronize()
            assert _rel_err(C32, ref) < 1e-5, gm
            outs.append(C32.cpu())
    finally:
        lib.mec_set_option(b'gemm_group_m', 8)
    assert all(torch.equal(o, outs[0]) for o in outs[1:])


@pytest.mark.parametrize('tile,M,N', [(10256, 2304 + 100, 768), (1128, 300, 512), (11064, 8192, 3072)])
def test_glds_group_order_bit_identical(dev, tile, M, N):
    """The same for the multi-stage engine (gemm_glds_group_m), on plain f16 operands and on
    split-f16 (fp32x3) operands at both term orders (pass-major on the tile itself, K-interleaved
    on its 7xxxx counterpart): every tile order writes the same bits."""
    lib = _lib.load()
    K = 768
    tile_x3i = {10256: 70256, 1128: 71128, 11064: 71064}[tile]
    g = torch.Generator().manual_seed(M + N + tile)
    A = (torch.rand(2, M, K, generator=g) * 2 - 1).half().to(dev)
    B = (torch.rand(2, N, K, generator=g) * 2 - 1).mul(K ** -0.5).half().to(dev)
    bias = torch.rand(N, generator=g).to(dev)
    outs, outs3 = [], {0: [], 1: []}
    try:
        for gm in (0, 2, 4, 8, 16):
            _lib.check(lib.mec_set_option(b'gemm_glds_group_m', gm), 'gemm_glds_group_m')
            C32 = torch.empty(M, N, device=dev)
            _forced(lib, tile, lambda: _lib.check(lib.mec_gemm_f16(_p(A[0]), _p(B[0]), _p(bias), None, 0, None,
                                                                   _p(C32), M, N, K, 0, _s()), f'gemm gm={gm}'))
            torch.cuda.synchronize()
            outs.append(C32.cpu())
            for order, t in ((0, tile), (1, tile_x3i)):
                _lib.check(lib.mec_set_option(b'gemm_x3_order', order), 'gemm_x3_order')
                D32 = torch.empty(M, N, device=dev)
                _forced(lib, t, lambda: _lib.check(lib.mec_gemm_f16x3(_p(A), M * K, _p(B), N * K, ctypes.c_float(1.0),
                                                                      _p(bias), None, None, 0, _p(D32), M, N, K, 0,
                                                                      _s()), f'split gemm gm={gm} order={order}'))
                torch.cuda.synchronize()
                outs3[order].append(D32.cpu())
    finally:
        lib.mec_set_option(b'gemm_glds_group_m', 8)
        lib.mec_set_option(b'gemm_x3_order', 1)
    ref = A[0].float() @ B[0].float().t() + bias
    assert _rel_err(outs[0].to(dev), ref) < 1e-5
    assert all(torch.equal(o, outs[0]) for o in outs[1:])
    for order in (0, 1):
        assert all(torch.equal(o, outs3[order][0]) for o in outs3[order][1:]), f'order {order}'


def test_gemm_f16_residual_f16_asymmetric(dev):
    """A = I with an asymmetric B catches a transposed C write."""
    lib = _lib.load()
    M = N = K = 128
    A = torch.eye(M, dtype=torch.float16, device=dev)
    B = torch.arange(N * K, dtype=torch.float32).reshape(N, K).remainder(97).half().to(dev)
    R = torch.ones(M, N, dtype=torch.float16, device=dev)
    C32 = torch.empty(M, N, device=dev)
    _lib.check(lib.mec_gemm_f16(_p(A), _p(B), None, _p(R), 0, None, _p(C32), M, N, K, 0, _s()), 'gemm')
    torch.cuda.synchronize()
    assert torch.equal(C32, B.float().t() + 1)


@pytest.mark.parametrize('n,H,C,Cout,ks,stride,pad', [(2, 14, 64, 64, 3, 1, 1), (3, 15, 128, 128, 3, 2, 1),
                                                     (2, 28, 256, 512, 1, 2, 0), (1, 7, 512, 128, 3, 1, 1)])
def test_conv_f16(dev, n, H, C, Cout, ks, stride, pad):
    lib = _lib.load()
    g = torch.Generator().manual_seed(H * C)
    x = torch.rand(n, C, H, H, generator=g).half()
    w = ((torch.rand(Cout, C, ks, ks, generator=g) * 2 - 1) * (C * ks * ks) ** -0.5).half()
    bias = torch.rand(Cout, generator=g)
    ref = torch.nn.functional.conv2d(x.float(), w.float(), bias, stride=stride, padding=pad)
    ref = torch.relu(ref)
    OH = ref.shape[2]
    xd = x.permute(0, 2, 3, 1).contiguous().to(dev)
    wd = w.permute(0, 2, 3, 1).contiguous().to(dev)
    y = torch.empty(n, OH, OH, Cout, dtype=torch.float16, device=dev)
    _lib.check(lib.mec_conv_f16(_p(xd), _p(wd), _p(bias.to(dev)), None, _p(y), n, H, H, C, Cout, ks, stride, pad,
                                1, _s()), 'conv')
    torch.cuda.synchronize()
    got = y.float().cpu().permute(0, 3, 1, 2)
    assert _rel_err(got, ref) < 2e-3


def test_resize_bit_exact(dev, golden):
    lib = _lib.load()
    g = golden('image_resize.npz')
    gray = torch.from_numpy(g['gray']).to(dev)
    out = torch.empty(gray.shape[0], 224, 224, dtype=torch.uint8, device=dev)
    _lib.check(lib.mec_resize_u8(_p(gray), gray.shape[0], 48, 48, _p(out), 224, 224, _s()), 'resize')
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), g['resized'])


def test_resize_bit_exact_many(dev):
    from mec import synthetic as syn
    from oracle.resize import resize_bilinear_u8
    lib = _lib.load()
    gray = syn.image_inputs(64, seed=99)
    gd = torch.from_numpy(gray).to(dev)
    out = torch.empty(64, 224, 224, dtype=torch.uint8, device=dev)
    _lib.check(lib.mec_resize_u8(_p(gd), 64, 48, 48, _p(out), 224, 224, _s()), 'resize')
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), resize_bilinear_u8(gray))


@pytest.mark.parametrize('B', [1, 7, 256])
def test_fusion_split_bit_identical(dev, B):
    """The three-launch fusion (projection / cross-attention per modality, then the head)
    against the single fused kernel at the same samples-per-block value: bit-identical.
    (R = 4 itself differs from R = 1 / 2 by an ulp in both forms: not compared across R.)"""
    from mec import engine, synthetic as syn
    lib = _lib.load()
    m = engine.FusionHead(device=dev)
    g = torch.Generator().manual_seed(B)
    args = [torch.randn(B, d, generator=g).to(dev) for d in (64, 768, 512)]
    args += [torch.softmax(torch.randn(B, 7, generator=g), 1).to(dev) for _ in range(3)]
    outs = {}
    for split in (0, 1):
        for r in (1, 2, 4):
            m.set_option('fusion_split', split)
            m.set_option('fusion_r', r)
            outs[split, r] = [t.cpu() for t in m.forward(*args)]
    for r in (1, 2, 4):
        for a, b in zip(outs[1, r], outs[0, r]):
            assert torch.equal(a, b), r


@pytest.mark.parametrize('n', [1, 3, 37, 75])
def test_conv3x3_c64_bit_identical(dev, n):
    """ResNet layer1's 3x3 conv (56x56, 64 -> 64) on the halo-tile kernel (conv3x3.hip) vs the
    implicit-GEMM path: bit-identical, and close to torch fp32. n = 37 / 75 give 259 / 525
    tiles, so workgroups walk several tiles through both halo buffers."""
    lib = _lib.load()
    g = torch.Generator().manual_seed(n)
    x = torch.rand(n, 56, 56, 64, generator=g).half().to(dev)
    w = ((torch.rand(64, 3, 3, 64, generator=g) * 2 - 1) * 576 ** -0.5).half().to(dev)
    bias = (torch.rand(64, generator=g) - 0.5).to(dev)
    outs = []
    for direct in (1, 0):
        _lib.check(lib.mec_set_option(b'conv3x3_direct', direct), 'option')
        y = torch.full((n, 56, 56, 64), float('nan'), dtype=torch.float16, device=dev)
        try:
            _lib.check(lib.mec_conv_f16(_p(x), _p(w), _p(bias), None, _p(y), n, 56, 56, 64, 64, 3, 1, 1, 1, _s()),
                       'conv')
        finally:
            lib.mec_set_option(b'conv3x3_direct', 1)
        torch.cuda.synchronize()
        outs.append(y.cpu())
    ref = torch.relu(torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(), bias,
                                                padding=1)).permute(0, 2, 3, 1).cpu()
    assert not torch.isnan(outs[0]).any()
    assert _rel_err(outs[0].float(), ref) < 2e-3
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize('H,C', [(28, 128), (14, 256)])
@pytest.mark.parametrize('n', [1, 6, 13])
def test_conv3x3_halo(dev, H, C, n):
    """ResNet layers 2-3's stride-1 3x3 convs (28x28x128, 14x14x256) on the halo kernel
    (conv3x3_halo.hip) vs the implicit-GEMM path and torch fp32: the same fp32 accumulation in
    another order, so within f16 output rounding of the GEMM path, not bit-identical. A batch
    split gives the same bits (image 0 alone = image 0 of the batch); n = 13 gives 52 / 26 tiles
    on partially filled XCD groups."""
    lib = _lib.load()
    g = torch.Generator().manual_seed(1000 * n + H)
    x = torch.rand(n, H, H, C, generator=g).half().to(dev)
    w = ((torch.rand(C, 3, 3, C, generator=g) * 2 - 1) * (9 * C) ** -0.5).half().to(dev)
    bias = (torch.rand(C, generator=g) - 0.5).to(dev)

    def run(halo, xx):
        y = torch.full(xx.shape, float('nan'), dtype=torch.float16, device=dev)
        _lib.check(lib.mec_set_option(b'conv3x3_halo', halo), 'option')
        try:
            _lib.check(lib.mec_conv_f16(_p(xx), _p(w), _p(bias), None, _p(y), xx.shape[0], H, H, C, C, 3, 1, 1, 1, _s()),
                       'conv')
        finally:
            lib.mec_set_option(b'conv3x3_halo', 1)
        torch.cuda.synchronize()
        return y.cpu()

    yh, yg = run(1, x), run(0, x)
    ref = torch.relu(torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(), bias,
                                                padding=1)).permute(0, 2, 3, 1).cpu()
    assert not torch.isnan(yh).any()
    assert _rel_err(yh.float(), ref) < 2e-3
    # both paths round an fp32 sum of the same products (reassociation error ~1e-5 absolute
    # at these magnitudes) to f16: one f16 ulp apart at most, plus that error near zero
    d = (yh.float() - yg.float()).abs()
    ulp = torch.maximum(yh.float().abs(), yg.float().abs()).clamp_min(2 ** -14) * 2 ** -10
    assert bool((d <= ulp + 1e-4).all()), float((d - ulp).max())
    assert torch.equal(run(1, x[:1].contiguous())[0], yh[0])


@pytest.mark.parametrize('B', [3, 37])
def test_pw_chain_bit_identical(dev, B):
    """ResNet50 with layer1's seam kernels (pw_chain.hip: block 1 -> 2 dual seam, block 2 -> 3
    and 3 -> layer2 residual seams, in both weight placements) and with the GEMMs they
    replace: identical features, logits and probabilities (B = 3: 147 tiles, fewer than the
    CUs; B = 37: 1813 tiles, several per workgroup through every buffer)."""
    from mec import engine, synthetic as syn
    lib = _lib.load()
    enc = engine.ImageEncoder(device=dev)
    gray = engine.to_device(syn.image_inputs(B, seed=77 + B), dev)
    outs = []
    for chain, form in ((0, 0), (1, 0), (2, 0), (2, 1), (2, 2)):
        enc.set_option('pw_chain', chain)
        enc.set_option('pw_chain_form', form)
        res = enc.forward(gray)
        torch.cuda.synchronize()
        outs.append([t.cpu() for t in res])
    for o in outs[1:]:
        for a, b in zip(o, outs[0]):
            assert torch.equal(a, b)


@pytest.mark.parametrize('precision', ['f16', 'fp32'])
def test_bert_layernorm_rows_per_wave_bit_identical(dev, precision):
    """bert_layernorm_kernel<RW> (bert_ln_rows 1 / 2 / 4): each row's arithmetic is the same at
    any rows-per-wave, so the encoder's outputs are the same bits."""
    from mec import engine, synthetic as syn
    m = engine.TextEncoder(device=dev, precision=precision)
    ids, mask = syn.text_inputs(9, 128, seed=77, ragged=True)
    args = (engine.to_device(ids, dev), engine.to_device(mask, dev))
    outs = []
    for rw in (1, 2, 4):
        m.set_option('bert_ln_rows', rw)
        outs.append([t.cpu() for t in m.forward(*args)])
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)
