"""fp32 path (mec_create_ex(..., MEC_PREC_FP32)): the precision the reference computes in
(inference/text_inference.py:91-93, inference/image_inference.py:116-118 — torch fp32).

Every BERT and ResNet50 GEMM runs on v_mfma_f32_32x32x2_f32 (an exact f32 fmaf chain);
the only deviation from the oracle is the summation order, so the bar is far tighter than
the f16 path's 1e-3: softmax probabilities within FP32_PROB_TOL of the oracle and argmax
exact on every row, with no near-tie exclusion.
"""
import ctypes

import numpy as np
import pytest
import torch

from mec import _lib, engine, synthetic as syn
from oracle import fusion as o_f, image as o_i, speech as o_s, text as o_t

pytestmark = pytest.mark.gpu

FP32_PROB_TOL = 1e-5   # probs, fp32 path vs the fp32 oracle (order of summation only)
FP32_FEAT_RTOL = 1e-4  # features, max |d| / max |ref|


def _np(ts):
    torch.cuda.synchronize()
    return [t.cpu().numpy() for t in ts]


def _report(name, got, ref):
    err = float(np.abs(got - ref).max())
    agree = int((got.argmax(1) == ref.argmax(1)).sum())
    s = np.sort(ref, axis=1)
    print(f'{name}: rows {len(got)}, probs max|d| {err:.3g}, argmax {agree}/{len(got)}, '
          f'min top-2 margin {(s[:, -1] - s[:, -2]).min():.3g}')
    return err, agree


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


@pytest.fixture
def tile_option():
    lib = _lib.load()
    yield lib
    assert lib.mec_set_option(b'gemm_f32_tile', 0) == 0


@pytest.mark.parametrize('M,N,K,act,res', [(300, 192, 256, 1, True), (256, 128, 768, 4, False),
                                           (1000, 256, 96, 0, True), (64, 64, 32, 0, False)])
def test_gemm_f32_vs_fp64(dev, tile_option, M, N, K, act, res):
    """mec_gemm_f32 against an fp64 reference; the tiles of one MFMA shape (32x32x2: 1-4,
    16x16x4: 5-8) give bit-identical results (each output is the same k-ordered fmaf chain)."""
    lib = tile_option
    g = torch.Generator().manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g)
    B = torch.randn(N, K, generator=g) / np.sqrt(K)
    bias = torch.randn(N, generator=g)
    R = torch.randn(M, N, generator=g) if res else None
    ref = A.double() @ B.double().T + bias.double()
    if res:
        ref = ref + R.double()
    if act == 1:
        ref = ref.clamp_min(0)
    elif act == 4:
        ref = torch.nn.functional.gelu(ref)
    outs = []
    for tile in range(1, 9):
        if N % {1: 128, 2: 128, 3: 64, 4: 256}[(tile - 1) % 4 + 1]:
            continue
        assert lib.mec_set_option(b'gemm_f32_tile', tile) == 0
        dA, dB, db = A.to(dev), B.to(dev), bias.to(dev)
        dR = R.to(dev) if res else None
        C = torch.empty(M, N, device=dev)
        _lib.check(lib.mec_gemm_f32(_ptr(dA), _ptr(dB), _ptr(db), _ptr(dR), _ptr(C), M, N, K, act, _stream(dev)),
                   'mec_gemm_f32')
        torch.cuda.synchronize()
        outs.append((tile, C.cpu()))
    scale = float((A.abs().double() @ B.abs().double().T).max()) + 1.0
    first = {}
    for tile, C in outs:
        err = float((C.double() - ref).abs().max())
        print(f'tile {tile}: max|d| {err:.3g} (scale {scale:.3g})')
        assert err <= 2e-6 * scale
        shape = 32 if tile <= 4 else 16  # tiles of one MFMA shape sum in one k order
        first.setdefault(shape, (tile, C))
        assert torch.equal(C, first[shape][1]), f'tile {tile} differs from tile {first[shape][0]}'


@pytest.mark.parametrize('H,C,Cout,ks,stride,pad', [(14, 64, 128, 3, 2, 1), (7, 128, 64, 3, 1, 1),
                                                    (8, 32, 64, 1, 2, 0)])
def test_conv_f32_vs_fp64(dev, H, C, Cout, ks, stride, pad):
    lib = _lib.load()
    g = torch.Generator().manual_seed(H * C)
    n = 3
    x = torch.randn(n, C, H, H, generator=g)
    w = torch.randn(Cout, C, ks, ks, generator=g) / np.sqrt(C * ks * ks)
    b = torch.randn(Cout, generator=g)
    ref = torch.nn.functional.conv2d(x.double(), w.double(), b.double(), stride=stride, padding=pad).clamp_min(0)
    OH = ref.shape[2]
    xn = x.permute(0, 2, 3, 1).contiguous().to(dev)
    wn = w.permute(0, 2, 3, 1).contiguous().to(dev)
    y = torch.empty(n, OH, OH, Cout, device=dev)
    _lib.check(lib.mec_conv_f32(_ptr(xn), _ptr(wn), _ptr(b.to(dev)), None, _ptr(y), n, H, H, C, Cout, ks, stride, pad,
                                1, _stream(dev)), 'mec_conv_f32')
    torch.cuda.synchronize()
    err = float((y.cpu().permute(0, 3, 1, 2).double() - ref).abs().max())
    print(f'conv f32 max|d| {err:.3g}')
    assert err <= 1e-5


def test_precision_query(dev):
    t = engine.TextEncoder(device=dev, precision='fp32')
    assert t.lib.mec_precision(t.handle) == 1
    s = engine.SpeechEncoder(device=dev)
    assert s.lib.mec_precision(s.handle) == 1  # speech is fp32 at either setting
    with pytest.raises(ValueError):
        engine.TextEncoder(device=dev, precision='bf16')
    m = engine.MobileNetImageEncoder(device=dev, precision='fp32')
    assert m.lib.mec_precision(m.handle) == 1


@pytest.mark.parametrize('precision', ['fp32', 'fp32x3'])
def test_text_fp32_golden(dev, golden, precision):
    """BERT at both fp32-class precisions (the exact-f32 engine, and fp32x3 -- the bench headline's)
    against the fixture pinned to HF BertForSequenceClassification (eager): probs within 1e-5, CLS
    feature within 1e-4 relative, argmax exact (inference/text_inference.py:124-127)."""
    gd = golden('text_bert.npz')
    enc = engine.TextEncoder(device=dev, precision=precision)
    cls, logits, probs = _np(enc.forward(engine.to_device(gd['ids'], dev), engine.to_device(gd['mask'], dev)))
    enc.check()
    err, agree = _report(f'text {precision} golden', probs, gd['probs'])
    ferr = float(np.abs(cls - gd['cls']).max() / np.abs(gd['cls']).max())
    print(f'  cls rel err {ferr:.3g}, logits max|d| {np.abs(logits - gd["logits"]).max():.3g}')
    assert agree == len(probs) and err <= FP32_PROB_TOL and ferr <= FP32_FEAT_RTOL


@pytest.mark.parametrize('precision', ['fp32', 'fp32x3'])
def test_image_fp32_golden(dev, golden, precision):
    """ResNet50 + head at both fp32-class precisions against the committed image fixture
    (tests/golden/image_full.npz: the oracle/image.py restatement, torchvision absent, so
    restatement-pinned; its resize is PIL-pinned): probs within 1e-5, 512-d feature within 1e-4
    relative, argmax exact (inference/image_inference.py:116-118)."""
    gd = golden('image_full.npz')
    enc = engine.ImageEncoder(device=dev, precision=precision)
    feat, logits, probs = _np(enc.forward(engine.to_device(gd['gray'], dev)))
    enc.check()
    err, agree = _report(f'image {precision} golden', probs, gd['probs'])
    ferr = float(np.abs(feat - gd['feat']).max() / np.abs(gd['feat']).max())
    print(f'  feat rel err {ferr:.3g}, logits max|d| {np.abs(logits - gd["logits"]).max():.3g}')
    assert agree == len(probs) and err <= FP32_PROB_TOL and ferr <= FP32_FEAT_RTOL


@pytest.mark.parametrize('B,ragged', [(16, True), (128, False)])
def test_text_fp32_vs_oracle(dev, B, ragged):
    ids, mask = syn.text_inputs(B, 128, seed=40 + B, ragged=ragged)
    enc = engine.TextEncoder(device=dev, precision='fp32')
    cls, logits, probs = _np(enc.forward(engine.to_device(ids, dev), engine.to_device(mask, dev)))
    sub = np.unique(np.r_[0, 1, np.arange(0, B, max(1, B // 12)), B - 1])
    rc, rl, rp = o_t.forward(syn.weights('text'), ids[sub], mask[sub])
    err, agree = _report(f'text fp32 B={B}', probs[sub], rp)
    ferr = float(np.abs(cls[sub] - rc).max() / np.abs(rc).max())
    print(f'  cls rel err {ferr:.3g}, logits max|d| {np.abs(logits[sub] - rl).max():.3g}')
    assert agree == len(sub) and err <= FP32_PROB_TOL and ferr <= FP32_FEAT_RTOL


@pytest.mark.parametrize('B', [3, 32])
def test_image_fp32_vs_oracle(dev, B):
    gray = syn.image_inputs(B, seed=50 + B)
    enc = engine.ImageEncoder(device=dev, precision='fp32')
    feat, logits, probs = _np(enc.forward(engine.to_device(gray, dev)))
    sub = np.unique(np.r_[0, np.arange(0, B, max(1, B // 6)), B - 1])
    rf, rl, rp = o_i.forward(syn.weights('image'), gray[sub])
    err, agree = _report(f'image fp32 B={B}', probs[sub], rp)
    ferr = float(np.abs(feat[sub] - rf).max() / np.abs(rf).max())
    print(f'  feat rel err {ferr:.3g}, logits max|d| {np.abs(logits[sub] - rl).max():.3g}')
    assert agree == len(sub) and err <= FP32_PROB_TOL and ferr <= FP32_FEAT_RTOL


def test_image_fp32_rgb_and_gray224(dev):
    """The already-resized entry points (mec_image_fwd_u8: [B,224,224,1] and RGB [B,224,224,3])."""
    rng = np.random.default_rng(5)
    enc = engine.ImageEncoder(device=dev, precision='fp32')
    for C in (1, 3):
        img = rng.integers(0, 256, (2, 224, 224, C), dtype=np.uint8)
        feat, logits, probs = _np(enc.forward_u8(engine.to_device(img, dev)))
        rf, rl, rp = o_i.forward_resized(syn.weights('image'), img[..., 0] if C == 1 else img)
        err, agree = _report(f'image fp32 224x224x{C}', probs, rp)
        assert agree == 2 and err <= FP32_PROB_TOL


@pytest.mark.parametrize('B', [1, 7, 64])
def test_image_fp32_gray_stem_matches_im2col(dev, B):
    """The gray-input stem as one conv + BN + ReLU + max-pool kernel (stem_pool_gray_f32_kernel:
    channels folded into (pixel, inside) taps) against the im2col GEMM + pool path it replaces:
    the same network output to fp32 reassociation (B = 64: 3,136 tiles, several per CU)."""
    gray = engine.to_device(syn.image_inputs(B, seed=90 + B), dev)
    enc = engine.ImageEncoder(device=dev, precision='fp32')
    outs = []
    for v in (0, 1):
        enc.set_option('stem_gray_f32', v)
        outs.append(_np(enc.forward(gray)))
    (f0, l0, p0), (f1, l1, p1) = outs
    assert not np.isnan(f1).any()
    ferr = float(np.abs(f1 - f0).max() / np.abs(f0).max())
    perr = float(np.abs(p1 - p0).max())
    print(f'gray stem vs im2col B={B}: feat rel {ferr:.3g}, probs max|d| {perr:.3g}')
    assert ferr <= 1e-5 and perr <= 1e-6 and (p1.argmax(1) == p0.argmax(1)).all()


def test_fused_fp32_end_to_end(dev):
    """Fused probs of the fp32 pipeline against the oracle chain o_f(o_s, o_t, o_i)
    (inference/multimodal_fusion.py:271-278), B = 24 with ragged text."""
    B = 24
    x = syn.speech_inputs(B, seed=61)
    ids, mask = syn.text_inputs(B, 128, seed=61, ragged=True)
    gray = syn.image_inputs(B, seed=61)
    pipe = engine.FusedPipeline(device=dev, precision='fp32')
    args = [engine.to_device(a, dev) for a in (x, ids, mask, gray)]
    pipe.forward(*args)
    out = pipe.forward(*args)
    pipe.wait()
    got = {k: _np(v) for k, v in out.items()}
    rs = o_s.forward(syn.weights('speech'), x)
    rt = o_t.forward(syn.weights('text'), ids, mask)
    ri = o_i.forward(syn.weights('image'), gray)
    rf = o_f.forward(syn.weights('fusion'), rs[0], rt[0], ri[0], rs[2], rt[2], ri[2])
    for name, g, r in (('speech', got['speech'][2], rs[2]), ('text', got['text'][2], rt[2]),
                       ('image', got['image'][2], ri[2]), ('fused', got['fusion'][1], rf[1])):
        err, agree = _report(f'fp32 pipeline {name}', g, r)
        assert agree == B and err <= FP32_PROB_TOL, name


@pytest.mark.parametrize('B', [3, 32])
def test_mobilenet_v2_fp32_vs_oracle(dev, B):
    """MobileNetV2 backbone (BASELINE config "Image-only: MobileNetV2 on 48x48x1") in fp32."""
    from oracle import image_mbv2 as o_mb
    gray = syn.image_inputs(B, seed=70 + B)
    enc = engine.MobileNetImageEncoder(device=dev, precision='fp32')
    feat, logits, probs = _np(enc.forward(engine.to_device(gray, dev)))
    sub = np.unique(np.r_[0, np.arange(0, B, max(1, B // 6)), B - 1])
    rf, rl, rp = o_mb.forward(syn.weights('image_mbv2'), gray[sub])
    err, agree = _report(f'mobilenet_v2 fp32 B={B}', probs[sub], rp)
    ferr = float(np.abs(feat[sub] - rf).max() / np.abs(rf).max())
    print(f'  feat rel err {ferr:.3g}, logits max|d| {np.abs(logits[sub] - rl).max():.3g}')
    assert agree == len(sub) and err <= FP32_PROB_TOL and ferr <= FP32_FEAT_RTOL


@pytest.mark.parametrize('enc,B', [('image', 256), ('text', 128)])
def test_fp32_batch_invariance(dev, enc, B):
    """With the fp32 autotune held to one MFMA family (gemm_f32_family 16, the default) every
    shape sums in one k order: rows of a full-size batch equal the same rows run as B = 16, bit
    for bit, although the tuned tiles differ between the two batch sizes."""
    if enc == 'image':
        m = engine.ImageEncoder(device=dev, precision='fp32')
        args = (engine.to_device(syn.image_inputs(B, seed=41), dev),)
    else:
        m = engine.TextEncoder(device=dev, precision='fp32')
        ids, mask = syn.text_inputs(B, 128, seed=41, ragged=True)
        args = (engine.to_device(ids, dev), engine.to_device(mask, dev))
    big = [t[:16].cpu() for t in m.forward(*args)]
    small = [t.cpu() for t in m.forward(*(a[:16] for a in args))]
    for i, (a, b) in enumerate(zip(big, small)):
        assert torch.equal(a, b), f'{enc} output {i}: rows of B={B} differ from the B=16 run'
