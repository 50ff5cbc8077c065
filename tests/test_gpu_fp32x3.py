"""GPU: the fp32x3 path (MEC_PREC_FP32X3) -- the fp32 path's arithmetic with every GEMM / conv
operand carried as a pair of f16 planes (hi + lo, 22 significant bits, activations at a per-tensor
power-of-two plane scale) on the f16 MFMA (three products per fp32 product, one fp32 accumulator) -- held to the fp32 path's own bars against the oracle: probs within
1e-5, features within 1e-4 relative, argmax exact on every row; and compared with the exact
fp32 path on the same inputs (the two differ by reassociation-scale amounts only)."""
import numpy as np
import pytest
import torch

from mec import engine, synthetic as syn
from oracle import image as o_i, text as o_t

pytestmark = pytest.mark.gpu

PROB_TOL, FEAT_RTOL = 1e-5, 1e-4


def _np(ts):
    torch.cuda.synchronize()
    return [t.cpu().numpy() for t in ts]


def _report(name, got, ref, got32):
    err = float(np.abs(got - ref).max())
    e32 = float(np.abs(got32 - ref).max())
    agree = int((got.argmax(1) == ref.argmax(1)).sum())
    s = np.sort(ref, axis=1)
    print(f'{name}: probs max|d| vs oracle {err:.3g} (exact fp32 path {e32:.3g}), argmax {agree}/{len(got)}, '
          f'min top-2 margin {(s[:, -1] - s[:, -2]).min():.3g}')
    return err, agree


@pytest.mark.parametrize('B,ragged', [(3, True), (64, True), (128, False)])
def test_text_fp32x3_vs_oracle(dev, B, ragged):
    ids, mask = syn.text_inputs(B, 128, seed=500 + B, ragged=ragged)
    args = (engine.to_device(ids, dev), engine.to_device(mask, dev))
    cls, logits, probs = _np(engine.TextEncoder(device=dev, precision='fp32x3').forward(*args))
    cls32, _, probs32 = _np(engine.TextEncoder(device=dev, precision='fp32').forward(*args))
    sub = np.unique(np.r_[0, np.arange(0, B, max(1, B // 24)), B - 1])
    rc, rl, rp = o_t.forward(syn.weights('text'), ids[sub], mask[sub])
    err, agree = _report(f'text fp32x3 B={B}', probs[sub], rp, probs32[sub])
    ferr = float(np.abs(cls[sub] - rc).max() / np.abs(rc).max())
    print(f'  cls rel err {ferr:.3g} (fp32 path {float(np.abs(cls32[sub] - rc).max() / np.abs(rc).max()):.3g}), '
          f'logits max|d| {np.abs(logits[sub] - rl).max():.3g}; fp32x3 vs fp32 probs {np.abs(probs - probs32).max():.3g}')
    assert agree == len(sub) and err <= PROB_TOL and ferr <= FEAT_RTOL


def test_text_fp32x3_batch_invariance(dev):
    """Rows of a B=128 batch equal the same rows run as B=16, bit for bit (every split tile sums
    each output in the same k order: pass 0, 1, 2, each in k order)."""
    m = engine.TextEncoder(device=dev, precision='fp32x3')
    ids, mask = syn.text_inputs(128, 128, seed=41, ragged=True)
    args = (engine.to_device(ids, dev), engine.to_device(mask, dev))
    big = [t[:16].cpu() for t in m.forward(*args)]
    small = [t.cpu() for t in m.forward(*(a[:16] for a in args))]
    for i, (a, b) in enumerate(zip(big, small)):
        assert torch.equal(a, b), f'output {i}'


@pytest.mark.parametrize('B', [5, 64])
def test_resnet_fp32x3_vs_oracle(dev, B):
    gray = syn.image_inputs(B, seed=600 + B)
    g = engine.to_device(gray, dev)
    feat, logits, probs = _np(engine.ImageEncoder(device=dev, precision='fp32x3').forward(g))
    feat32, _, probs32 = _np(engine.ImageEncoder(device=dev, precision='fp32').forward(g))
    sub = np.unique(np.r_[0, np.arange(0, B, max(1, B // 16)), B - 1])
    rf, rl, rp = o_i.forward(syn.weights('image'), gray[sub])
    err, agree = _report(f'resnet50 fp32x3 B={B}', probs[sub], rp, probs32[sub])
    ferr = float(np.abs(feat[sub] - rf).max() / np.abs(rf).max())
    print(f'  feat rel err {ferr:.3g} (fp32 path {float(np.abs(feat32[sub] - rf).max() / np.abs(rf).max()):.3g}), '
          f'logits max|d| {np.abs(logits[sub] - rl).max():.3g}')
    assert agree == len(sub) and err <= PROB_TOL and ferr <= FEAT_RTOL


def test_resnet_fp32x3_rgb_and_224_gray_inputs(dev):
    """The other u8 entry shapes (already-resized 224 gray, RGB) through the fp32x3 stem."""
    from oracle import image as oi
    enc = engine.ImageEncoder(device=dev, precision='fp32x3')
    rgb = np.stack([syn.image_inputs(2, seed=70 + c).repeat(4, axis=1).repeat(4, axis=2)[:, :224, :224]
                    for c in range(3)], -1)
    rgb = np.ascontiguousarray(np.pad(rgb, ((0, 0), (0, 32), (0, 32), (0, 0)))[:, :224, :224])
    _, _, probs = _np(enc.forward_u8(engine.to_device(rgb, dev)))
    _, _, rp = oi.forward_resized(syn.weights('image'), rgb)
    assert np.abs(probs - rp).max() <= PROB_TOL and (probs.argmax(1) == rp.argmax(1)).all()
    g224 = np.ascontiguousarray(rgb[..., 0])
    _, _, probs = _np(enc.forward_u8(engine.to_device(g224[..., None], dev)))
    _, _, rp = oi.forward_resized(syn.weights('image'), g224)
    assert np.abs(probs - rp).max() <= PROB_TOL


def test_fused_fp32x3_b256_vs_oracle(dev):
    """The whole fused step at the headline config (B=256) on the fp32x3 path against the oracle
    chain o_f(o_s, o_t, o_i) on 32 rows spread over the batch (every row: bench.py's parity)."""
    from oracle import fusion as o_f, speech as o_s
    B = 256
    x = syn.speech_inputs(B, seed=71)
    ids, mask = syn.text_inputs(B, 128, seed=71, ragged=True)
    gray = syn.image_inputs(B, seed=71)
    pipe = engine.FusedPipeline(device=dev, precision='fp32x3')
    args = [engine.to_device(a, dev) for a in (x, ids, mask, gray)]
    pipe.forward(*args)
    out = pipe.forward(*args)
    pipe.check()
    got = {k: _np(v) for k, v in out.items()}
    sub = np.unique(np.r_[np.arange(0, B, 8), B - 1])
    rs = o_s.forward(syn.weights('speech'), x[sub])
    rt = o_t.forward(syn.weights('text'), ids[sub], mask[sub])
    ri = o_i.forward(syn.weights('image'), gray[sub])
    rf = o_f.forward(syn.weights('fusion'), rs[0], rt[0], ri[0], rs[2], rt[2], ri[2])
    for name, g, r in (('text', got['text'][2][sub], rt[2]), ('image', got['image'][2][sub], ri[2]),
                       ('fused', got['fusion'][1][sub], rf[1])):
        err = float(np.abs(g - r).max())
        print(f'fp32x3 fused step {name}: probs max|d| {err:.3g}')
        assert err <= PROB_TOL and (g.argmax(1) == r.argmax(1)).all(), name


def _split(a, scale=1.0):
    x = (np.asarray(a, np.float32) * np.float32(scale)).astype(np.float32)
    hi = x.astype(np.float16)
    lo = (x - hi.astype(np.float32)).astype(np.float16)
    return np.concatenate([hi.ravel(), lo.ravel()]).reshape((2,) + x.shape)


SPLIT_TILES = {0: [64, 128, 256, 1128, 1064, 10064, 10128, 10256, 11128, 11064, 20256, 30256, 20128, 50128, 60128,
                   50256, 40256, 41256],
               1: [70256, 70128, 71128, 71064, 70064, 72128]}


class x3_order:
    """The split engine's term order (option gemm_x3_order: 0 pass-major, 1 K-interleaved, the
    default) as the process default for the handle-less entry points, restored on exit."""

    def __init__(self, order):
        from mec import _lib
        self.lib, self.order = _lib.load(), order

    def __enter__(self):
        from mec import _lib
        _lib.check(self.lib.mec_set_option(b'gemm_x3_order', self.order), 'gemm_x3_order')

    def __exit__(self, *exc):
        self.lib.mec_set_option(b'gemm_x3_order', 1)


@pytest.mark.parametrize('order', [0, 1])
@pytest.mark.parametrize('M,N,K,act', [(512, 256, 768, 0), (1000, 768, 3072, 4), (300, 512, 128, 1),
                                       (1000, 3072, 768, 5)])
def test_split_gemm_vs_fp64_and_every_tile_bit_identical(dev, M, N, K, act, order):
    """mec_gemm_f16x3 (the fp32x3 engine) against float64 A . B^T of the fp32 operands: within the
    fp32 GEMM engine's bar (2e-6 x sum |a b|, tests/test_gpu_fp32.py), with the weights pre-scaled
    by 2^8 and undone by oscale; and, per term order, every tile computes the same bits (each
    output's terms and k chain are tile-independent)."""
    import ctypes
    from mec import _lib
    lib = _lib.load()
    with x3_order(order):
        _split_gemm_tiles(dev, lib, M, N, K, act, order)


def _split_gemm_tiles(dev, lib, M, N, K, act, order):
    import ctypes
    from mec import _lib
    rng = np.random.default_rng(M + N + K)
    A = rng.standard_normal((M, K)).astype(np.float32)
    Bw = (rng.standard_normal((N, K)) * 0.03).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32)
    R = rng.standard_normal((M, N)).astype(np.float32) if act == 0 else None
    Ad = torch.from_numpy(_split(A)).to(dev)
    Bd = torch.from_numpy(_split(Bw, 256.0)).to(dev)
    bd = torch.from_numpy(bias).to(dev)
    Rd = torch.from_numpy(R).to(dev) if R is not None else None
    p = lambda t: ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)  # noqa: E731
    ref = A.astype(np.float64) @ Bw.astype(np.float64).T + bias
    if R is not None:
        ref = ref + R
    if act == 1:
        ref = np.maximum(ref, 0)
    elif act in (4, 5):  # 5: the branch-free erf GELU of the fp32x3 FFN1 (gemm_common.h gelu_f32)
        from scipy.special import erf
        ref = 0.5 * ref * (1 + erf(ref / np.sqrt(2)))
    bound = 2e-6 * (np.abs(A).astype(np.float64) @ np.abs(Bw).astype(np.float64).T + np.abs(bias) + 1)
    outs = {}
    for tile in [0] + SPLIT_TILES[order]:
        width = (256 if 40000 <= tile < 50000 else tile % 1000 if tile >= 70000 else
                 tile % 10000 if tile % 10000 < 1000 else tile % 10000 - 1000)
        if tile and N % width:
            continue
        _lib.check(lib.mec_set_option(b'gemm_bn', tile), 'gemm_bn')
        C = torch.empty((M, N), device=dev)
        try:
            _lib.check(lib.mec_gemm_f16x3(p(Ad), M * K, p(Bd), N * K, ctypes.c_float(1 / 256), p(bd), p(Rd), None, 0,
                                          p(C), M, N, K, act, ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)),
                       f'split gemm tile {tile}')
        finally:
            lib.mec_set_option(b'gemm_bn', 0)
        outs[tile] = C.cpu().numpy()
    got = outs[0]
    err = np.abs(got - ref)
    print(f'split GEMM (order {order}) {M}x{N}x{K} act {act}: max err {err.max():.3g}, '
          f'max err / bound {(err / bound).max():.3g}, tiles {len(outs) - 1}')
    assert (err <= bound).all()
    for tile, o in outs.items():
        assert np.array_equal(o, got), f'tile {tile} differs from the autotuned tile'


@pytest.mark.parametrize('order', [0, 1])
@pytest.mark.parametrize('M,N,K', [(4096, 768, 768), (4096, 768, 3072), (2048, 512, 4608)])
def test_split_gemm_error_vs_exact_fp32_gemm(dev, M, N, K, order):
    """Against float64 on the same fp32 operands (BERT-like scales: activations O(1), weights
    ~0.02-0.05), the split-f16 engine's error is of the exact-fp32 MFMA engine's size (the
    split's 2^-22 operand rounding sits below the fp32 accumulation error): max and RMS error of
    both printed; the split's max error may exceed the exact engine's by at most 50%, at either
    term order."""
    from mec import _lib
    with x3_order(order):
        _split_vs_exact(dev, _lib.load(), M, N, K, order)


def _split_vs_exact(dev, lib, M, N, K, order):
    import ctypes
    from mec import _lib
    rng = np.random.default_rng(K)
    A = rng.standard_normal((M, K)).astype(np.float32)
    W = (rng.standard_normal((N, K)) * (0.02 if K < 4000 else 0.05)).astype(np.float32)
    ref = A.astype(np.float64) @ W.astype(np.float64).T
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    # device operands held in locals until the launches have completed (a temporary passed as a raw
    # pointer is freed on return and its block handed to the next allocation)
    Ad, Wd = torch.from_numpy(A).to(dev), torch.from_numpy(W).to(dev)
    e = float(np.ceil(np.log2(16384 / np.abs(W).max())) - 1)
    Axd, Wxd = torch.from_numpy(_split(A)).to(dev), torch.from_numpy(_split(W, 2.0 ** e)).to(dev)
    C32 = torch.empty((M, N), device=dev)
    _lib.check(lib.mec_gemm_f32(p(Ad), p(Wd), None, None, p(C32), M, N, K, 0, st), 'mec_gemm_f32')
    Cx = torch.empty((M, N), device=dev)
    _lib.check(lib.mec_gemm_f16x3(p(Axd), M * K, p(Wxd), N * K, ctypes.c_float(2.0 ** -e),
                                  None, None, None, 0, p(Cx), M, N, K, 0, st), 'mec_gemm_f16x3')
    torch.cuda.synchronize()
    e32 = np.abs(C32.cpu().numpy() - ref)
    ex3 = np.abs(Cx.cpu().numpy() - ref)
    print(f'{M}x{N}x{K}: exact-fp32 engine max {e32.max():.3g} rms {np.sqrt((e32 ** 2).mean()):.3g}; '
          f'split-f16 engine (order {order}) max {ex3.max():.3g} rms {np.sqrt((ex3 ** 2).mean()):.3g}')
    # both engines within the fp32 GEMM bar (so the comparison below has a sound reference)
    bound = 2e-6 * (np.abs(A).astype(np.float64) @ np.abs(W).astype(np.float64).T + 1)
    assert (e32 <= bound).all() and (ex3 <= bound).all()
    assert ex3.max() <= 1.5 * e32.max()


@pytest.mark.parametrize('order,tile', [(0, 0), (0, 40256), (0, 10256), (0, 11128), (1, 0), (1, 70256), (1, 71128)])
def test_split_gemm_plane_output(dev, order, tile):
    """C16 written as hi / lo planes (c_lo): hi = f16(v), lo = f16(v - hi), for v the fp32 result
    the same launch writes to C32 on another call; on the ping-pong tile this is its staged
    f16 fast-path epilogue run once per plane."""
    from mec import _lib
    with x3_order(order):
        _plane_output(dev, _lib.load(), tile)


def _plane_output(dev, lib, tile):
    import ctypes
    from mec import _lib
    M, N, K = 700, 512, 768
    rng = np.random.default_rng(7)
    A = rng.standard_normal((M, K)).astype(np.float32)
    Bw = (rng.standard_normal((N, K)) * 0.03).astype(np.float32)
    bias = rng.standard_normal(N).astype(np.float32)
    Ad = torch.from_numpy(_split(A)).to(dev)
    Bd = torch.from_numpy(_split(Bw, 256.0)).to(dev)
    bd = torch.from_numpy(bias).to(dev)
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    C32 = torch.empty((M, N), device=dev)
    C16 = torch.empty((2, M, N), device=dev, dtype=torch.float16)
    _lib.check(lib.mec_set_option(b'gemm_bn', tile), 'gemm_bn')
    try:
        _lib.check(lib.mec_gemm_f16x3(p(Ad), M * K, p(Bd), N * K, ctypes.c_float(1 / 256), p(bd), None, None, 0, p(C32),
                                      M, N, K, 4, st), 'f32 out')
        _lib.check(lib.mec_gemm_f16x3(p(Ad), M * K, p(Bd), N * K, ctypes.c_float(1 / 256), p(bd), None, p(C16), M * N,
                                      None, M, N, K, 4, st), 'plane out')
    finally:
        lib.mec_set_option(b'gemm_bn', 0)
    v = C32.cpu().numpy()
    hi, lo = C16[0].cpu().numpy(), C16[1].cpu().numpy()
    assert np.array_equal(hi, v.astype(np.float16))
    assert np.array_equal(lo, (v - hi.astype(np.float32)).astype(np.float16))


# ------------------------------------------------------------------ the fp32x3 range envelope
# Weights are split after a per-matrix power-of-two pre-scale (csrc/runtime.hip split_planes).
# Activations are split at a per-tensor power-of-two scale fixed at handle creation (models.h
# activation_exp): hi = f16(x 2^s), lo = f16(x 2^s - hi), which holds 22 significant bits while
# 2^-3 <= |x 2^s| < 65520; the consumer's epilogue scale folds in 2^-s (exact). At |x 2^s| >= 65520
# hi is inf: every producer of activation planes raises the handle's range flag and mec_model_check
# fails the forward (INTEGRATION.md "fp32x3 envelope").


def _gemm_pair(dev, A, W, s_a=0):
    """(exact-f32 engine, split engine with A's planes at 2^s_a) outputs of A . W^T, and the float64
    reference."""
    import ctypes
    from mec import _lib
    lib = _lib.load()
    M, K = A.shape
    N = W.shape[0]
    st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    Ad, Wd = torch.from_numpy(A).to(dev), torch.from_numpy(W).to(dev)
    e = float(np.ceil(np.log2(16384 / np.abs(W).max())) - 1)
    Axd, Wxd = torch.from_numpy(_split(A, 2.0 ** s_a)).to(dev), torch.from_numpy(_split(W, 2.0 ** e)).to(dev)
    C32, Cx = torch.empty((M, N), device=dev), torch.empty((M, N), device=dev)
    _lib.check(lib.mec_gemm_f32(p(Ad), p(Wd), None, None, p(C32), M, N, K, 0, st), 'mec_gemm_f32')
    _lib.check(lib.mec_gemm_f16x3(p(Axd), M * K, p(Wxd), N * K, ctypes.c_float(2.0 ** (-e - s_a)), None, None, None, 0,
                                  p(Cx), M, N, K, 0, st), 'mec_gemm_f16x3')
    torch.cuda.synchronize()
    return C32.cpu().numpy(), Cx.cpu().numpy(), A.astype(np.float64) @ W.astype(np.float64).T


def _act_exp(bound, target=32768.0):
    """csrc/runtime.hip activation_exp: the largest s with bound 2^s <= target."""
    s = int(np.floor(np.log2(target / bound)))
    while bound * 2.0 ** s > target:
        s -= 1
    return s


def test_split_gemm_mixed_magnitude_activations_1e6_to_1e4(dev):
    """Activations whose magnitudes span 1e-6 .. 1e4 inside every row (log-uniform, random signs),
    split at the plane scale the model rule gives (max |a| 2^s <= 2^15): the split engine stays within
    the fp32 GEMM bar (2e-6 x sum |a w|) of float64, as the exact-f32 engine does; tiny entries lose
    relative bits, but the bar is relative to the row's sum and both engines are held to it."""
    rng = np.random.default_rng(11)
    M, N, K = 1024, 768, 768
    A = (np.sign(rng.standard_normal((M, K))) * 10.0 ** rng.uniform(-6, 4, (M, K))).astype(np.float32)
    W = (rng.standard_normal((N, K)) * 0.02).astype(np.float32)
    c32, cx, ref = _gemm_pair(dev, A, W, _act_exp(float(np.abs(A).max())))
    bound = 2e-6 * (np.abs(A).astype(np.float64) @ np.abs(W).astype(np.float64).T + 1)
    e32, ex3 = np.abs(c32 - ref), np.abs(cx - ref)
    print(f'mixed 1e-6..1e4: exact-f32 max err/bound {(e32 / bound).max():.3g}, split {(ex3 / bound).max():.3g}')
    assert (e32 <= bound).all() and (ex3 <= bound).all()


@pytest.mark.parametrize('scale', [1e-1, 1e-3, 1e-5])
def test_split_gemm_small_activations_scaled_planes(dev, scale):
    """Activations uniformly small (N(0,1) x scale) split at their plane scale (max |a| 2^s <= 2^15,
    the rule activation_exp applies to the models' bounds): the split engine holds the plain fp32 GEMM
    bar, 2e-6 x sum |a w|, with no absolute term, as the exact-f32 engine does. Unscaled planes (s = 0)
    would leave the lo plane an f16 subnormal below 2^-3 (an absolute error of 2^-25 per operand): that
    error is printed beside it."""
    rng = np.random.default_rng(12)
    M, N, K = 1024, 768, 768
    A = (rng.standard_normal((M, K)) * scale).astype(np.float32)
    W = (rng.standard_normal((N, K)) * 0.02).astype(np.float32)
    s_a = _act_exp(float(np.abs(A).max()))
    c32, cx, ref = _gemm_pair(dev, A, W, s_a)
    _, cu, _ = _gemm_pair(dev, A, W, 0)
    aw = np.abs(A).astype(np.float64) @ np.abs(W).astype(np.float64).T
    e32, ex3, eu = np.abs(c32 - ref), np.abs(cx - ref), np.abs(cu - ref)
    print(f'A ~ N(0,1) x {scale:g} (planes at 2^{s_a}): max err / sum|a w|: exact-f32 {(e32 / aw).max():.3g}, '
          f'split {(ex3 / aw).max():.3g} (unscaled planes {(eu / aw).max():.3g})')
    assert (e32 <= 2e-6 * aw + 1e-30).all()
    assert (ex3 <= 2e-6 * aw + 1e-30).all()


def _edit(kind, edits):
    """A copy of the seeded weights with edits {name: factor | (index, value)} applied (syn.weights
    returns the cached dict every handle shares)."""
    w = dict(syn.weights(kind))
    for name, e in edits.items():
        a = np.array(w[name], np.float32)
        if isinstance(e, tuple):
            a.flat[e[0]] = e[1]
        else:
            a = (a * np.float32(e)).astype(np.float32)
        w[name] = a
    return w


def _raises_then_clears(enc):
    from mec._lib import MecError
    torch.cuda.synchronize()
    with pytest.raises(MecError, match='f16 hi / lo range'):
        enc.check()
    enc.check()  # the check cleared the flag


# Non-finite values are no fp32 operands: whichever producer first writes one as planes raises the
# flag. BERT's plane scales come from rigorous bounds, so only a NaN / inf can reach the guard there.
@pytest.mark.parametrize('name,idx,value,fused', [
    ('bert.embeddings.word_embeddings.weight', 101 * 768 + 5, np.nan, 1),   # embedding LayerNorm
    ('bert.encoder.layer.0.attention.self.query.weight', 0, np.inf, 1),      # fused QKV + attention kernel
    ('bert.encoder.layer.0.attention.self.value.weight', 0, np.inf, 0),      # split QKV GEMM epilogue
    ('bert.encoder.layer.0.intermediate.dense.weight', 0, np.inf, 1)])       # FFN1 GEMM epilogue
def test_text_fp32x3_nonfinite_raises_at_check(dev, name, idx, value, fused):
    """A NaN / inf in the weights reaches an activation plane: the forward completes and check() raises
    MecError (mec_model_check) instead of returning NaN probabilities unannounced; the check clears the
    flag, so a second check passes."""
    w = _edit('text', {name: (idx, value)})
    ids, mask = syn.text_inputs(4, 128, seed=3, ragged=True)
    enc = engine.TextEncoder(w, device=dev, precision='fp32x3')
    enc.set_option('bert_qkv_attn', fused)
    enc.check()  # clean handle
    enc.forward(engine.to_device(ids, dev), engine.to_device(mask, dev))
    _raises_then_clears(enc)


@pytest.mark.parametrize('name', ['bert.encoder.layer.0.intermediate.dense.weight', 'bert.embeddings.LayerNorm.weight'])
def test_text_fp32x3_large_weights_adapt_plane_scale(dev, name):
    """A weight scaled by 1e5 (FFN1 outputs near 1e5, or embedding LayerNorm outputs near 3e6: past the
    f16 range unscaled): the bound-derived plane exponents follow (models.h activation_exp), so the
    forward raises no flag and matches the oracle on the same weights at the fp32 bars."""
    w = _edit('text', {name: 1e5})
    ids, mask = syn.text_inputs(4, 128, seed=3, ragged=True)
    enc = engine.TextEncoder(w, device=dev, precision='fp32x3')
    cls, _, probs = _np(enc.forward(engine.to_device(ids, dev), engine.to_device(mask, dev)))
    enc.check()
    rc, _, rp = o_t.forward(w, ids, mask)
    err, agree = float(np.abs(probs - rp).max()), int((probs.argmax(1) == rp.argmax(1)).sum())
    ferr = float(np.abs(cls - rc).max() / np.abs(rc).max())
    print(f'{name} x 1e5: probs max|d| {err:.3g}, cls rel err {ferr:.3g}')
    assert agree == 4 and err <= PROB_TOL and ferr <= FEAT_RTOL


# ResNet50 / MobileNetV2 plane scales come from BatchNorm estimates: activations far above what the BN
# parameters predict (a conv weight scaled, BN unchanged) overflow and raise the flag.
@pytest.mark.parametrize('name,seam', [('base.layer1.0.conv1.weight', 2),  # conv1 GEMM epilogue
                                       ('base.layer1.0.conv3.weight', 2),  # layer1 dual seam (pw_chain_x3)
                                       ('base.layer1.1.conv3.weight', 2),  # layer1 residual seam
                                       ('base.layer1.1.conv3.weight', 0),  # conv3 GEMM epilogue (residual)
                                       ('base.layer3.0.conv3.weight', 2),  # dual conv3 + downsample GEMM
                                       ('base.layer2.1.conv3.weight', 2),  # layer2 seam (pw_seam_x3), conv3
                                       ('base.layer2.2.conv1.weight', 2)])  # layer2 seam, conv1 epilogue
def test_resnet_fp32x3_overflow_raises_at_check(dev, name, seam):
    """A conv weight scaled by 1e6 with its BN unchanged: the activations leave the estimate's 64x
    headroom and the f16 range -> check() raises; a handle with the seeded weights checks clean.
    `seam` sets both seam families (pw_chain_x3 for layer1, pw_seam_x3 > 0 for layer2)."""
    enc = engine.ImageEncoder(_edit('image', {name: 1e6}), device=dev, precision='fp32x3')
    enc.set_option('pw_chain_x3', seam)
    enc.set_option('pw_seam_x3', min(seam, 1))
    enc.forward(engine.to_device(syn.image_inputs(2, seed=5), dev))
    _raises_then_clears(enc)
    ok = engine.ImageEncoder(device=dev, precision='fp32x3')
    ok.forward(engine.to_device(syn.image_inputs(2, seed=5), dev))
    torch.cuda.synchronize()
    ok.check()


@pytest.mark.parametrize('name,layered', [('base.features.2.conv.2.weight', 8),   # fused block input split
                                          ('base.features.7.conv.2.weight', 8),   # layered tail's first split
                                          ('base.features.9.conv.2.weight', 8),   # layered project epilogue
                                          ('base.features.16.conv.2.weight', 0)])  # features[17]'s layered input
def test_mobilenet_v2_fp32x3_overflow_raises_at_check(dev, name, layered):
    """A MobileNetV2 projection weight scaled by 1e6 (its BN unchanged): the block output overflows the
    next producer of planes (the fused block kernel's input split, mbv2_split_pad_kernel, the layered
    project GEMM; with every other block fused, features[17]'s split_pad) -> check() raises, then clears."""
    enc = engine.MobileNetImageEncoder(_edit('image_mbv2', {name: 1e6}), device=dev, precision='fp32x3')
    enc.set_option('mbv2_layered', layered)
    enc.forward(engine.to_device(syn.image_inputs(2, seed=5), dev))
    _raises_then_clears(enc)


# ------------------------------------------------------------------ small activations, model level
def _resnet_scaled(c):
    """ResNet50 weights computing the seeded network's function with every activation tensor c times
    smaller: every BN's gamma and beta x c, every conv after the stem x 1/c (its input is c times
    smaller; its BN sees the same pre-BN values), fc[1] x 1/c."""
    w = dict(syn.weights('image'))
    for k in list(w):
        a = np.asarray(w[k], np.float32)
        if (k.endswith('.weight') or k.endswith('.bias')) and a.ndim == 1 and ('bn' in k or 'downsample.1' in k):
            w[k] = (a * np.float32(c)).astype(np.float32)
        elif k.startswith('base.layer') and a.ndim == 4:
            w[k] = (a / np.float32(c)).astype(np.float32)
    w['base.fc.1.weight'] = (np.asarray(w['base.fc.1.weight']) / np.float32(c)).astype(np.float32)
    return w


@pytest.mark.parametrize('how', ['gamma_1e-3', 'activations_2^-14', 'activations_2^12'])
def test_resnet_fp32x3_scaled_activations_vs_oracle(dev, how):
    """Activations far from O(1) end to end on the fp32x3 path against the oracle on the same weights, at
    the fp32 bars (probs 1e-5, feature 1e-4 relative, argmax exact):
      * gamma_1e-3: every BN gamma x 1e-3 (activations near |beta| ~ 0.1 and below, the f16 lo plane's
        subnormal range without a plane scale);
      * activations_2^-14 / 2^12: every activation tensor 2^-14 / 2^12 times the seeded network's
        (_resnet_scaled: the same function, so the probs must also equal the seeded network's; at 2^12
        the largest activations, ~1e5, are past the f16 range without a plane scale).
    The plane exponents follow the BN estimates (models.h activation_exp): no flag, no subnormal lo plane."""
    if how == 'gamma_1e-3':
        w = dict(syn.weights('image'))
        for k in list(w):
            if k.endswith('.weight') and np.asarray(w[k]).ndim == 1:
                w[k] = (np.asarray(w[k]) * np.float32(1e-3)).astype(np.float32)
    else:
        w = _resnet_scaled(2.0 ** int(how.split('^')[1]))
    gray = syn.image_inputs(8, seed=77)
    enc = engine.ImageEncoder(w, device=dev, precision='fp32x3')
    feat, _, probs = _np(enc.forward(engine.to_device(gray, dev)))
    enc.check()
    rf, _, rp = o_i.forward(w, gray)
    err = float(np.abs(probs - rp).max())
    ferr = float(np.abs(feat - rf).max() / np.abs(rf).max())
    print(f'resnet50 fp32x3 {how}: probs max|d| {err:.3g}, feat rel err {ferr:.3g}')
    assert err <= PROB_TOL and ferr <= FEAT_RTOL and (probs.argmax(1) == rp.argmax(1)).all()
    if how != 'gamma_1e-3':
        _, _, rp0 = o_i.forward(syn.weights('image'), gray)
        assert np.abs(probs - rp0).max() <= PROB_TOL


def test_text_fp32x3_small_activations_vs_oracle(dev):
    """BERT with the LayerNorm outputs, Q, V and the context 2^-12 times the seeded network's and K 2^12
    times (every LN gamma / beta, bq, bv, bo, Wo2, bo2 x c; bk, Wi, the pooler x 1/c; Wk x 1/c^2: the
    same function) on the fp32x3 path against the oracle at the fp32 bars; the plane exponents follow
    the bounds (one each for Q, K, V)."""
    c = np.float32(2.0 ** -12)
    w = dict(syn.weights('text'))
    for k in list(w):
        a = np.asarray(w[k], np.float32)
        if 'LayerNorm' in k or k.endswith(('query.bias', 'value.bias', 'attention.output.dense.bias',
                                           'output.dense.weight', 'output.dense.bias')):
            if not k.endswith('attention.output.dense.weight'):
                w[k] = (a * c).astype(np.float32)
        elif k.endswith(('intermediate.dense.weight', 'pooler.dense.weight', 'key.bias')):
            w[k] = (a / c).astype(np.float32)
        elif k.endswith('key.weight'):  # K = K_seeded / c, so the scores Q K^T are unchanged
            w[k] = (a / (c * c)).astype(np.float32)
    ids, mask = syn.text_inputs(6, 128, seed=78, ragged=True)
    enc = engine.TextEncoder(w, device=dev, precision='fp32x3')
    cls, _, probs = _np(enc.forward(engine.to_device(ids, dev), engine.to_device(mask, dev)))
    enc.check()
    rc, _, rp = o_t.forward(w, ids, mask)
    _, _, rp0 = o_t.forward(syn.weights('text'), ids, mask)
    err = float(np.abs(probs - rp).max())
    ferr = float(np.abs(cls - rc).max() / np.abs(rc).max())
    print(f'bert fp32x3 activations x 2^-12: probs max|d| {err:.3g} (seeded net {np.abs(probs - rp0).max():.3g}), '
          f'cls rel err {ferr:.3g}, |cls| max {np.abs(rc).max():.3g}')
    assert err <= PROB_TOL and ferr <= FEAT_RTOL and (probs.argmax(1) == rp.argmax(1)).all()


def test_mobilenet_v2_fp32x3_small_activations_vs_oracle(dev):
    """MobileNetV2 with every block output 2^-14 times the seeded network's (each projection BN's gamma /
    beta x c, every expand conv and features[18]'s conv x 1/c: the same function), fused blocks and the
    layered tail, against the oracle at the fp32 bars."""
    from oracle import image_mbv2 as o_mb
    c = np.float32(2.0 ** -14)
    w = dict(syn.weights('image_mbv2'))
    for i, (t, cin, hid, cout, st) in enumerate(syn.mbv2_blocks()):
        p = f'base.features.{i + 1}.conv.'
        bn = p + ('2' if t == 1 else '3')
        for sfx in ('.weight', '.bias'):
            w[bn + sfx] = (np.asarray(w[bn + sfx]) * c).astype(np.float32)
        if t != 1:
            w[p + '0.0.weight'] = (np.asarray(w[p + '0.0.weight']) / c).astype(np.float32)
    w['base.features.18.0.weight'] = (np.asarray(w['base.features.18.0.weight']) / c).astype(np.float32)
    gray = syn.image_inputs(6, seed=79)
    rf, _, rp = o_mb.forward(w, gray)
    for layered in (8, 0):
        enc = engine.MobileNetImageEncoder(w, device=dev, precision='fp32x3')
        enc.set_option('mbv2_layered', layered)
        feat, _, probs = _np(enc.forward(engine.to_device(gray, dev)))
        enc.check()
        err = float(np.abs(probs - rp).max())
        ferr = float(np.abs(feat - rf).max() / np.abs(rf).max())
        print(f'mobilenet_v2 fp32x3 block outputs x 2^-14, mbv2_layered {layered}: probs max|d| {err:.3g}, '
              f'feat rel err {ferr:.3g}')
        assert err <= PROB_TOL and ferr <= FEAT_RTOL and (probs.argmax(1) == rp.argmax(1)).all()


def test_fp32x3_untuned_tiles_match_autotuned(dev):
    """gemm_autotune 0 (the untuned fallback, also what a first launch inside graph capture runs):
    K-interleaved split GEMMs take an interleaved tile (heuristic_bn), so the fp32x3 text and image
    forwards run and give the autotuned handle's bits (every interleaved tile sums in one k order)."""
    ids, mask = syn.text_inputs(8, 128, seed=9, ragged=True)
    targs = (engine.to_device(ids, dev), engine.to_device(mask, dev))
    g = engine.to_device(syn.image_inputs(8, seed=9), dev)
    outs = []
    for autotune in (1, 0):
        t = engine.TextEncoder(device=dev, precision='fp32x3')
        i = engine.ImageEncoder(device=dev, precision='fp32x3')
        t.set_option('gemm_autotune', autotune)
        i.set_option('gemm_autotune', autotune)
        outs.append(_np(t.forward(*targs)) + _np(i.forward(g)))
        t.check()
        i.check()
    for k, (a, b) in enumerate(zip(*outs)):
        assert np.array_equal(a, b), f'output {k}'


@pytest.mark.parametrize('B,ragged', [(3, True), (64, True), (256, False)])
def test_text_fp32x3_fused_qkv_attention_bit_identical(dev, B, ragged):
    """bert_qkv_attn 1 (the default: bert_qkv_attn_x3_kernel, Q / K / V planes kept in LDS) against
    0 (the split QKV GEMM, then bert_attention_x3_kernel): the same products in the same term and k
    order and the same attention code, so CLS feature, logits and probs are equal bit for bit."""
    ids, mask = syn.text_inputs(B, 128, seed=800 + B, ragged=ragged)
    args = (engine.to_device(ids, dev), engine.to_device(mask, dev))
    outs = []
    for fused, heads in ((0, 2), (1, 2), (1, 1)):  # heads per workgroup of the fused kernel: 2 or 1
        enc = engine.TextEncoder(device=dev, precision='fp32x3')
        enc.set_option('bert_qkv_attn', fused)
        enc.set_option('bert_qkv_attn_x3_heads', heads)
        outs.append(_np(enc.forward(*args)))
        enc.check()
        enc.close()
    for form, o in zip(('fused, 2 heads', 'fused, 1 head'), outs[1:]):
        for k, (a, b) in enumerate(zip(outs[0], o)):
            assert np.array_equal(a, b), f'{form}, output {k}: max |d| {np.abs(a - b).max()}'


# ------------------------------------------------------------------ MobileNetV2 on the fp32x3 path
@pytest.mark.parametrize('B', [3, 64, 256])
def test_mobilenet_v2_fp32x3_vs_oracle(dev, B):
    """MobileNetV2 (BASELINE configs[1], parity unpinned: no reference code) on the fp32x3 path
    (csrc/mobilenet_x3.hip: one fused kernel per block, 1x1 products on split f16 operands, fp32
    depthwise and block outputs) against the oracle at the fp32 bars: probs within 1e-5, feature
    within 1e-4 relative, argmax exact; the exact-fp32 path's error printed beside it."""
    from oracle import image_mbv2 as o_mb
    gray = syn.image_inputs(B, seed=90 + B)
    g = engine.to_device(gray, dev)
    enc = engine.MobileNetImageEncoder(device=dev, precision='fp32x3')
    feat, logits, probs = _np(enc.forward(g))
    enc.check()
    feat32, _, probs32 = _np(engine.MobileNetImageEncoder(device=dev, precision='fp32').forward(g))
    sub = np.unique(np.r_[0, np.arange(0, B, max(1, B // 16)), B - 1])
    rf, rl, rp = o_mb.forward(syn.weights('image_mbv2'), gray[sub])
    err, agree = _report(f'mobilenet_v2 fp32x3 B={B}', probs[sub], rp, probs32[sub])
    ferr = float(np.abs(feat[sub] - rf).max() / np.abs(rf).max())
    print(f'  feat rel err {ferr:.3g} (fp32 path {float(np.abs(feat32[sub] - rf).max() / np.abs(rf).max()):.3g}), '
          f'logits max|d| {np.abs(logits[sub] - rl).max():.3g}')
    assert agree == len(sub) and err <= PROB_TOL and ferr <= FEAT_RTOL


@pytest.mark.parametrize('first', [0, 7, 11, 15, 17])
def test_mobilenet_v2_fp32x3_layered_tail_vs_oracle(dev, first):
    """mbv2_layered k: features[k..17] as expand GEMM -> depthwise kernel -> project GEMM on split
    planes (csrc/mobilenet_x3.hip; 0 = every block fused) against the oracle at the fp32 bars, and
    batch invariance of the layered form (rows of a B=24 batch equal the same rows run as B=5)."""
    from oracle import image_mbv2 as o_mb
    gray = syn.image_inputs(24, seed=120 + first)
    g = engine.to_device(gray, dev)
    enc = engine.MobileNetImageEncoder(device=dev, precision='fp32x3')
    enc.set_option('mbv2_layered', first)
    feat, logits, probs = _np(enc.forward(g))
    small = _np(enc.forward(g[:5]))
    enc.check()
    for i, (a, b) in enumerate(zip((feat, logits, probs), small)):
        assert np.array_equal(a[:5], b), f'output {i}'
    sub = np.array([0, 7, 15, 23])
    rf, rl, rp = o_mb.forward(syn.weights('image_mbv2'), gray[sub])
    err = float(np.abs(probs[sub] - rp).max())
    ferr = float(np.abs(feat[sub] - rf).max() / np.abs(rf).max())
    print(f'mbv2_layered {first}: probs max|d| {err:.3g}, feat rel err {ferr:.3g}')
    assert err <= PROB_TOL and ferr <= FEAT_RTOL and (probs[sub].argmax(1) == rp.argmax(1)).all()


@pytest.mark.parametrize('B', [3, 256])
def test_mobilenet_v2_fp32x3_tiles_per_workgroup_bit_identical(dev, B):
    """mbv2_x3_tpw k (each fused-block workgroup walks k output tiles, the next tile's input loaded
    while one computes; the stem block, RGB and gray, included) against one tile per workgroup: the
    same per-tile arithmetic, so the same bits, also when k does not divide the tile count (B = 3);
    every block fused (mbv2_layered 0: all but features[17]) so all the fused shapes run."""
    g = engine.to_device(syn.image_inputs(B, seed=210 + B), dev)
    enc = engine.MobileNetImageEncoder(device=dev, precision='fp32x3')
    enc.set_option('mbv2_layered', 0)
    outs = {}
    for k in (1, 3, 4):
        enc.set_option('mbv2_x3_tpw', k)
        outs[k] = [t.cpu() for t in enc.forward(g)]
    enc.check()
    for k in (3, 4):
        for i, (a, b) in enumerate(zip(outs[1], outs[k])):
            assert torch.equal(a, b), f'tpw {k}, output {i}: max |d| {float((a - b).abs().max())}'


def test_mobilenet_v2_fp32x3_batch_invariance_and_entry_shapes(dev):
    """Rows of a B=64 batch equal the same rows run as B=8 bit for bit (per-tile kernels, and the
    features[18] split GEMM's interleaved tiles share one k order); the RGB and already-resized
    224 gray entry shapes through the fp32x3 stem against the oracle."""
    from oracle import image_mbv2 as o_mb
    enc = engine.MobileNetImageEncoder(device=dev, precision='fp32x3')
    g = engine.to_device(syn.image_inputs(64, seed=99), dev)
    big = [t[:8].cpu() for t in enc.forward(g)]
    small = [t.cpu() for t in enc.forward(g[:8])]
    for i, (a, b) in enumerate(zip(big, small)):
        assert torch.equal(a, b), f'output {i}'
    rgb = np.stack([syn.image_inputs(2, seed=170 + c).repeat(4, axis=1).repeat(4, axis=2)[:, :224, :224]
                    for c in range(3)], -1)
    rgb = np.ascontiguousarray(np.pad(rgb, ((0, 0), (0, 32), (0, 32), (0, 0)))[:, :224, :224])
    _, _, probs = _np(enc.forward_u8(engine.to_device(rgb, dev)))
    _, _, rp = o_mb.forward_resized(syn.weights('image_mbv2'), rgb)
    assert np.abs(probs - rp).max() <= PROB_TOL and (probs.argmax(1) == rp.argmax(1)).all()
    g224 = np.ascontiguousarray(rgb[..., 0])
    _, _, probs = _np(enc.forward_u8(engine.to_device(g224[..., None], dev)))
    _, _, rp = o_mb.forward_resized(syn.weights('image_mbv2'), g224)
    assert np.abs(probs - rp).max() <= PROB_TOL
    enc.check()


def test_resnet_fp32x3_chunked_layers_bit_identical(dev):
    """resnet_chunk n (layers 1-2 over chunks of n images, the rest over the batch) gives the
    unchunked forward's bits: every split GEMM / conv row is computed the same way at any M."""
    g = engine.to_device(syn.image_inputs(40, seed=44), dev)
    outs = []
    for chunk in (0, 16):
        enc = engine.ImageEncoder(device=dev, precision='fp32x3')
        enc.set_option('resnet_chunk', chunk)
        outs.append(_np(enc.forward(g)))
        enc.check()
        enc.close()
    for k, (a, b) in enumerate(zip(*outs)):
        assert np.array_equal(a, b), f'output {k}'


@pytest.mark.parametrize('B,chunk', [(3, 0), (40, 0), (40, 16)])
def test_resnet_fp32x3_seams_bit_identical(dev, B, chunk):
    """pw_chain_x3 1 / 2 (layer1's conv3 + downsample-or-residual + ReLU and the next block's conv1
    in one kernel, csrc/pw_chain_x3.hip) against 0 (the two split GEMMs): the same K-interleaved
    terms in the same k order and the same epilogue, so every output is equal bit for bit, also
    over image chunks (resnet_chunk)."""
    g = engine.to_device(syn.image_inputs(B, seed=47 + B), dev)
    outs = []
    for seam in (0, 1, 2):
        enc = engine.ImageEncoder(device=dev, precision='fp32x3')
        enc.set_option('pw_chain_x3', seam)
        enc.set_option('resnet_chunk', chunk)
        outs.append(_np(enc.forward(g)))
        enc.check()
        enc.close()
    for seam, o in zip((1, 2), outs[1:]):
        for k, (a, b) in enumerate(zip(outs[0], o)):
            assert np.array_equal(a, b), f'pw_chain_x3 {seam}, output {k}: max |d| {np.abs(a - b).max()}'


@pytest.mark.parametrize('B,chunk', [(3, 0), (5, 0), (40, 0), (40, 16), (256, 0)])
def test_resnet_fp32x3_layer2_seams_bit_identical(dev, B, chunk):
    """pw_seam_x3 1 / 2 (layer2's conv3 + identity residual + ReLU and the next block's conv1 -- layer3's
    first conv1 at 2 -- in one kernel that walks the block output in 32-channel chunks,
    csrc/pw_seam_x3.hip) against 0 (the two split GEMMs): conv1's k steps are summed in the same
    ascending order with the same three terms each, and both epilogues are the GEMM's, so every output
    is equal bit for bit. B = 3 / 5 leave row tails (784 B rows: 16 or 48 rows past the last 64-row
    tile); resnet_chunk 16 runs layer2 per image chunk (the layer3 seam then stays unfused)."""
    g = engine.to_device(syn.image_inputs(B, seed=53 + B), dev)
    outs = []
    for seam in (0, 1, 2):
        enc = engine.ImageEncoder(device=dev, precision='fp32x3')
        enc.set_option('pw_seam_x3', seam)
        enc.set_option('resnet_chunk', chunk)
        outs.append(_np(enc.forward(g)))
        enc.check()
        enc.close()
    for seam, o in zip((1, 2), outs[1:]):
        for k, (a, b) in enumerate(zip(outs[0], o)):
            assert np.array_equal(a, b), f'pw_seam_x3 {seam}, output {k}: max |d| {np.abs(a - b).max()}'


def test_mobilenet_v2_fp32x3_tile_forms_bit_identical(dev):
    """mbv2_x3_tile 4 (4x4 output tiles for the stride-2 blocks at 56 / 28 outputs) computes every
    output pixel with the same arithmetic as the 8x8 / 7x7 tiles: the same bits."""
    g = engine.to_device(syn.image_inputs(6, seed=46), dev)
    outs = []
    for t in (0, 4):
        enc = engine.MobileNetImageEncoder(device=dev, precision='fp32x3')
        enc.set_option('mbv2_x3_tile', t)
        outs.append(_np(enc.forward(g)))
        enc.close()
    for k, (a, b) in enumerate(zip(*outs)):
        assert np.array_equal(a, b), f'output {k}'
