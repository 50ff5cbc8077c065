"""GPU: the fp32x3 path on data outside its activation-plane envelope, and the knobs ADVICE r05 asked
to pin.

1. Range recovery (engine.HipModel.recover). ResNet50 / MobileNetV2 plane exponents come from the
   BatchNorm parameters (64x headroom over a 6-sigma estimate, models.h activation_exp); a conv weight
   scaled by 256 with its BN left alone produces activations past that envelope. The drop-in paths
   (ImageInference.predict_batch, MultimodalFusion.predict_batch / predict_multimodal) and
   FusedPipeline.check() must then ANSWER, not raise: the batch is re-run on the exact-fp32 HIP engine
   (an fp32 twin handle, not the oracle) and matches the oracle on the same weights at the fp32 bars
   (probs 1e-5, feature 1e-4 relative, argmax exact); the fp32x3 handle is re-created with 8 more
   binades of plane headroom (mec_create_opt "x3_headroom"), so a later batch runs fp32x3 with no
   re-run and still matches.
2. Bit identity of the schedule knobs ADVICE r05 names: gemm_x3_restage 0 / 1 / 2 (BERT and ResNet50
   fp32x3), mbv2_x3_occ 3 / 4 and mbv2_x3_sesw 0 / 1 (MobileNetV2 fp32x3).
3. GEMM shapes first launched inside hipGraph capture (include/mec.h): replay and a later eager launch
   compute the same bits; a split (fp32x3) shape stays untuned through the capture and is tuned by its
   first eager launch.
4. The FFN pins (gemm_x3_tag) step aside for small batches (grid < 128 tiles) with the same bits.
"""
import ctypes

import numpy as np
import pytest
import torch

from mec import _lib, engine, synthetic as syn
from oracle import image as o_i

pytestmark = pytest.mark.gpu

PROB_TOL, FEAT_RTOL = 1e-5, 1e-4
SCALED = 'base.layer2.1.conv2.weight'  # a 3x3 conv of layer2 (the halo / implicit-GEMM epilogue writes planes)


def _edit(kind, edits):
    w = dict(syn.weights(kind))
    for name, f in edits.items():
        w[name] = (np.asarray(w[name], np.float32) * np.float32(f)).astype(np.float32)
    return w


W256 = None


def _w256():
    global W256
    if W256 is None:
        W256 = _edit('image', {SCALED: 256.0})
    return W256


def _vs_oracle(name, w, gray, feat, probs):
    rf, _, rp = o_i.forward(w, gray)
    err = float(np.abs(probs - rp).max())
    ferr = float(np.abs(feat - rf).max() / np.abs(rf).max())
    print(f'{name}: probs max|d| {err:.3g}, feat rel err {ferr:.3g}')
    assert err <= PROB_TOL and ferr <= FEAT_RTOL and (probs.argmax(1) == rp.argmax(1)).all(), name


def test_scaled_conv_trips_the_unwidened_handle(dev):
    """The premise: with the default headroom the scaled network raises the range flag."""
    enc = engine.ImageEncoder(_w256(), device=dev, precision='fp32x3')
    enc.forward(engine.to_device(syn.image_inputs(4, seed=61), dev))
    torch.cuda.synchronize()
    with pytest.raises(_lib.X3RangeError, match='f16 hi / lo range'):
        enc.check()
    assert 'x3_headroom=0' in enc.x3_report()


def test_image_predict_batch_recovers_then_runs_fp32x3(dev):
    from inference.image_inference import ImageInference
    inf = ImageInference(weights=_w256(), device=dev, precision='fp32x3')
    gray = syn.image_inputs(16, seed=62)
    feat, _, probs = inf.predict_batch(engine.to_device(gray, dev))
    assert inf.model.x3_reruns == 1 and inf.model.x3_headroom == 8
    _vs_oracle('predict_batch, re-run on fp32', _w256(), gray, feat.cpu().numpy(), probs.cpu().numpy())
    # the re-created handle: fp32x3 again, no re-run, same bars
    gray2 = syn.image_inputs(16, seed=63)
    feat2, _, probs2 = inf.predict_batch(engine.to_device(gray2, dev))
    assert inf.model.x3_reruns == 1, 'the widened handle tripped again'
    assert 'x3_headroom=8' in inf.model.x3_report()
    _vs_oracle('predict_batch, widened fp32x3', _w256(), gray2, feat2.cpu().numpy(), probs2.cpu().numpy())


def test_predict_multimodal_image_recovers(dev, tmp_path):
    from PIL import Image
    from inference.multimodal_fusion import MultimodalFusion
    fusion = MultimodalFusion(weights={'image': _w256()}, seed=1234, device=dev, precision='fp32x3')
    faces = syn.image_inputs(2, seed=64)
    _, _, rp = o_i.forward(_w256(), faces)
    for i in range(2):
        p = tmp_path / f'face{i}.png'
        Image.fromarray(faces[i], 'L').save(p)
        res = fusion.predict_multimodal(image_path=str(p))
        got = np.array(res['image']['all_probabilities'])
        print(f'request {i}: probs max|d| {np.abs(got - rp[i]).max():.3g}')
        assert np.abs(got - rp[i]).max() <= PROB_TOL and int(got.argmax()) == int(rp[i].argmax())
    m = fusion.image_inference.model
    assert m.x3_reruns == 1 and m.x3_headroom == 8  # the second request ran fp32x3 without a re-run


def test_multimodal_predict_batch_and_pipeline_check_recover(dev):
    """The tri-modal batch paths: MultimodalFusion.predict_batch and FusedPipeline.forward + check()
    with the scaled image network; the repaired image outputs and the fusion outputs computed from them
    equal a fused run on fp32 image weights' oracle chain."""
    from inference.multimodal_fusion import MultimodalFusion
    from oracle import fusion as o_f, speech as o_s, text as o_t
    B = 8
    x = syn.speech_inputs(B, seed=65)
    ids, mask = syn.text_inputs(B, 128, seed=66, ragged=True)
    gray = syn.image_inputs(B, seed=67)
    w = {k: syn.weights(k) for k in ('speech', 'text', 'fusion')}
    w['image'] = _w256()
    sf, _, sp = o_s.forward(w['speech'], x)
    tf, _, tp = o_t.forward(w['text'], ids, mask)
    imf, _, ip = o_i.forward(w['image'], gray)
    _, fp, _, _ = o_f.forward(w['fusion'], sf, tf, imf, sp, tp, ip)
    args = [engine.to_device(a, dev) for a in (x, ids, mask, gray)]
    mf = MultimodalFusion(weights={'image': _w256()}, seed=1234, device=dev, precision='fp32x3')
    out = mf.predict_batch(*args)
    mf.check()
    assert mf.image_inference.model.x3_reruns == 1
    for name, got, ref in (('image', out['image'][2], ip), ('fusion', out['fusion'][1], fp)):
        err = float(np.abs(got.cpu().numpy() - ref).max())
        print(f'MultimodalFusion.predict_batch {name}: probs max|d| {err:.3g}')
        assert err <= PROB_TOL
    pipe = engine.FusedPipeline(seed=1234, device=dev, weights={'image': _w256()}, precision='fp32x3')
    for rnd in range(2):  # the first (serial) batch trips and is repaired; the second runs widened
        out = pipe.forward(*args)
        redo = pipe.check()
        assert redo == (['image'] if rnd == 0 else []), (rnd, redo)
        for name, got, ref in (('image', out['image'][2], ip), ('fusion', out['fusion'][1], fp)):
            err = float(np.abs(got.cpu().numpy() - ref).max())
            print(f'FusedPipeline batch {rnd} {name}: probs max|d| {err:.3g}')
            assert err <= PROB_TOL
    assert pipe.image.x3_reruns == 1 and pipe.image.x3_headroom == 8


def test_x3_creation_knobs_are_creation_time(dev):
    """x3_headroom / x3_plane_scale go through mec_create_opt; a live handle rejects them."""
    enc = engine.TextEncoder(device=dev, precision='fp32x3', opts={'x3_headroom': 3})
    rep = enc.x3_report()
    assert rep.startswith('x3_headroom=3') and 'layer11.ffn s=' in rep
    base = engine.TextEncoder(device=dev, precision='fp32x3').x3_report()
    s3 = {ln.split()[0]: int(ln.split()[1][2:]) for ln in rep.splitlines()[1:]}
    s0 = {ln.split()[0]: int(ln.split()[1][2:]) for ln in base.splitlines()[1:]}
    assert s3.keys() == s0.keys() and all(s3[k] == s0[k] - 3 for k in s0)  # 3 binades lower each
    for key in ('x3_headroom', 'x3_plane_scale'):
        with pytest.raises(_lib.MecError, match='creation-time'):
            enc.set_option(key, 1)
    img = engine.ImageEncoder(device=dev, precision='fp32x3')
    assert 'layer3.out s=' in img.x3_report() and 'stem s=' in img.x3_report()
    assert engine.ImageEncoder(device=dev, precision='fp32').x3_report() == ''


# ------------------------------------------------------------------ schedule knobs: the same bits
@pytest.mark.parametrize('knob,values', [('gemm_x3_restage', (0, 1, 2)), ('gemm_x3_late_dma', (1, 0, 2, 3)),
                                         ('gemm_x3_stagger', (0, 20)), ('gemm_x3_prio', (0, 1)),
                                         ('qkv_x3_late_dma', (0, 1, 2))])
@pytest.mark.parametrize('enc_kind', ['text', 'image'])
def test_x3_schedule_knobs_bit_identical(dev, enc_kind, knob, values):
    """Split-tile schedule knobs against their default: gemm_x3_restage 1 / 2 (2-stage split tiles
    refilled for k step t + 2 as soon as every wave holds step t's fragments, in every A mode / the convs
    only), gemm_x3_late_dma 0 / 2 / 3 against the default 1 (where the second wave of each SIMD issues its DMA
    share), gemm_x3_stagger (co-resident workgroups started apart), gemm_x3_prio (MFMA sections at wave
    priority 1), qkv_x3_late_dma 1 / 2 (the fused QKV + attention kernel's refill issued late by every other
    block of workgroups): the same fragments and MFMA order."""
    if knob == 'qkv_x3_late_dma' and enc_kind == 'image':
        pytest.skip('a BERT kernel')
    if enc_kind == 'text':
        ids, mask = syn.text_inputs(48 if knob == 'qkv_x3_late_dma' else 32, 128, seed=71, ragged=True)
        enc = engine.TextEncoder(device=dev, precision='fp32x3')
        # the unfused QKV GEMM too (the fused kernel for its own knob: 576 workgroups, past block 256)
        enc.set_option('bert_qkv_attn', 1 if knob == 'qkv_x3_late_dma' else 0)
        args = (engine.to_device(ids, dev), engine.to_device(mask, dev))
    else:
        enc = engine.ImageEncoder(device=dev, precision='fp32x3')
        args = (engine.to_device(syn.image_inputs(16, seed=72), dev),)
    enc.set_option('gemm_autotune', 0)  # heuristic tiles: 70256 / 71128 / 71064 (2 stages)
    outs = {}
    for v in values:
        enc.set_option(knob, v)
        outs[v] = [t.cpu() for t in enc.forward(*args)]
    enc.check()
    for v in values[1:]:
        for i, (a, b) in enumerate(zip(outs[values[0]], outs[v])):
            assert torch.equal(a, b), f'{knob} {v}, output {i}: max |d| {float((a - b).abs().max())}'


def test_mobilenet_v2_fp32x3_occ_and_sesw_bit_identical(dev):
    g = engine.to_device(syn.image_inputs(12, seed=73), dev)
    enc = engine.MobileNetImageEncoder(device=dev, precision='fp32x3')
    enc.set_option('mbv2_layered', 0)  # every fused block shape runs
    outs = {}
    for occ, sesw in ((3, 1), (4, 1), (3, 0), (4, 0)):
        enc.set_option('mbv2_x3_occ', occ)
        enc.set_option('mbv2_x3_sesw', sesw)
        outs[occ, sesw] = [t.cpu() for t in enc.forward(g)]
    enc.check()
    for k in ((4, 1), (3, 0), (4, 0)):
        for i, (a, b) in enumerate(zip(outs[3, 1], outs[k])):
            assert torch.equal(a, b), f'occ / sesw {k}, output {i}: max |d| {float((a - b).abs().max())}'


# ------------------------------------------------------------------ graph capture, then eager
def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def test_capture_then_eager_gemm_same_bits(dev):
    """A GEMM shape whose first launch is inside hipGraph capture (no timing possible there): the
    f16 engine caches the heuristic tile, so a later eager launch runs the replayed tile (same bits);
    a split (fp32x3) shape is left untuned through the capture (query 0) and tuned by its first eager
    launch, again with the replay's bits (every split tile sums in one k order)."""
    lib = _lib.load()
    g = torch.Generator().manual_seed(5)
    M, N, K, KX = 1544, 384, 640, 576  # shapes no other test runs (the process-default tune cache)
    A = (torch.rand(M, K, generator=g) * 2 - 1).half().to(dev)
    B = (torch.rand(N, K, generator=g) * 2 - 1).mul(K ** -0.5).half().to(dev)
    ax = torch.rand(M, KX, generator=g) * 2 - 1
    bx = (torch.rand(N, KX, generator=g) * 2 - 1) * KX ** -0.5
    A2 = torch.cat([ax.half(), (ax - ax.half().float()).half()]).contiguous().to(dev)  # hi | lo planes
    B2 = torch.cat([bx.half(), (bx - bx.half().float()).half()]).contiguous().to(dev)
    C_g, C_e, X_g, X_e = (torch.empty(M, N, dtype=torch.float32, device=dev) for _ in range(4))
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    assert lib.mec_gemm_query(0, M, N, K) == 0 and lib.mec_gemm_query(0, M, N, KX) == 0

    def f16(out, st):
        _lib.check(lib.mec_gemm_f16(_p(A), _p(B), None, None, 0, None, _p(out), M, N, K, 0, ctypes.c_void_p(st)), 'f16')

    def x3(out, st):
        _lib.check(lib.mec_gemm_f16x3(_p(A2), M * KX, _p(B2), N * KX, 1.0, None, None, None, 0, _p(out), M, N, KX, 0,
                                      ctypes.c_void_p(st)), 'x3')
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=s):
        f16(C_g, s.cuda_stream)
        x3(X_g, s.cuda_stream)
    graph.replay()
    torch.cuda.synchronize()
    t_f16 = lib.mec_gemm_query(0, M, N, K)
    assert t_f16 != 0  # cached during capture: the f16 engine's heuristic tile
    assert lib.mec_gemm_query(0, M, N, KX) == 0  # the split shape: not cached during capture
    f16(C_e, torch.cuda.current_stream(dev).cuda_stream)
    x3(X_e, torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize()
    assert lib.mec_gemm_query(0, M, N, K) == t_f16  # the eager launch kept the captured tile
    assert 70000 <= lib.mec_gemm_query(0, M, N, KX) < 80000  # tuned by the eager launch
    assert torch.equal(C_g, C_e)
    assert torch.equal(X_g, X_e)


# ------------------------------------------------------------------ FFN pins at small batches
def test_ffn_pins_step_aside_at_small_batch(dev):
    """BERT FFN1 / FFN2 pins (70256 / 72128) apply from 128 / 512 tiles; at B = 16 (48 / 24 tiles) the
    handle autotunes among the 7xxxx tiles instead: the same bits as at B = 64 (FFN1 pinned)."""
    m = engine.TextEncoder(device=dev, precision='fp32x3')
    ids, mask = syn.text_inputs(64, 128, seed=74, ragged=True)
    args = [engine.to_device(a, dev) for a in (ids, mask)]
    big = [t[:16].cpu() for t in m.forward(*args)]
    small = [t.cpu() for t in m.forward(*(a[:16] for a in args))]
    m.check()
    for i, (a, b) in enumerate(zip(big, small)):
        assert torch.equal(a, b), f'output {i}'
    t_small = m.gemm_tile(16 * 128, 768, 3072)  # FFN2 at B = 16: autotuned, not the pin
    assert t_small != 0 and 70000 <= t_small < 80000
