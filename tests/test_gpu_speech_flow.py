"""speech_flow_kernel (csrc/speech_fusion.hip): the speech DNN of
model_training/train_speech_model.py:55-90 as one launch whose layers are split by output
columns over workgroups, with in-launch hand-offs between the stages of each 16-sample chunk.

Checks: parity with the fp32 oracle across chunk edges, a forced expired wait (probe build)
reported by mec_model_check and NOT leaking into the next launch, bit-stable results over many
back-to-back launches (the per-launch counter reset), under uneven load from a concurrent stream (MI355X_MICROARCH.md: test every hand-off
under uneven load, checking every word), inside a captured graph, and batch invariance (chunks
are independent, so a row's result does not depend on the batch around it).
"""
import numpy as np
import pytest
import torch

from mec import engine, synthetic as syn
from oracle import speech as o_s

pytestmark = pytest.mark.gpu

PROB_TOL = 1e-5
FEAT_RTOL = 2e-5


@pytest.fixture(scope='module')
def enc(dev):
    return engine.SpeechEncoder(device=dev)


def _run(enc, x):
    out = enc.forward(x)
    torch.cuda.synchronize()
    return [t.cpu().numpy() for t in out]


@pytest.mark.parametrize('B', [1, 15, 16, 17, 33, 100, 256, 1000])
def test_flow_vs_oracle(enc, dev, B):
    x = syn.speech_inputs(B, seed=300 + B)
    feat, logits, probs = _run(enc, engine.to_device(x, dev))
    rf, rl, rp = o_s.forward(syn.weights('speech'), x)
    assert not np.isnan(probs).any()
    ferr = float(np.abs(feat - rf).max() / max(1.0, np.abs(rf).max()))
    perr = float(np.abs(probs - rp).max())
    print(f'B={B}: feat rel {ferr:.3g}, logits {np.abs(logits - rl).max():.3g}, probs {perr:.3g}')
    assert ferr < FEAT_RTOL and perr < PROB_TOL
    assert np.array_equal(probs.argmax(1), rp.argmax(1))


def test_expired_wait_is_reported_and_does_not_poison_the_next_launch(dev):
    """The probe build's speech_spin_limit 0 makes every stage give up on its first poll: some
    waits expire (their chunks' probs come out NaN) and mec_model_check reports it. The next
    launch on the same handle, at the normal limit, starts from zeroed counters and error word:
    finite probs equal to the product library's, and a clean check. One forced run, not
    repeated (the expiry depends on timing; the assertions hold either way)."""
    import ctypes
    from mec import _lib
    x = syn.speech_inputs(256, seed=8)
    xd = engine.to_device(x, dev)
    ref = _run(engine.SpeechEncoder(device=dev), xd)
    plib = _lib.load(_lib.PROBES_LIB_PATH)
    assert plib.mec_build_flags() == 1
    blob = syn.pack('speech', syn.weights('speech'))
    h = ctypes.c_void_p()
    assert plib.mec_create_ex(0, blob.ctypes.data_as(_lib.c_fp), blob.size, dev.index, 1, ctypes.byref(h)) == 0
    try:
        outs = []
        for limit in (0, -1):
            assert plib.mec_model_set_option(h, b'speech_spin_limit', limit) == 0
            feat, logits, probs = (torch.empty((256, d), device=dev) for d in (64, 7, 7))
            ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
            assert plib.mec_speech_fwd(h, ptr(xd), 256, ptr(feat), ptr(logits), ptr(probs),
                                       ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)) == 0
            torch.cuda.synchronize()
            outs.append((probs.cpu().numpy(), plib.mec_model_check(h)))
        (p0, rc0), (p1, rc1) = outs
        n_nan = int(np.isnan(p0).any(1).sum())
        print(f'forced expiry: {n_nan} of 256 rows NaN, check rc {rc0}; next launch: check rc {rc1}')
        assert rc0 == (-1 if n_nan else 0)  # reported iff some chunk's wait expired
        assert rc1 == 0 and not np.isnan(p1).any()
        assert np.array_equal(p1, ref[2])
    finally:
        plib.mec_destroy(h)


def test_check_is_clean_after_normal_launches(enc, dev):
    x = engine.to_device(syn.speech_inputs(100, seed=10), dev)
    for _ in range(5):
        enc.forward(x)
    torch.cuda.synchronize()
    enc.check()  # raises MecError if any wait expired


def test_flow_repeat_bit_stable(enc, dev):
    """200 back-to-back launches (each starts from the counters its memset zeroed)."""
    x = engine.to_device(syn.speech_inputs(32, seed=3), dev)
    ref = _run(enc, x)
    outs = [enc.forward(x) for _ in range(200)]
    torch.cuda.synchronize()
    for o in outs:
        for r, t in zip(ref, o):
            assert np.array_equal(r, t.cpu().numpy())


def test_flow_alternating_inputs(enc, dev):
    """Back-to-back launches over different inputs into the same hand-off buffers: a consumer
    that accepted a previous launch's granules would return the other input's result."""
    xs = [engine.to_device(syn.speech_inputs(40, seed=s), dev) for s in (11, 12, 13)]
    refs = [_run(enc, x) for x in xs]
    outs = [(i % 3, enc.forward(xs[i % 3])) for i in range(150)]
    torch.cuda.synchronize()
    for i, o in outs:
        for r, t in zip(refs[i], o):
            assert np.array_equal(r, t.cpu().numpy())


def test_flow_under_uneven_load(enc, dev):
    """Speech launches on the current stream while a side stream keeps the CUs busy with GEMMs;
    every word of every launch must equal the idle run."""
    x = engine.to_device(syn.speech_inputs(256, seed=4), dev)
    ref = _run(enc, x)
    side = torch.cuda.Stream(dev)
    a = torch.randn(4096, 4096, device=dev, dtype=torch.float16)
    outs = []
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        for _ in range(10):
            a = (a @ a).clamp_(-1, 1)
    for _ in range(30):
        outs.append(enc.forward(x))
    torch.cuda.synchronize()
    for o in outs:
        for r, t in zip(ref, o):
            assert np.array_equal(r, t.cpu().numpy())


def test_flow_graph_replay(enc, dev):
    x = engine.to_device(syn.speech_inputs(48, seed=5), dev)
    ref = _run(enc, x)
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        enc.forward(x)  # warm on the capture stream
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        out = enc.forward(x)
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    for r, t in zip(ref, out):
        assert np.array_equal(r, t.cpu().numpy())


def test_flow_batch_invariance(enc, dev):
    x = syn.speech_inputs(256, seed=6)
    full = _run(enc, engine.to_device(x, dev))
    for lo in (0, 100, 240):
        part = _run(enc, engine.to_device(x[lo:lo + 16], dev))
        for f, p in zip(full, part):
            assert np.array_equal(f[lo:lo + 16], p)
