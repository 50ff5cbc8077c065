"""Benchmark: fused tri-modal samples/s; per-modality logits max-abs-err (BASELINE.json metric).

One step = one pass of the whole hot path over one synthetic batch already resident in
HBM: speech DNN + BERT-base (L=128) + ResNet50 (48x48 u8 -> 224) encoders, then the
attention-MLP fusion, then (N>1) the RCCL all-gather of the 34-float result rows.
Weak scaling: every rank processes its own batch (256 at N=1 = BASELINE configs[3]; 1024 per
rank at N>1 = configs[4]'s global 8192 on 8 GPUs). Consecutive batches are pipelined
(engine.FusedPipeline): batch i's fusion and gather overlap batch i+1's encoders; the timed
region ends after the last batch's gather (device synchronize).

The path runs at three precisions on the same inputs; rank 0 prints ONE JSON line:
  headline  "fp32x3": the reference's fp32 arithmetic (inference/text_inference.py:91-93,
            inference/image_inference.py:116-118) with every GEMM / conv operand carried as a
            pair of f16 planes (hi + lo: 22 significant bits; activations at a per-tensor
            power-of-two plane scale fixed at handle creation, weights at a per-matrix one; a range
            flag that check() raises if a plane leaves the f16 range: INTEGRATION.md "fp32x3
            envelope") and each product as hi.hi + hi.lo + lo.hi on the f16 MFMA into one fp32
            accumulator; LayerNorm, softmax, attention, GELU, residual stream, heads,
            speech and fusion in fp32 as on the exact path. Held to the fp32 path's parity bars,
            and closer to float64 than the exact-f32 MFMA engine per GEMM (its 32-deep MFMA sums
            round the accumulator 8x less often: tests/test_gpu_fp32x3.py) -- `value`;
  nested    "fp32_exact_path": every operand and product in fp32 (v_mfma_f32_16x16x4_f32);
  nested    "f16_fast_path": BERT / ResNet50 on f16 MFMA operands with fp32 accumulation,
            LayerNorm, softmax, GELU, residual stream and heads: a speed option, narrower than the
            reference's arithmetic, reported beside the headline, not as it. Its text probs error sits
            near the north_star's 1e-3 bar with rows at risk, so its parity.north_star verdict reads
            "outside the contract margin" (margin = half the bar, no at-risk rows).
Each carries `parity`: the oracle (CPU fp32 restatement of the reference) on rows of the timed
batch -- every row at B <= 256, rows from every quarter of the batch beyond -- with logits /
probs max-abs-err, argmax agreement and the count of at-risk rows (oracle top-2 margin below
twice the measured probs error), the fused output checked end to end against o_f(o_s, o_t, o_i).
At N>1 rank 0 also checks two gathered rows of EVERY rank against the oracle run on that rank's
inputs (the all-gather's order and content).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--precision all|both|fp32x3|fp32|f16]

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py starts
`python -m torch.distributed.run --nproc-per-node N ... bench.py` as a child process BEFORE any
GPU call and exits with its status (one process per GPU; the driver's own torchrun launch
sets WORLD_SIZE and skips this). With no GPU visible (or --stub) each rank runs a stub step on
the CPU over gloo -- the launcher, sharding, all-gather order and max-over-ranks timing only;
its line has `value` null.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'multimodal-emotion-classification_amd'))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = 'fused tri-modal samples/sec @ batch 256; per-modality logits max-abs-err'
# Algorithmic work (BASELINE.md "Work per unit")
FLOP_PER_SAMPLE = {'text': 2 * 11_174_221_056, 'image': 2 * 4_088_188_416, 'speech': 2 * 463_296,
                   'fusion': 2 * 2_020_000}
# MI355X_MICROARCH.md: dense f16 MFMA ~2.5 PF; f32-input MFMA 157.3 TF (= the f32 vector peak)
PEAK_TFLOPS = {'f16': 2500.0, 'fp32': 157.3, 'fp32x3': 2500.0}
# fp32x3: every GEMM FLOP is three f16 MFMA FLOPs (hi.hi + hi.lo + lo.hi), priced against the f16 peak
MFMA_FLOP_PER_FLOP = {'f16': 1, 'fp32': 1, 'fp32x3': 3}
DTYPE = {'f16': 'f16 MFMA operands / fp32 accumulate, LN & softmax & residual fp32; speech+fusion fp32',
         'fp32': 'fp32 (exact-f32 MFMA GEMMs; every operand and product fp32)',
         'fp32x3': 'fp32 (GEMM/conv operands as f16 hi+lo plane pairs, 22 significant bits, activations at '
                   'per-tensor power-of-two plane scales; hi.hi + hi.lo + lo.hi on the f16 MFMA into '
                   'one fp32 accumulator: per GEMM closer to float64 than the exact-f32 MFMA; LN, softmax, '
                   'attention, GELU, residual stream, heads, speech and fusion fp32)'}
ROW = 34  # packed result row: 3x7 modality probs | 7 fused probs | 3 attention | 3 decision weights


def tile_name(tile: int, M: int) -> str:
    """Kernel + grid for an f16 GEMM tile id (gemm_glds.hip, launch_bn)."""
    if tile in (40256, 41256):
        bm = 256 if tile == 40256 else 128
        return f'gemm_pp_kernel<{bm}x256x64 ping-pong, mfma16x16x32> grid={((M + bm - 1) // bm) * (3072 // 256)}'
    v, w = divmod(tile, 10000)
    bm, bn = (128, w - 1000) if w > 1000 else (256, w)
    if bn <= 0:
        return f'gemm tile {tile}'
    mf = 32 if v == 0 else 16
    bk = 32 if v >= 2 else 64
    x3i = ' K-interleaved split terms' if v == 7 else ''
    return f'gemm_glds_kernel<{bm}x{bn}x{bk}, mfma{mf}{x3i}> grid={((M + bm - 1) // bm) * (3072 // bn)}'


def tile_name_f32(tile: int, M: int) -> str:
    """Kernel + grid for an fp32 GEMM tile id (gemm_f32.hip, launch_tile)."""
    bm, bn = {1: (256, 128), 2: (128, 128), 3: (128, 64), 4: (256, 256)}.get((tile - 1) % 4 + 1, (0, 0))
    if not bm or not 1 <= tile <= 8:
        return f'gemm_f32 tile {tile}'
    mf = 'mfma_f32_32x32x2f32' if tile <= 4 else 'mfma_f32_16x16x4f32'
    return f'gemm_f32_kernel<{bm}x{bn}x32, {mf}> grid={((M + bm - 1) // bm) * (3072 // bn)}'


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--batch', type=int, default=0, help='samples per rank (default 256 at N=1, 1024 at N>1)')
    ap.add_argument('--precision', default='all', choices=['all', 'both', 'f16', 'fp32', 'fp32x3'],
                    help='all: fp32x3 (headline) + fp32 exact + f16 (nested); both: fp32 (headline) + f16; '
                         'or one precision')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-parity', action='store_true')
    ap.add_argument('--oracle-rows', type=int, default=256,
                    help='check every row of the batch against the oracle up to this batch size; '
                         'beyond it, rows from every quarter (parity_rows)')
    ap.add_argument('--serial', action='store_true', help='run the encoders on one stream (A/B of the concurrency)')
    ap.add_argument('--no-pipeline', action='store_true',
                    help="run each batch's fusion on the main stream (A/B of the cross-batch overlap)")
    ap.add_argument('--no-configs', action='store_true', help='skip the per-config (single-encoder) timings')
    ap.add_argument('--text-priority', type=int, default=1, help='0: BERT on the default-priority stream (A/B)')
    ap.add_argument('--image-priority', type=int, default=0,
                    help='1: speech + image stream at high priority, BERT at normal (A/B)')
    ap.add_argument('--stub', action='store_true',
                    help='CPU stub step over gloo (launcher / gather check; automatic with no GPU visible)')
    ap.add_argument('--json-out', default=None, help='also write the result line to this file (rank 0)')
    return ap.parse_args(argv)


# ----------------------------------------------------------------------------- launcher


def _free_port() -> int:
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch(a, argv) -> int:
    """--gpus N > 1 without WORLD_SIZE: run N ranks through torch.distributed.run as a CHILD
    process (never exec: this process has not touched the GPU, and must not replace itself)."""
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={a.gpus}',
           '--master-addr', '127.0.0.1', f'--master-port={_free_port()}', os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    return subprocess.run(cmd, env=env).returncode


def parity_rows(B: int, limit: int):
    """Rows the oracle recomputes: all of them up to `limit`; beyond, the batch edges, the
    64/128/256-row tile edges of every quarter of the batch and a seeded spread (so rows
    256..B-1 of a 1024-per-rank batch are covered)."""
    if B <= limit:
        return list(range(B))
    rows = {0, 1, 2, B - 2, B - 1}
    for q in range(4):
        base = q * B // 4
        for off in (0, 1, 63, 64, 127, 128, 255):
            if base + off < B:
                rows.add(base + off)
    rng = np.random.default_rng(B)
    rows.update(int(r) for r in rng.choice(B, size=min(B, 16), replace=False))
    return sorted(rows)


# ----------------------------------------------------------------------------- oracle side


def host_cpus():
    """(threads usable by this process, physical cores of the host, logical CPUs in the
    affinity mask, physical cores in the affinity mask). The GPU box shares a many-core host; its
    share is OMP_NUM_THREADS (16)."""
    mask = os.sched_getaffinity(0)
    avail = len(mask)
    try:
        threads = min(avail, int(os.environ.get('OMP_NUM_THREADS', avail)))
    except ValueError:
        threads = avail
    phys, phys_mask = set(), set()
    try:
        cpu = pid = None
        with open('/proc/cpuinfo') as fh:
            for line in fh:
                if line.startswith('processor'):
                    cpu = int(line.split(':')[1])
                elif line.startswith('physical id'):
                    pid = line.split(':')[1].strip()
                elif line.startswith('core id'):
                    core = (pid, line.split(':')[1].strip())
                    phys.add(core)
                    if cpu in mask:
                        phys_mask.add(core)
    except (OSError, ValueError):
        pass
    return threads, (len(phys) or None), avail, (len(phys_mask) or None)


# BERT's executed work per sample when the last layer runs on the [CLS] rows only (bert_cls_last,
# DESIGN.md §4): K / V for every token, Q / O-projection / FFN for the [CLS] row, and the [CLS]
# attention kernel's 32 query rows (it runs the full kernel's instruction sequence for queries 0..31)
_BERT_LAYER_MAC = 128 * 768 * 2304 + 2 * 128 * 128 * 768 + 128 * 768 * 768 + 2 * 128 * 768 * 3072
_BERT_CLS_LAYER_MAC = 128 * 768 * 1536 + 768 * 768 + 2 * 32 * 128 * 768 + 768 * 768 + 2 * 768 * 3072
EXEC_FLOP_PER_SAMPLE = dict(FLOP_PER_SAMPLE, text=FLOP_PER_SAMPLE['text'] - 2 * (_BERT_LAYER_MAC - _BERT_CLS_LAYER_MAC))


def _oracle_chain(w, x, ids, mask, gray, sel, times=None):
    """The oracle chain on rows `sel`: per modality (feat, logits, probs) and the fused chain
    o_f(o_s, o_t, o_i) (inference/multimodal_fusion.py:271-278); `times` collects per-modality
    seconds."""
    from oracle import fusion as o_f, image as o_i, speech as o_s, text as o_t
    t = [time.perf_counter()]
    rs = o_s.forward(w['speech'], x[sel])
    t.append(time.perf_counter())
    rt = o_t.forward(w['text'], ids[sel], mask[sel])
    t.append(time.perf_counter())
    ri = o_i.forward(w['image'], gray[sel])
    t.append(time.perf_counter())
    rf = o_f.forward(w['fusion'], rs[0], rt[0], ri[0], rs[2], rt[2], ri[2])
    t.append(time.perf_counter())
    if times is not None:
        for k, (a, b) in zip(('speech', 'text', 'image', 'fusion'), zip(t, t[1:])):
            times.setdefault(k, []).append(b - a)
        times.setdefault('fused', []).append(t[-1] - t[0])
    return {'speech': rs, 'text': rt, 'image': ri, 'fusion': rf}


# cpu_baseline (BASELINE.md "CPU baseline"): the whole timed batch (up to CPU_SAMPLE_ROWS rows), median
# of CPU_PASSES passes at the box's CPU share; the physical-core repeat is a secondary, smaller sample
CPU_SAMPLE_ROWS, CPU_PASSES = 256, 5
CPU_PHYS_ROWS, CPU_PHYS_PASSES = 32, 3


def oracle_run(x, ids, mask, gray, rows, timed: bool):
    """The CPU oracle (fp32 torch-CPU / numpy restatement of the reference arithmetic) on `rows`
    of the batch: the parity reference. timed=True also returns the cpu_baseline record (SURVEY
    §8(d)): the oracle chain on the first CPU_SAMPLE_ROWS rows of the timed batch (all
    256 at the headline config), after a 2-row warm-up, CPU_PASSES timed passes -> median, at torch
    threads = OMP_NUM_THREADS (the box's CPU share for one GPU: `value`). When the sample is the
    parity rows, the first timed pass's outputs are the parity reference (the same computation, not
    run twice). Secondary: CPU_PHYS_PASSES passes over CPU_PHYS_ROWS rows at every physical core in
    the affinity mask; per-modality rates at both."""
    sys.path.insert(0, ROOT)
    from mec import synthetic as syn
    threads, phys, avail, phys_mask = host_cpus()
    prev = torch.get_num_threads()
    w = {k: syn.weights(k) for k in ('speech', 'text', 'image', 'fusion')}
    r = np.asarray(rows)
    torch.set_num_threads(threads)
    sample = np.arange(min(CPU_SAMPLE_ROWS, len(x)))
    shared = timed and len(r) == len(sample) and np.array_equal(r, sample)
    ref, ref_s = None, None
    if not shared:
        t0 = time.perf_counter()
        ref = _oracle_chain(w, x, ids, mask, gray, r)
        ref_s = time.perf_counter() - t0
    cb = None
    if timed:
        def run(nt, rows_, passes):
            nonlocal ref, ref_s
            torch.set_num_threads(nt)
            _oracle_chain(w, x, ids, mask, gray, rows_[:2])  # warm-up
            times = {}
            for i in range(passes):
                out = _oracle_chain(w, x, ids, mask, gray, rows_, times)
                if ref is None and nt == threads and i == 0:
                    ref, ref_s = out, times['fused'][0]
            med = {k: float(np.median(v)) for k, v in times.items()}
            return {'rows': len(rows_), 'passes': passes, 'fused_samples_per_s': len(rows_) / med['fused'],
                    'per_modality_samples_per_s': {k: len(rows_) / med[k] for k in ('speech', 'text', 'image', 'fusion')},
                    'median_pass_s': med['fused'], 'passes_s': [round(v, 3) for v in times['fused']]}
        head = run(threads, sample, CPU_PASSES)
        physrun = None
        if phys_mask and phys_mask != threads:
            physrun = {'cores': phys_mask, **run(phys_mask, sample[:CPU_PHYS_ROWS], CPU_PHYS_PASSES)}
        cb = {'value': head['fused_samples_per_s'], 'unit': 'fused samples/s', 'cores': threads, 'kind': 'port',
              'sample': f'the {len(sample)} rows of the timed batch (L=128 full rows, 48x48 u8) through oracle/ '
                        f'(fp32 torch-CPU restatement: speech DNN, BERT, ResNet50, fusion), 2-row warm-up, median of '
                        f'{CPU_PASSES} passes' + ('; the first pass is also the parity reference' if shared else ''),
              'per_modality_samples_per_s': head['per_modality_samples_per_s'],
              'median_pass_s': head['median_pass_s'], 'passes_s': head['passes_s'],
              'threads_note': 'cores = torch threads = OMP_NUM_THREADS, the CPU share the GPU box gives one GPU; '
                              '`at_physical_cores_in_affinity_mask` repeats a smaller sample on every physical core '
                              'this process may run on (secondary)',
              'at_physical_cores_in_affinity_mask': physrun,
              'parity_pass': {'rows': len(r), 'seconds': ref_s, 'fused_samples_per_s': len(r) / ref_s,
                              'cores': threads, 'shared_with_timed_pass': shared},
              'host_physical_cores': phys, 'host_logical_cpus_in_affinity': avail,
              'host_physical_cores_in_affinity': phys_mask}
    torch.set_num_threads(prev)
    return ref, cb


def parity(out, ref, rows):
    """Per modality logits / probs max-abs-err, argmax agreement and at-risk rows against the
    oracle outputs `ref` for `rows` of the timed batch; fusion = the end-to-end oracle chain."""
    torch.cuda.synchronize()
    idx = torch.as_tensor(rows, device=out['fusion'][1].device)
    g = {k: [t.index_select(0, idx).cpu().numpy() for t in v] for k, v in out.items()}
    res = {}
    for name, (gl, gp), (rl, rp) in (('speech', g['speech'][1:3], ref['speech'][1:3]),
                                      ('text', g['text'][1:3], ref['text'][1:3]),
                                      ('image', g['image'][1:3], ref['image'][1:3]),
                                      ('fusion', g['fusion'][0:2], ref['fusion'][0:2])):
        perr = float(np.abs(gp - rp).max())
        s = np.sort(rp, axis=1)
        margin = s[:, -1] - s[:, -2]
        res[name] = {'logits_max_abs_err': float(np.abs(gl - rl).max()), 'probs_max_abs_err': perr,
                     'argmax_agree': f'{int((gp.argmax(1) == rp.argmax(1)).sum())}/{len(rows)}',
                     'min_oracle_top2_margin': float(margin.min()),
                     'at_risk_rows': int((margin < 2 * perr).sum())}
    for k, j in (('attention_weights', 2), ('decision_weights', 3)):
        res['fusion'][k + '_max_abs_err'] = float(np.abs(g['fusion'][j] - ref['fusion'][j]).max())
    res['rows'] = (f'all {len(rows)} rows of the timed batch' if len(rows) == out['fusion'][1].shape[0]
                   else f'{len(rows)} rows spread over the timed batch (first {rows[:4]}, last {rows[-3:]})')
    res['fused_reference'] = 'end-to-end oracle chain o_f(o_s, o_t, o_i) (multimodal_fusion.py:271-278)'
    # north_star: argmax exact, probs within 1e-3. "with_margin": every modality's probs error at most half
    # the bar and no row whose oracle top-2 margin is below twice that error (a path that meets the bar only
    # narrowly, as the f16 one does, is reported as outside the contract's margin)
    mods = [res[k] for k in ('speech', 'text', 'image', 'fusion')]
    exact = all(m['argmax_agree'].split('/')[0] == m['argmax_agree'].split('/')[1] for m in mods)
    within = all(m['probs_max_abs_err'] <= 1e-3 for m in mods)
    margin = all(m['probs_max_abs_err'] <= 5e-4 and m['at_risk_rows'] == 0 for m in mods)
    res['north_star'] = {'argmax_exact': exact, 'probs_within_1e-3': within, 'with_margin': margin,
                         'verdict': ('held' if exact and within and margin else
                                     'met on this batch, outside the contract margin' if exact and within else
                                     'not met')}
    return res


def gather_check(gathered, world, B):
    """Rank 0: two rows of every rank's shard in the gathered [world*B, 34] block against the
    oracle run on that rank's own (seed = rank) inputs."""
    sys.path.insert(0, ROOT)
    from mec import synthetic as syn
    errs, agree, n = [], 0, 0
    for r in range(world):
        x = syn.speech_inputs(B, seed=r)
        ids, mask = syn.text_inputs(B, 128, seed=r, ragged=False)
        gray = syn.image_inputs(B, seed=r)
        sel = [0, B - 1]
        ref, _ = oracle_run(x, ids, mask, gray, sel, timed=False)
        want = np.concatenate([ref['speech'][2], ref['text'][2], ref['image'][2], ref['fusion'][1],
                               ref['fusion'][2], ref['fusion'][3]], axis=1)
        got = gathered[[r * B + s for s in sel]]
        errs.append(float(np.abs(got - want).max()))
        agree += int((got[:, 21:28].argmax(1) == want[:, 21:28].argmax(1)).sum())
        n += len(sel)
    return {'rows_per_rank': 2, 'ranks': world, 'max_abs_err_vs_oracle': max(errs), 'fused_argmax_agree': f'{agree}/{n}'}


# ----------------------------------------------------------------------------- GPU run


def per_config(pipe, dev, precision, iters=10):
    """Single-encoder throughput on the other BASELINE configs (rank 0, N=1; informational,
    not `value`): speech B=32, image B=256 (ResNet50 and the MobileNetV2 backbone),
    text B=128 (L=128). hipEvents around `iters` back-to-back calls, inputs in HBM."""
    from mec import engine, synthetic as syn
    xs = engine.to_device(syn.speech_inputs(32, seed=7), dev)
    ids, mask = syn.text_inputs(128, 128, seed=7)
    ids, mask = engine.to_device(ids, dev), engine.to_device(mask, dev)
    g = engine.to_device(syn.image_inputs(256, seed=7), dev)
    runs = {'speech_b32': (32, lambda: pipe.speech.forward(xs)),
            'image_resnet50_b256': (256, lambda: pipe.image.forward(g)),
            'text_bert_b128': (128, lambda: pipe.text.forward(ids, mask))}
    # speech from waveforms (§8(f) row 4): GPU features (csrc/audio.hip) then the DNN, B = 32
    # clips of 3 s at 22050 Hz (config.py:57-58)
    af = engine.AudioFeaturizer(device=dev)
    wv = torch.from_numpy(np.random.default_rng(7).standard_normal((32, 66150)).astype(np.float32)).to(dev)
    runs['speech_waveform_b32'] = (32, lambda: pipe.speech.forward(af.forward(wv)))
    mb = engine.MobileNetImageEncoder(device=dev, precision=precision)
    runs['image_mobilenet_v2_b256'] = (256, lambda: mb.forward(g))
    out = {}
    for name, (b, fn) in runs.items():
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / iters
        out[name] = {'samples_per_s': b / ms * 1e3, 'ms_per_batch': ms}
    # speech B=32 with the host out of the loop: 20 forwards captured in one graph, replayed
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(s):
        pipe.speech.forward(xs)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=s):
        for _ in range(20):
            pipe.speech.forward(xs)
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        gr.replay()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / (iters * 20)
    out['speech_b32_graph'] = {'samples_per_s': 32 / ms * 1e3, 'ms_per_batch': ms}
    del gr
    mb.close()
    af.close()
    return out


def run(a, precision, B, world, rank, dev, inputs):
    """Time K pipelined steps at one precision; returns (result line or None, last outputs,
    gathered rows or None)."""
    from mec import _lib, dist as mdist, engine
    # the product library: no probe build (probe option values skip work and return wrong
    # results), and every knob of the pipeline's handles at its default (handles own their knobs)
    # apart from the pipeline's own pin (BERT FFN2 on the ping-pong tile in the concurrent step)
    if _lib.load().mec_build_flags() != 0:
        raise SystemExit(f'bench.py: {_lib.LIB_PATH} is a probe build (MEC_PROBES); use the product library')
    pipe = engine.FusedPipeline(seed=1234, device=dev, concurrent=not a.serial, pipelined=not a.no_pipeline,
                                text_priority=bool(a.text_priority), image_priority=bool(a.image_priority),
                                precision=precision)
    x, ids, mask, gray = (engine.to_device(v, dev) for v in inputs)
    gather_ev = []
    last = {}

    def finish(out):  # runs on the fusion's stream (FusedPipeline: batch i's fusion overlaps batch i+1)
        rows = pipe.pack_rows(out)
        last['out'] = out
        if world > 1:  # one RCCL all-gather of the 34-float result rows
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rows = mdist.all_gather_rows(rows, world * B)
            e1.record()
            gather_ev.append((e0, e1))
        last['rows'] = rows
        return rows

    def step():
        return pipe.forward(x, ids, mask, gray, epilogue=finish)[1]

    for _ in range(a.warmup):
        step()
    # fence: every warm-up kernel (all streams) retires BEFORE the opening profiler marker, so a
    # rocprofv3 window between the two markers holds exactly the timed steps' dispatches
    torch.cuda.synchronize()
    gather_ev.clear()
    # hipEvent timing of the dominant kernel (BERT FFN1 GEMM) inside the timed region
    pipe.text.prof_enable('bert_ffn1')
    torch.cuda._sleep(1)  # opening marker for tools/prof_summary.py --window spin (outside the timing)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    torch.cuda._sleep(1)  # closing marker
    pipe.check()  # an after-the-fact kernel error (mec_model_check) fails the run, never a silent NaN
    ffn_ms, ffn_n = pipe.text.prof_read()
    gather_ms = [e0.elapsed_time(e1) for e0, e1 in gather_ev]
    # the same kernel with BERT alone on the GPU (no concurrent image stream), untimed region
    pipe.text.prof_enable('bert_ffn1')
    for _ in range(2):
        pipe.text.forward(ids, mask)
    torch.cuda.synchronize()
    iso_ms, iso_n = pipe.text.prof_read()
    pipe.text.prof_enable(0)
    t = torch.tensor([el], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    el = float(t.item())
    gathered = last['rows'].cpu().numpy() if world > 1 else None
    if rank != 0:
        for m in pipe.models():
            m.close()
        return None, None, None

    M = B * 128
    peak = PEAK_TFLOPS[precision]
    mf = MFMA_FLOP_PER_FLOP[precision]
    ffn_flop = 2.0 * M * 3072 * 768 * mf  # MFMA FLOPs per launch (fp32x3: three f16 products per product)
    avg_s = (ffn_ms / max(ffn_n, 1)) / 1e3
    achieved = ffn_flop / avg_s / 1e12 if ffn_n else None
    iso = ffn_flop / ((iso_ms / max(iso_n, 1)) / 1e3) / 1e12 if iso_n else None
    tile = pipe.text.gemm_tile(M, 3072, 768)  # the text handle's own autotune choice
    if precision == 'fp32x3' and not tile:
        # the split FFN1 is pinned, never autotuned (csrc/gemm.hip: launch_gemm): 70256 at the default
        # K-interleaved term order (gemm_x3_order 1), 10256 at the pass-major order
        tile = 70256
    if precision == 'f16':
        kname = tile_name(tile, M) + ' + GELU'
        ebytes, tfile = 2, 'ffn1_traffic.json'
    elif precision == 'fp32x3':
        kname = tile_name(tile, M) + ' split-f16 (hi.hi + hi.lo + lo.hi) + erf-GELU, hi/lo f16 out'
        ebytes, tfile = 4, 'ffn1_x3_traffic.json'
    else:
        kname = tile_name_f32(tile, M) + ' + erf-GELU'
        ebytes, tfile = 4, 'ffn1_f32_traffic.json'
    traffic, tsrc = None, None
    tf = os.path.join(ROOT, 'profiles', tfile)
    if os.path.exists(tf):  # PMC passes (tools/pmc.sh), FETCH_SIZE x2 per MI355X_MICROARCH gfx950 note
        with open(tf) as fh:
            tj = json.load(fh)
        if tj.get('tile') == tile and tj.get('M') == M:
            traffic, tsrc = tj['bytes_per_launch'], tj['source']
    roof = {'bound': 'mfma', 'kernel': f'{kname} (BERT FFN1, M={M} N=3072 K=768)',
            'achieved': achieved, 'peak': peak, 'unit': 'TFLOP/s',
            'frac': (achieved / peak) if achieved else None, 'traffic': traffic, 'traffic_source': tsrc,
            'algorithmic_flop_per_launch': ffn_flop / mf, 'mfma_flop_per_launch': ffn_flop,
            'algorithmic_bytes_per_launch': ebytes * (M * 768 + 3072 * 768 + M * 3072),
            'avg_launch_ms': avg_s * 1e3, 'launches': ffn_n,
            # 11 of BERT's 12 layers run FFN1 over all M tokens; the last one (bert_cls_last) runs it
            # on the B [CLS] rows only, as an untagged launch of its own shape
            'launches_expected': 11 * a.steps,
            'note': 'achieved: live in the timed region (CUs shared with the image stream); '
                    'achieved_isolated: BERT alone',
            'achieved_isolated': iso, 'frac_isolated': (iso / peak) if iso else None}
    if precision == 'fp32x3' and achieved:
        # the same launch priced as fp32 work: algorithmic FLOPs / time, against the f32 MFMA peak
        # (157.3 TF) the exact-fp32 engine is bound by, and against 2.5 PF / 3 (three f16 products
        # per fp32 product)
        fp32_eq = achieved / mf
        roof['fp32_equivalent'] = {'achieved_tflops': fp32_eq, 'vs_f32_mfma_peak': fp32_eq / PEAK_TFLOPS['fp32'],
                                   'vs_f16_peak_over_3': fp32_eq / (peak / mf)}
    total = world * B * a.steps
    flop = sum(FLOP_PER_SAMPLE.values()) * total
    flop_exec = sum(EXEC_FLOP_PER_SAMPLE.values()) * total
    res = {
        'metric': METRIC,
        'value': total / el, 'unit': 'samples/s', 'n_gpus': world, 'steps': a.steps, 'warmup': a.warmup,
        # samples each rank runs per step: a SCALE N = 8 line (1024 per rank) divides by an N = 1 line of
        # the same per_rank_batch (bench.py --batch 1024), not by the 256-sample headline
        'per_rank_batch': B,
        'ms_per_step': el / a.steps * 1e3, 'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
        'dtype': DTYPE[precision], 'precision': precision,
        'data': 'synthetic (seeded inputs: 56-d features, 128-token ids, 48x48 u8; seeded synthetic weights)',
        'config': {'workload': 'fused tri-modal: speech DNN + BERT-base L=128 + ResNet50@224 + attention fusion'
                               + (' (BASELINE configs[3])' if world == 1 and B == 256 else
                                  ' (BASELINE configs[4] per-rank shard)' if B == 1024 else ''),
                   'batch_per_gpu': B, 'global_batch': world * B, 'seq_len': 128,
                   # BASELINE.json's metric string names batch 256 (configs[3]); at N > 1 each rank
                   # runs batch_per_gpu samples (configs[4]: 8192 over 8 GPUs)
                   'metric_batch_note': None if B == 256 else f'metric string names batch 256; this run: {B} per GPU',
                   'parallelism': f'dp{world} (sample-sharded, all-gather of 34-float rows)'},
        'achieved_tflops_whole_step': flop / el / 1e12,
        'whole_step_frac_of_peak': flop * mf / el / 1e12 / peak,
        # the same step counted by what the GPU executes: BERT's last layer on the [CLS] rows only
        'achieved_tflops_whole_step_executed': flop_exec / el / 1e12,
        'whole_step_frac_of_peak_executed': flop_exec * mf / el / 1e12 / peak,
        'flop_per_sample': {'reference_count': sum(FLOP_PER_SAMPLE.values()),
                            'executed': sum(EXEC_FLOP_PER_SAMPLE.values()),
                            'note': 'reference_count: the reference forward per sample (BERT 12 full layers, '
                                    'ResNet50, speech, fusion); executed: BERT last layer [CLS]-only '
                                    '(bert_cls_last), other encoders as counted'},
        'roofline': roof,
    }
    if world > 1:
        res['distributed'] = {'world_size': dist.get_world_size(), 'backend': dist.get_backend(),
                              'rccl_version': '.'.join(map(str, torch.cuda.nccl.version())),
                              'all_gather_ms_per_step': (sum(gather_ms) / len(gather_ms)) if gather_ms else None,
                              'all_gather_bytes_per_step': world * B * ROW * 4}
    if world == 1 and not a.no_configs:
        res['per_config'] = per_config(pipe, dev, precision)
    out = last.get('out')
    return res, (out, pipe), gathered


def main_gpu(a, world, rank, local):
    from mec import synthetic as syn
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    dev = torch.device('cuda', local)
    torch.cuda.set_device(dev)
    B = a.batch or (256 if world == 1 else 1024)
    inputs = (syn.speech_inputs(B, seed=rank), *syn.text_inputs(B, 128, seed=rank, ragged=False),
              syn.image_inputs(B, seed=rank))
    precs = {'all': ['f16', 'fp32x3', 'fp32'], 'both': ['f16', 'fp32']}.get(a.precision, [a.precision])
    lines, outs, gathered = {}, {}, {}
    for p in precs:
        res, o, gth = run(a, p, B, world, rank, dev, inputs)
        lines[p], outs[p], gathered[p] = res, o, gth
    if rank == 0:
        rows = parity_rows(B, a.oracle_rows)
        need_oracle = not a.no_parity or (world == 1 and not a.no_cpu_baseline)
        ref, cb = (oracle_run(*inputs, rows, timed=(world == 1 and not a.no_cpu_baseline))
                   if need_oracle else (None, None))
        for p in precs:
            out, pipe = outs[p]
            if not a.no_parity and out is not None:
                lines[p]['parity'] = parity(out, ref, rows)
                if world > 1:
                    lines[p]['parity']['all_gather_rows'] = gather_check(gathered[p], world, B)
            for m in pipe.models():
                m.close()
            if cb is not None:
                lines[p]['cpu_baseline'] = cb
        hp = next(p for p in ('fp32x3', 'fp32', 'f16') if p in lines)
        head = lines[hp]
        for p, key in (('fp32', 'fp32_exact_path'), ('f16', 'f16_fast_path'), ('fp32x3', 'fp32x3_path')):
            if p != hp and p in lines:
                f = lines[p]
                head[key] = {k: f[k] for k in ('value', 'unit', 'ms_per_step', 'dtype',
                                               'achieved_tflops_whole_step', 'whole_step_frac_of_peak',
                                               'achieved_tflops_whole_step_executed',
                                               'roofline', 'parity', 'per_config', 'distributed') if k in f}
        print(json.dumps(head), flush=True)
        if a.json_out:
            with open(a.json_out, 'w') as fh:
                json.dump(head, fh)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


# ----------------------------------------------------------------------------- CPU stub


def stub_rows(lo: int, hi: int) -> torch.Tensor:
    """Deterministic stand-in for the packed 34-float result rows of samples [lo, hi)."""
    g = torch.arange(lo, hi, dtype=torch.float64)[:, None] * ROW + torch.arange(ROW, dtype=torch.float64)[None]
    return torch.sin(g).float()


def main_stub(a, world, rank):
    """No GPU: the launcher, sharding, all-gather order and max-over-ranks timing over gloo."""
    from mec import dist as mdist
    if world > 1:
        dist.init_process_group('gloo')
    B = a.batch or (8 if world == 1 else 16)
    rows = None
    for i in range(a.warmup + a.steps):
        if i == a.warmup:
            if world > 1:
                dist.barrier()
            t0 = time.perf_counter()
        lo, hi = mdist.shard(world * B, world, rank)
        rows = stub_rows(lo, hi)
        if world > 1:
            rows = mdist.all_gather_rows(rows, world * B)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    t = torch.tensor([el], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ok = bool(torch.equal(rows, stub_rows(0, world * B)))
    if rank == 0:
        line = {'metric': METRIC, 'value': None, 'unit': 'samples/s', 'n_gpus': world, 'steps': a.steps,
                'warmup': a.warmup, 'per_rank_batch': B, 'ms_per_step': float(t.item()) / max(a.steps, 1) * 1e3,
                'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': None,
                'data': 'stub: no GPU visible, CPU stand-in rows', 'stub': True,
                'config': {'workload': 'launcher / sharding / all-gather check (no encoders run)',
                           'batch_per_gpu': B, 'global_batch': world * B,
                           'parallelism': f'dp{world} (gloo)'},
                'distributed': {'world_size': dist.get_world_size() if world > 1 else 1,
                                'backend': dist.get_backend() if world > 1 else None,
                                'gathered_rows_in_order': ok}}
        print(json.dumps(line), flush=True)
        if a.json_out:
            with open(a.json_out, 'w') as fh:
                json.dump(line, fh)
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        raise SystemExit('bench.py stub: gathered rows out of order')


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if 'WORLD_SIZE' not in os.environ and a.gpus > 1:
        sys.exit(launch(a, argv))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if a.stub or torch.cuda.device_count() == 0:  # device_count does not initialise the GPU
        if not a.stub:
            print('bench.py: no GPU visible -- running the CPU stub step (value null)', file=sys.stderr)
        main_stub(a, world, rank)
    else:
        main_gpu(a, world, rank, local)


if __name__ == '__main__':
    main()
