"""Benchmark: fused tri-modal samples/s @ batch 256 per GPU; per-modality logits max-abs-err
(BASELINE.json metric).

One step = one pass of the whole hot path over one synthetic batch already resident in
HBM: speech DNN + BERT-base (L=128) + ResNet50 (48x48 u8 -> 224) encoders, then the
attention-MLP fusion, then (N>1) the RCCL all-gather of the 34-float result rows.
Weak scaling: every rank processes its own batch (256 at N=1; 1024 per rank at N>1, i.e.
BASELINE configs[4]'s global 8192 on 8 GPUs). Consecutive batches are pipelined
(engine.FusedPipeline): batch i's fusion and gather overlap batch i+1's encoders; the timed
region ends after the last batch's gather (device synchronize).

The path runs at two precisions, each timed and checked on the same inputs, and rank 0
prints one JSON line per precision:
  1. "f16"  BERT / ResNet50 on f16 MFMA operands, fp32 accumulation, LayerNorm, softmax, GELU,
           residual stream and heads (the fast path, north_star's >=10k/s mode);
  2. "fp32" every operand and product in fp32 (v_mfma_f32_32x32x2_f32), the reference's own
           precision: the same-precision counterpart, printed second.
Each line carries `parity`: the oracle (CPU fp32 restatement of the reference) run on a fixed
subset of the timed batch — logits / probs max-abs-err and argmax agreement per modality,
the fused output checked end to end against o_f(o_s, o_t, o_i).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--precision both|f16|fp32]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, 'multimodal-emotion-classification_amd'))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# Algorithmic work (BASELINE.md "Work per unit")
FLOP_PER_SAMPLE = {'text': 2 * 11_174_221_056, 'image': 2 * 4_088_188_416, 'speech': 2 * 463_296,
                   'fusion': 2 * 2_020_000}
# MI355X_MICROARCH.md: dense f16 MFMA ~2.5 PF; f32-input MFMA 157.3 TF (= the f32 vector peak)
PEAK_TFLOPS = {'f16': 2500.0, 'fp32': 157.3}
DTYPE = {'f16': 'f16 MFMA operands / fp32 accumulate, LN & softmax & residual fp32; speech+fusion fp32',
         'fp32': 'fp32 (v_mfma_f32_32x32x2_f32 exact-f32 GEMMs; every operand and product fp32)'}
# rows of the timed batch the oracle recomputes: batch edges, tile edges and a spread
PARITY_ROWS = [0, 1, 63, 64, 100, 127, 128, 129, 170, 191, 200, 230, 254, 255]


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
    return f'gemm_glds_kernel<{bm}x{bn}x{bk}, mfma{mf}> grid={((M + bm - 1) // bm) * (3072 // bn)}'


def tile_name_f32(tile: int, M: int) -> str:
    """Kernel + grid for an fp32 GEMM tile id (gemm_f32.hip, launch_tile)."""
    bm, bn = {1: (256, 128), 2: (128, 128), 3: (128, 64), 4: (256, 256)}.get((tile - 1) % 4 + 1, (0, 0))
    if not bm or not 1 <= tile <= 8:
        return f'gemm_f32 tile {tile}'
    mf = 'mfma_f32_32x32x2f32' if tile <= 4 else 'mfma_f32_16x16x4f32'
    return f'gemm_f32_kernel<{bm}x{bn}x32, {mf}> grid={((M + bm - 1) // bm) * (3072 // bn)}'


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--batch', type=int, default=0, help='samples per rank (default 256 at N=1, 1024 at N>1)')
    ap.add_argument('--precision', default='both', choices=['both', 'f16', 'fp32'])
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-parity', action='store_true')
    ap.add_argument('--cpu-batch', type=int, default=32, help='fused samples per CPU-oracle run')
    ap.add_argument('--serial', action='store_true', help='run the encoders on one stream (A/B of the concurrency)')
    ap.add_argument('--no-pipeline', action='store_true',
                    help="run each batch's fusion on the main stream (A/B of the cross-batch overlap)")
    ap.add_argument('--no-configs', action='store_true', help='skip the per-config (single-encoder) timings')
    ap.add_argument('--text-priority', type=int, default=1, help='0: BERT on the default-priority stream (A/B)')
    ap.add_argument('--image-priority', type=int, default=0,
                    help='1: speech + image stream at high priority, BERT at normal (A/B)')
    return ap.parse_args()


def host_cpus():
    """(threads usable by this process, physical cores of the host, logical CPUs in the
    affinity mask). The GPU box shares a many-core host; its share is OMP_NUM_THREADS (16)."""
    avail = len(os.sched_getaffinity(0))
    try:
        threads = min(avail, int(os.environ.get('OMP_NUM_THREADS', avail)))
    except ValueError:
        threads = avail
    phys = set()
    try:
        pid = None
        with open('/proc/cpuinfo') as fh:
            for line in fh:
                if line.startswith('physical id'):
                    pid = line.split(':')[1].strip()
                elif line.startswith('core id'):
                    phys.add((pid, line.split(':')[1].strip()))
    except OSError:
        pass
    return threads, (len(phys) or None), avail


def cpu_baseline(batch: int):
    """the CPU oracle (fp32 torch-CPU restatement of the reference arithmetic, our
    'port') on a bounded fused batch: 2 warm-up runs, then the median of 5 timed runs, at
    torch.set_num_threads(threads usable by this process)."""
    sys.path.insert(0, ROOT)
    from mec import synthetic as syn
    from oracle import fusion as o_f, image as o_i, speech as o_s, text as o_t
    threads, phys, avail = host_cpus()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    w = {k: syn.weights(k) for k in ('speech', 'text', 'image', 'fusion')}
    x = syn.speech_inputs(batch, seed=0)
    ids, mask = syn.text_inputs(batch, 128, seed=0)
    gray = syn.image_inputs(batch, seed=0)

    def one():
        sf, _, sp = o_s.forward(w['speech'], x)
        tf, _, tp = o_t.forward(w['text'], ids, mask)
        imf, _, ip = o_i.forward(w['image'], gray)
        o_f.forward(w['fusion'], sf, tf, imf, sp, tp, ip)

    for _ in range(2):
        one()
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        one()
        ts.append(time.perf_counter() - t0)
    torch.set_num_threads(prev)
    med = statistics.median(ts)
    return {'value': batch / med, 'unit': 'fused samples/s', 'cores': threads, 'kind': 'port',
            'sample': f'fused batch of {batch} (L=128 full rows, 48x48 u8) through oracle/ fp32 torch-CPU, '
                      f'median of 5 runs after 2 warm-ups ({med:.2f} s/run)',
            'host_physical_cores': phys, 'host_logical_cpus_in_affinity': avail}


def parity(out, x, ids, mask, gray, rows):
    """Oracle on `rows` of the timed batch: per modality logits / probs max-abs-err and argmax
    agreement; fused end to end (the oracle fusion on the ORACLE encoders' outputs,
    inference/multimodal_fusion.py:271-278)."""
    sys.path.insert(0, ROOT)
    from mec import synthetic as syn
    from oracle import fusion as o_f, image as o_i, speech as o_s, text as o_t
    torch.cuda.synchronize()
    g = {k: [t[rows].cpu().numpy() for t in v] for k, v in out.items()}
    rs = o_s.forward(syn.weights('speech'), x[rows])
    rt = o_t.forward(syn.weights('text'), ids[rows], mask[rows])
    ri = o_i.forward(syn.weights('image'), gray[rows])
    rf = o_f.forward(syn.weights('fusion'), rs[0], rt[0], ri[0], rs[2], rt[2], ri[2])
    res = {}
    for name, (gl, gp), (rl, rp) in (('speech', g['speech'][1:3], rs[1:3]), ('text', g['text'][1:3], rt[1:3]),
                                      ('image', g['image'][1:3], ri[1:3]), ('fusion', g['fusion'][0:2], rf[0:2])):
        res[name] = {'logits_max_abs_err': float(np.abs(gl - rl).max()),
                     'probs_max_abs_err': float(np.abs(gp - rp).max()),
                     'argmax_agree': f'{int((gp.argmax(1) == rp.argmax(1)).sum())}/{len(rows)}'}
    res['rows'] = f'{len(rows)} fixed rows of the timed batch; fusion = end-to-end oracle chain'
    return res


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
    sys.path.insert(0, ROOT)
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
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(20):
            pipe.speech.forward(xs)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / (iters * 20)
    out['speech_b32_graph'] = {'samples_per_s': 32 / ms * 1e3, 'ms_per_batch': ms}
    del g
    mb.close()
    af.close()
    return out


def run(a, precision, B, world, rank, dev):
    """Time K pipelined steps at one precision; returns the result line (rank 0) or None."""
    from mec import _lib, dist as mdist, engine, synthetic as syn
    # the product library: no probe build (probe option values skip work and return wrong
    # results), and every knob of the pipeline's handles at its default (handles own their knobs)
    # apart from the pipeline's own pin (BERT FFN2 on the ping-pong tile in the concurrent step)
    if _lib.load().mec_build_flags() != 0:
        raise SystemExit(f'bench.py: {_lib.LIB_PATH} is a probe build (MEC_PROBES); use the product library')
    pipe = engine.FusedPipeline(seed=1234, device=dev, concurrent=not a.serial, pipelined=not a.no_pipeline,
                                text_priority=bool(a.text_priority), image_priority=bool(a.image_priority),
                                precision=precision)
    x_np = syn.speech_inputs(B, seed=rank)
    ids_np, mask_np = syn.text_inputs(B, 128, seed=rank, ragged=False)
    gray_np = syn.image_inputs(B, seed=rank)
    x, ids, mask, gray = (engine.to_device(v, dev) for v in (x_np, ids_np, mask_np, gray_np))
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
        return rows

    def step():
        return pipe.forward(x, ids, mask, gray, epilogue=finish)[1]

    for _ in range(a.warmup):
        step()
    gather_ev.clear()
    # hipEvent timing of the dominant kernel (BERT FFN1 GEMM) inside the timed region
    pipe.text.prof_enable('bert_ffn1')
    torch.cuda._sleep(1)  # marker dispatch for tools/prof_summary.py --window spin (outside the timing)
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
    if rank != 0:
        for m in pipe.models():
            m.close()
        return None

    M = B * 128
    peak = PEAK_TFLOPS[precision]
    ffn_flop = 2.0 * M * 3072 * 768
    avg_s = (ffn_ms / max(ffn_n, 1)) / 1e3
    achieved = ffn_flop / avg_s / 1e12 if ffn_n else None
    iso = ffn_flop / ((iso_ms / max(iso_n, 1)) / 1e3) / 1e12 if iso_n else None
    tile = pipe.text.gemm_tile(M, 3072, 768)  # the text handle's own autotune choice
    if precision == 'f16':
        kname = tile_name(tile, M) + ' + GELU'
        ebytes, tfile = 2, 'ffn1_traffic.json'
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
            'algorithmic_flop_per_launch': ffn_flop,
            'algorithmic_bytes_per_launch': ebytes * (M * 768 + 3072 * 768 + M * 3072),
            'avg_launch_ms': avg_s * 1e3, 'launches': ffn_n,
            'note': 'achieved: live in the timed region (CUs shared with the image stream); '
                    'achieved_isolated: BERT alone',
            'achieved_isolated': iso, 'frac_isolated': (iso / peak) if iso else None}
    total = world * B * a.steps
    flop = sum(FLOP_PER_SAMPLE.values()) * total
    res = {
        'metric': 'fused tri-modal samples/sec @ batch 256; per-modality logits max-abs-err',
        'value': total / el, 'unit': 'samples/s', 'n_gpus': world, 'steps': a.steps, 'warmup': a.warmup,
        'ms_per_step': el / a.steps * 1e3, 'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
        'dtype': DTYPE[precision], 'precision': precision,
        'data': 'synthetic (seeded inputs: 56-d features, 128-token ids, 48x48 u8; seeded synthetic weights)',
        'config': {'workload': 'fused tri-modal: speech DNN + BERT-base L=128 + ResNet50@224 + attention fusion',
                   'batch_per_gpu': B, 'global_batch': world * B, 'seq_len': 128,
                   'parallelism': f'dp{world} (sample-sharded, all-gather of 34-float rows)'},
        'achieved_tflops_whole_step': flop / el / 1e12,
        'whole_step_frac_of_peak': flop / el / 1e12 / peak,
        'roofline': roof,
    }
    if world > 1:
        res['distributed'] = {'world_size': dist.get_world_size(), 'backend': dist.get_backend(),
                              'rccl_version': '.'.join(map(str, torch.cuda.nccl.version())),
                              'all_gather_ms_per_step': (sum(gather_ms) / len(gather_ms)) if gather_ms else None,
                              'all_gather_bytes_per_step': world * B * 34 * 4}
    if not a.no_parity and 'out' in last:
        rows = [r for r in PARITY_ROWS if r < B]
        res['parity'] = parity(last['out'], x_np, ids_np, mask_np, gray_np, rows)
    if world == 1 and not a.no_configs:
        res['per_config'] = per_config(pipe, dev, precision)
    for m in pipe.models():
        m.close()
    return res


def main():
    a = parse()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    dev = torch.device('cuda', local)
    torch.cuda.set_device(dev)
    B = a.batch or (256 if world == 1 else 1024)
    precs = ['f16', 'fp32'] if a.precision == 'both' else [a.precision]
    lines = [run(a, p, B, world, rank, dev) for p in precs]
    if rank == 0:
        if world == 1 and not a.no_cpu_baseline:
            cb = cpu_baseline(a.cpu_batch)
            for r in lines:
                r['cpu_baseline'] = cb
        for r in lines:  # f16 (the fast path) first, then its fp32 same-precision counterpart
            print(json.dumps(r), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
