"""Benchmark: fused tri-modal samples/s @ batch 256 per GPU (BASELINE.json metric).

One step = one pass of the whole hot path over one synthetic batch already resident in
HBM: speech DNN + BERT-base (L=128) + ResNet50 (48x48 u8 -> 224) encoders, then the
attention-MLP fusion, then (N>1) the RCCL all-gather of the 34-float result rows.
Weak scaling: every rank processes its own batch of 256. Consecutive batches are
pipelined (engine.FusedPipeline): batch i's fusion and gather overlap batch i+1's
encoders; the timed region ends after the last batch's gather (device synchronize).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--no-cpu-baseline]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
import argparse
import json
import os
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
MI355X_F16_DENSE_TFLOPS = 2500.0  # MI355X_MICROARCH.md: ~2.5 PF dense bf16/f16 MFMA


def tile_name(tile: int, M: int) -> str:
    """Kernel + grid for a GEMM tile id (gemm_glds.hip, launch_bn)."""
    if tile in (40256, 41256):
        bm = 256 if tile == 40256 else 128
        return f'gemm_pp_kernel<{bm}x256x64 ping-pong, mfma16x16x32> grid={((M + bm - 1) // bm) * (3072 // 256)}'
    v, w = divmod(tile, 10000)
    bm, bn = (128, w - 1000) if w > 1000 else (256, w)
    mf = 32 if v == 0 else 16
    bk = 32 if v >= 2 else 64
    return f'gemm_glds_kernel<{bm}x{bn}x{bk}, mfma{mf}> grid={((M + bm - 1) // bm) * (3072 // bn)}'


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--batch', type=int, default=256)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--cpu-seconds', type=float, default=12.0)
    ap.add_argument('--serial', action='store_true', help='run the encoders on one stream (A/B of the concurrency)')
    ap.add_argument('--no-pipeline', action='store_true',
                    help="run each batch's fusion on the main stream (A/B of the cross-batch overlap)")
    ap.add_argument('--no-configs', action='store_true', help='skip the per-config (single-encoder) timings')
    ap.add_argument('--text-priority', type=int, default=1, help='0: BERT on the default-priority stream (A/B)')
    ap.add_argument('--image-priority', type=int, default=0,
                    help='1: speech + image stream at high priority, BERT at normal (A/B)')
    return ap.parse_args()


def cpu_baseline(seconds: float):
    """Time the CPU oracle (fp32 restatement: our 'port' of the reference arithmetic) on a
    bounded sample of the same workload: fused samples in batches of 2 until `seconds`."""
    sys.path.insert(0, ROOT)
    from mec import synthetic as syn
    from oracle import fusion as o_f, image as o_i, speech as o_s, text as o_t
    w = {k: syn.weights(k) for k in ('speech', 'text', 'image', 'fusion')}
    Bc = 2
    x = syn.speech_inputs(Bc, seed=0)
    ids, mask = syn.text_inputs(Bc, 128, seed=0)
    gray = syn.image_inputs(Bc, seed=0)

    def one():
        sf, _, sp = o_s.forward(w['speech'], x)
        tf, _, tp = o_t.forward(w['text'], ids, mask)
        imf, _, ip = o_i.forward(w['image'], gray)
        o_f.forward(w['fusion'], sf, tf, imf, sp, tp, ip)

    one()  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        one()
        n += Bc
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    return {'value': n / el, 'unit': 'fused samples/s', 'cores': torch.get_num_threads(), 'kind': 'port',
            'sample': f'{n} fused samples (batches of {Bc}, L=128, 48x48 u8) through oracle/ fp32 torch-CPU, '
                      f'{el:.1f}s'}


def per_config(pipe, dev, iters=10):
    """Single-encoder throughput on the other BASELINE configs (rank 0, N=1; informational,
    not `value`): speech B=32, image B=256 (ResNet50 and the MobileNetV2 backbone), text B=128
    (L=128). hipEvents around `iters` back-to-back calls on the current stream, inputs in HBM."""
    from mec import engine, synthetic as syn
    mb = engine.MobileNetImageEncoder(device=dev)
    xs = engine.to_device(syn.speech_inputs(32, seed=7), dev)
    ids, mask = syn.text_inputs(128, 128, seed=7)
    ids, mask = engine.to_device(ids, dev), engine.to_device(mask, dev)
    g = engine.to_device(syn.image_inputs(256, seed=7), dev)
    runs = {'speech_b32': (32, lambda: pipe.speech.forward(xs)),
            'image_resnet50_b256': (256, lambda: pipe.image.forward(g)),
            'image_mobilenet_v2_b256': (256, lambda: mb.forward(g)),
            'text_bert_b128': (128, lambda: pipe.text.forward(ids, mask))}
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
    mb.close()
    return out


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

    from mec import engine, synthetic as syn
    B = a.batch
    pipe = engine.FusedPipeline(seed=1234, device=dev, concurrent=not a.serial, pipelined=not a.no_pipeline,
                                text_priority=bool(a.text_priority), image_priority=bool(a.image_priority))
    x = engine.to_device(syn.speech_inputs(B, seed=rank), dev)
    ids_np, mask_np = syn.text_inputs(B, 128, seed=rank, ragged=False)
    ids, mask = engine.to_device(ids_np, dev), engine.to_device(mask_np, dev)
    gray = engine.to_device(syn.image_inputs(B, seed=rank), dev)
    from mec import dist as mdist

    def finish(out):  # runs on the fusion's stream (FusedPipeline: batch i's fusion overlaps batch i+1)
        rows = pipe.pack_rows(out)
        if world > 1:  # one RCCL all-gather of the 34-float result rows
            rows = mdist.all_gather_rows(rows, world * B)
        return rows

    def step():
        return pipe.forward(x, ids, mask, gray, epilogue=finish)[1]

    for _ in range(a.warmup):
        step()
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

    if rank == 0:
        M = B * 128
        ffn_flop = 2.0 * M * 3072 * 768
        avg_s = (ffn_ms / max(ffn_n, 1)) / 1e3
        achieved = ffn_flop / avg_s / 1e12 if ffn_n else None
        tile = pipe.text.lib.mec_gemm_query(0, M, 3072, 768)
        kname = tile_name(tile, M) + f' (BERT FFN1 + GELU epilogue, M={M} N=3072 K=768)'
        iso = ffn_flop / ((iso_ms / max(iso_n, 1)) / 1e3) / 1e12 if iso_n else None
        traffic, tsrc = None, None
        tf = os.path.join(ROOT, 'profiles', 'ffn1_traffic.json')
        if os.path.exists(tf):  # PMC passes (tools/pmc.sh), FETCH_SIZE x2 per MI355X_MICROARCH gfx950 note
            with open(tf) as fh:
                t = json.load(fh)
            if t.get('tile') == tile and t.get('M') == M:
                traffic, tsrc = t['bytes_per_launch'], t['source']
        roof = {'bound': 'mfma', 'kernel': kname,
                'achieved': achieved, 'peak': MI355X_F16_DENSE_TFLOPS, 'unit': 'TFLOP/s',
                'frac': (achieved / MI355X_F16_DENSE_TFLOPS) if achieved else None, 'traffic': traffic,
                'traffic_source': tsrc, 'algorithmic_flop_per_launch': ffn_flop,
                'algorithmic_bytes_per_launch': 2 * (M * 768 + 3072 * 768 + M * 3072),
                'avg_launch_ms': avg_s * 1e3, 'launches': ffn_n,
                'note': 'achieved = live, inside the timed region, sharing CUs with the concurrent image '
                        'stream; achieved_isolated = same kernel with BERT alone',
                'achieved_isolated': iso,
                'frac_isolated': (iso / MI355X_F16_DENSE_TFLOPS) if iso else None}
        total = world * B * a.steps
        flop = sum(FLOP_PER_SAMPLE.values()) * total
        res = {
            'metric': 'fused tri-modal samples/sec @ batch 256',
            'value': total / el, 'unit': 'samples/s', 'n_gpus': world, 'steps': a.steps, 'warmup': a.warmup,
            'ms_per_step': el / a.steps * 1e3, 'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None,
            'dtype': 'f16 MFMA operands / fp32 accumulate, LN & softmax & residual fp32; speech+fusion fp32',
            'data': 'synthetic (seeded inputs: 56-d features, 128-token ids, 48x48 u8; seeded synthetic weights)',
            'config': {'workload': 'fused tri-modal: speech DNN + BERT-base L=128 + ResNet50@224 + attention fusion',
                       'batch_per_gpu': B, 'global_batch': world * B, 'seq_len': 128,
                       'parallelism': f'dp{world} (sample-sharded, all-gather of 34-float rows)'},
            'achieved_tflops_whole_step': flop / el / 1e12,
            'roofline': roof,
        }
        if world == 1 and not a.no_configs:
            res['per_config'] = per_config(pipe, dev)
        if world == 1 and not a.no_cpu_baseline:
            res['cpu_baseline'] = cpu_baseline(a.cpu_seconds)
        print(json.dumps(res))
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
