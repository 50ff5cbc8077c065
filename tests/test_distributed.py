"""CPU, world_size 2 over gloo: the sample-sharded path end to end — each rank runs the
(oracle) per-sample arithmetic on its own contiguous shard, packs 34-float rows and the
all-gather reassembles the global batch in order. The GPU run uses the
same mec.dist code with backend nccl (RCCL)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rows_for(lo, hi, total):
    """Deterministic per-sample rows (stand-in for the pipeline's 34-float output)."""
    from mec import synthetic as syn
    from oracle import fusion as o_f
    g = {m: syn.uniform(5, f'dist/{m}', (total, d), 0.0, 1.0)
         for m, d in (('s', 64), ('t', 768), ('i', 512), ('sp', 7), ('tp', 7), ('ip', 7))}
    w = syn.weights('fusion')
    sl = slice(lo, hi)
    logits, probs, aw, dw = o_f.forward(w, g['s'][sl], g['t'][sl], g['i'][sl], g['sp'][sl], g['tp'][sl], g['ip'][sl])
    return np.concatenate([g['sp'][sl], g['tp'][sl], g['ip'][sl], probs, aw, dw], axis=1)


def _worker(rank, world, port, total, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, 'multimodal-emotion-classification_amd'))
    sys.path.insert(0, ROOT)
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from mec import dist as mdist
    lo, hi = mdist.shard(total, world, rank)
    rows = torch.from_numpy(_rows_for(lo, hi, total)).float()
    out = mdist.all_gather_rows(rows, total)
    if rank == 0:
        q.put(out.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('total', [8, 7])
def test_sharded_gather_world2(total):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, total, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = _rows_for(0, total, total)
    assert got.shape == (total, 34)
    np.testing.assert_allclose(got, ref, atol=1e-6)


def _bench_worker(rank, world, port, per_rank, q):
    """bench.py's finish(): FusedPipeline.pack_rows on the rank's outputs, then
    mec.dist.all_gather_rows over the global batch (gloo, CPU tensors)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, 'multimodal-emotion-classification_amd'))
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from mec import dist as mdist
    from mec.engine import FusedPipeline, ROW
    g = torch.Generator().manual_seed(100 + rank)
    t = lambda d: torch.rand(per_rank, d, generator=g)  # noqa: E731
    out = {'speech': (t(64), t(7), t(7)), 'text': (t(768), t(7), t(7)), 'image': (t(512), t(7), t(7)),
           'fusion': (t(7), t(7), t(3), t(3))}
    rows = FusedPipeline.pack_rows(out)
    assert rows.shape == (per_rank, ROW)
    got = mdist.all_gather_rows(rows, world * per_rank)
    q.put((rank, rows.numpy(), got.numpy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_bench_finish_pack_and_gather(world):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    per_rank = 5
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, per_rank, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r, rows, got = q.get(timeout=120)
        res[r] = (rows, got)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    full = np.concatenate([res[r][0] for r in range(world)])
    for r in range(world):
        assert np.array_equal(res[r][1], full)  # every rank holds the global batch, in rank order
    # the packed layout: 3x7 modality probs | 7 fused probs | 3 attention | 3 decision weights
    assert full.shape == (world * per_rank, 34)
