"""CPU: bench.py's multi-GPU launcher and sharding, without a GPU.

`python bench.py --gpus N` with no WORLD_SIZE starts N ranks through torch.distributed.run as a
child process (before any GPU call); with no GPU visible each rank runs the stub step over gloo:
the same sharding (mec.dist.shard), all-gather (mec.dist.all_gather_rows) and max-over-ranks
timing as the GPU run, on deterministic stand-in rows. The JSON line must report N ranks as
torch.distributed saw them and the gathered rows in global sample order."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run_bench(*args, timeout=240):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES='', HIP_VISIBLE_DEVICES='', OMP_NUM_THREADS='1')
    env.pop('WORLD_SIZE', None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), *args], capture_output=True, text=True,
                       timeout=timeout, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, p.stdout[-2000:]  # rank 0 prints ONE line
    return json.loads(lines[0])


@pytest.mark.parametrize('n', [2, 3])
def test_bench_gpus_n_launches_n_ranks(n):
    r = _run_bench('--gpus', str(n), '--steps', '2', '--warmup', '1', '--batch', '5')
    assert r['n_gpus'] == n and r['stub'] is True and r['value'] is None
    d = r['distributed']
    assert d['world_size'] == n and d['backend'] == 'gloo'
    assert d['gathered_rows_in_order'] is True
    assert r['config']['global_batch'] == 5 * n and r['scaling'] == 'weak'


def test_bench_single_rank_stub():
    r = _run_bench('--steps', '1', '--warmup', '0')
    assert r['n_gpus'] == 1 and r['distributed']['gathered_rows_in_order'] is True


def test_stub_rows_and_shards_tile_the_global_batch():
    sys.path.insert(0, ROOT)
    import bench
    from mec import dist as mdist
    world, B = 4, 7
    parts = [bench.stub_rows(*mdist.shard(world * B, world, r)) for r in range(world)]
    full = bench.stub_rows(0, world * B)
    assert np.array_equal(np.concatenate([p.numpy() for p in parts]), full.numpy())


@pytest.mark.parametrize('B', [256, 1024, 300])
def test_parity_rows_cover_every_quarter(B):
    sys.path.insert(0, ROOT)
    import bench
    rows = bench.parity_rows(B, 256)
    if B <= 256:
        assert rows == list(range(B))
        return
    assert rows == sorted(set(rows)) and rows[0] == 0 and rows[-1] == B - 1
    for q in range(4):
        lo, hi = q * B // 4, (q + 1) * B // 4
        assert sum(lo <= r < hi for r in rows) >= 4, (q, rows)
    assert any(r >= 256 for r in rows)
