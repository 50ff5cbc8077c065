"""GPU: the RCCL branch of mec.dist.all_gather_rows (BASELINE configs[4]'s one collective,
SURVEY.md §8e) on real hardware. A world-size-1 process group on the "nccl" backend (RCCL on
ROCm) runs bench.py's epilogue -- pack the 34-float result rows, all-gather them on the fusion
stream of the pipelined FusedPipeline (bench.py run(): finish) -- and the gathered rows must equal
the packed rows bit for bit. The group lives in this pytest process (initialised over TCP on
127.0.0.1 and destroyed at the end): a child process would have to be exec'd from a process that
has already initialised the GPU. Multi-rank ordering is covered by the gloo tests
(tests/test_distributed.py, tests/test_bench_launcher.py); 8-GPU runs are the driver's."""
import socket

import pytest
import torch
import torch.distributed as dist

from mec import dist as mdist, engine, synthetic as syn

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def nccl_world1(dev):
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    torch.cuda.set_device(dev)
    dist.init_process_group('nccl', init_method=f'tcp://127.0.0.1:{port}', rank=0, world_size=1, device_id=dev)
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize('precision', ['fp32x3', 'f16'])
def test_rccl_world1_all_gather_on_fusion_stream(dev, nccl_world1, precision):
    assert dist.get_backend() == 'nccl' and dist.get_world_size() == 1
    B = 128
    pipe = engine.FusedPipeline(device=dev, precision=precision)
    x = engine.to_device(syn.speech_inputs(B, seed=0), dev)
    ids, mask = (engine.to_device(a, dev) for a in syn.text_inputs(B, 128, seed=0, ragged=False))
    gray = engine.to_device(syn.image_inputs(B, seed=0), dev)
    got = []

    def finish(out):  # on the fusion stream, as bench.py's epilogue
        rows = pipe.pack_rows(out)
        gathered = mdist.all_gather_rows(rows, B)
        got.append((rows, gathered, torch.cuda.current_stream(dev).cuda_stream))
        return gathered

    for _ in range(3):  # 1st: serial (autotune); then concurrent + pipelined (batch i's gather under batch i+1)
        pipe.forward(x, ids, mask, gray, epilogue=finish)
    pipe.wait()
    torch.cuda.synchronize()
    pipe.check()
    print(f'{precision}: backend {dist.get_backend()}, RCCL {".".join(map(str, torch.cuda.nccl.version()))}, '
          f'{len(got)} gathers of {tuple(got[-1][1].shape)}')
    for rows, gathered, _ in got:
        assert tuple(gathered.shape) == (B, 34)
        assert torch.equal(rows, gathered)
        assert torch.isfinite(gathered).all()
    # the pipelined batches' gathers ran on the fusion (tail) stream, not the caller's
    assert all(sid == pipe._tail.cuda_stream for _, _, sid in got[1:])
    for m in pipe.models():
        m.close()
