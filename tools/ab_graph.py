"""A/B: the fused step launched eagerly (FusedPipeline, stream priorities, cross-batch
fusion overlap) vs the same step captured once into a HIP graph (torch.cuda.CUDAGraph
over the library's launches on all three streams) and replayed. Prints ms/step of each,
interleaved rounds in one process, and checks the graph's outputs equal the eager ones."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'multimodal-emotion-classification_amd'))


def main():
    from mec import engine, synthetic as syn
    dev = torch.device('cuda', 0)
    B = int(os.environ.get('B', '256'))
    steps = int(os.environ.get('STEPS', '20'))
    pipe = engine.FusedPipeline(seed=1234, device=dev)
    x = engine.to_device(syn.speech_inputs(B, seed=0), dev)
    ids_np, mask_np = syn.text_inputs(B, 128, seed=0, ragged=False)
    ids, mask = engine.to_device(ids_np, dev), engine.to_device(mask_np, dev)
    gray = engine.to_device(syn.image_inputs(B, seed=0), dev)

    def step():
        return pipe.forward(x, ids, mask, gray, epilogue=pipe.pack_rows)[1]

    for _ in range(3):
        ref = step()
    pipe.wait()
    torch.cuda.synchronize()
    ref = ref.clone()

    g = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream(device=dev)
    cs.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(cs):
        g.capture_begin()
        gout = pipe.forward(x, ids, mask, gray, epilogue=pipe.pack_rows)[1]
        pipe.wait()
        g.capture_end()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    same = torch.equal(gout, ref)
    print(f'graph output bit-identical to eager: {same}', flush=True)

    def t_eager():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        pipe.wait()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    def t_graph():
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            g.replay()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / steps * 1e3

    for r in range(4):
        e, gr = t_eager(), t_graph()
        print(f'round {r}: eager {e:.3f} ms/step ({B / e * 1e3:.0f}/s)  graph {gr:.3f} ms/step ({B / gr * 1e3:.0f}/s)',
              flush=True)
    if not same:
        sys.exit(1)


if __name__ == '__main__':
    main()
