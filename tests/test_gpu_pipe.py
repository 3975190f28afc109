"""Two batches in flight through the device API (vpcsum_pipe_*).

The pipe forks two streams of its own from the caller's stream (`begin`), alternates launches
between them, and joins them back (`join`).  Checked here: the fork orders the pipe's launches after
work queued on the caller's stream before `begin` (the batches are generated there, right before);
the join orders work queued on the caller's stream after `join` behind every launch (the results
are copied on the caller's stream, no device-wide synchronise in between); every batch's sums equal
the oracle's, for batches of different shapes in one series.
"""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def V():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vproxy_amd import vpcsum
    vpcsum.lib()
    return vpcsum


@pytest.mark.parametrize("series", [2, 7])
def test_pipe_fork_join_and_results(V, orc, series):
    import torch
    stream = torch.cuda.Stream()
    works = [O.SYNTH_C1, O.SYNTH_C3, O.SYNTH_C2, O.SYNTH_C5]
    n, stride = 20000, 2048
    pipe = V.Pipe(stream)
    arenas = [torch.zeros(n * stride, dtype=torch.uint8, device="cuda") for _ in range(series)]
    descs = [torch.zeros(n * 16, dtype=torch.uint8, device="cuda") for _ in range(series)]
    outs = [torch.zeros(n, dtype=torch.int32, device="cuda") for _ in range(series)]
    sts = [torch.zeros(n, dtype=torch.uint8, device="cuda") for _ in range(series)]
    torch.cuda.synchronize()
    with torch.cuda.stream(stream):
        for rep in range(3):
            for b in range(series):   # the batches are made on the caller's stream, right before begin
                V.synth(arenas[b], n, stride, 14, works[b % len(works)], O.SEED, 1000 * rep + b, descs[b], stream=stream)
                outs[b].fill_(-1)
            pipe.begin()
            for b in range(series):
                pipe.compute(arenas[b], descs[b], n, outs[b], sts[b], V.MODE_VERIFY if b % 3 == 2 else V.MODE_COMPUTE)
            pipe.join()
            got = [o.to("cpu", non_blocking=False) for o in outs]   # queued on the caller's stream
            stream.synchronize()
            for b in range(series):
                a = arenas[b].cpu().numpy()
                d = descs[b].cpu().numpy().view(O.DESC_DTYPE)
                want, _ = orc.process(a, d, O.MODE_VERIFY if b % 3 == 2 else O.MODE_COMPUTE)
                assert np.array_equal(got[b].numpy().view(np.uint32), want), (rep, b)
    pipe.close()


def test_pipe_rejects_null(V):
    import ctypes
    L = V.lib()
    assert L.vpcsum_pipe_begin(None) != 0
    assert L.vpcsum_pipe_join(None) != 0
    assert L.vpcsum_pipe_compute_async(None, None, 0, None, 0, None, None, 0) != 0
    assert L.vpcsum_pipe_destroy(None) == 0
    assert ctypes is not None
