"""Multi-rank control plane on CPU (gloo, world size 2): packet sharding is disjoint and
complete, and bench.py's max-over-ranks timing / all-ranks verify gate reduce correctly.
The data path itself has no collective."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from vproxy_amd.shard import shard_by_bytes, shard_range


def test_shard_range_disjoint_complete():
    for n in (0, 1, 7, 1000, 1 << 20):
        for world in (1, 2, 3, 8):
            rs = [shard_range(n, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            for a, b in zip(rs, rs[1:]):
                assert a[1] == b[0]
            sizes = [b - a for a, b in rs]
            assert max(sizes) - min(sizes) <= 1


def test_shard_by_bytes_balanced():
    rng = np.random.default_rng(1)
    lens = rng.choice([64, 576, 1500, 9000], 10000)
    for world in (1, 2, 4, 8):
        rs = shard_by_bytes(lens, world)
        assert rs[0][0] == 0 and rs[-1][1] == len(lens)
        tot = [int(lens[a:b].sum()) for a, b in rs]
        assert max(tot) - min(tot) <= 2 * 9000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from vproxy_amd.shard import all_ranks_ok, gather_over_ranks, max_over_ranks, rank_seed_first_index, shard_range
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dist.barrier()
    m = max_over_ranks(float(rank) + 0.5)
    ok = all_ranks_ok(rank != 1)
    ok_all = all_ranks_ok(True)
    lo, hi = shard_range(1000, rank, world)
    g = gather_over_ranks({"rank": rank, "kernel_ms": 0.1 * (rank + 1)})
    q.put((rank, m, ok, ok_all, lo, hi, rank_seed_first_index(1 << 20, rank), g))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_reductions():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [1.5, 1.5]                 # max over ranks
    assert [r[2] for r in res] == [False, False]             # one rank failed -> all fail
    assert [r[3] for r in res] == [True, True]
    assert [(r[4], r[5]) for r in res] == [(0, 500), (500, 1000)]
    assert [r[6] for r in res] == [0, 1 << 20]               # disjoint synthetic sub-streams
    for r in res:                                            # every rank sees every rank, in order
        assert r[7] == [{"rank": 0, "kernel_ms": 0.1}, {"rank": 1, "kernel_ms": 0.2}]


def _bench_cpu(args, env_extra=None):
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(repo, "bench.py")] + args, capture_output=True,
                          text=True, timeout=120, cwd=repo, env=env)


def test_bench_refuses_ranks_beyond_visible_gpus():
    """bench.py never prints an N-GPU line from ranks sharing cards unless told to: here (no GPU)
    --gpus 2 fails before launching anything, and so does a launcher's WORLD_SIZE=2 without --gpus
    (the count is taken from the launcher)."""
    r = _bench_cpu(["--gpus", "2", "--steps", "1"])
    assert r.returncode != 0 and "share-gpu" in r.stderr
    r = _bench_cpu(["--steps", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "2 ranks but 0 visible" in r.stderr
    r = _bench_cpu(["--gpus", "3", "--steps", "1"], {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "matching counts" in r.stderr
