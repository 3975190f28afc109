"""Multi-rank runs of the HIP path (world size 2 on one GPU): `bench.py --gpus 2` starts its own
ranks (no torchrun from the caller), every rank runs the checksum kernel on its shard and checks a
block of it against the oracle, and rank 0 reports the whole job.  Weak scaling (a batch per rank,
disjoint sub-streams) and strong scaling (one global batch, byte-balanced shards)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--ramp-ms", "0", "--no-cpu-baseline", "--share-gpu"] + list(args)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=REPO)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout   # rank 0 alone prints
    j = json.loads(lines[0])
    c = j["config"]
    # two ranks on this box's one card: the line says so, and names each rank's kernel time
    ndev = torch.cuda.device_count()
    assert c["devices_distinct"] == min(2, ndev)
    assert c["shared_gpu_rehearsal"] is (ndev < 2)
    assert [r["rank"] for r in c["ranks"]] == [0, 1]
    assert c["kernel_ms_over_ranks"]["min"] <= c["kernel_ms_over_ranks"]["max"]
    return j


@pytest.mark.parametrize("workload", ["c2", "c3", "c1"])
def test_bench_two_ranks_weak(workload):
    """c1: its 64-MB batch is below the bench's 1-GiB rotation floor, so the launches rotate over
    16 batches per rank; the gates still check batch 0."""
    j = _bench("--workload", workload)
    assert j["n_gpus"] == 2 and j["scaling"] == "weak"
    c = j["config"]
    assert c["batches_rotated"] == (16 if workload == "c1" else 1)
    assert c["verify_all_packets"] is True
    assert c["oracle_gate"]["sample_equal"] is True
    assert c["global_batch"] == 2 * c["packets_rank0"]
    assert c["algorithmic_bytes_per_step_all_ranks"] > 1.9 * c["algorithmic_bytes_per_step_rank0"]
    assert j["value"] > 0


@pytest.mark.parametrize("workload", ["c3", "c4"])
def test_bench_two_ranks_strong(workload):
    """One global batch split by bytes: each rank's slice starts where the previous one ends,
    and the two slices together are the whole batch."""
    j = _bench("--workload", workload, "--strong")
    assert j["n_gpus"] == 2 and j["scaling"] == "strong"
    c = j["config"]
    assert c["verify_all_packets"] is True and c["oracle_gate"]["sample_equal"] is True
    assert c["packets_rank0"] < c["global_batch"]
    assert abs(c["algorithmic_bytes_per_step_all_ranks"] - 2 * c["algorithmic_bytes_per_step_rank0"]) \
        < 0.01 * c["algorithmic_bytes_per_step_all_ranks"]


def test_bench_two_ranks_strong_shards_per_rank_with_cpu_baseline():
    """Strong C4 over two ranks: each rank generates and holds only its own byte-balanced slice of
    the global batch (rank 1 starts where rank 0 ends; a rank's peak allocation is about half the
    global arena, not all of it), and the N > 1 line carries the CPU baseline (VERIFY r3 item 2)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--ramp-ms", "0", "--share-gpu", "--workload", "c4", "--strong", "--cpu-budget", "0.3"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=REPO)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    j = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    c = j["config"]
    r0, r1 = c["ranks"]
    assert r0["first_packet"] == 0 and r1["first_packet"] == r0["packets"]
    assert r0["packets"] + r1["packets"] == c["global_batch"] == 1 << 18
    global_arena = (1 << 18) * 9216
    for rr in (r0, r1):
        assert rr["peak_alloc_bytes"] < 0.6 * global_arena, rr
    assert j["cpu_baseline"] and j["cpu_baseline"]["value"] > 0 and j["cpu_baseline"]["cores"] >= 1
    assert c["oracle_gate"]["oracle_equal"] is True and c["oracle_gate"]["sample_equal"] is True
    # the two-stream pass ran on every rank (its second batch not counted in the peak above)
    assert j["pipelined_two_streams"]["value"] > 0 and j["pipelined_two_streams"]["ms_per_step"] > 0


def test_descriptor_only_synth_equals_full_synth():
    """vpcsum_synth_async with a NULL arena writes the same descriptors as the full generator (the
    lengths a strong rank cuts the global batch with)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from vproxy_amd import vpcsum as V
    for wl, stride in ((V.SYNTH_C3, 2048), (V.SYNTH_FUZZ, 9216), (V.SYNTH_C4, 9216)):
        n = 5000
        arena = torch.zeros(n * stride, dtype=torch.uint8, device="cuda")
        d1 = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
        d2 = torch.full((n * 16,), 0x5a, dtype=torch.uint8, device="cuda")
        V.synth(arena, n, stride, 14, wl, 99, 12345, d1)
        V.synth(None, n, stride, 14, wl, 99, 12345, d2)
        torch.cuda.synchronize()
        assert torch.equal(d1, d2), wl


def test_bench_refuses_more_ranks_than_gpus():
    """Without --share-gpu, more ranks than visible cards is an error (no "N-GPU" line from ranks
    sharing one card)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    n = torch.cuda.device_count() + 1
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n), "--steps", "1"],
                       capture_output=True, text=True, timeout=120, cwd=REPO)
    assert r.returncode != 0 and "share-gpu" in r.stderr


@pytest.mark.parametrize("ndev", [1, 3])
@pytest.mark.parametrize("registered", [False, True])
def test_device_group_splits_by_bytes(orc, ndev, registered):
    """vpcsum_group_*: one host batch cut into per-device ranges of nearly equal bytes (three
    contexts on this box's one GPU stand for three GPUs); results in batch order equal the oracle's,
    in-place writes land in the caller's frames, two batches can be in flight."""
    import numpy as np
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import oracle as O
    from vproxy_amd import vpcsum as V
    a, d = orc.synth(3000, 9088, 14, O.SYNTH_FUZZ, O.SEED, 77 + ndev)
    arena = np.concatenate([a, np.zeros(4096, np.uint8)])
    want, want_st = orc.process(arena, d, O.MODE_VERIFY)
    g = V.Group([0] * ndev, max_arena=arena.nbytes, max_pkts=len(d))
    if registered:
        g.register(arena)
    out, st = g.run(arena, d, O.MODE_VERIFY)
    assert np.array_equal(out, want) and np.array_equal(st, want_st)
    want_arena = arena.copy()
    wout, _ = orc.process(want_arena, d, O.MODE_COMPUTE, write=True)
    o1, o2 = np.zeros(1000, np.uint32), np.zeros(2000, np.uint32)
    t1 = g.submit(arena, d[:1000], o1, None, O.MODE_WRITE)
    t2 = g.submit(arena, d[1000:], o2, None, O.MODE_WRITE)
    g.wait(t2)
    g.wait(t1)
    assert np.array_equal(np.concatenate([o1, o2]), wout) and np.array_equal(arena, want_arena)
    g.close()


def test_device_group_failed_submit_joins_submitted_ranges(orc):
    """A range that a context refuses (here the second one holds more packets than a context's
    capacity) fails the group submit only after the ranges already submitted have finished: their
    results are in the caller's buffers when the error is returned, and the group keeps working."""
    import numpy as np
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import oracle as O
    from vproxy_amd import vpcsum as V
    a4, d4 = orc.synth(100, 9216, 14, O.SYNTH_C4, O.SEED, 0)       # 100 jumbo packets first
    a1, d1 = orc.synth(3000, 128, 14, O.SYNTH_C1, O.SEED, 100)     # then 3000 small ones
    d1 = d1.copy()
    d1["l3_off"] += len(a4)
    arena = np.concatenate([a4, a1])
    d = np.concatenate([d4, d1])
    want, _ = orc.process(arena, d, O.MODE_COMPUTE)
    # the library's byte-balanced cut of two ranges (vpcsum_group_submit)
    acc = np.cumsum(d["l3_len"].astype(np.int64))
    cut = int(np.argmax(acc * 2 >= acc[-1])) + 1
    assert cut < 1000 < len(d) - cut   # range 0 fits a context, range 1 does not
    g = V.Group([0, 0], max_arena=arena.nbytes, max_pkts=1000)
    out = np.zeros(len(d), np.uint32)
    with pytest.raises(V.VpcsumError, match="capacity"):
        g.submit(arena, d, out, None, O.MODE_COMPUTE)
    assert np.array_equal(out[:cut], want[:cut])   # range 0 finished before the error
    assert not out[cut:].any()
    small = d[:cut]
    o2, _ = g.run(arena, small, O.MODE_COMPUTE)
    assert np.array_equal(o2, want[:cut])
    g.close()


def test_survey_entry_points_over_the_default_group(orc):
    """vpcsum_init(dev_mask) / vpcsum_register_arena / vpcsum_batch_submit / vpcsum_batch_wait /
    vpcsum_nat_submit / vpcsum_shutdown: a checksum batch and a NAT batch over
    the process-wide group, results equal to the oracle's; a second init is refused."""
    import ctypes
    import numpy as np
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import oracle as O
    from vproxy_amd import vpcsum as V
    L = V.lib()
    mask = (1 << torch.cuda.device_count()) - 1
    arena, d = orc.synth(3000, 2048, 14, O.SYNTH_C3, O.SEED, 4321)
    arena = np.concatenate([arena, np.zeros(4096, np.uint8)])
    want_out, want_st = orc.process(arena, d, O.MODE_VERIFY)
    assert L.vpcsum_init(mask, arena.nbytes, len(d)) == 0
    try:
        assert L.vpcsum_init(mask, arena.nbytes, len(d)) != 0
        assert L.vpcsum_register_arena(arena.ctypes.data, arena.nbytes) == 0
        out, st = np.zeros(len(d), np.uint32), np.zeros(len(d), np.uint8)
        h = ctypes.c_uint64()
        assert L.vpcsum_batch_submit(arena.ctypes.data, arena.nbytes, d.ctypes.data, len(d), out.ctypes.data,
                                     st.ctypes.data, O.MODE_VERIFY, ctypes.byref(h)) == 0
        assert L.vpcsum_batch_wait(h.value) == 0
        assert np.array_equal(out, want_out) and np.array_equal(st, want_st)
        # NAT over the group: valid sums first, then rewrites, equal to Java's setters + recompute
        orc.process(arena, d, O.MODE_COMPUTE, write=True)
        rng = np.random.default_rng(9)
        rw = np.zeros(len(d), O.NAT_DTYPE)
        rw["src"][:, :4] = rng.integers(0, 256, (len(d), 4))
        rw["dport"] = rng.integers(0, 256, (len(d), 2))
        rw["mask"] = O.NAT_SRC | O.NAT_DPORT
        want = arena.copy()
        want_nst = orc.nat_java(want, d, rw)
        nst = np.zeros(len(d), np.uint8)
        assert L.vpcsum_nat_submit(arena.ctypes.data, arena.nbytes, d.ctypes.data, rw.ctypes.data, len(d),
                                   nst.ctypes.data, V.NAT_STRICT_JAVA, ctypes.byref(h)) == 0
        assert L.vpcsum_batch_wait(h.value) == 0
        assert np.array_equal(arena, want) and np.array_equal(nst, want_nst)
    finally:
        assert L.vpcsum_shutdown() == 0
