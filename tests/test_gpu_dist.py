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
           "--ramp-ms", "0", "--no-cpu-baseline"] + list(args)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=REPO)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout   # rank 0 alone prints
    return json.loads(lines[0])


@pytest.mark.parametrize("workload", ["c2", "c3"])
def test_bench_two_ranks_weak(workload):
    j = _bench("--workload", workload)
    assert j["n_gpus"] == 2 and j["scaling"] == "weak"
    c = j["config"]
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
