"""bench.py's strong-scaling share options on one GPU (--assign cost / --share R/N): the share a rank of an N-rank
run would replay, bin-packed on shard.doc_costs, runs, reports itself as that share, and its documents replay
without error. The N > 1 path itself (shard / gather over a process group) is tests/test_distributed.py."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("assign", ["uniform", "cost"])
def test_bench_share_of_a_strong_run(assign):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", "3", "--docs", "96", "--ops-per-doc", "512",
           "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--assign", assign, "--share", "1/4"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    c = out["config"]
    assert c["docs_per_node"] == 96
    assert c["docs_rank0"] == 24 if assign == "uniform" else 16 <= c["docs_rank0"] <= 32
    assert c["docs_in_error_rank0"] == 0
    assert "share 1/4" in c["parallelism"] and assign in c["parallelism"]
    assert out["value"] > 0


@pytest.mark.gpu
def test_bench_two_rank_rehearsal_on_one_gpu():
    """The multi-rank path of bench.py end to end on real hardware: torch.distributed.run with two ranks, both on
    device 0 with gloo collectives (--rehearse): the node's documents bin-packed over the ranks, the barriers, the
    max-reduced interval, the summed work and the digest all-gather. RCCL itself needs one GPU per rank (the driver's
    8-GPU runs); this rehearses everything around it."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rehearse",
           "--config", "3", "--docs", "96", "--ops-per-doc", "512", "--steps", "1", "--warmup", "0",
           "--no-cpu-baseline", "--no-e2e"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads([l for l in r.stdout.strip().splitlines() if l.startswith("{")][-1])
    c = out["config"]
    assert out["n_gpus"] == 2 and c["docs_per_node"] == 96 and c["docs_rank0"] == 48
    assert c["docs_in_error_rank0"] == 0 and "REHEARSAL" in c["parallelism"]
    assert out["value"] > 0
