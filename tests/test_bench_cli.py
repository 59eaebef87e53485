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
