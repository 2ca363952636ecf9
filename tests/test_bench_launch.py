"""bench.py --gpus N launches its own ranks (the replacement for the
reference's in-process nn.DataParallel, train_patch.py:63-71): started
without a torchrun environment it runs N processes through
torch.distributed.run and rank 0 prints one JSON line for the whole job.
On the CPU, --dry-run exercises exactly that launch, each rank's shard of the
global batch and the fused all-reduce of the patch gradient (gloo)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT


def _bench(*args, timeout=240):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + list(args), cwd=ROOT, env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout          # one JSON line for the job, from rank 0 only
    return json.loads(lines[0])


@pytest.mark.parametrize("n,B", [(2, 16), (3, 5)])
def test_bench_gpus_n_launches_n_ranks(n, B):
    line = _bench("--dry-run", "--gpus", str(n), "--dist-backend", "gloo", "--batch", str(B), "--steps", "2")
    assert line["n_gpus"] == n and line["dry_run"] and line["value"] is None
    assert line["config"]["global_batch"] == n * B and line["config"]["parallelism"] == "dp%d" % n
    # contiguous shards of one global batch, in rank order, covering it exactly
    assert line["shards"] == [[r * B, (r + 1) * B] for r in range(n)]
    assert line["allreduce_bytes"] == 4 * (3 * 224 * 224 + 6)
    assert line["dist_backend"] == "gloo"


def test_bench_single_rank_dry_run():
    line = _bench("--dry-run", "--steps", "1")
    assert line["n_gpus"] == 1 and line["shards"] == [[0, 16]]


def test_bench_refuses_more_rccl_ranks_than_gpus():
    """RCCL needs one GPU per rank: asking for more ranks than visible GPUs
    fails loudly instead of measuring fewer (no GPU here: any N > 1)."""
    import torch
    n = torch.cuda.device_count() + 1
    if n < 2:
        n = 2
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n)], cwd=ROOT,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=120,
                       env={k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")})
    assert p.returncode != 0 and "GPU(s) visible" in p.stderr
