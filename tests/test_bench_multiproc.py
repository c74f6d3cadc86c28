"""bench.py under torchrun with two processes on the one GPU of the test box (gloo for the final
reduction, host tensors): the HIP path of the N > 1 layout.  Each process encodes, decodes and
verifies its own block of a small job; together they must cover every rank once."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_two_processes_share_the_job():
    env = dict(os.environ, CDCX_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    port = 29600 + os.getpid() % 300
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "1",
           "--world", "12", "--events", "200000", "--ranks-per-gpu", "4", "--streams", "2", "--cpu-baseline", "0",
           "--host-io", "0", "--solo", "0", "--oracle-ranks", "1"]
    out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
    d = json.loads(line)
    assert d["n_gpus"] == 2
    cfg = d["config"]
    assert cfg["ranks_processed"] == 12 and cfg["batches_per_gpu"] == 2
    assert cfg["verify"]["decode_ranks"] == 12 and cfg["verify_failures"] == 0
    assert cfg["verify"]["encode_ranks"] >= 1 and cfg["verify"]["encode_failures"] == 0
    assert d["value"] > 0 and cfg["records_per_step"] > 12 * 190000
