"""bench.py's multi-rank path on the GPU (BASELINE config 4's code: RCCL process
group, the timed gather of the int16 maps to rank 0, the max-over-ranks
all-reduce and the ``distributed`` block) run at world size 1 on one MI355X.

The bench runs as a CHILD of ``torch.distributed.run`` started from this test;
this module never touches the GPU itself, and it sorts before every module that
does, so the pytest process has not initialised HIP when the child starts."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
def test_bench_rank_path_rccl_world1():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--dist", "--steps", "5", "--warmup", "2", "--cpu-baseline-pairs", "0",
           "--host-surface-calls", "0"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    H, W = 375, 1242
    assert d["n_gpus"] == 1 and d["value"] > 0
    assert d["config"]["gather"] is True
    dd = d["distributed"]
    assert dd["backend"] == "nccl"
    assert dd["world_size"] == 1
    # world 1: rank 0 computes straight into its rows of the double-buffered result, so no
    # byte travels; the overlapped gather's buffer / launch / drain path runs all the same
    assert dd["gather_bytes_to_root"] == 0
    assert dd["gathered_in_pair_order"] is True
    assert dd["gather_ms_per_step_max"] >= 0 and dd["gather_exposed_ms_per_step"] >= 0
    assert "double-buffered" in dd["gather"]
