"""bench.py's RCCL calls on a GPU box (one rank: RCCL refuses two ranks on
one GPU, and 8-GPU runs are the driver's): tests/rccl_world1.py under
torch.distributed.run with the nccl backend — barrier, all_reduce(MAX),
all_gather, and shard.redistribute's all_to_all_single."""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
def test_rccl_collectives_world1(gpu):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=1", "--master-addr", "127.0.0.1", "--master-port",
                        str(_port()), os.path.join(HERE, "rccl_world1.py")],
                       env=env, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["backend"] == "nccl" and line["world"] == 1
    assert line["all_reduce_max"] == 1.25
    assert line["all_gather"] == [[10, 20, 30, -1, 5]]
    assert line["redistributed_equal"]
