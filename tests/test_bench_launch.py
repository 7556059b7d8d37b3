"""bench.py's multi-rank path on the CPU: `--gpus N` without a launcher
starts N ranks (torch.distributed.run child), every rank runs bench.main()
and rank 0 prints one line with n_gpus == N. The ranks run config 5 (one file
split by bytes) over gloo with the oracle as codec (tests/bench_rehearsal.py),
so the redistribution, the boundary exchange and verify()'s record-count and
re-encode checks are bench.py's own code at world size 2 and 3."""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    return env


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("world", [2, 3, 8])
def test_gpus_flag_launches_ranks(world):
    n = 2000
    r = subprocess.run([sys.executable, os.path.join(HERE, "bench_rehearsal.py"),
                        "--gpus", str(world), "--config", "5", "--records", str(n),
                        "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                        "--no-copy-ceiling"],
                       env=_env(), cwd="/tmp", capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    line = _line(r.stdout)
    assert line["n_gpus"] == world
    assert line["config"]["records_total"] == n * world
    assert line["steps"] == 2 and line["scaling"] == "weak"
    assert "all_to_all_single" in line["config"]["parallelism"]
    # whole-job bytes: the file is every rank's encode output
    assert line["value"] > 0
    # each rank holds the next range's first bytes up to the file's longest
    # record (config 3 records: at most 4 x 5 + 2 x (5 + 32) + ... < 128 B)
    assert 4096 <= line["config"]["overlap_bytes"] <= 1 << 20


def test_local_rank_maps_to_its_gpu(monkeypatch):
    """`bench.py --gpus 8` under torch.distributed.run: rank LOCAL_RANK runs
    on cuda:LOCAL_RANK (CudaRuntime.setup), one process per GPU."""
    import torch

    seen = []
    monkeypatch.setattr(torch.cuda, "device_count", lambda: 8)
    monkeypatch.setattr(torch.cuda, "set_device", lambda d: seen.append(d))
    rt = bench.CudaRuntime()
    for local in range(8):
        assert rt.setup(local) == torch.device("cuda", local)
    assert seen == list(range(8))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("WORLD_SIZE", "8")
    monkeypatch.setenv("RANK", "6")
    monkeypatch.setenv("LOCAL_RANK", "6")
    world, rank, local = bench.resolve_world(8)
    assert (world, rank, local) == (8, 6, 6) and rt.setup(local) == torch.device("cuda", 6)


def test_overlap_is_the_longest_record():
    """Config 5's overlap: the longest record of the whole file (every rank's
    index), so the record straddling a range's end is always held."""
    import torch

    class W(bench.FileShards):
        def __init__(self, offs):
            self.n = len(offs) - 1
            self.offs = torch.tensor(offs, dtype=torch.int64)
            self.wire = torch.zeros(int(offs[-1]), dtype=torch.uint8)
            self.wire_bytes = int(offs[-1])
            self.record_bytes = 56

        def _gather(self, vals):  # a 3-rank file: the other ranks' longest records
            return [vals, [100, 9000], [100, 20]]

    w = W([0, 10, 60, 5000, 5010])
    assert w.longest_record() == 4940
    w.setup_file(0, torch.device("cpu"))
    assert w.overlap == 9000 and w.file_len == 5010 + 200


def test_world_mismatch_exits_nonzero():
    env = _env()
    env.update(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4",
                        "--config", "2"], env=env, cwd="/tmp", capture_output=True, text=True,
                       timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_resolve_world(monkeypatch):
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    assert bench.resolve_world(None) == (1, 0, 0)
    assert bench.resolve_world(1) == (1, 0, 0)
    assert bench.resolve_world(8) == (None, None, None)  # this process launches
    monkeypatch.setenv("WORLD_SIZE", "8")
    monkeypatch.setenv("RANK", "5")
    monkeypatch.setenv("LOCAL_RANK", "5")
    assert bench.resolve_world(8) == (8, 5, 5)
    assert bench.resolve_world(None) == (8, 5, 5)
    with pytest.raises(SystemExit):
        bench.resolve_world(2)


# ---- the same path on a GPU box ---------------------------------------------
# Two ranks share the box's one MI355X over gloo (RCCL refuses two ranks on one
# GPU): the real GPU chain of config 5 — device encode, all_to_all_single of
# the byte ranges (gloo's CUDA path), tgpu_decode_stream as the speculative
# index, the boundary all-gather — and config 2's independent shards.
@pytest.mark.gpu
@pytest.mark.parametrize("config,n", [(5, 1 << 20), (2, 1 << 20)])
def test_gpu_two_ranks_one_gpu(gpu, config, n):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--backend", "gloo", "--config", str(config), "--records", str(n),
                        "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                        "--no-copy-ceiling"],
                       env=_env(), cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    line = _line(r.stdout)
    assert line["n_gpus"] == 2 and line["config"]["records_total"] == 2 * n
