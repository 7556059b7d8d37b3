"""Run under torch.distributed.run with one rank on the box's one MI355X
(tests/test_rccl_world1.py): the RCCL (torch "nccl" backend) calls bench.py's
multi-GPU path issues — init_process_group with the rank's device, barrier,
the max-over-ranks all_reduce of the elapsed time, config 5's all_gather of
the boundary tuples and all_to_all_single of the file bytes
(fbthrift_amd/shard.py redistribute) — executed through RCCL at world size 1
(RCCL refuses two ranks on one GPU). Prints one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from fbthrift_amd import shard  # noqa: E402


def main():
    local = int(os.environ["LOCAL_RANK"])
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("nccl", device_id=dev)
    world, rank = dist.get_world_size(), dist.get_rank()
    out = {"backend": dist.get_backend(), "world": world}
    dist.barrier()
    t = torch.tensor([1.25 + rank], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    out["all_reduce_max"] = t.item()
    row = torch.tensor([10, 20, 30, -1, 5], dtype=torch.int64, device=dev)
    rows = [torch.empty_like(row) for _ in range(world)]
    dist.all_gather(rows, row)
    out["all_gather"] = [r.tolist() for r in rows]
    # the file redistribution of config 5: rank 0 encoded the whole file
    file_len, overlap = 1 << 20, 4096
    data = torch.arange(file_len, device=dev, dtype=torch.int64).to(torch.uint8)
    ranges = shard.byte_ranges(file_len, world)
    buf = torch.empty(file_len + overlap, dtype=torch.uint8, device=dev)
    got = shard.redistribute(data, [(0, file_len)], ranges, overlap, file_len, rank, buf,
                             dist.all_to_all_single)
    torch.cuda.synchronize()
    out["redistributed_equal"] = bool(torch.equal(got, data))
    dist.barrier()
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
