"""CPU rehearsal of bench.py's multi-rank path (test infrastructure).

Runs bench.main() unchanged — its --gpus launcher (torch.distributed.run
child re-running this script), the per-rank setup, the barrier + max-over-
ranks timing and the JSON line — with two substitutions that only a test may
make: ranks run on the CPU over gloo (CpuRuntime), and config 5's FileShards
workload uses the oracle as its codec (CpuFileShards: oracle encode, the
oracle's sequential record walk as the speculative index, oracle decode).
Everything between those calls is bench.py's own: the file's byte split,
shard.redistribute over all_to_all_single, shard.exchange_boundaries over
all_gather, the record-count check and the re-encode check of verify().

    python tests/bench_rehearsal.py --gpus 2 --config 5 --records 3000 \
        --steps 2 --warmup 1 --no-cpu-baseline --no-copy-ceiling
"""
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "golden"))

import numpy as np  # noqa: E402

import bench  # noqa: E402


class CpuEvent:
    def record(self, stream=None):
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3


class CpuRuntime:
    backend = "gloo"

    def setup(self, local):
        import torch

        return torch.device("cpu")

    def init_group(self, dev):
        import torch.distributed as dist

        dist.init_process_group(self.backend)

    def sync(self):
        pass

    def event(self):
        return CpuEvent()


class _Status:
    code = 0

    def as_tuple(self):
        return (0,)


def _records(schema, first, n):
    import datagen
    import helpers

    table = datagen.SCHEMAS["mixed"]
    vals = datagen.flatten_values(table, [datagen.gen_mixed(i) for i in range(first, first + n)])
    rec, sarena, _ = helpers.pack(schema, vals, n)
    return rec.view(np.uint8).reshape(-1), sarena


class CpuFileShards(bench.FileShards):
    """Config 5 with the oracle as codec: same records (datagen.gen_mixed of
    the global record index), same Compact bytes as the GPU writes."""

    def __init__(self, n, rank, dev):
        import torch

        from fbthrift_amd.schema import Schema
        from oracle import oracle
        import datagen

        self.oracle = oracle
        self.schema = Schema.from_table(datagen.SCHEMAS["mixed"])
        self.n = n
        self.record_bytes = self.schema.record_size
        self.stream = None
        self.dec_kernel = self.enc_kernel = "oracle (CPU rehearsal)"
        self.rec_np, self.sarena = _records(self.schema, rank * n, n)
        st, wire, offs = oracle.encode(self.schema, 2, self.rec_np, n, self.sarena)
        assert st.code == 0
        self.wire = torch.frombuffer(bytearray(wire), dtype=torch.uint8)
        self.offs = torch.from_numpy(offs.astype(np.int64))
        self.wire_bytes = len(wire)
        self.side_bytes = int(self.sarena.size)
        self.setup_file(rank, dev)

    def encode(self):
        import torch

        st, wire, _ = self.oracle.encode(self.schema, 2, self.rec_np, self.n, self.sarena)
        assert st.code == 0 and len(wire) == self.wire_bytes
        self.wire.copy_(torch.frombuffer(bytearray(wire), dtype=torch.uint8))

    def index_range(self, local, begin, end, speculative):
        import torch

        buf = local.numpy()
        o = self.oracle

        def walk(p):
            count = 0
            while p < end:
                length = o.record_length(2, buf, p)
                if length <= 0:
                    return None
                p += length
                count += 1
            return count, p

        found = None
        for c in (range(begin, end) if speculative else [begin]):
            r = walk(c)
            if r is not None and r[0] > 0:
                found = (r[0], c, r[1])
                break
        if found is None:
            return 0, 0, 0, _Status()
        n, first, last = found
        st, rec, _, nd, _ = o.decode(self.schema, 2, buf[first:last], n,
                                     offsets=None)
        assert st.code == 0 and nd == n
        rs = self.record_bytes
        rec = rec.view(np.uint8).reshape(n, rs).copy()
        for so in (16, 32):  # string spans: relative to `local`, like the GPU's views
            v = rec[:, so:so + 8].view(np.uint64).reshape(n)
            v += np.uint64(first)
        self.back[: n * rs] = torch.from_numpy(rec.reshape(-1))
        return n, first, last, _Status()

    def expected_records(self, base, n):
        import torch

        rec, _ = _records(self.schema, base, n)
        return torch.from_numpy(rec.copy())

    def reencode(self, records, n, local):
        import torch

        st, wire, _ = self.oracle.encode(self.schema, 2, records.numpy(), n, local.numpy())
        assert st.code == 0
        return torch.frombuffer(bytearray(wire), dtype=torch.uint8)


def install():
    bench.RUNTIME = CpuRuntime()
    bench.WORKLOADS[5] = CpuFileShards


if __name__ == "__main__":
    install()
    sys.exit(bench.main())
