"""One record file split by bytes across ranks (BASELINE config 5: a Compact
file sharded over 8 GPUs).

Rank k owns the records that START in its byte range [B_k, B_{k+1}) of the
file and holds the bytes [B_k, min(B_{k+1} + overlap, L)) so the record that
straddles B_{k+1} can be read. No rank knows where its first record starts:
it indexes its range speculatively (tgpu_index_stream, speculative=1), and the
only exchange between ranks is each range's (first start, last end) pair —
rank k's first start must equal rank k-1's last end, which is where the
reference's sequential reader (repeated deserialize<T>(Cursor&),
Serializer.h:97-100) would be after reading rank k-1's records. A rank whose
speculation disagrees re-indexes from the confirmed position; repeated until
the chain agrees (at most world rounds). Record numbering is an exclusive scan
of the per-rank counts.

Everything here is host logic over small per-rank tuples; the collective is an
all-gather of 4 int64 per rank (RCCL over xGMI on the GPU path, gloo in the
CPU tests). The bulk bytes never cross ranks except the caller's own
redistribution of the file.
"""
NONE = (1 << 64) - 1


def byte_ranges(total_len, world):
    """[B_k, B_{k+1}) for every rank: equal byte split of the file."""
    return [(total_len * k // world, total_len * (k + 1) // world) for k in range(world)]


def need_range(ranges, overlap, file_len, rank):
    """File bytes rank `rank` must hold: its range plus `overlap` bytes of the
    next one (the record straddling its end; overlap >= the longest record)."""
    b, e = ranges[rank]
    return b, min(e + overlap, file_len)


def redistribution(enc_ranges, ranges, overlap, file_len, rank):
    """The byte moves that turn "rank k holds the file bytes it encoded"
    (enc_ranges[k], contiguous and in file order) into "rank k holds
    need_range(k)". Returns (send, recv): send[d] / recv[s] = (lo, hi) file
    offsets this rank sends to rank d / receives from rank s (lo == hi:
    nothing). The received pieces are ascending and tile need_range(rank)."""
    world = len(ranges)
    mine = enc_ranges[rank]
    lo, hi = need_range(ranges, overlap, file_len, rank)
    send, recv = [], []
    for d in range(world):
        nlo, nhi = need_range(ranges, overlap, file_len, d)
        a0, a1 = max(mine[0], nlo), min(mine[1], nhi)
        send.append((a0, max(a0, a1)))
        s0, s1 = enc_ranges[d]
        r0, r1 = max(s0, lo), min(s1, hi)
        recv.append((r0, max(r0, r1)))
    return send, recv


def redistribute(local, enc_ranges, ranges, overlap, file_len, rank, out, all_to_all_single):
    """Moves the file bytes (one all-to-all; RCCL over xGMI on the GPU path,
    gloo in the CPU tests): `local` (uint8 tensor) holds this rank's encoded
    bytes enc_ranges[rank]; `out` receives need_range(rank). Returns the
    filled prefix of `out`."""
    import torch

    send, recv = redistribution(enc_ranges, ranges, overlap, file_len, rank)
    base = enc_ranges[rank][0]
    pieces = [local[a - base: b - base] for a, b in send if b > a]
    inp = torch.cat(pieces) if pieces else local[:0]
    lo, hi = need_range(ranges, overlap, file_len, rank)
    all_to_all_single(out[: hi - lo], inp, [b - a for a, b in recv], [b - a for a, b in send])
    return out[: hi - lo]


def tensor_gather(all_gather, device, world):
    """all_gather(list_of_ints) over torch.distributed for
    exchange_boundaries: one int64 tensor per rank. Positions may be NONE
    (2**64 - 1, no record start in a range), which int64 cannot hold: it
    travels as -1 and comes back as NONE (no real position is negative)."""
    import torch

    def gather(vals):
        enc = [-1 if v == NONE else int(v) for v in vals]
        if world == 1:
            rows = [enc]
        else:
            t = torch.tensor(enc, dtype=torch.int64, device=device)
            out = [torch.empty_like(t) for _ in range(world)]
            all_gather(out, t)
            rows = [o.tolist() for o in out]
        return [[NONE if v == -1 else int(v) for v in r] for r in rows]

    return gather


def resolve(begins, ends, firsts, lasts):
    """Given every rank's range [begins[k], ends[k]) and its index result
    (first start, last end; NONE when no record start was found), return the
    confirmed first start per rank and the ranks whose index must be redone
    from that position (non-speculatively). Positions are file offsets.

    Rank 0 starts at its begin (the file's first record). Walking ranks in
    order, the expected first start of rank k is the previous rank's confirmed
    last end, or — when that lies past rank k's range (one record covers the
    whole range) — the range holds no record start and the expectation moves
    on unchanged.
    """
    world = len(begins)
    expect = begins[0]
    confirmed, redo = [], []
    for k in range(world):
        if expect >= ends[k]:
            # no record starts inside this range
            confirmed.append(NONE)
            if firsts[k] != NONE:
                redo.append(k)
            continue
        confirmed.append(expect)
        if firsts[k] != expect:
            redo.append(k)
            # the redone index will report its own last end next round; until
            # then nothing after k can be confirmed
            for j in range(k + 1, world):
                confirmed.append(None)
            return confirmed, redo
        expect = lasts[k]
    return confirmed, redo


def exchange_boundaries(index_fn, rank, world, begin, end, all_gather):
    """Runs the speculative index and the boundary exchange for this rank.

    index_fn(begin, speculative) -> (n_records, first_start, last_end) for this
    rank's range (file offsets), re-runnable; all_gather(list_of_ints) ->
    list (one per rank) of such lists. Returns (n_records, first_start,
    last_end, record_base, rounds)."""
    n, first, last = index_fn(begin, rank > 0)
    rounds = 1
    while True:
        rows = all_gather([begin, end, first, last, n])
        begins = [r[0] for r in rows]
        ends = [r[1] for r in rows]
        firsts = [r[2] for r in rows]
        lasts = [r[3] for r in rows]
        counts = [r[4] for r in rows]
        confirmed, redo = resolve(begins, ends, firsts, lasts)
        if not redo:
            base = sum(counts[:rank])
            return n, first, last, base, rounds
        if rank in redo:
            c = confirmed[rank]
            if c == NONE:
                n, first, last = 0, NONE, NONE
            else:
                n, first, last = index_fn(c, False)
        rounds += 1
        if rounds > world + 1:
            raise RuntimeError("shard boundary exchange did not converge")
