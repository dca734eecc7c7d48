"""N > 1 path on the CPU: world_size-2 gloo.  Each rank checksums its own
contiguous shard with the product's per-datagram CPU entry point
(lnl_crc32c; the batch kernels need a GPU -- bench.py's spawn path is
covered by tests/test_bench_spawn.py), and the shards reassemble to the
oracle's single-process answer (the oracle is only the checker here)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from litenetlibpp_amd.shard import max_over_ranks, shard_range, sum_over_ranks


def test_shard_range_partitions():
    for n in (0, 1, 7, 64, 1000, 1 << 20):
        for world in (1, 2, 3, 4, 8):
            seen = 0
            for r in range(world):
                s, c = shard_range(n, r, world)
                assert s == seen and c >= 0
                seen += c
            assert seen == n
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import litenetlibpp_amd as P
    n, L = 1000, 1400
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, n * L, dtype=np.uint8)   # every rank can regenerate the job's data
    s, c = shard_range(n, rank, world)
    mine = np.array([P.crc32c(data[(s + i) * L:(s + i + 1) * L]) for i in range(c)], dtype=np.uint32)
    parts = [None] * world
    dist.all_gather_object(parts, (s, mine.tolist()))
    t = max_over_ranks(1.0 + rank)
    b = sum_over_ranks(c * L)
    if rank == 0:
        import oracle
        full = np.zeros(n, np.uint32)
        for st, vals in parts:
            full[st:st + len(vals)] = vals
        ok = np.array_equal(full, oracle.batch_fixed(data, L, L, n))
        q.put((ok, t, b))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_shards_reassemble():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    ok, t, b = q.get(timeout=10)
    assert ok
    assert t == 2.0           # MAX over ranks
    assert b == 1000 * 1400   # bytes of all shards
