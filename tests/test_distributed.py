"""Multi-rank path on CPU: world_size-2 gloo processes shard certificates,
verify their shard (the oracle stands in for the device here), all-gather the
verdict bitmaps, and must reproduce the single-process verdicts exactly."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, certs_per_rank, cache_dir, result_path):
    import oracle_ffi as O
    import workload as W

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pool = W.build_pool(R=4, k=1, P=64, P_f=16, cache_dir=cache_dir)
    s = W.make_batch(pool, certs_per_rank, first_cert=rank * certs_per_rank)  # bench.py's weak-scaling shard
    v = O.verify_batch(pool.moduli, s.batch, 4, True, 1)
    local = torch.from_numpy(v.cert_accept_bits.view(np.int32).copy())
    gathered = shard.allgather_bitmaps(local, world)
    if rank == 0:
        np.save(result_path, gathered.numpy().view(np.uint32))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("certs_per_rank", [37, 64])
def test_two_rank_allgather_matches_single_process(tmp_path, certs_per_rank):
    import oracle_ffi as O
    import workload as W

    world = 2
    cache = str(tmp_path / "cache")
    W.build_pool(R=4, k=1, P=64, P_f=16, cache_dir=cache)  # sign once, ranks load the cache
    out = str(tmp_path / "gathered.npy")
    mp.start_processes(_worker, args=(world, _free_port(), certs_per_rank, cache, out), nprocs=world,
                       start_method="spawn")
    gathered = np.load(out)
    got = shard.unpack_gathered(gathered, certs_per_rank, world)
    pool = W.build_pool(R=4, k=1, P=64, P_f=16, cache_dir=cache)
    full = W.make_batch(pool, certs_per_rank * world)
    v = O.verify_batch(pool.moduli, full.batch, 4, True, 2)
    assert np.array_equal(got, v.cert_accept)
    assert (~got).any()  # the fault mix produced rejects in the gathered set


def test_shard_range_partitions():
    for n in (0, 1, 7, 1000, 1001):
        for w in (1, 2, 3, 8):
            cover = []
            for r in range(w):
                lo, hi = shard.shard_range(n, w, r)
                cover.extend(range(lo, hi))
            assert cover == list(range(n))
