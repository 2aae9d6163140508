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


def _lib_worker(rank, world, port, n_certs, cache_dir, result_path):
    """One rank of the library's multi-GPU logic with gloo standing in for RCCL and the
    oracle for the device: libmochi_hip's shard plan (mochi_shard_plan) picks this rank's
    32-aligned certificate range, the shard's bitmap is padded to the plan's slot size
    (mochi_shard_words) and all-gathered, and libmochi_hip assembles the batch bitmap
    (mochi_bits_assemble) -- the host half of mochi_mverify_batch / bench.py N > 1."""
    import mochi_hip as mh
    import oracle_ffi as O
    import workload as W

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    pool = W.build_pool(R=4, k=1, P=64, P_f=16, cache_dir=cache_dir)
    full = W.make_batch(pool, n_certs)
    plan = mh.shard_plan(n_certs, world, full.batch.cert_grant_off)
    lo, hi = int(plan[rank]), int(plan[rank + 1])
    s = W.make_batch(pool, hi - lo, first_cert=lo)  # this rank's shard of the seeded stream
    v = O.verify_batch(pool.moduli, s.batch, 4, True, 1)
    words = mh.shard_words(plan)
    slot = np.zeros(words, np.uint32)
    slot[:v.cert_accept_bits.shape[0]] = v.cert_accept_bits
    gathered = torch.zeros(world * words, dtype=torch.int32)
    dist.all_gather_into_tensor(gathered, torch.from_numpy(slot.view(np.int32)))
    if rank == 0:
        np.save(result_path, mh.bits_assemble(plan, gathered.numpy().view(np.uint32)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_certs", [(2, 1000), (3, 777)])
def test_library_shard_plan_and_assembly_multi_rank(tmp_path, world, n_certs):
    import mochi_hip as mh
    import oracle_ffi as O
    import workload as W

    cache = str(tmp_path / "cache")
    W.build_pool(R=4, k=1, P=64, P_f=16, cache_dir=cache)
    out = str(tmp_path / "bits.npy")
    mp.start_processes(_lib_worker, args=(world, _free_port(), n_certs, cache, out), nprocs=world,
                       start_method="spawn")
    got = mh.unpack_bits(np.load(out), n_certs)
    pool = W.build_pool(R=4, k=1, P=64, P_f=16, cache_dir=cache)
    v = O.verify_batch(pool.moduli, W.make_batch(pool, n_certs).batch, 4, True, 2)
    assert np.array_equal(got, v.cert_accept)
    assert (~got).any()


def test_shard_plan_properties():
    import mochi_hip as mh

    rng = np.random.default_rng(3)
    for n in (0, 1, 31, 32, 33, 1000, 4_000_000):
        for w in (1, 2, 3, 8):
            cgo = np.concatenate([[0], np.cumsum(rng.integers(1, 9, n))]).astype(np.uint32) if n < 100000 else None
            lo = mh.shard_plan(n, w, cgo)
            assert lo[0] == 0 and lo[-1] == n and (np.diff(lo.astype(np.int64)) >= 0).all()
            assert all(int(x) % 32 == 0 or int(x) == n for x in lo[1:-1])
            if n >= 64 * w:  # balanced to within one 32-certificate step of the ideal
                work = (cgo[lo] if cgo is not None else lo).astype(np.int64)
                ideal = work[-1] / w
                assert np.abs(np.diff(work) - ideal).max() <= (cgo[32] - cgo[0] if cgo is not None else 32) * 2 + 16
