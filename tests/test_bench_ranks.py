"""bench.py's N > 1 plumbing rehearsed on CPU before any multi-GPU run: gloo
ranks (world 2 and 3) drive bench.py's own helpers -- rank_shard (the
libmochi_hip shard plan and each rank's first_cert stream), timed_steps (barrier
+ sync around the timed span), reduce_over_ranks (MAX of the span, SUM of the
grants, AND of the correctness gates) and gathered_matches_rank0 (bitmap
assembly of the gathered slots) -- with the oracle standing in for the device
verify and a gloo all-gather for the RCCL one.  The gathered bitmap must be the
single-process oracle's verdicts for the whole batch."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


SLEEP = 0.03  # rank r's step sleeps r * SLEEP: the MAX over ranks must see the slowest


def _worker(rank, world, port, total_grants, cache_dir, out_dir):
    sys.path.insert(0, ROOT)
    import bench
    import mochi_hip as mh
    import oracle_ffi as O
    import workload as W

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    R, k = 4, 1
    C_total, plan, c_lo, c_hi = bench.rank_shard(total_grants, R, k, world, rank, mh.shard_plan)
    C = c_hi - c_lo
    pool = W.build_pool(R=R, k=k, P=64, P_f=16, cache_dir=cache_dir)
    s = W.make_batch(pool, C, first_cert=c_lo)  # this rank's slice of the one stream
    words = mh.shard_words(plan)
    gathered = torch.zeros(world * words, dtype=torch.int32)
    state = {}

    def step():
        v = O.verify_batch(pool.moduli, s.batch, R, True, 1)
        slot = torch.zeros(words, dtype=torch.int32)
        bits = torch.from_numpy(v.cert_accept_bits.view(np.int32).copy())
        slot[:bits.shape[0]] = bits
        parts = [torch.zeros(words, dtype=torch.int32) for _ in range(world)]
        dist.all_gather(parts, slot)
        gathered.copy_(torch.cat(parts))
        state["v"] = v
        import time

        time.sleep(SLEEP * rank)

    ev_s, wall = bench.timed_steps(step, 2, 1, stream=None, dist=dist, sync=lambda: None)
    ok = bool(np.array_equal(state["v"].grant_flags, s.expected_flags))
    t_max, wall_max, all_ok, n_total = bench.reduce_over_ranks(dist, ev_s, wall, ok, s.batch.n_grants, "cpu")
    if rank == 0:
        match = bench.gathered_matches_rank0(plan, gathered.numpy(), C_total, state["v"].cert_accept, mh.bits_assemble,
                                             mh.unpack_bits)
        full = mh.bits_assemble(plan, gathered.numpy().view(np.uint32))
        np.savez(os.path.join(out_dir, "r0.npz"), full=full, t_max=t_max, own=ev_s, all_ok=all_ok, n_total=n_total,
                 match=match, C_total=C_total, plan=plan)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,total_grants", [(2, 4 * 150), (3, 4 * 200 + 4)])
def test_bench_rank_plumbing_gloo(tmp_path, world, total_grants):
    import mochi_hip as mh
    import oracle_ffi as O
    import workload as W

    cache = str(tmp_path / "cache")
    pool = W.build_pool(R=4, k=1, P=64, P_f=16, cache_dir=cache)  # sign once, ranks load the cache
    mp.start_processes(_worker, args=(world, _free_port(), total_grants, cache, str(tmp_path)), nprocs=world,
                       start_method="spawn")
    z = np.load(tmp_path / "r0.npz")
    C_total = int(z["C_total"])
    full = W.make_batch(pool, C_total)
    ref = O.verify_batch(pool.moduli, full.batch, 4, True, 2)
    assert np.array_equal(mh.unpack_bits(z["full"], C_total), ref.cert_accept)  # the gathered batch bitmap
    assert (~ref.cert_accept).any()  # the fault mix produced rejects
    assert bool(z["match"]) and bool(z["all_ok"])
    assert int(z["n_total"]) == full.batch.n_grants  # SUM over ranks = the whole batch
    assert float(z["t_max"]) >= 2 * SLEEP * (world - 1) > float(z["own"]) - 1.0  # MAX saw the slowest rank
    assert float(z["t_max"]) >= float(z["own"])
    plan = z["plan"]
    assert plan[0] == 0 and plan[-1] == C_total and all(int(p) % 32 == 0 for p in plan[1:-1])
