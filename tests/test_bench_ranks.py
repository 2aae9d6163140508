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


def _bench_cmd(world, total_grants, cache, extra=()):
    return [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--steps", "2", "--warmup", "1",
            "--grants-total", str(total_grants), "--cache-dir", cache] + list(extra)


def _plain_env(**kv):
    """A plain shell's environment: no launcher variables at all."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
                        "GROUP_RANK")}
    env.update(kv)
    return env


@pytest.mark.parametrize("world,total_grants", [(2, 4 * 300), (4, 4 * 333 + 4), (8, 4 * 520)])
def test_bench_self_launch_gloo(tmp_path, world, total_grants):
    """`python bench.py --gpus N` with no launcher env starts its own N ranks (bench.self_launch)
    and rank 0 prints the one JSON line; the gathered bitmap == the single-process oracle."""
    import json
    import subprocess

    import mochi_hip as mh
    import oracle_ffi as O
    import workload as W

    cache = str(tmp_path / "cache")
    pool = W.build_pool(R=4, k=1, P=64, P_f=16, cache_dir=cache)  # sign once, ranks load the cache
    out = str(tmp_path / "r0.npz")
    env = _plain_env(MOCHI_BENCH_REHEARSAL=os.path.join(ROOT, "tests", "bench_rehearsal.py"),
                     MOCHI_REHEARSAL_OUT=out, OMP_NUM_THREADS="1")
    p = subprocess.run(_bench_cmd(world, total_grants, cache), env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout  # only rank 0 prints, one line
    res = json.loads(lines[0])
    assert res["n_gpus"] == world and res["correct_vs_ground_truth"] and res["gathered_bitmap_matches_rank0"]
    z = np.load(out)
    C_total = int(z["C_total"])
    full = W.make_batch(pool, C_total)
    ref = O.verify_batch(pool.moduli, full.batch, 4, True, 2)
    assert np.array_equal(mh.unpack_bits(z["full"], C_total), ref.cert_accept)
    assert (~ref.cert_accept).any()
    assert res["grants_total"] == full.batch.n_grants
    plan = z["plan"]
    assert len(plan) == world + 1 and plan[-1] == C_total


def test_bench_self_launch_rank_failure_ends_job(tmp_path):
    """A rank that dies after the rendezvous must not leave its peers waiting in the first
    barrier: the launcher stops them and exits with the failed rank's code."""
    import subprocess
    import time

    cache = str(tmp_path / "cache")
    import workload as W

    W.build_pool(R=4, k=1, P=64, P_f=16, cache_dir=cache)
    env = _plain_env(MOCHI_BENCH_REHEARSAL=os.path.join(ROOT, "tests", "bench_rehearsal.py"),
                     MOCHI_REHEARSAL_FAIL_RANK="1", OMP_NUM_THREADS="1")
    t0 = time.time()
    p = subprocess.run(_bench_cmd(3, 4 * 200, cache), env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 3, (p.returncode, p.stderr[-2000:])
    assert time.time() - t0 < 240
    assert not p.stdout.strip()


def test_bench_self_launch_needs_devices(tmp_path):
    """Without the rehearsal hook, --gpus N with fewer than N visible GPUs fails fast
    (this container has none) instead of starting ranks."""
    import subprocess

    p = subprocess.run(_bench_cmd(2, 4 * 100, str(tmp_path)), env=_plain_env(HIP_VISIBLE_DEVICES=""),
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 2 and "GPU(s) visible" in p.stderr
