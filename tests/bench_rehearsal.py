"""CPU stand-in for one bench.py rank (test infrastructure, loaded by bench.py
only when MOCHI_BENCH_REHEARSAL names this file): the rank plumbing of
`python bench.py --gpus N` -- bench.py's own self-launch (RANK / WORLD_SIZE /
MASTER_* per child), rank_shard (libmochi_hip's shard plan), timed_steps
(barrier + sync around the timed span), reduce_over_ranks (MAX of the span, SUM
of the grants, AND of the gates) and gathered_matches_rank0 -- on gloo, with the
oracle standing in for the device verify and a gloo all-gather for the RCCL one.

Env: MOCHI_REHEARSAL_OUT (rank 0 saves the assembled batch bitmap there),
MOCHI_REHEARSAL_FAIL_RANK (that rank exits 3 right after the rendezvous: its
peers then wait in the first barrier until bench.py's launcher stops them)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "mochi-db_amd"))


def rank_main(args, world, rank, local_rank):
    import numpy as np
    import torch
    import torch.distributed as dist

    import bench
    import mochi_hip as mh
    import oracle_ffi as O
    import workload as W

    dist.init_process_group("gloo", rank=rank, world_size=world)
    if os.environ.get("MOCHI_REHEARSAL_FAIL_RANK") == str(rank):
        sys.exit(3)
    R, k = args.replication or 4, args.ops_per_txn
    C_total, plan, c_lo, c_hi = bench.rank_shard(args.grants_total, R, k, world, rank, mh.shard_plan)
    pool = W.build_pool(R=R, k=k, P=64, P_f=16, cache_dir=args.cache_dir)
    s = W.make_batch(pool, c_hi - c_lo, first_cert=c_lo)
    words = mh.shard_words(plan)
    gathered = torch.zeros(world * words, dtype=torch.int32)
    state = {}

    def step():
        v = O.verify_batch(pool.moduli, s.batch, R, not args.client_predicate, 1)
        slot = np.zeros(words, np.uint32)
        slot[:v.cert_accept_bits.shape[0]] = v.cert_accept_bits
        dist.all_gather_into_tensor(gathered, torch.from_numpy(slot.view(np.int32)))
        state["v"] = v

    ev_s, wall = bench.timed_steps(step, args.steps, args.warmup, stream=None, dist=dist, sync=lambda: None)
    ok = bool(np.array_equal(state["v"].grant_flags, s.expected_flags))
    t_max, wall_max, all_ok, n_total = bench.reduce_over_ranks(dist, ev_s, wall, ok, s.batch.n_grants, "cpu")
    result = None
    if rank == 0:
        full = mh.bits_assemble(plan, gathered.numpy().view(np.uint32))
        out = os.environ.get("MOCHI_REHEARSAL_OUT")
        if out:
            np.savez(out, full=full, C_total=C_total, plan=plan)
        result = {"metric": bench.METRIC, "value": round(n_total * args.steps / t_max, 1), "unit": "grants/s",
                  "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                  "ms_per_step": round(t_max / args.steps * 1e3, 4), "scaling": "strong",
                  "data": "synthetic (CPU rehearsal: oracle verify, gloo all-gather)",
                  "correct_vs_ground_truth": all_ok, "grants_total": n_total,
                  "gathered_bitmap_matches_rank0": bench.gathered_matches_rank0(
                      plan, gathered.numpy(), C_total, state["v"].cert_accept, mh.bits_assemble, mh.unpack_bits)}
    dist.barrier()
    dist.destroy_process_group()
    return result
