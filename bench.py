#!/usr/bin/env python3
"""Benchmark: verified grant signatures/sec on MI355X (BASELINE.json metric).

One step = one pass of the Write2 certificate-verification hot path over one
batch already resident in HBM: grant prep (proto3 parse + SHA-256), signer
bucketing, RSA-2048 verify (k_rsa_pow + k_rsa_final), certificate tally, and
for N > 1 the RCCL all-gather of the per-rank certificate-verdict bitmaps
(the only collective).

Headline (default --config c4): BASELINE.json config C4, the 16M-grant
certificate batch (R = 4).  It fits one MI355X, so N = 1 verifies all of it;
N > 1 shards its certificate-index range contiguously over the ranks (strong
scaling: 16M/N grants per GPU) and all-gathers the verdict bitmaps.  At N = 1
the run also reports a C3 leg (4M grants, R = 7, server and client
predicates, own roofline), the PCIe-inclusive host path, the Write2ToServer
wire path, producer signing and the CPU baseline.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4|c3|c2]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mochi-db_amd"))

METRIC = "verified grant signatures/sec (1/2/4/8 GPU) + % of INT32 VALU roofline"

# Algorithmic work: RSA-2048, e = 65537 -> 17 Montgomery
# multiplications of 2048-bit operands, each a CIOS modmul over s = 64 32-bit
# limbs = 2s^2 + s = 8,256 32x32->64 multiply-accumulates; the squaring chain
# (k_rsa_pow) is 16 of them, the whole path 17.
MAC_PER_MODMUL = 8256
MAC_PER_GRANT = 17 * MAC_PER_MODMUL  # 140,352
MAC_POW_PER_GRANT = 16 * MAC_PER_MODMUL  # 132,096 (CIOS-equivalent work of the squaring chain)
# Peak VALU issue: one wave64 v_mad_u64_u32 per 4 cycles per SIMD =
# 256 CU x 4 SIMD x 16 lanes x 2.4 GHz = 3.93e13 lane-ops/s (microbench/int_peak.hip
# measured 3.41-3.57e13 v_mad_u64_u32/s, 87-91 %).
PEAK_MAC_PER_S = 256 * 4 * 32 / 2 * 2.4e9
# k_rsa_pow (rsa_pow.hip, csrc/fold.h) per grant and squaring: x^2 on the VALU
# and the fold t_hi x W on the matrix cores (296 x 300 int8 MACs, 200
# v_mfma_i32_32x32x32_i8 per 64 grants, each holding the SIMD's issue for 8 cycles
# = 2 wave-instruction slots = 128 lane-slots).  Its roofline is the SIMD issue
# port both share.  The work is counted the way Strassen GEMMs report FLOPs:
# classical-equivalent -- the schoolbook x^2 (2,775 28-bit v_mad_u64_u32) + the
# fold = 3,175 lane-slots per grant-squaring, the same figure as round 2 -- while
# the kernel does one level of Karatsuba (kara_dev.h: 3 x 703 = 2,109 mads), so
# the issue slots it actually needs are 2,109 + 400 = 2,509 (reported beside).
POW_SQR = 16
POW_VALU_MAC = 2775
POW_VALU_MAC_KARATSUBA = 3 * 703
POW_MFMA_I8_MAC = 296 * 300
POW_ISSUE_SLOTS = POW_VALU_MAC + 200 * 128 // 64  # 3,175 (classical-equivalent)
POW_ISSUE_SLOTS_IMPL = POW_VALU_MAC_KARATSUBA + 200 * 128 // 64  # 2,509 (what the kernel needs)
INT8_DENSE_PEAK = 2 * 2.5e15 / 2  # MACs/s: i8 = 2x bf16 dense (MICROARCH.md), 2.5 PFLOP bf16 = 1.25e15 MAC/s

# BASELINE.json configs (index 1..3): total grants, replication factor
CONFIGS = {
    "c2": dict(grants=1_000_000, R=4, name="C2: 1M synthetic signed write grants batch-verified on one MI355X"),
    "c3": dict(grants=4_000_000, R=7, name="C3: 7-server (f=2) certificates, 4M grants, quorum tally fused with verify"),
    "c4": dict(grants=16_000_000, R=4, name="C4: 16M-grant certificate batch sharded across the GPUs, RCCL all-gather "
                                            "of verdict bitmaps"),
}


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c4")
    ap.add_argument("--grants-total", type=int, default=0, help="override the config's batch size (all GPUs)")
    ap.add_argument("--replication", type=int, default=0, help="override the config's R")
    ap.add_argument("--ops-per-txn", type=int, default=1)
    ap.add_argument("--client-predicate", action="store_true", help="count >= M instead of the server's count > M")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU work (core-seconds) per baseline run")
    ap.add_argument("--cpu-runs", type=int, default=5, help="timed CPU-baseline runs (median reported)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-wire", action="store_true", help="skip the Write2ToServer wire-path measurement")
    ap.add_argument("--no-c3", action="store_true", help="skip the C3 leg")
    ap.add_argument("--headline-only", action="store_true",
                    help="only the timed device-resident steps (no side legs): the profiled run")
    ap.add_argument("--cache-dir", default=os.environ.get("MOCHI_CACHE", "/tmp/mochi_bench_cache"))
    ap.add_argument("--no-native", action="store_true", help="skip the native batcher load driver leg")
    ap.add_argument("--no-cluster", action="store_true", help="skip the in-process cluster (C1 / C5 proxy) leg")
    ap.add_argument("--no-shard-sizes", action="store_true", help="skip the per-rank shard-size leg (16M/2, /4, /8)")
    ap.add_argument("--shard-sizes", action="store_true", help="run the shard-size leg even with --headline-only")
    ap.add_argument("--no-separate", action="store_true", help="skip the separate-copies C4 leg")
    ap.add_argument("--layout", choices=("shared", "separate"), default="shared",
                    help="headline grant-byte layout (separate: workload.separate_copies; profiling runs)")
    return ap.parse_args()


def timed_steps(step, steps, warmup, stream=None, dist=None, sync=None):
    """W untimed steps, then K steps bracketed by barrier + synchronize on both
    sides; returns (event seconds, wall seconds) of this rank.  With a CUDA
    `stream` the event time comes from HIP events on it; without one (the CPU
    rehearsal of the rank plumbing, tests/test_bench_ranks.py) it is the wall
    time.  `sync` defaults to torch.cuda.synchronize."""
    import torch

    if sync is None:
        sync = torch.cuda.synchronize
    for _ in range(warmup):
        step()
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    e0 = e1 = None
    if stream is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    if e0 is not None:
        e0.record(stream)
    for _ in range(steps):
        step()
    if e1 is not None:
        e1.record(stream)
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    wall = time.perf_counter() - t0
    return (e0.elapsed_time(e1) / 1e3 if e0 is not None else wall), wall


def rank_shard(total_grants, R, k, world, rank, shard_plan):
    """This rank's certificate shard of the config's batch: libmochi_hip's plan
    (contiguous, 32-aligned, so the per-rank verdict bitmaps concatenate word by
    word after the all-gather).  Returns (C_total, plan, c_lo, c_hi); the rank
    generates the SURVEY §8d stream from certificate c_lo on (first_cert)."""
    import workload as W

    C_total = W.n_certs_for_grants(total_grants, R, k)
    plan = shard_plan(C_total, world)
    return C_total, plan, int(plan[rank]), int(plan[rank + 1])


def reduce_over_ranks(dist, ev_s, wall, ok, n_grants, device):
    """MAX of the timed span over ranks (the job is as slow as its slowest
    rank), AND of the per-rank correctness gates, SUM of the grants verified.
    Returns (t_max, wall_max, all_ok, total_grants)."""
    import torch

    t = torch.tensor([ev_s, wall, 1.0 if ok else 0.0], dtype=torch.float64, device=device)
    n_all = torch.tensor([n_grants], dtype=torch.int64, device=device)
    if dist is not None:
        tt = t[:2].clone()
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        ok_t = t[2:].clone()
        dist.all_reduce(ok_t, op=dist.ReduceOp.MIN)
        t = torch.cat([tt, ok_t])
        dist.all_reduce(n_all)
    return float(t[0]), float(t[1]), bool(t[2] >= 1.0), int(n_all.item())


def gathered_matches_rank0(plan, gathered_words, C_total, local_accept, bits_assemble, unpack_bits):
    """Rank 0's check of the all-gather: the whole batch's bitmap, assembled from
    the gathered per-rank slots, holds rank 0's own shard verdicts."""
    import numpy as np

    g = bits_assemble(plan, np.ascontiguousarray(gathered_words).view(np.uint32))
    C0 = int(plan[1]) - int(plan[0])
    return bool(np.array_equal(unpack_bits(g, C_total)[:C0], np.asarray(local_accept)[:C0]))


def roofline(n_grants, pow_ms, traffic=None):
    """k_rsa_pow against the SIMD issue port (VALU + MFMA issue): algorithmic issue
    slots per launch (n_grants x 16 x 3,175) / kernel time vs 3.93e13 slots/s.
    Also: the VALU-resident MACs alone, the int8 MFMA rate, and the CIOS-equivalent
    work (SURVEY §8d, 132,096 MAC/grant) against the VALU-only peak the previous
    Montgomery kernel was bound by."""
    t = pow_ms / 1e3 if pow_ms > 0 else float("inf")
    slots = n_grants * POW_SQR * POW_ISSUE_SLOTS
    achieved = slots / t
    cios = n_grants * MAC_POW_PER_GRANT / t
    mfma = n_grants * POW_SQR * POW_MFMA_I8_MAC / t
    impl = n_grants * POW_SQR * POW_ISSUE_SLOTS_IMPL / t
    return {"bound": "valu", "kernel": "k_rsa_pow", "achieved": round(achieved / 1e12, 3),
            "peak": round(PEAK_MAC_PER_S / 1e12, 3),
            "unit": "T issue-slots/s (v_mad_u64_u32 lane-ops + MFMA issue), classical-equivalent work "
                    "(schoolbook x^2 + fold: 3,175 slots per grant-squaring)",
            "frac": round(achieved / PEAK_MAC_PER_S, 4), "traffic": traffic,
            "algorithmic_slots_per_launch": slots, "kernel_ms": round(pow_ms, 4),
            "implemented": {"slots_per_grant_squaring": POW_ISSUE_SLOTS_IMPL,
                            "achieved": round(impl / 1e12, 3), "frac": round(impl / PEAK_MAC_PER_S, 4),
                            "note": "Karatsuba x^2 (3 x 703 mads) + fold: the issue the kernel's own algorithm needs"},
            "valu_mac_tmac_per_s": round(n_grants * POW_SQR * POW_VALU_MAC_KARATSUBA / t / 1e12, 3),
            "mfma_i8": {"tmac_per_s": round(mfma / 1e12, 1), "peak_tmac_per_s": INT8_DENSE_PEAK / 1e12,
                        "frac": round(mfma / INT8_DENSE_PEAK, 4)},
            "cios_equiv": {"tmac_per_s": round(cios / 1e12, 3),
                           "vs_valu_only_peak": round(cios / PEAK_MAC_PER_S, 4)}}


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def visible_devices():
    """GPUs this process may use, counted without initialising the GPU
    (torch.cuda.device_count() does not create a HIP context on this image)."""
    import torch

    return torch.cuda.device_count()


def self_launch(n, argv, poll_s=0.2, grace_s=10.0):
    """`python bench.py --gpus N` (N > 1) with no launcher environment: start the
    N rank processes here, before this process makes any GPU call, exactly as
    `torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1` would
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT per child), and
    wait for them.  Rank 0's stdout is this process's stdout (the one JSON
    line); the other ranks' stdout goes to stderr.  The first rank to fail ends
    the job: the others are terminated (then killed after `grace_s`) so no rank
    is left waiting in a collective for a peer that is gone, and its exit code
    is returned.  Fails fast (exit 2) when fewer than N devices are visible.
    With MOCHI_BENCH_REHEARSAL set (tests/bench_rehearsal.py: gloo on the CPU,
    the oracle standing in for the device) no device is needed."""
    import subprocess

    if not os.environ.get("MOCHI_BENCH_REHEARSAL"):
        have = visible_devices()
        if have < n:
            print(f"bench.py: --gpus {n} but {have} GPU(s) visible", file=sys.stderr, flush=True)
            return 2
    import threading

    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr, text=r == 0))

    def relay(f):  # rank 0's JSON line to stdout; library chatter (gloo / RCCL banners) to stderr
        for line in f:
            (sys.stdout if line.lstrip().startswith("{") else sys.stderr).write(line)
            sys.stdout.flush()

    reader = threading.Thread(target=relay, args=(procs[0].stdout,), daemon=True)
    reader.start()
    rc = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [c for c in codes if c not in (None, 0)]
        if bad:
            rc = bad[0]
            break
        if all(c == 0 for c in codes):
            reader.join()
            return 0
        time.sleep(poll_s)
    print(f"bench.py: a rank exited with {rc}; stopping the others", file=sys.stderr, flush=True)
    for p in procs:
        if p.poll() is None:
            p.terminate()
    t_end = time.time() + grace_s
    for p in procs:
        try:
            p.wait(timeout=max(0.1, t_end - time.time()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    return rc if rc > 0 else 1


def rank_env(gpus):
    """(world, rank, local_rank) from the launcher's environment."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world != gpus:
        raise SystemExit(f"--gpus {gpus} but WORLD_SIZE={world}")
    return world, rank, local_rank


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args.gpus, sys.argv[1:]))
    rehearsal = os.environ.get("MOCHI_BENCH_REHEARSAL")
    if rehearsal:  # CPU rehearsal of the rank plumbing (tests only): no device, gloo, the oracle verifies
        import importlib.util

        spec = importlib.util.spec_from_file_location("bench_rehearsal", rehearsal)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        result = mod.rank_main(args, *rank_env(args.gpus))
        if result is not None:
            print(json.dumps(result), flush=True)
        return
    import numpy as np
    import torch

    import mochi_hip as mh
    import workload as W

    world, rank, local_rank = rank_env(args.gpus)
    if local_rank >= visible_devices():
        raise SystemExit(f"rank {rank}: LOCAL_RANK {local_rank} but {visible_devices()} GPU(s) visible")
    cfg = CONFIGS[args.config]
    R, k = args.replication or cfg["R"], args.ops_per_txn
    strict = not args.client_predicate
    total_grants = args.grants_total or cfg["grants"]
    C_total, plan, c_lo, c_hi = rank_shard(total_grants, R, k, world, rank, mh.shard_plan)
    C = c_hi - c_lo
    # CPU baseline (rank 0, N = 1 only): a child process started BEFORE this
    # process touches the GPU (it forks its workers and must hold no HIP
    # state); it waits for the sample file written below and times the oracle.
    cpu_child = None
    cpu_flags = os.path.join(args.cache_dir, "cpu_baseline_flags.npz")
    batch_file = os.path.join(args.cache_dir, f"bench_batch_{os.getpid()}.npz")
    cpu_certs = min(C, 250_000)  # the baseline's sample: the stream's first certificates (~1M grants at R = 4)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu_child = start_cpu_baseline(args, R, k, cpu_flags, batch_file)
    # native batcher load driver (microbench/batcher_load): also started before this
    # process touches the GPU; it waits for the Write2 input file the wire leg writes
    args.native_child = args.native_input = None
    if rank == 0 and world == 1 and not (args.headline_only or args.no_wire or args.no_native):
        args.native_input = os.path.join(args.cache_dir, f"w2_native_{os.getpid()}.bin")
        args.native_child = start_batcher_native(args, args.native_input)
    torch.cuda.set_device(local_rank)
    dist = None
    comm = None
    if world > 1:
        import torch.distributed as dist

        # torch.distributed only for the rendezvous, barriers and the timing reduction; the
        # verdict all-gather goes through libmochi_hip's own RCCL communicator (mochi_comm)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        uid = [mh.Comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = mh.Comm(uid[0], world, rank, local_rank)

    # SURVEY §8d stream, unique grant bytes per certificate, signed on this GPU (k_rsa_sign)
    t_gen = time.perf_counter()
    synth = W.make_batch_unique(R, C, k, first_cert=c_lo, device=local_rank)
    if args.layout == "separate":
        synth = W.separate_copies(synth)
    gen_s = time.perf_counter() - t_gen
    moduli = [mh.pem_modulus(p) for p in W.load_keys(R)]
    if cpu_child is not None:
        os.makedirs(args.cache_dir, exist_ok=True)
        tmp = batch_file + ".tmp.npz"
        W.save_batch(tmp, W.head_certs(synth, cpu_certs))
        os.replace(tmp, batch_file)
    batch = synth.batch
    N = batch.n_grants

    ver = mh.Verifier(moduli, device=local_rank)
    ver.moduli = moduli  # for the second context of the pipelined wire leg
    dev = mh.DeviceBatch(batch, local_rank)
    out = mh.DeviceVerdicts(dev.n_grants, dev.n_certs, local_rank, full=True, n_ops=dev.n_ops)
    stream = torch.cuda.current_stream()
    words = mh.shard_words(plan)  # equal all-gather slots; this rank's bitmap fills the head of its slot
    out.cert_accept_bits = torch.zeros(words, dtype=torch.int32, device="cuda")
    gathered = torch.zeros(world * words, dtype=torch.int32, device="cuda")

    def step():
        ver.verify_device(dev, out, R, strict, stream=stream.cuda_stream)
        if comm is not None:  # the only collective: RCCL all-gather of the verdict bitmaps
            comm.allgather_bits(out.cert_accept_bits, gathered, stream.cuda_stream)
            return gathered
        return out.cert_accept_bits

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # correctness gate on this rank's shard (ground truth of the seeded fault mix)
    host = out.to_host()
    flags_ok = bool(np.array_equal(host.grant_flags, synth.expected_flags))

    ver.set_profiling(True)
    ev_s, wall = timed_steps(step, args.steps, 0, stream, dist)
    ver.set_profiling(False)
    prof = ver.read_profile()
    stage_ms = [prof[name] for name in ver.STAGES]
    t_max, wall_max, all_ok, total_grants_verified = reduce_over_ranks(dist, ev_s, wall, flags_ok, N, "cuda")
    value = total_grants_verified * args.steps / t_max

    result = None
    if rank == 0:
        # HBM bytes of one k_rsa_pow launch from the committed rocprofv3 PMC summary
        # (FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md), per grant x this launch's grants
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_rsa_pow.json")
        if os.path.exists(pmc):
            try:
                z = json.load(open(pmc))
                traffic = round(z["hbm_bytes_per_launch"] / z["grants_per_launch"] * N)
            except Exception:
                traffic = None
        if cpu_child is not None:
            cpu = finish_cpu_baseline(cpu_child)
            if os.path.exists(cpu_flags) and "error" not in cpu:
                z = np.load(cpu_flags)
                n = z["grant_flags"].shape[0]
                cpu["agrees_with_gpu"] = bool(np.array_equal(z["grant_flags"], host.grant_flags[:n]) and
                                              np.array_equal(z["cert_reason"], host.cert_reason[:z["cert_reason"].shape[0]]))
        else:
            cpu = None
        if os.path.exists(batch_file):
            os.remove(batch_file)
        extras = world == 1 and not args.headline_only  # side measurements: single-GPU runs only
        shard_leg = None
        if world == 1 and (args.shard_sizes or (extras and not args.no_shard_sizes)):
            shard_leg = shard_sizes_leg(args, ver, synth, C_total, R, strict, local_rank, stream, stage_ms[2])
        separate = separate_copies_leg(args, ver, synth, host, R, strict, local_rank, stream, t_max / args.steps) \
            if extras and not args.no_separate else None
        head = W.head_certs(synth, min(C, 1_000_000 // (R * k) * 4)) if extras else None  # ~4M grants
        hostp = host_path(ver, head.batch, R, strict) if extras else None
        wire_s = W.head_certs(synth, min(C, 250_000)) if extras and not args.no_wire else None
        wire = wire_path(ver, wire_s, R, strict, local_rank, stream, args) if wire_s is not None else None
        signing = sign_path(W.load_keys(1)[0], batch, local_rank, stream, args) if extras else None
        c3 = c3_leg(args, local_rank, stream) if extras and not args.no_c3 and args.config != "c3" else None
        cluster = cluster_leg(local_rank) if extras and not args.no_cluster else None
        result = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "grants/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_max / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic",
            "config": {
                "workload": f"{cfg['name']}: {total_grants_verified} SHA256withRSA-2048 signed grants "
                            f"({C_total} certificates) in total, R={R} (f={R // 3}), k={k} op/txn, "
                            f"{'server' if strict else 'client'} quorum predicate, 2.75% fault mix, unique grant "
                            "bytes per certificate (SURVEY §8d stream; signed on the GPU by k_rsa_sign, "
                            "bit-identical to OpenSSL)",
                "config": args.config,
                "workload_generation_s": round(gen_s, 2),
                "grants_total": total_grants_verified,
                "grants_per_gpu": N,
                "certs_per_gpu": C,
                "replication_factor": R,
                "majority": mh.majority(R),
                "parallelism": f"dp{world}: contiguous 32-aligned certificate shards (mochi_shard_plan) + one "
                               "RCCL all-gather of the verdict bitmaps through libmochi_hip (mochi_comm)"
                               if world > 1 else "dp1",
            },
            "roofline": roofline(N, stage_ms[2], traffic),
            "path_cios_equiv_vs_valu_peak": round(value / world * MAC_PER_GRANT / PEAK_MAC_PER_S, 4),
            "stage_ms": {"prep_sha256": round(stage_ms[0], 4), "bucket": round(stage_ms[1], 4),
                         "rsa_pow": round(stage_ms[2], 4), "rsa_final": round(stage_ms[3], 4),
                         "tally": round(stage_ms[4], 4),
                         "outside_serial_stages": round(t_max / args.steps * 1e3 - sum(stage_ms[1:]), 4),
                         "note": "prep_sha256 = k_grant_prep_cert + k_grant_prep_rare on the aux stream, "
                                 "launched beside k_rsa_pow (its blocks run in pow's tail; serialised before "
                                 "it with MOCHI_PREP_SERIAL=1): its span ends after pow's; "
                                 "outside_serial_stages = step - bucket - pow - final - tally"},
            "cpu_baseline": cpu,
            # the side legs in full; the compact `summary` below comes LAST so a tail of the line carries it
            "c3": c3,
            "shard_sizes": shard_leg,
            "c4_separate_copies": separate,
            "host_path_pcie_inclusive_grants_per_s": hostp["pinned_grants_per_s"] if hostp else None,
            "host_path": hostp,
            "write2_wire_path": wire,
            "producer_signing": signing,
            "cluster_c5_proxy": cluster,
            "wall_s": round(wall_max, 4),
            "correct_vs_ground_truth": all_ok,
            "prep_dedup": prep_dedup(batch) if rank == 0 else None,
        }
        result["summary"] = summary(result, stage_ms, t_max / args.steps * 1e3)
    if dist is not None:
        # the gathered bitmap is the whole batch's: rank 0 checks it holds its own shard's verdicts
        if rank == 0 and result is not None:
            result["gathered_bitmap_matches_rank0"] = gathered_matches_rank0(
                plan, gathered.cpu().numpy(), C_total, host.cert_accept, mh.bits_assemble, mh.unpack_bits)
        dist.barrier()
        comm.close()
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if getattr(args, "native_child", None) is not None and args.native_child.poll() is None:
        args.native_child.kill()  # the wire leg never wrote its input
    ver.close()


def summary(res, stage_ms, step_ms):
    """The figures a reader checks first, compact, as the line's last key: the
    headline's stage split and roofline fractions, the grant-prep dedup, the C3
    fractions, the per-rank shard sizes and the separate-copies C4 step."""
    def g(d, *path):
        for k in path:
            if not isinstance(d, dict) or k not in d:
                return None
            d = d[k]
        return d

    out = {"value": res["value"], "ms_per_step": res["ms_per_step"],
           "stage_ms": {k: round(v, 4) for k, v in zip(("prep_sha256", "bucket", "rsa_pow", "rsa_final", "tally"),
                                                      stage_ms)},
           "outside_serial_stages_ms": round(step_ms - sum(stage_ms[1:]), 4),
           "roofline_frac": g(res, "roofline", "frac"), "roofline_frac_implemented": g(res, "roofline", "implemented",
                                                                                          "frac"),
           "prep_dedup": {k: g(res, "prep_dedup", k) for k in ("grants", "prepped", "ratio")},
           "correct_vs_ground_truth": res["correct_vs_ground_truth"]}
    if res.get("c3"):
        out["c3"] = {k: {"grants_per_s": g(res, "c3", k, "grants_per_s"), "frac": g(res, "c3", k, "roofline", "frac")}
                     for k in ("server_gt", "client_ge")}
    if res.get("shard_sizes"):
        out["shard_sizes"] = [{"world": r["world"], "grants_per_s": r["grants_per_s"],
                               "pow_per_grant_vs_full": r["pow_per_grant_vs_full"], "frac": r["roofline_frac"]}
                              for r in res["shard_sizes"]["rows"]]
    sep = res.get("c4_separate_copies")
    if sep:
        out["c4_separate_copies"] = {k: sep.get(k) for k in ("grants_per_s", "ms_per_step", "vs_shared_layout",
                                                             "verdicts_equal_shared_layout", "flags_equal_ground_truth")}
        out["c4_separate_copies"]["stage_ms"] = sep.get("stage_ms")
    wire = res.get("write2_wire_path")
    if wire:
        out["write2_wire_grants_per_s"] = wire.get("grants_per_s")
        nat = g(wire, "batcher_native", "rows") or []
        out["batcher_native"] = [{"mode": r.get("mode"), "threads": r.get("threads"), "contexts": r.get("contexts"),
                                  "requests_per_s": r.get("requests_per_s"), "p50_us": g(r, "latency_us", "p50"),
                                  "mismatches": r.get("verdict_mismatches")} for r in nat]
    if res.get("cpu_baseline"):
        out["cpu_baseline_grants_per_s"] = g(res, "cpu_baseline", "value")
    return out


def separate_copies_leg(args, ver, synth, head_host, R, strict, dev, stream, head_step_s):
    """C4 with every grant its own copy of its bytes at a mixed alignment
    (workload.separate_copies: the layout of grant slices of received
    Write2ToServer messages -- each replica builds its own Grant,
    InMemoryDataStore.java:131-140, and the client ships all R MultiGrants,
    MochiDBClient.java:333-338), timed exactly like the headline.  Grant prep
    then finds a slot's equal grants by comparing bytes (no shared offsets).
    Its verdicts and per-op outputs must equal the headline's."""
    import numpy as np

    import mochi_hip as mh
    import workload as W

    t0 = time.perf_counter()
    sc = W.separate_copies(synth)
    build_s = time.perf_counter() - t0
    d = mh.DeviceBatch(sc.batch, dev)
    o = mh.DeviceVerdicts(d.n_grants, d.n_certs, dev, full=True, n_ops=d.n_ops)
    ver.set_profiling(True)
    ev_s, _ = timed_steps(lambda: ver.verify_device(d, o, R, strict, stream=stream.cuda_stream), args.steps,
                          args.warmup, stream)
    ver.set_profiling(False)
    prof = ver.read_profile()
    h = o.to_host()
    same = all(np.array_equal(getattr(h, k), getattr(head_host, k)) for k in
               ("grant_flags", "grant_ts", "cert_accept_bits", "cert_reason", "cert_fail_op", "op_decision", "op_g0",
                "op_ts"))
    n = sc.batch.n_grants
    step_s = ev_s / args.steps
    del d, o
    return {"grants_per_s": round(n * args.steps / ev_s, 1), "ms_per_step": round(step_s * 1e3, 4),
            "vs_shared_layout": round(head_step_s / step_s, 4),
            "stage_ms": {k: round(prof[k], 4) for k in ver.STAGES},
            "verdicts_equal_shared_layout": bool(same),
            "flags_equal_ground_truth": bool(np.array_equal(h.grant_flags, synth.expected_flags)),
            "blob_bytes": int(sc.batch.grant_bytes.nbytes), "layout_build_s": round(build_s, 2),
            "note": "every grant its own copy after 0-15 filler bytes; vs_shared_layout = headline step / this step"}


def c3_leg(args, dev, stream):
    """BASELINE.json C3: 7-server certificates (f = 2), 4M grants on one GPU, the
    quorum tally fused into the verify path; timed like the headline for the
    server predicate (count > M, 6-of-7, InMemoryDataStore.java:590) and the
    client one (count >= M, the '5-of-7', MochiDBClient.java:172,379)."""
    import numpy as np

    import mochi_hip as mh
    import workload as W

    R = 7
    C = W.n_certs_for_grants(CONFIGS["c3"]["grants"], R)
    t0 = time.perf_counter()
    s = W.make_batch_unique(R, C, 1, first_cert=0, device=dev)
    gen = time.perf_counter() - t0
    v = mh.Verifier([mh.pem_modulus(p) for p in W.load_keys(R)], device=dev)
    d = mh.DeviceBatch(s.batch, dev)
    o = mh.DeviceVerdicts(d.n_grants, d.n_certs, dev, full=True)
    res = {"workload": f"C3: {s.batch.n_grants} grants, {C} certificates, R=7 (M=5), unique grant bytes",
           "generation_s": round(gen, 2)}
    for name, strict in (("server_gt", True), ("client_ge", False)):
        v.set_profiling(True)
        # a longer warmup than the headline's: the leg starts right after 4M grants were signed on
        # the GPU (k_rsa_sign, ~1.5 s at full power) and the power-capped clock settles over it
        ev_s, _ = timed_steps(lambda: v.verify_device(d, o, R, strict, stream=stream.cuda_stream), args.steps,
                              max(args.warmup, 10), stream)
        v.set_profiling(False)
        prof = v.read_profile()
        h = o.to_host()
        res[name] = {"grants_per_s": round(s.batch.n_grants * args.steps / ev_s, 1),
                     "ms_per_step": round(ev_s / args.steps * 1e3, 4),
                     "accepted": int(h.cert_accept.sum()),
                     "flags_equal_ground_truth": bool(np.array_equal(h.grant_flags, s.expected_flags)),
                     "roofline": roofline(s.batch.n_grants, prof["rsa_pow"])}
    v.close()
    return res


def shard_sizes_leg(args, ver, synth, C_total, R, strict, dev, stream, head_pow_ms):
    """The per-GPU work of the headline at N = 2 / 4 / 8, measured on this GPU:
    rank 0's shard of the same C4 stream (mochi_shard_plan over the whole
    batch, contiguous from certificate 0 -- exactly what rank 0 verifies at
    that N), timed like the headline.  Reports grants/s, per-stage device ms
    and k_rsa_pow's per-grant cost against the full batch's (strong-scaling
    ceiling of one rank)."""
    import numpy as np

    import mochi_hip as mh
    import workload as W

    N_full = synth.batch.n_grants
    head_ns = head_pow_ms * 1e6 / N_full
    rows = []
    for world in (2, 4, 8):
        plan = mh.shard_plan(C_total, world)
        C0 = int(plan[1]) - int(plan[0])
        s = W.head_certs(synth, C0)
        d = mh.DeviceBatch(s.batch, dev)
        o = mh.DeviceVerdicts(d.n_grants, d.n_certs, dev, full=True, n_ops=d.n_ops)
        ver.set_profiling(True)
        ev_s, _ = timed_steps(lambda: ver.verify_device(d, o, R, strict, stream=stream.cuda_stream), args.steps,
                              max(1, args.warmup), stream)
        ver.set_profiling(False)
        prof = ver.read_profile()
        h = o.to_host()
        n = s.batch.n_grants
        pow_ns = prof["rsa_pow"] * 1e6 / n
        rows.append({"world": world, "grants": n, "certs": C0, "grants_per_s": round(n * args.steps / ev_s, 1),
                     "ms_per_step": round(ev_s / args.steps * 1e3, 4),
                     "stage_ms": {k: round(prof[k], 4) for k in ver.STAGES},
                     "pow_ns_per_grant": round(pow_ns, 4), "pow_per_grant_vs_full": round(pow_ns / head_ns, 4),
                     "roofline_frac": roofline(n, prof["rsa_pow"])["frac"],
                     "flags_equal_ground_truth": bool(np.array_equal(h.grant_flags, s.expected_flags))})
        del d, o
    return {"rows": rows, "full_pow_ns_per_grant": round(head_ns, 4),
            "note": "rank 0's shard of the C4 stream at each N, on this one GPU (strong scaling: what each rank "
                    "runs); pow_per_grant_vs_full = k_rsa_pow ns/grant at that size / at 16M"}


def prep_dedup(batch):
    """Grants k_grant_prep_cert + k_grant_prep_rare parse and hash:
    the first grant of each (certificate, key slot) plus every later grant of the
    slot whose bytes differ from it (in the SoA stream a distinct byte string is
    stored once per certificate, so equal bytes <=> equal offset and length)."""
    import numpy as np

    cgo = np.asarray(batch.cert_grant_off, np.int64)
    n = int(cgo[-1])
    cert = np.repeat(np.arange(len(cgo) - 1, dtype=np.int64), np.diff(cgo))
    key = cert * 256 + np.asarray(batch.grant_key[:n], np.int64)
    _, first, inv = np.unique(key, return_index=True, return_inverse=True)
    lead = first[inv]
    off = np.asarray(batch.grant_off[:n], np.uint64)
    ln = np.asarray(batch.grant_len[:n], np.uint32)
    rare = int(np.count_nonzero((off != off[lead]) | (ln != ln[lead])))
    return {"grants": n, "prepped": int(len(first)) + rare, "leaders": int(len(first)), "rare": rare,
            "ratio": round((len(first) + rare) / max(1, n), 4),
            "note": "grants parsed + SHA-256'd per step; every other grant takes its slot leader's results"}


def host_path(ver, batch, R, strict, reps=3):
    """PCIe-inclusive rate of mochi_verify_batch (host buffers in, verdicts out):
    the chunked upload/compute/download pipeline timed by its own stream events
    (first H2D start -> last D2H end), best of `reps`, for pinned in-place arrays
    (mochi_host_alloc, the intended drop-in layout) and for pageable arrays
    (staged through pinned buffers; `wall` also counts that host memcpy)."""
    N = batch.n_grants
    out = {}
    pinned = batch.pinned()
    for name, b in (("pinned", pinned), ("pageable", batch)):
        best_dev, best_wall = float("inf"), float("inf")
        for _ in range(reps):
            t0 = time.perf_counter()
            v = ver.verify(b, R, strict)
            best_wall = min(best_wall, time.perf_counter() - t0)
            best_dev = min(best_dev, v.timing_ms["total"] / 1e3)
        out[f"{name}_grants_per_s"] = round(N / best_dev, 1)
        out[f"{name}_wall_grants_per_s"] = round(N / best_wall, 1)
    out["note"] = "chunked pipeline, 262144-grant chunks; device-event span unless *_wall_*"
    return out


def wire_path(ver, synth, R, strict, dev, stream, args):
    """Device-resident Write2ToServer wire messages -> verdicts (mochi_verify_write2_device):
    the device protobuf decode (k_w2_count + scans + k_w2_emit) + the same verify
    path + status fix-up, timed like the headline (events around K calls).
    Reported beside the headline; the headline stays the SoA batch path."""
    import numpy as np
    import torch

    import mochi_hip as mh
    import workload as W

    t0 = time.perf_counter()
    wb = W.encode_wire_batch(synth)
    enc_s = time.perf_counter() - t0
    ver.set_server_ids(W.SERVER_IDS[:R])
    dwb = mh.DeviceWireBatch(wb, dev)
    out = mh.DeviceVerdicts(0, wb.n_msgs, dev, full=True)
    out.grant_flags = out.grant_ts = None
    for _ in range(max(1, args.warmup)):
        ver.verify_write2_device(dwb, out, R, strict, stream=stream.cuda_stream)
    torch.cuda.synchronize()
    host = out.to_host()
    ref = ver.verify(synth.batch, R, strict)
    same = bool(np.array_equal(host.cert_reason, ref.cert_reason) and
                np.array_equal(host.cert_accept_bits, ref.cert_accept_bits) and
                int(dwb.status.max().item()) == 0)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(args.steps):
        ver.verify_write2_device(dwb, out, R, strict, stream=stream.cuda_stream)
    e1.record(stream)
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 1e3 / args.steps
    N = synth.batch.n_grants
    pipe = wire_pipelined(ver, dwb, R, strict, dev, args, N, host)
    # PCIe-inclusive: host wire bytes in, verdicts out (mochi_verify_write2's chunked pipeline)
    best_dev, best_wall, host_same = float("inf"), float("inf"), True
    for _ in range(3):
        t0 = time.perf_counter()
        hv, hst = ver.verify_write2(wb, R, strict)
        best_wall = min(best_wall, time.perf_counter() - t0)
        best_dev = min(best_dev, hv.timing_ms["total"] / 1e3)
        host_same &= bool(np.array_equal(hv.cert_reason, host.cert_reason))
    # the same with the wire batch in pinned memory (mochi_host_alloc): DMA'd in place, no staging copy
    pwb, keep = pinned_wire(wb)
    best_pdev, best_pwall, pin_same = float("inf"), float("inf"), True
    for _ in range(3):
        t0 = time.perf_counter()
        hv, hst = ver.verify_write2(pwb, R, strict)
        best_pwall = min(best_pwall, time.perf_counter() - t0)
        best_pdev = min(best_pdev, hv.timing_ms["total"] / 1e3)
        pin_same &= bool(np.array_equal(hv.cert_reason, host.cert_reason))
    del pwb, keep
    del dwb, out
    ver2 = mh.Verifier(ver.moduli, device=dev)  # a second context: two batches in flight
    ver2.set_server_ids(W.SERVER_IDS[:R])
    batch_legs = [batcher_leg(vs, wb, synth.batch.cert_grant_off, R, strict, th, host)
                  for vs in ([ver], [ver, ver2]) for th in (2, 20)]
    async_leg = batcher_async_leg([ver, ver2], wb, synth.batch.cert_grant_off, R, strict, host)
    ver2.close()
    native = batcher_native_leg(args, wb, R, host, synth.batch.cert_grant_off)
    return {"grants_per_s": round(N / t, 1), "ms_per_step": round(t * 1e3, 4), "messages": wb.n_msgs,
            "wire_bytes": int(wb.wire.nbytes), "verdicts_equal_soa_path": same,
            "host_encode_s": round(enc_s, 2),
            "note": "Write2ToServer bodies resident in HBM; includes one host wait on the decoded totals per step",
            "pipelined_2ctx": pipe,
            "host_pcie_inclusive_pinned": {"grants_per_s": round(N / best_pdev, 1),
                                           "wall_grants_per_s": round(N / best_pwall, 1),
                                           "wire_gb_per_s": round(wb.wire.nbytes / best_pdev / 1e9, 2),
                                           "verdicts_equal": pin_same,
                                           "note": "wire bytes, offsets, hashes and op flags in mochi_host_alloc memory: "
                                                   "DMA'd in place by the chunked pipeline"},
            "host_pcie_inclusive": {"grants_per_s": round(N / best_dev, 1), "wall_grants_per_s": round(N / best_wall, 1),
                                    "verdicts_equal": host_same,
                                    "note": "mochi_verify_write2: pageable wire bytes staged + chunked H2D / decode+"
                                            "verify / D2H pipeline; device-event span, wall includes host staging"},
            "batcher": batch_legs, "batcher_async": async_leg, "batcher_native": native}


def pinned_wire(wb):
    """A copy of the WireBatch whose arrays live in mochi_host_alloc memory."""
    import copy

    import numpy as np

    import mochi_hip as mh

    keep = []

    def pin(a):
        if a is None:
            return None
        a = np.ascontiguousarray(a)
        h = mh.PinnedHost(a.nbytes)
        keep.append(h)
        v = h.view()[:a.nbytes].view(a.dtype).reshape(a.shape)
        v[...] = a
        return v

    p = copy.copy(wb)
    for k in ("wire", "msg_off", "msg_len", "op_flags_off", "op_flags", "expected_hash", "op_object_ts"):
        setattr(p, k, pin(getattr(wb, k)))
    return p, keep


def batcher_leg(vers, wb, cert_grant_off, R, strict, threads, ref, max_msgs=4096, max_wait_us=100, n_req=20000):
    """The drop-in as a MochiDB server would drive it (C5 proxy): `threads` worker
    threads -- the reference's request pool is core 2 / max 20
    (MochiServer.java:36-40) -- each blocking in mochi_batcher_verify on one
    Write2ToServer body at a time (host bytes in, verdict out); the batcher
    coalesces whatever is in flight into one GPU call (one batch in flight per
    context in `vers`).  Reports per-request latency percentiles and throughput."""
    import threading

    import numpy as np

    import mochi_hip as mh

    M = min(wb.n_msgs, n_req)
    msgs = [wb.wire[int(wb.msg_off[i]):int(wb.msg_off[i]) + int(wb.msg_len[i])].tobytes() for i in range(M)]
    hashes = [wb.expected_hash[i].tobytes() for i in range(M)]
    b = mh.Batcher(vers, R, strict, max_msgs=max_msgs, max_wait_us=max_wait_us)
    lat = [[] for _ in range(threads)]
    res = [None] * M

    def worker(tid):
        for i in range(tid, M, threads):
            t0 = time.perf_counter()
            res[i] = b.verify(msgs[i], hashes[i])
            lat[tid].append(time.perf_counter() - t0)

    for i in range(min(M, 64)):  # warm
        b.verify(msgs[i], hashes[i])
    nb0, nm0 = b.stats()
    th = [threading.Thread(target=worker, args=(x,)) for x in range(threads)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    wall = time.perf_counter() - t0
    nb, nm = b.stats()
    b.close()
    ls = np.sort(np.concatenate([np.asarray(x) for x in lat])) * 1e6
    reasons = np.array([r[1] for r in res], np.uint8)
    n_grants = int(cert_grant_off[M])
    return {"threads": threads, "contexts": len(vers), "requests": M, "requests_per_s": round(M / wall, 1),
            "grants_per_s": round(n_grants / wall, 1),
            "latency_us": {"p50": round(float(np.percentile(ls, 50)), 1), "p99": round(float(np.percentile(ls, 99)), 1),
                           "max": round(float(ls[-1]), 1)},
            "gpu_batches": nb - nb0, "mean_batch_msgs": round((nm - nm0) / max(1, nb - nb0), 2),
            "verdicts_equal_one_shot": bool(np.array_equal(reasons, ref.cert_reason[:M])),
            "max_wait_us": max_wait_us}


def batcher_async_leg(vers, wb, cert_grant_off, R, strict, ref, n_req=100000, window=8192, max_msgs=4096,
                      max_wait_us=200):
    """The event-loop form (mochi_batcher_submit): one producer thread keeps up to
    `window` Write2ToServer bodies in flight and each completion callback frees a
    slot -- how a Netty handler completing futures would drive the library.
    Reports requests/s, grants/s and submit->callback latency percentiles."""
    import threading

    import numpy as np

    import mochi_hip as mh

    M = min(wb.n_msgs, n_req)
    msgs = [wb.wire[int(wb.msg_off[i]):int(wb.msg_off[i]) + int(wb.msg_len[i])].tobytes() for i in range(M)]
    hashes = [wb.expected_hash[i].tobytes() for i in range(M)]
    b = mh.Batcher(vers, R, strict, max_msgs=max_msgs, max_wait_us=max_wait_us)
    slots = threading.Semaphore(window)
    t_sub = np.zeros(M)
    lat = np.zeros(M)
    reasons = np.zeros(M, np.uint8)
    left = [M]
    cv = threading.Condition()

    def done_for(i):
        def done(rc, accepted, reason, fail_op, status):
            lat[i] = time.perf_counter() - t_sub[i]
            reasons[i] = reason if rc == mh.OK else 255
            slots.release()
            with cv:
                left[0] -= 1
                if left[0] == 0:
                    cv.notify()
        return done

    nb0, nm0 = b.stats()
    t0 = time.perf_counter()
    for i in range(M):
        slots.acquire()
        t_sub[i] = time.perf_counter()
        b.submit(msgs[i], hashes[i], done_for(i))
    with cv:
        cv.wait_for(lambda: left[0] == 0, timeout=300)
    wall = time.perf_counter() - t0
    nb, nm = b.stats()
    b.close()
    ls = np.sort(lat) * 1e6
    return {"requests": M, "contexts": len(vers), "window": window, "requests_per_s": round(M / wall, 1),
            "grants_per_s": round(int(cert_grant_off[M]) / wall, 1),
            "latency_us": {"p50": round(float(np.percentile(ls, 50)), 1),
                           "p99": round(float(np.percentile(ls, 99)), 1)},
            "gpu_batches": nb - nb0, "mean_batch_msgs": round((nm - nm0) / max(1, nb - nb0), 1),
            "verdicts_equal_one_shot": bool(np.array_equal(reasons, ref.cert_reason[:M])),
            "note": "one Python producer thread (ctypes call + callback per request bound the rate)"}


# the reference's Write2 pool is core 2 / max 20 on an unbounded queue (MochiServer.java:36-39,51-52),
# so it runs 2 workers: sync:2 is the blocking drop-in at that concurrency, async:2 the same 2 workers
# submitting and completing each request from the callback (INTEGRATION.md's handler form)
NATIVE_CONFIGS = ["sync:2:1::20000", "sync:2:2::20000", "async:2:1:16384:400000", "async:2:2:16384:400000",
                  "sync:20:1::40000", "sync:20:2::40000", "sync:64:2::100000", "async:4:2:16384:400000"]


def start_batcher_native(args, input_path):
    """microbench/batcher_load: native threads calling mochi_batcher_verify (2, 20
    and 64 of them -- the reference's worker pool is core 2 / max 20,
    MochiServer.java:36-40) and an event-loop form on mochi_batcher_submit, over
    real Write2ToServer bodies.  Started before this process uses the GPU; it
    waits for `input_path`."""
    import subprocess

    exe = os.path.join(ROOT, "microbench", "batcher_load")
    if not os.path.exists(exe):
        return None
    os.makedirs(args.cache_dir, exist_ok=True)
    cfgs = [c.replace("::", ":8192:") for c in NATIVE_CONFIGS]
    return subprocess.Popen([exe, input_path, "20000", "4096", "100"] + cfgs, stdout=subprocess.PIPE,
                            stderr=subprocess.PIPE, text=True)


def write_native_input(path, wb, R, ref):
    """The driver's input (format in microbench/batcher_load.cpp): keys, server ids,
    the Write2ToServer bodies and the expected verdict of each (the device one-shot
    path's, itself equal to the oracle's in tests/test_write2_wire_gpu.py)."""
    import struct

    import numpy as np

    import mochi_hip as mh
    import workload as W

    ids, id_off = W.server_id_table(R)
    moduli = b"".join(mh.pem_modulus(p) for p in W.load_keys(R))
    M = wb.n_msgs
    off = np.ascontiguousarray(wb.msg_off, np.uint64)
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(b"MOCHIW2\0" + struct.pack("<II", R, M) + moduli)
        f.write(struct.pack("<I", ids.nbytes) + ids.tobytes() + np.ascontiguousarray(id_off, np.uint32).tobytes())
        f.write(struct.pack("<Q", wb.wire.nbytes) + wb.wire.tobytes() + off.tobytes())
        f.write(np.ascontiguousarray(wb.msg_len, np.uint32).tobytes() + np.ascontiguousarray(wb.expected_hash).tobytes())
        f.write(ref.cert_reason[:M].astype(np.uint8).tobytes() + ref.cert_accept[:M].astype(np.uint8).tobytes())
    os.replace(tmp, path)


def batcher_native_leg(args, wb, R, ref, cert_grant_off):
    child = getattr(args, "native_child", None)
    if child is None:
        return None
    try:
        write_native_input(args.native_input, wb, R, ref)
        out, err = child.communicate(timeout=600)
    except Exception as ex:  # reported, never required
        child.kill()
        return {"error": f"batcher_load failed: {ex}"}
    finally:
        if os.path.exists(args.native_input):
            os.remove(args.native_input)
    rows = []
    for line in out.splitlines():
        try:
            r = json.loads(line)
        except ValueError:
            continue
        r["grants_per_s"] = round(r["requests_per_s"] * float(cert_grant_off[-1]) / max(1, len(cert_grant_off) - 1), 1)
        rows.append(r)
    res = {"rows": rows, "messages": wb.n_msgs, "rc": child.returncode,
           "verdicts_equal_one_shot": bool(rows) and all(r["verdict_mismatches"] == 0 for r in rows),
           "note": "microbench/batcher_load: native threads, no Python on the request path; request i sends "
                   "message i % M; max_msgs 4096, max_wait 100 us"}
    if child.returncode not in (0, 3):
        res["stderr"] = err[-2000:]
    return res


def cluster_leg(dev, clients=256, txns_per_client=8, keys=2000, seed=11, backend="device"):
    """In-process 4-server cluster from the reference's config/sample_config
    (tests/cluster_harness.py) under a write-heavy multi-client KV load -- the C5
    configuration's proxy (no JVM here): every Write1 grant signed on the device
    (k_rsa_sign), Write1 rounds classified and responses tallied on the device,
    every Write2 certificate verified through the batcher's request API with the
    receiving server's stored state, its per-op decisions applied to the model.
    Reports transactions/s and per-transaction latency (Write1 -> result)."""
    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import cluster_harness as H

    c = H.Cluster(backend=backend, seed=seed, device=dev, max_wait_us=50)
    rng = np.random.default_rng(seed)
    t_done, lat, errors = [], [], []
    n_reads = [0]

    def script(cl):
        import time as _t
        written = []
        for j in range(txns_per_client):
            t0 = _t.perf_counter()
            try:
                if written and rng.random() < 0.1:  # read back a key this client wrote (a never-written key
                    # has no container on the servers: processRead throws, the reference client hangs)
                    r = yield ("read", H.read_ops(written[int(rng.integers(0, len(written)))]))
                    n_reads[0] += 1
                else:
                    nk = 1 if rng.random() < 0.7 else 2
                    ks = sorted({f"DEMO_KEY_STRESS_TEST_{int(x)}" for x in rng.integers(0, keys, nk)})
                    r = yield ("write", H.write_ops(*[(k, f"v{cl.id}-{j}") for k in ks]))
                    written.extend(ks)
            except H.ClientError as ex:  # the reference client's exception for this transaction
                errors.append(type(ex).__name__)
                continue
            lat.append(_t.perf_counter() - t0)

    # warm the contexts (first launches, buffer sizing)
    H.run_clients(c, [H.ScriptedClient(c, lambda cl: (yield ("write", H.write_ops(("WARM", "x")))))])
    st0 = dict(c.stats)
    t0 = time.perf_counter()
    cl = [H.ScriptedClient(c, script) for _ in range(clients)]
    try:
        H.run_clients(c, cl)
    except H.Hung as ex:
        errors.append(str(ex))
    wall = time.perf_counter() - t0
    st = {k: c.stats[k] - st0.get(k, 0) for k in c.stats}
    nb, nm = c.batcher.stats() if c.batcher else (0, 0)
    c.close()
    ls = np.sort(np.asarray(lat)) * 1e3 if lat else np.zeros(1)
    n = len(lat)
    return {"clients": clients, "transactions": n, "reads": n_reads[0], "transactions_per_s": round(n / wall, 1),
            "write2_verifies_per_s": round(st["write2"] / wall, 1), "grants_signed_per_s": round(st["signed"] / wall, 1),
            "latency_ms": {"p50": round(float(np.percentile(ls, 50)), 2), "p99": round(float(np.percentile(ls, 99)), 2)},
            "write1_retries": st["retries"], "read_branch_ops": st["read_branch"], "scheduler_steps": st["steps"],
            "client_errors": errors[:8], "n_client_errors": len(errors), "batcher_batches": nb,
            "mean_batch_msgs": round(nm / max(1, nb), 1),
            "note": "R=4 replicas of config/sample_config, 90% writes (70% 1-key, 30% 2-key), 10% reads over "
                    f"{keys} keys; deterministic scheduler delivering random subsets of in-flight messages per step; "
                    "wall clock includes the Python server/client models"}


def wire_pipelined(ver, dwb, R, strict, dev, args, N, ref_host):
    """Two batches in flight: a second context (own streams and scratch) driven by a
    second host thread, so one batch's latency-bound decode runs beside the other's
    k_rsa_pow -- how a server keeps the GPU busy with back-to-back batches (the
    batcher's next batch accumulates while one is on the GPU).  Wall-clock over
    2 x steps batches, both streams synchronised on both sides."""
    import copy
    import threading

    import numpy as np
    import torch

    import mochi_hip as mh
    import workload as W

    ver_b = mh.Verifier(ver.moduli, device=dev)
    ver_b.set_server_ids(W.SERVER_IDS[:R])
    dwb_b = copy.copy(dwb)  # same read-only wire bytes, own status array
    dwb_b.status = torch.zeros_like(dwb.status)
    lanes = [(ver, dwb, torch.cuda.Stream(dev)), (ver_b, dwb_b, torch.cuda.Stream(dev))]
    outs = [mh.DeviceVerdicts(0, dwb.n_msgs, dev, full=True) for _ in lanes]
    for o in outs:
        o.grant_flags = o.grant_ts = None
    errs = []

    def run(i, n):
        v, d, st = lanes[i]
        try:
            for _ in range(n):
                v.verify_write2_device(d, outs[i], R, strict, stream=st.cuda_stream)
            st.synchronize()
        except Exception as e:  # surfaced after join
            errs.append(e)

    def both(n):
        th = [threading.Thread(target=run, args=(i, n)) for i in range(2)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        if errs:
            raise errs[0]

    both(max(1, args.warmup))
    same = all(np.array_equal(o.to_host().cert_reason, ref_host.cert_reason) for o in outs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    both(args.steps)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ver_b.close()
    t = wall / (2 * args.steps)
    return {"grants_per_s": round(N / t, 1), "ms_per_batch": round(t * 1e3, 4), "contexts": 2,
            "batches": 2 * args.steps, "verdicts_equal": bool(same), "timing": "host wall clock"}


def sign_path(pem, batch, dev, stream, args, n_gpu=262144, n_cpu=16384):
    """Producer side (Write1 signing site): SHA256withRSA-2048 of grants with one
    server key on the device (k_rsa_sign, CRT) vs OpenSSL on the host cores."""
    import numpy as np
    import torch

    import mochi_hip as mh

    n = min(n_gpu, batch.n_grants)
    off = np.ascontiguousarray(batch.grant_off[:n], np.uint64)
    ln = np.ascontiguousarray(batch.grant_len[:n], np.uint32)
    d = torch.device("cuda", dev)
    blob_t = torch.from_numpy(np.ascontiguousarray(batch.grant_bytes)).to(d)
    off_t = torch.from_numpy(off.view(np.int64)).to(d)
    len_t = torch.from_numpy(ln.view(np.int32)).to(d)
    sig_t = torch.empty((n, 256), dtype=torch.uint8, device=d)
    s = mh.DeviceSigner(pem, dev)
    s.sign_device(blob_t, off_t, len_t, n, sig_t, stream.cuda_stream)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 3
    e0.record(stream)
    for _ in range(reps):
        s.sign_device(blob_t, off_t, len_t, n, sig_t, stream.cuda_stream)
    e1.record(stream)
    torch.cuda.synchronize()
    t_gpu = e0.elapsed_time(e1) / 1e3 / reps
    got = sig_t[:64].cpu().numpy()
    s.close()
    threads = min(16, os.cpu_count() or 1)
    t0 = time.perf_counter()
    ref = mh.sign_grants(pem, batch.grant_bytes, off[:n_cpu], ln[:n_cpu], threads)
    t_cpu = time.perf_counter() - t0
    return {"gpu_signatures_per_s": round(n / t_gpu, 1), "gpu_ms_per_launch": round(t_gpu * 1e3, 3), "grants": n,
            "cpu_signatures_per_s": round(n_cpu / t_cpu, 1), "cpu_threads": threads, "cpu_sample": n_cpu,
            "bit_exact_sample": bool(np.array_equal(got, ref[:64]))}


def start_cpu_baseline(args, R, k, flags_out, batch_file):
    """The oracle (OpenSSL SHA256withRSA verify + the restated quorum logic)
    timed on this host's cores over a bounded sample of the same workload (the
    stream's first certificates), in a child process (tests/cpu_baseline.py)
    that forks its workers without any HIP state; it waits for the sample file
    the parent writes after generating the stream on the GPU."""
    import subprocess

    os.makedirs(args.cache_dir, exist_ok=True)
    cmd = [sys.executable, os.path.join(ROOT, "tests", "cpu_baseline.py"), "--replication", str(R), "--ops-per-txn",
           str(k), "--cache-dir", args.cache_dir, "--seconds", str(args.cpu_seconds), "--runs", str(args.cpu_runs),
           "--flags-out", flags_out, "--batch-file", batch_file, "--stream", args.config.upper()]
    if args.client_predicate:
        cmd.append("--client-predicate")
    return subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)


def finish_cpu_baseline(child):
    try:
        out, err = child.communicate(timeout=900)
        return json.loads(out.strip().splitlines()[-1])
    except Exception as ex:  # the baseline is reported, never required
        child.kill()
        return {"error": f"cpu baseline failed: {ex}"}


if __name__ == "__main__":
    main()
