#!/usr/bin/env python3
"""CPU baseline for bench.py: the oracle verifier timed on this host's cores.

Runs as its own process (bench.py starts it with subprocess before touching
the GPU), so its worker processes are forked from a process that never
initialised HIP.  OpenSSL 3.0 serialises threads of one process on shared
provider state (8 threads: ~1.4x one thread here), so the grant signatures are
split over worker PROCESSES, as `openssl speed -multi` does; the certificate
tally (restated InMemoryDataStore.java:576-640) then runs in the parent and is
included in the timed region.

Prints one JSON object; with --flags-out also saves the grant flags / reasons
so bench.py can check them against the GPU's verdicts for the same grants.
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mochi-db_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

_G = {}


def _work(rng):
    import oracle_ffi as O

    b, e = rng
    flags, ts = O.verify_grants(_G["moduli"], _G["batch"], b, e, 1)
    return b, e, flags[b:e].copy(), ts[b:e].copy()


def _wait_for(path, timeout_s=900):
    t0 = time.time()
    while not os.path.exists(path):
        if time.time() - t0 > timeout_s:
            raise TimeoutError(path)
        time.sleep(0.2)


def cpu_share():
    """Worker count: every CPU this process may run on, capped by the job's CPU
    share when the host declares one (the GPU pool gives a 1-GPU job 16 CPUs and
    exports OMP_NUM_THREADS=16; nproc there reports the whole machine)."""
    aff = len(os.sched_getaffinity(0))
    share = os.environ.get("OMP_NUM_THREADS")
    n = min(aff, int(share)) if share and share.isdigit() and int(share) > 0 else aff
    return max(1, n), aff, os.cpu_count() or aff, share


def run(R, k, cache_dir, n_certs, procs, seconds, runs, strict, flags_out=None, batch_file=None, stream="C4",
        pool_size=4096):
    import numpy as np

    import mochi_hip as mh
    import oracle_ffi as O
    import workload as W

    if batch_file:
        # the bench's own stream (unique grants, signed on the GPU by the parent
        # process); this process never touches the GPU
        _wait_for(batch_file)
        full = W.load_batch(batch_file)
        moduli = [mh.pem_modulus(p) for p in W.load_keys(R)]
        probe = W.head_certs(full, 256)
        make = lambda n: W.head_certs(full, n)
        n_certs = min(n_certs, full.batch.n_certs)
    else:
        pool = W.build_pool(R=R, k=k, P=pool_size, P_f=256, cache_dir=cache_dir)
        moduli = pool.moduli
        probe = W.make_batch(pool, 256)
        make = lambda n: W.make_batch(pool, n)
    # calibrate: one process, a few hundred grants
    t0 = time.perf_counter()
    O.verify_grants(moduli, probe.batch, 0, probe.batch.n_grants, 1)
    rate1 = probe.batch.n_grants / max(1e-6, time.perf_counter() - t0)
    want = int(rate1 * seconds / (R * k))  # `seconds` of CPU work (core-seconds) per run
    n = max(64, min(n_certs, want))
    s = make(n)
    N = s.batch.n_grants
    _G["moduli"], _G["batch"] = moduli, s.batch.normalized()
    chunks = max(procs * 4, 1)
    ranges = [(N * i // chunks, N * (i + 1) // chunks) for i in range(chunks)]
    ctx = mp.get_context("fork")
    times = []
    with ctx.Pool(procs) as p:
        p.map(_work, ranges[:procs])  # warm the workers (library load, key setup)
        for _ in range(max(1, runs)):
            t0 = time.perf_counter()
            flags = np.zeros(N, np.uint8)
            ts = np.zeros(N, np.int64)
            for b, e, f, t in p.imap_unordered(_work, ranges):
                flags[b:e] = f
                ts[b:e] = t
            v = O.tally(s.batch, flags, ts, R, strict)
            times.append(time.perf_counter() - t0)
    dt = float(np.median(times))
    if flags_out:
        np.savez(flags_out, grant_flags=flags, cert_reason=v.cert_reason, cert_accept_bits=v.cert_accept_bits)
    cpu = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    cpu = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    _, aff, nproc, share = cpu_share()
    return {
        "value": round(N / dt, 1),
        "unit": "grants/s",
        "cores": procs,
        "kind": "port",
        "sample": f"first {n} certificates ({N} grants) of the {stream} stream (unique grants); OpenSSL 3.0.2 SHA-256 + "
                  f"RSA-2048 PKCS#1 v1.5 verify per grant + restated InMemoryDataStore.java:576-640 tally; {procs} "
                  f"worker processes on '{cpu}' (nproc {nproc}, affinity {aff}, job CPU share "
                  f"OMP_NUM_THREADS={share}); median of {len(times)} runs, {dt:.2f} s wall each = "
                  f"{dt * procs:.1f} core-seconds",
        "runs_s": [round(x, 3) for x in times],
        "single_core_grants_per_s": round(rate1, 1),
        "whole_host_extrapolated_grants_per_s": round(N / dt / procs * nproc, 1),
        "nproc": nproc,
        "n_certs": n,
        "n_grants": N,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replication", type=int, default=4)
    ap.add_argument("--ops-per-txn", type=int, default=1)
    ap.add_argument("--pool", type=int, default=4096)
    ap.add_argument("--cache-dir", default="/tmp/mochi_bench_cache")
    ap.add_argument("--max-certs", type=int, default=250_000)
    ap.add_argument("--procs", type=int, default=0)
    ap.add_argument("--seconds", type=float, default=12.0, help="CPU work (core-seconds) per timed run")
    ap.add_argument("--runs", type=int, default=5)
    ap.add_argument("--client-predicate", action="store_true")
    ap.add_argument("--flags-out", default=None)
    ap.add_argument("--batch-file", default=None, help="wait for and load this saved batch (bench's unique stream)")
    ap.add_argument("--stream", default="C4")
    a = ap.parse_args()
    procs = a.procs or cpu_share()[0]
    res = run(a.replication, a.ops_per_txn, a.cache_dir, a.max_certs, procs, a.seconds, a.runs,
              not a.client_predicate, a.flags_out, a.batch_file, a.stream, a.pool)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
