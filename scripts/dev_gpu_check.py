import sys, time, os
sys.path.insert(0, 'mochi-db_amd'); sys.path.insert(0, 'tests')
import numpy as np
import workload as W, oracle_ffi as O, mochi_hip as mh
pool = W.build_pool(R=4, k=1, P=256, P_f=64, cache_dir='/tmp/mochi_cache')
s = W.make_batch(pool, 2000)
b = s.batch
v = O.verify_batch(pool.moduli, b, 4, True, 8)
ver = mh.Verifier(pool.moduli, 0)
t = time.time(); g = ver.verify(b, 4, True); print('gpu first call', time.time()-t, g.timing_ms, flush=True)
print('flags equal', np.array_equal(g.grant_flags, v.grant_flags), 'ts equal', np.array_equal(g.grant_ts, v.grant_ts))
print('valid bits equal', np.array_equal(g.grant_valid_bits, v.grant_valid_bits))
print('accept equal', np.array_equal(g.cert_accept_bits, v.cert_accept_bits), 'reason equal', np.array_equal(g.cert_reason, v.cert_reason), 'failop eq', np.array_equal(g.cert_fail_op, v.cert_fail_op))
print('gpu flags hist', np.bincount(g.grant_flags, minlength=4), 'oracle', np.bincount(v.grant_flags, minlength=4))
bad = np.nonzero(g.grant_flags != v.grant_flags)[0]
print('mismatch idx', bad[:10])
# timing on a bigger batch
s2 = W.make_batch(pool, 250000)
for i in range(3):
    g2 = ver.verify(s2.batch, 4, True); print('N', s2.batch.n_grants, g2.timing_ms, flush=True)
print('big flags match expected', np.array_equal(g2.grant_flags, s2.expected_flags))
