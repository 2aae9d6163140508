"""The vectorized bench-stream encoder (workload.encode_grants_vec) produces exactly
Grant.toByteArray() (MochiProtocol.java:7556-7574) -- checked against the scalar
encoder and the oracle's restated Grant.writeTo on every length class."""
import hashlib

import numpy as np

import oracle_ffi as O
import workload as W


def test_encode_grants_vec_matches_scalar_encoder():
    rng = np.random.default_rng(5)
    n = 3000
    oid = rng.integers(0, 200, n)
    ts = np.concatenate([[0, 1, 127, 128, 16383, 16384, (1 << 21) - 1], rng.integers(0, 64000, n - 7)])
    hashes = np.frombuffer(b"".join(hashlib.sha512(f"t{i}".encode()).hexdigest().encode() for i in range(n)),
                           np.uint8).reshape(n, 128)
    blob, off, ln = W.encode_grants_vec(oid, ts, hashes)
    for i in range(n):
        exp = W.encode_grant(f"DEMO_KEY_STRESS_TEST_{oid[i]}", int(ts[i]), hashes[i].tobytes().decode())
        got = blob[int(off[i]):int(off[i]) + int(ln[i])].tobytes()
        assert got == exp, i
        if i % 97 == 0:
            assert got == O.grant_encode(f"DEMO_KEY_STRESS_TEST_{oid[i]}".encode(), int(ts[i]), hashes[i].tobytes())
    assert int(off[-1] + ln[-1]) == blob.size


def test_txn_hashes():
    h = W._txn_hashes(np.array([0, 5, 123456789], np.uint64))
    assert h[1].tobytes().decode() == hashlib.sha512(b"txn-5").hexdigest()
    assert h[2].tobytes().decode() == W.txn_hash_hex(123456789)


def test_separate_copies_layout(tmp_path):
    """workload.separate_copies: every grant its own copy at a mixed alignment, the same
    bytes per grant, and the oracle's verdicts unchanged (the C4 separate-copy leg)."""
    import numpy as np

    import oracle_ffi as O
    import workload as W

    pool = W.build_pool(R=4, k=2, P=64, P_f=16, cache_dir=str(tmp_path))
    s = W.make_batch(pool, 700, first_cert=5)
    t = W.separate_copies(s)
    b, c = s.batch, t.batch
    for i in range(b.n_grants):
        x = b.grant_bytes[int(b.grant_off[i]):int(b.grant_off[i]) + int(b.grant_len[i])]
        y = c.grant_bytes[int(c.grant_off[i]):int(c.grant_off[i]) + int(c.grant_len[i])]
        assert np.array_equal(x, y)
    assert len(np.unique(c.grant_off)) == c.n_grants  # no two grants share a copy
    assert len(set((c.grant_off % 16).tolist())) == 16  # every alignment occurs
    v1 = O.verify_batch(pool.moduli, b, 4, True, 4)
    v2 = O.verify_batch(pool.moduli, c, 4, True, 4)
    for k in ("grant_flags", "grant_ts", "cert_accept_bits", "cert_reason", "cert_fail_op"):
        assert np.array_equal(getattr(v1, k), getattr(v2, k)), k
