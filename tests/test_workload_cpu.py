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
