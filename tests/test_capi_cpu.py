"""C-ABI checks that need no GPU: the library loads, exports every symbol the
header declares, rejects bad arguments, and its host-side client tally
matches the oracle restatement of MochiDBClient.java:148-175 / 355-382."""
import ctypes
import os
import re

import numpy as np
import pytest

import mochi_hip as mh
import oracle_ffi as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "mochi_hip.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(mochi_[a-z_0-9]+)\s*\(", hdr)))


def test_library_exports_every_declared_symbol():
    lib = mh.load_library()
    syms = declared_symbols()
    assert "mochi_verify_batch" in syms and "mochi_verify_batch_device" in syms
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(lib, s), f"{s} declared in include/mochi_hip.h but not exported"


def test_abi_version():
    assert mh.load_library().mochi_abi_version() == mh.ABI_VERSION == 3


def test_ctx_create_rejects_bad_keys():
    lib = mh.load_library()
    bad = np.zeros(256, np.uint8)  # not a 2048-bit odd modulus
    assert not lib.mochi_ctx_create(0, bad.ctypes.data, 1, 256, 65537)
    good = np.frombuffer(O.pem_modulus(open(os.path.join(ROOT, "tests/golden/keys/server0.pem"), "rb").read()),
                         np.uint8).copy()
    assert not lib.mochi_ctx_create(0, good.ctypes.data, 1, 256, 3)  # e must be 65537
    assert not lib.mochi_ctx_create(0, good.ctypes.data, 1, 128, 65537)  # RSA-2048 only
    assert not lib.mochi_ctx_create(0, good.ctypes.data, 0, 256, 65537)


def test_verify_rejects_null_ctx():
    lib = mh.load_library()
    b = mh.Batch_C()
    p = mh.Params_C(replication_factor=4, strict_gt=1)
    v = mh.Verdicts_C()
    assert lib.mochi_verify_batch(None, ctypes.byref(b), ctypes.byref(p), ctypes.byref(v)) == mh.EINVAL


def test_sign_grants_roundtrip_cpu():
    pem = open(os.path.join(ROOT, "tests/golden/keys/server1.pem"), "rb").read()
    from workload import encode_grant
    msgs = [encode_grant(f"K{i}", 1000 + i, "b" * 128) for i in range(5)]
    blob = np.frombuffer(b"".join(msgs), np.uint8).copy()
    off = np.cumsum([0] + [len(m) for m in msgs[:-1]]).astype(np.uint64)
    ln = np.array([len(m) for m in msgs], np.uint32)
    sigs = mh.sign_grants(pem, blob, off, ln, n_threads=2)
    n = mh.pem_modulus(pem)
    assert n == O.pem_modulus(pem)
    for i, m in enumerate(msgs):
        assert O.rsa_verify(n, m, sigs[i].tobytes())


def _random_responses(rng, n_req):
    resps, n_ops = [], []
    for _ in range(n_req):
        k = int(rng.integers(1, 5))
        n_ops.append(k)
        r = []
        for _ in range(int(rng.integers(0, 7))):
            kk = k if rng.random() > 0.05 else k + 1
            r.append([int(x) for x in (rng.random(kk) < 0.2)])
        resps.append(r)
    return resps, n_ops


@pytest.mark.parametrize("R", [4, 5, 7])
def test_client_tally_matches_oracle(R):
    rng = np.random.default_rng(1234 + R)
    resps, n_ops = _random_responses(rng, 300)
    a1, r1, c1 = mh.tally_responses(resps, n_ops, R)
    a2, r2, c2 = O.tally_responses(resps, n_ops, R)
    assert np.array_equal(a1, a2)
    assert np.array_equal(r1, r2)
    for x, y in zip(c1, c2):
        assert np.array_equal(x, y)
    assert a1.any() and (~a1).any()


def test_client_tally_reference_semantics():
    # 4 responses, all OK -> accept; chosen = last response index (MochiDBClient.java:166,373)
    acc, why, ch = mh.tally_responses([[[0], [0], [0], [0]]], [1], 4)
    assert acc[0] and why[0] == 0 and ch[0][0] == 3
    # two WRONG_SHARD of 4 -> 2 < M=3 -> InconsistentWriteException
    acc, why, ch = mh.tally_responses([[[0], [1], [0], [1]]], [1], 4)
    assert not acc[0] and why[0] == 2 and ch[0][0] == 2
    # op-count mismatch -> InconsistentReadException path
    acc, why, _ = mh.tally_responses([[[0, 0], [0]]], [2], 4)
    assert not acc[0] and why[0] == 1


def _random_write1(rng, n):
    reqs = []
    for _ in range(n):
        R = int(rng.integers(1, 8))
        k = int(rng.integers(1, 4))
        base = rng.integers(0, 5, size=k) * 1000
        resps = []
        for q in range(R):
            u = rng.random()
            kind = mh.W1_OK if u < 0.85 else mh.W1_REFUSED if u < 0.93 else mh.W1_REQUEST_FAILED if u < 0.97 else mh.W1_OTHER
            sid = q if rng.random() > 0.05 else int(rng.integers(0, R))  # occasional duplicate serverId
            grants = []
            for j in range(k):
                if rng.random() < 0.05:
                    continue
                ts = int(base[j] + (1 if rng.random() < 0.08 else 0))
                st = 1 if rng.random() < 0.01 else 0
                grants.append((j, ts, st))
            if rng.random() < 0.1:
                grants.append((0xFF, int(rng.integers(0, 9999)), 0))  # a grant for no op key
            resps.append((kind, sid, grants))
        reqs.append(resps)
    return reqs


def test_write1_classify_matches_oracle():
    rng = np.random.default_rng(77)
    reqs = _random_write1(rng, 3000)
    got = mh.write1_classify(reqs)
    exp = O.write1_classify(reqs)
    assert np.array_equal(got, exp)
    assert set(np.unique(got).tolist()) == {0, 1, 2, 3, 4}


def test_write1_classify_reference_semantics():
    ok = lambda sid, g: (mh.W1_OK, sid, g)
    # all OK, uniform -> Write2 (MochiDBClient.java:320-324)
    assert mh.write1_classify([[ok(0, [(0, 5, 0)]), ok(1, [(0, 5, 0)])]])[0] == mh.W1_PROCEED
    # non-uniform -> retry (:310-318), even when another server refused
    assert mh.write1_classify([[ok(0, [(0, 5, 0)]), ok(1, [(0, 6, 0)]),
                                (mh.W1_REFUSED, 2, [(0, 9, 0)])]])[0] == mh.W1_RETRY
    # refused grants are not part of the uniformity check -> RequestRefusedException (:325-328)
    assert mh.write1_classify([[ok(0, [(0, 5, 0)]), (mh.W1_REFUSED, 1, [(0, 9, 0)])]])[0] == mh.W1_THROW_REFUSED
    # REQUESTFAILED anywhere throws first (:281-283)
    assert mh.write1_classify([[ok(0, [(0, 5, 0)]), ok(1, [(0, 6, 0)]),
                                (mh.W1_REQUEST_FAILED, 2, [])]])[0] == mh.W1_THROW_FAILED
    # a WRONG_SHARD grant -> removal from the read-only map view throws (:221-228)
    assert mh.write1_classify([[ok(0, [(0, 5, 1)])]])[0] == mh.W1_THROW_UNSUPPORTED
    # a later OK response with the same serverId replaces the earlier one (HashMap.put, :299)
    assert mh.write1_classify([[ok(0, [(0, 5, 0)]), ok(1, [(0, 6, 0)]), ok(0, [(0, 6, 0)])]])[0] == mh.W1_PROCEED
    # grants for keys outside the transaction are never consulted (:202-205)
    assert mh.write1_classify([[ok(0, [(0, 5, 0), (0xFF, 1, 0)]), ok(1, [(0, 5, 0), (0xFF, 2, 0)])]])[0] == mh.W1_PROCEED
    # OTHER payloads clear allWriteOk only (:284-287)
    assert mh.write1_classify([[ok(0, [(0, 5, 0)]), (mh.W1_OTHER, 1, [])]])[0] == mh.W1_THROW_REFUSED



@pytest.mark.parametrize("n", [2, 3, 8])
def test_gather_protocol_never_strands_a_peer(n):
    """The per-device protocol mochi_mverify_* run around the RCCL all-gather
    (multi.cpp run_gather), on the CPU with simulated devices: a device whose
    selection fails keeps every device out of the collective; one whose slot fill
    fails still joins it (its peers complete) and the error is reported; one
    whose enqueue fails makes every device abort instead of waiting.  No device
    ever waits for a peer that never comes (timed_out == 0) and every case
    returns an error, not a hang."""
    import ctypes

    import mochi_hip as mh

    lib = mh.load_library()
    entered, timed_out = ctypes.c_uint32(), ctypes.c_uint32()

    def run(sel=0, fill=0, enq=0):
        rc = lib.mochi_test_gather_protocol(n, sel, fill, enq, 5000, ctypes.byref(entered), ctypes.byref(timed_out))
        return rc, entered.value, timed_out.value

    assert run() == (mh.OK, n, 0)
    rc, e, t = run(sel=1 << 1)
    assert rc != mh.OK and e == 0 and t == 0
    rc, e, t = run(sel=1 << (n - 1) | 1)
    assert rc != mh.OK and e == 0 and t == 0
    rc, e, t = run(fill=1 << 1)
    assert rc != mh.OK and e == n and t == 0
    assert "slot fill" in lib.mochi_last_error().decode()
    rc, e, t = run(enq=1 << (n - 1))
    assert rc != mh.OK and e == n - 1 and t == 0
    assert "enqueue" in lib.mochi_last_error().decode()
