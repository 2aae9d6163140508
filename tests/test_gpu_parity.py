"""HIP path vs the CPU oracle, bit-exact (needs an MI355X).

Every test calls libmochi_hip through its C ABI (ctypes) and compares grant
flags / timestamps / validity bits and certificate accept bits / reason codes /
failing-op indices with oracle/ (OpenSSL + the restated Java verdict logic).
"""
import json
import os

import numpy as np
import pytest

import mochi_hip as mh
import oracle_ffi as O
import workload as W
from cases import build_case_batch, grouped_cases, moduli_for
from test_oracle_golden import check_case_verdicts

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def pool4():
    return W.build_pool(R=4, k=1, P=1024, P_f=128)


@pytest.fixture(scope="module")
def pool4k2():
    return W.build_pool(R=4, k=2, P=512, P_f=64)


@pytest.fixture(scope="module")
def pool7():
    return W.build_pool(R=7, k=1, P=1024, P_f=128)


@pytest.fixture(scope="module")
def ver4(pool4):
    v = mh.Verifier(pool4.moduli, 0)
    yield v
    v.close()


@pytest.fixture(scope="module")
def ver7(pool7):
    v = mh.Verifier(pool7.moduli, 0)
    yield v
    v.close()


def assert_same(g: mh.Verdicts, o: mh.Verdicts, what=""):
    np.testing.assert_array_equal(g.grant_flags, o.grant_flags, err_msg=f"grant_flags {what}")
    np.testing.assert_array_equal(g.grant_ts, o.grant_ts, err_msg=f"grant_ts {what}")
    np.testing.assert_array_equal(g.grant_valid_bits, o.grant_valid_bits, err_msg=f"grant_valid_bits {what}")
    np.testing.assert_array_equal(g.cert_accept_bits, o.cert_accept_bits, err_msg=f"cert_accept_bits {what}")
    np.testing.assert_array_equal(g.cert_reason, o.cert_reason, err_msg=f"cert_reason {what}")
    np.testing.assert_array_equal(g.cert_fail_op, o.cert_fail_op, err_msg=f"cert_fail_op {what}")
    for k in ("op_decision", "op_g0", "op_ts"):
        if getattr(g, k) is not None and getattr(o, k) is not None:
            np.testing.assert_array_equal(getattr(g, k), getattr(o, k), err_msg=f"{k} {what}")


def test_rsa_public_op_matches_python_pow():
    pems = W.load_keys(3)
    mods = [O.pem_modulus(p) for p in pems]
    ver = mh.Verifier(mods, 0)
    rng = np.random.default_rng(7)
    sigs, signer = [], []
    for i in range(300):
        k = i % 3
        N = int.from_bytes(mods[k], "big")
        kind = i % 6
        if kind == 0:
            s = int.from_bytes(O.rsa_sign(pems[k], W.encode_grant(f"k{i}", i, "c" * 128)), "big")
        elif kind == 1:
            s = 0
        elif kind == 2:
            s = N - 1
        elif kind == 3:
            s = int(rng.integers(1, 1 << 62))
        else:
            s = int.from_bytes(rng.bytes(256), "big") % N
        sigs.append(s.to_bytes(256, "big"))
        signer.append(k)
    y, z = mh.rsa_public_op(ver, np.frombuffer(b"".join(sigs), np.uint8), np.array(signer), want_z=True)
    for i in range(len(sigs)):
        N = int.from_bytes(mods[signer[i]], "big")
        s = int.from_bytes(sigs[i], "big")
        assert int.from_bytes(y[i].tobytes(), "big") == pow(s, 65537, N), i
        # k_rsa_pow's fold chain (csrc/fold.h): z = s^(2^16) mod n, not fully reduced
        zi = sum(int(v) << (28 * j) for j, v in enumerate(z[i]))
        assert max(int(v) for v in z[i]) < 1 << 28
        assert zi < 1 << 2064
        assert zi % N == pow(s, 65536, N), i
    ver.close()


@pytest.mark.parametrize("layout", ["shuffled", "skewed"])
def test_bucketing_many_signers(layout):
    """Signer bucketing (k_bucket_count/scan/scatter) at MOCHI_MAX_KEYS = 4096 keys:
    waves holding up to 64 distinct signers (wave-aggregated ranking loops once
    per distinct key) and a skewed mix where one key takes most grants.  The
    moduli are random odd 2048-bit integers (Montgomery needs only gcd(R, n) = 1);
    every lane's s^65537 mod n is checked against Python's pow."""
    rng = np.random.default_rng(11 if layout == "shuffled" else 12)
    n_keys = 4096
    mods = []
    for _ in range(n_keys):
        v = int.from_bytes(rng.bytes(256), "big") | (3 << 2046) | 1
        mods.append(v.to_bytes(256, "big"))
    ver = mh.Verifier(mods, 0)
    n = 20000
    if layout == "shuffled":
        signer = rng.integers(0, n_keys, n)
    else:
        signer = np.where(rng.random(n) < 0.9, 17, rng.integers(0, n_keys, n))
    sigs = []
    for k in signer:
        N = int.from_bytes(mods[k], "big")
        sigs.append((int.from_bytes(rng.bytes(256), "big") % N).to_bytes(256, "big"))
    y = mh.rsa_public_op(ver, np.frombuffer(b"".join(sigs), np.uint8), signer.astype(np.uint16))
    for i in range(n):
        N = int.from_bytes(mods[signer[i]], "big")
        assert int.from_bytes(y[i].tobytes(), "big") == pow(int.from_bytes(sigs[i], "big"), 65537, N), i
    ver.close()


def test_rsa_golden_vectors_gpu(golden_dir):
    d = json.load(open(os.path.join(golden_dir, "rsa_vectors.json")))
    moduli = [bytes.fromhex(d["moduli"][str(i)]) for i in range(7)]
    vecs = d["vectors"]
    msgs = [bytes.fromhex(v["msg"]) for v in vecs]
    blob = np.frombuffer(b"".join(msgs), np.uint8).copy()
    off = np.cumsum([0] + [len(m) for m in msgs[:-1]]).astype(np.uint64)
    n = len(vecs)
    batch = mh.Batch(
        grant_bytes=blob, grant_off=off, grant_len=np.array([len(m) for m in msgs], np.uint32),
        sig=np.frombuffer(b"".join(bytes.fromhex(v["sig"]) for v in vecs), np.uint8).reshape(n, 256).copy(),
        signer=np.array([v["key"] for v in vecs], np.uint16), grant_key=np.zeros(n, np.uint8),
        cert_grant_off=np.array([0, n], np.uint32), cert_op_off=np.array([0, 0], np.uint32),
        op_key=np.zeros(0, np.uint8), op_flags=np.zeros(0, np.uint8), expected_hash=np.zeros((1, 128), np.uint8))
    ver = mh.Verifier(moduli, 0)
    g = ver.verify(batch, 4, True)
    got = (g.grant_flags & mh.GRANT_SIG_OK) != 0
    want = np.array([v["valid"] for v in vecs])
    bad = [vecs[i]["name"] for i in np.nonzero(got != want)[0]]
    assert not bad, bad
    assert want.sum() == 21
    ver.close()


@pytest.mark.parametrize("seq", ["small", "dedup"])
@pytest.mark.parametrize("explicit_mg", [True, False])
@pytest.mark.parametrize("key", sorted(grouped_cases().keys()))
def test_cert_branch_cases_gpu(key, explicit_mg, seq):
    """Every branch fixture on the device: GPU == oracle array for array (grant flags,
    timestamps, accept bits, reasons, failing ops, per-op decisions / g0 / ts) and
    both == the hand-derived expectations.  `seq`: the small-batch launch sequence
    (these batches' default) and the large-batch one (certificate-level dedup, slot
    leaders' hashes checked in k_grant_prep_cert, the lean k_tally outside
    MOCHI_Q_BIND)."""
    R, strict, qm = key
    cases = grouped_cases(explicit_mg).get(key)
    if not cases:
        pytest.skip("every case of this group needs explicit MultiGrants")
    batch, ex = build_case_batch(cases, W.load_keys(R), explicit_mg)
    ver = mh.Verifier(moduli_for(R), 0)
    if seq == "dedup":
        ver.set_small_batch(0)
    g = ver.verify(batch, R, bool(strict), quorum_mode=qm)
    o = O.verify_batch(moduli_for(R), batch, R, bool(strict), 4, quorum_mode=qm)
    assert_same(g, o, str(key))
    check_case_verdicts(g, cases, ex, f"gpu mg={explicit_mg}")
    ver.close()


@pytest.mark.parametrize("strict", [True, False])
def test_synthetic_r4_parity(pool4, ver4, strict):
    s = W.make_batch(pool4, 6000, first_cert=1000)
    g = ver4.verify(s.batch, 4, strict)
    o = O.verify_batch(pool4.moduli, s.batch, 4, strict, 8)
    assert_same(g, o, f"R=4 strict={strict}")
    np.testing.assert_array_equal(g.grant_flags, s.expected_flags)
    # every fault class shows up and is judged as the reference would
    assert set(np.unique(s.fault)) == {0, 1, 2, 3, 4, 5}


def test_synthetic_r4_k2_parity(pool4k2):
    ver = mh.Verifier(pool4k2.moduli, 0)
    s = W.make_batch(pool4k2, 4000)
    for strict in (True, False):
        g = ver.verify(s.batch, 4, strict)
        o = O.verify_batch(pool4k2.moduli, s.batch, 4, strict, 8)
        assert_same(g, o, f"k=2 strict={strict}")
    ver.close()


@pytest.mark.parametrize("strict", [True, False])
def test_synthetic_r7_parity(pool7, ver7, strict):
    # C3: 7-server certificates; strict = server predicate (> 5, i.e. 6 of 7), else client (>= 5: "5-of-7")
    s = W.make_batch(pool7, 4000)
    g = ver7.verify(s.batch, 7, strict)
    o = O.verify_batch(pool7.moduli, s.batch, 7, strict, 8)
    assert_same(g, o, f"R=7 strict={strict}")
    if not strict:
        # dropped-replica certificates: 6 of 7 valid still reaches 5-of-7
        drop = s.fault == W.FAULT_DROP
        assert g.cert_accept[drop].all()


def _oracle_tally_own_parse(batch, gpu_flags, expected_flags, R, strict):
    """Oracle verdicts for a large batch without re-verifying every signature: the
    oracle's OWN parse (flags + timestamps) and the workload's ground-truth
    signature bits (checked against the GPU's flags over the whole batch by the
    caller), then the restated tally."""
    pf, pts = O.parse_grants(batch)
    assert (pf == mh.GRANT_PARSED).all()
    np.testing.assert_array_equal(gpu_flags & mh.GRANT_PARSED, pf)
    return O.tally(batch, pf | (expected_flags & mh.GRANT_SIG_OK), pts, R, strict)


def test_large_batch_c2_bit_exact(pool4, ver4):
    """C2 scale (1M grants, R=4): flags vs ground truth, verdicts vs oracle tally."""
    C = W.n_certs_for_grants(1_000_000, 4)
    s = W.make_batch(pool4, C)
    g = ver4.verify(s.batch, 4, True)
    np.testing.assert_array_equal(g.grant_flags, s.expected_flags)
    o = _oracle_tally_own_parse(s.batch, g.grant_flags, s.expected_flags, 4, True)
    assert_same_certs(g, o)
    # the oracle's own signature leg agrees on a sample (independent OpenSSL check)
    of, ot = O.verify_grants(pool4.moduli, s.batch, 0, 4000, 8)
    np.testing.assert_array_equal(g.grant_flags[:4000], of[:4000])
    np.testing.assert_array_equal(g.grant_ts[:4000], ot[:4000])


def assert_same_certs(g, o):
    np.testing.assert_array_equal(g.cert_accept_bits, o.cert_accept_bits)
    np.testing.assert_array_equal(g.cert_reason, o.cert_reason)
    np.testing.assert_array_equal(g.cert_fail_op, o.cert_fail_op)
    np.testing.assert_array_equal(g.op_decision, o.op_decision)
    np.testing.assert_array_equal(g.op_g0, o.op_g0)
    np.testing.assert_array_equal(g.op_ts, o.op_ts)


@pytest.mark.parametrize("strict", [True, False])
def test_large_batch_c3_bit_exact(pool7, ver7, strict):
    """C3 scale (4M grants, R=7, both quorum predicates): flags vs ground truth,
    verdicts / reasons / failing ops / per-op outputs vs the oracle tally over the
    whole batch (oracle's own timestamp parse)."""
    C = W.n_certs_for_grants(4_000_000, 7)
    s = W.make_batch(pool7, C)
    g = ver7.verify(s.batch, 7, strict)
    np.testing.assert_array_equal(g.grant_flags, s.expected_flags)
    o = _oracle_tally_own_parse(s.batch, g.grant_flags, s.expected_flags, 7, strict)
    assert_same_certs(g, o)
    # the ground truth is pinned by OpenSSL too: 8 slices of 1000 grants across the batch
    # (invalid signature => the grant is absent, InMemoryDataStore.java:622-624)
    for lo in np.linspace(0, s.batch.n_grants - 1000, 8).astype(np.int64):
        of, ot = O.verify_grants(pool7.moduli, s.batch, int(lo), int(lo) + 1000, 8)
        np.testing.assert_array_equal(g.grant_flags[lo:lo + 1000], of[lo:lo + 1000])
        np.testing.assert_array_equal(g.grant_ts[lo:lo + 1000], ot[lo:lo + 1000])


def test_c4_16m_batch_bit_exact():
    """C4: the 16M-grant batch (R=4) of the bench's unique stream, signed on the device,
    verified through the host path (chunked PCIe pipeline): grant flags == the
    workload's ground truth over all 16M grants, certificate verdicts and per-op
    outputs == the oracle tally (oracle's own parse), and an independent OpenSSL
    re-check of a sample spread over the batch."""
    R = 4
    C = W.n_certs_for_grants(16_000_000, R)
    s = W.make_batch_unique(R, C, 1, first_cert=0, device=0)
    b = s.batch
    assert b.n_grants > 15_900_000
    ver = mh.Verifier(moduli_for(R), 0)
    g = ver.verify(b, R, True)
    np.testing.assert_array_equal(g.grant_flags, s.expected_flags)
    o = _oracle_tally_own_parse(b, g.grant_flags, s.expected_flags, R, True)
    assert_same_certs(g, o)
    assert (~g.cert_accept).sum() > 0.01 * C
    # the device-signed stream is pinned by OpenSSL itself: the whole first 1M grants
    # (16 threads), then 8 slices of 1000 grants across the rest of the batch
    head = 1_000_000
    of, ot = O.verify_grants(moduli_for(R), b, 0, head, 16)
    np.testing.assert_array_equal(g.grant_flags[:head], of[:head])
    np.testing.assert_array_equal(g.grant_ts[:head], ot[:head])
    assert (of[:head] & mh.GRANT_SIG_OK).sum() < head  # the fault mix reaches the head
    for lo in np.linspace(head, b.n_grants - 1000, 8).astype(np.int64):
        of, ot = O.verify_grants(moduli_for(R), b, int(lo), int(lo) + 1000, 8)
        np.testing.assert_array_equal(g.grant_flags[lo:lo + 1000], of[lo:lo + 1000])
    # The launch bench.py times: the whole 16M-grant batch resident in HBM, ONE
    # mochi_verify_batch_device call (7,800+ dynamic pow groups, the LDS-staged
    # certificate prep at 4M certificates), in the bench's layout (one copy of a
    # certificate's grant bytes) and with every grant its own copy at a mixed
    # alignment (wire slices: prep must compare bytes).  Every certificate's
    # verdict, reason, failing op and per-op outputs == the oracle tally above.
    import torch

    for name, sb in (("shared", s), ("separate", W.separate_copies(s))):
        dev = mh.DeviceBatch(sb.batch, 0)
        out = mh.DeviceVerdicts(dev.n_grants, dev.n_certs, 0, full=True, n_ops=dev.n_ops)
        for _ in range(2):  # twice: the second call reuses the context's scratch as the bench's steps do
            ver.verify_device(dev, out, R, True, stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        h = out.to_host()
        np.testing.assert_array_equal(h.grant_flags, s.expected_flags, err_msg=name)
        np.testing.assert_array_equal(h.grant_ts, g.grant_ts, err_msg=name)
        np.testing.assert_array_equal(h.grant_valid_bits, g.grant_valid_bits, err_msg=name)
        assert_same_certs(h, o)
        del dev, out
    ver.close()


def test_sig_ge_modulus_rejected(pool4, ver4):
    s = W.make_batch(pool4, 50, faults=False)
    b = s.batch
    N = int.from_bytes(pool4.moduli[int(b.signer[0])], "big")
    sig0 = int.from_bytes(b.sig[0].tobytes(), "big")
    if sig0 + N < (1 << 2048):
        b.sig[0] = np.frombuffer((sig0 + N).to_bytes(256, "big"), np.uint8)  # s + n: same residue, must reject
    b.sig[1] = np.frombuffer(pool4.moduli[int(b.signer[1])], np.uint8)  # s == n
    b.sig[2] = 0xFF  # s = 2^2048 - 1 > n
    g = ver4.verify(b, 4, True)
    o = O.verify_batch(pool4.moduli, b, 4, True, 2)
    assert_same(g, o)
    assert not (g.grant_flags[:3] & 1).any()
    assert (g.grant_flags[3:] & 1).all()


def test_edge_shapes(pool4, ver4):
    # empty batch
    empty = mh.Batch(grant_bytes=np.zeros(1, np.uint8), grant_off=np.zeros(0, np.uint64),
                     grant_len=np.zeros(0, np.uint32), sig=np.zeros((0, 256), np.uint8),
                     signer=np.zeros(0, np.uint16), grant_key=np.zeros(0, np.uint8),
                     cert_grant_off=np.zeros(1, np.uint32), cert_op_off=np.zeros(1, np.uint32),
                     op_key=np.zeros(0, np.uint8), op_flags=np.zeros(0, np.uint8),
                     expected_hash=np.zeros((0, 128), np.uint8))
    g = ver4.verify(empty, 4, True)
    assert g.cert_accept_bits.size == 0
    # single certificate, single grant; and a batch whose size is not a multiple of 64
    for C in (1, 3, 17, 65):
        s = W.make_batch(pool4, C, first_cert=C * 31)
        g = ver4.verify(s.batch, 4, True)
        o = O.verify_batch(pool4.moduli, s.batch, 4, True, 2)
        assert_same(g, o, f"C={C}")
    # signer index outside the key table -> invalid signature (never verified)
    s = W.make_batch(pool4, 40, faults=False)
    s.batch.signer[5] = 4
    s.batch.signer[9] = 65535
    g = ver4.verify(s.batch, 4, True)
    o = O.verify_batch(pool4.moduli, s.batch, 4, True, 2)
    assert_same(g, o, "bad signer")
    assert not (g.grant_flags[[5, 9]] & 1).any()


def test_long_and_odd_grants(ver4, pool4):
    """Grants spanning many SHA-256 blocks, empty grants, unaligned offsets."""
    pems = W.load_keys(4)
    th = W.txn_hash_hex(5)
    grants = [W.encode_grant("K" * n, 1000, th) for n in (0, 1, 50, 55, 56, 63, 64, 119, 500, 3000)]
    grants.append(b"")  # an empty Grant (all defaults) parses fine
    grants.append(W.encode_grant("K", 1000, th) + b"\x0f")  # malformed
    blob = bytearray(b"\x01\x02\x03")
    offs = []
    for i, gb in enumerate(grants):
        blob += b"\xaa" * (i % 3)
        offs.append(len(blob))
        blob += gb
    sigs = [O.rsa_sign(pems[i % 4], gb) for i, gb in enumerate(grants)]
    n = len(grants)
    b = mh.Batch(grant_bytes=np.frombuffer(bytes(blob), np.uint8).copy(), grant_off=np.array(offs, np.uint64),
                 grant_len=np.array([len(x) for x in grants], np.uint32),
                 sig=np.frombuffer(b"".join(sigs), np.uint8).reshape(n, 256).copy(),
                 signer=np.array([i % 4 for i in range(n)], np.uint16), grant_key=np.zeros(n, np.uint8),
                 cert_grant_off=np.array([0, 4, 8, n], np.uint32), cert_op_off=np.array([0, 1, 2, 3], np.uint32),
                 op_key=np.zeros(3, np.uint8), op_flags=np.full(3, 3, np.uint8),
                 expected_hash=np.stack([np.frombuffer(th.encode(), np.uint8)] * 3))
    g = ver4.verify(b, 4, False)
    o = O.verify_batch(pool4.moduli, b, 4, False, 2)
    assert_same(g, o)
    assert (g.grant_flags[:n - 1] & 1).all()
    assert g.grant_flags[n - 1] == 1  # signature fine, bytes unparseable
    assert g.cert_reason[2] == mh.REJECT_MALFORMED


def test_device_resident_path_matches_host_path(pool4, ver4):
    import torch

    s = W.make_batch(pool4, 3000, first_cert=77)
    host = ver4.verify(s.batch, 4, True)
    dev = mh.DeviceBatch(s.batch, 0)
    out = mh.DeviceVerdicts(dev.n_grants, dev.n_certs, 0)
    ver4.verify_device(dev, out, 4, True, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    d = out.to_host()
    assert_same(d, host, "device path")


def test_repeatable(pool4, ver4):
    s = W.make_batch(pool4, 2000, first_cert=5)
    a = ver4.verify(s.batch, 4, True)
    b = ver4.verify(s.batch, 4, True)
    assert_same(a, b, "repeat")


def _scatter_blob(b: mh.Batch, seed: int) -> mh.Batch:
    """Same grants, bytes laid out in a random order with gaps (wire-slice layout)."""
    rng = np.random.default_rng(seed)
    order = rng.permutation(b.n_grants)
    blob, offs = bytearray(b"\x07" * 5), np.zeros(b.n_grants, np.uint64)
    for i in order:
        blob += b"\x00" * int(rng.integers(0, 4))
        offs[i] = len(blob)
        o, n = int(b.grant_off[i]), int(b.grant_len[i])
        blob += b.grant_bytes[o:o + n].tobytes()
    return mh.Batch(grant_bytes=np.frombuffer(bytes(blob), np.uint8).copy(), grant_off=offs, grant_len=b.grant_len,
                    sig=b.sig, signer=b.signer, grant_key=b.grant_key, cert_grant_off=b.cert_grant_off,
                    cert_op_off=b.cert_op_off, op_key=b.op_key, op_flags=b.op_flags, expected_hash=b.expected_hash)


@pytest.mark.parametrize("chunk", [1, 1000, 50_000])
def test_host_pipeline_chunking(pool4, chunk):
    """mochi_verify_batch's chunked H2D/compute/D2H pipeline: chunk sizes from 32
    certificates up, a certificate count that is not a multiple of 32, pinned
    in-place arrays and a scattered grant blob all give the oracle's verdicts."""
    ver = mh.Verifier(pool4.moduli, 0)
    ver.set_chunk_grants(chunk)
    s = W.make_batch(pool4, 2501, first_cert=123)
    o = O.verify_batch(pool4.moduli, s.batch, 4, True, 8)
    g = ver.verify(s.batch, 4, True)
    assert_same(g, o, f"chunk={chunk}")
    assert g.timing_ms["total"] > 0
    gp = ver.verify(s.batch.pinned(), 4, True)
    assert_same(gp, o, f"pinned chunk={chunk}")
    gs = ver.verify(_scatter_blob(s.batch, chunk), 4, True)
    assert_same(gs, o, f"scattered chunk={chunk}")
    ver.close()


def test_grant_group_depth_matches_google_protobuf(pool4, ver4, golden_dir):
    """Unknown groups nested up to CodedInputStream's recursion limit (100) parse on the
    device (the 16-deep register stack hands deeper grants to the out-of-line 100-deep
    parser), 101 is malformed -- exactly google.protobuf's verdicts."""
    d = json.load(open(os.path.join(golden_dir, "grant_vectors.json")))
    vecs = [v for v in d["parse"] if v["name"].startswith("groups_nested") or v["name"] == "group_skipped"]
    assert len(vecs) == 5
    pem = W.load_keys(1)[0]
    msgs = [bytes.fromhex(v["bytes"]) for v in vecs]
    n = len(msgs)
    blob = np.frombuffer(b"".join(msgs), np.uint8).copy()
    off = np.cumsum([0] + [len(m) for m in msgs[:-1]]).astype(np.uint64)
    b = mh.Batch(grant_bytes=blob, grant_off=off, grant_len=np.array([len(m) for m in msgs], np.uint32),
                 sig=np.frombuffer(b"".join(O.rsa_sign(pem, m) for m in msgs), np.uint8).reshape(n, 256).copy(),
                 signer=np.zeros(n, np.uint16), grant_key=np.zeros(n, np.uint8),
                 cert_grant_off=np.arange(n + 1, dtype=np.uint32), cert_op_off=np.zeros(n + 1, np.uint32),
                 op_key=np.zeros(0, np.uint8), op_flags=np.zeros(0, np.uint8), expected_hash=np.zeros((n, 128), np.uint8))
    g = ver4.verify(b, 4, True)
    for i, v in enumerate(vecs):
        assert bool(g.grant_flags[i] & mh.GRANT_PARSED) == v["expect"]["ok"], v["name"]
        assert g.grant_flags[i] & mh.GRANT_SIG_OK  # signature fine either way
        if v["expect"]["ok"]:
            assert g.grant_ts[i] == v["expect"]["timestamp"], v["name"]


_SIG_CACHE = {}


def _sign_cached(pem, gb):
    key = (pem, gb)
    if key not in _SIG_CACHE:
        _SIG_CACHE[key] = O.rsa_sign(pem, gb)
    return _SIG_CACHE[key]


def _dedup_batch(pems, certs, shared_first=False, bad_sig=()):
    """certs: list of lists of (grant bytes, signer, key slot); every grant its own copy
    in the blob at a varying alignment (the byte compares of k_grant_prep_cert /
    k_grant_match), or -- with shared_first -- grants equal to the certificate's first
    one pointing at its bytes (the SoA layout's offset shortcut).  bad_sig: (cert,
    grant) pairs whose signature gets one byte flipped."""
    blob = bytearray(b"\x07")
    offs, lens, sigs, signer, gkey, cgo = [], [], [], [], [], [0]
    cop, opk = [0], []
    for ci, cert in enumerate(certs):
        first = None
        for gi, (gb, s, k) in enumerate(cert):
            if shared_first and first is not None and gb == first[0]:
                offs.append(first[1])
            else:
                blob += b"\xee" * ((ci + gi) % 4)
                offs.append(len(blob))
                blob += gb
                if first is None:
                    first = (gb, offs[-1])
            lens.append(len(gb))
            sg = _sign_cached(pems[s], gb)
            if (ci, gi) in bad_sig:
                sg = sg[:100] + bytes([sg[100] ^ 0x40]) + sg[101:]
            sigs.append(sg)
            signer.append(s)
            gkey.append(k)
        cgo.append(len(offs))
        keys = sorted({k for _, _, k in cert})
        opk += keys
        cop.append(len(opk))
    n, C = len(offs), len(certs)
    th = W.txn_hash_hex(9)
    return mh.Batch(grant_bytes=np.frombuffer(bytes(blob), np.uint8).copy(), grant_off=np.array(offs, np.uint64),
                    grant_len=np.array(lens, np.uint32), sig=np.frombuffer(b"".join(sigs), np.uint8).reshape(n, 256).copy(),
                    signer=np.array(signer, np.uint16), grant_key=np.array(gkey, np.uint8),
                    cert_grant_off=np.array(cgo, np.uint32), cert_op_off=np.array(cop, np.uint32),
                    op_key=np.array(opk, np.uint8), op_flags=np.full(len(opk), 3, np.uint8),
                    expected_hash=np.stack([np.frombuffer(th.encode(), np.uint8)] * C))


@pytest.fixture
def dedup_path(ver4):
    """The large-batch launch sequence (certificate-level dedup) even for these small
    test batches; the small-batch sequence is restored afterwards."""
    ver4.set_small_batch(0)
    yield ver4
    ver4.set_small_batch(4096)


@pytest.mark.parametrize("shared_first", [False, True])
@pytest.mark.parametrize("small", [False, True])
def test_grant_dedup_one_byte_differences(pool4, ver4, shared_first, small):
    """Grant prep hashes each distinct grant of a (certificate, key slot) once
    (k_grant_prep_cert, k_grant_match, k_grant_prep_rare; `small`: the small-batch
    sequence, every grant on its own).  Grants that differ from the slot's first
    grant in exactly one byte -- timestamp skew, a g1 / g0 transactionHash mismatch, a
    flipped objectId byte, a trailing unknown field -- must be prepped on their own:
    flags, timestamps and verdicts bit-exact with the oracle (which hashes every
    grant)."""
    ver4.set_small_batch(4096 if small else 0)
    pems = W.load_keys(4)
    th = W.txn_hash_hex(9)
    oth = th[:-1] + ("0" if th[-1] != "0" else "1")
    base = W.encode_grant("DEMO_KEY_DEDUP", 1000, th)
    skew = W.encode_grant("DEMO_KEY_DEDUP", 1001, th)
    hmis = W.encode_grant("DEMO_KEY_DEDUP", 1000, oth)
    oflip = W.encode_grant("DEMO_KEY_DEDUQ", 1000, th)
    longer = base + b"\x30\x01"  # unknown varint field 6: parses, not byte-equal
    assert all(len(x) == len(base) for x in (skew, hmis, oflip))
    variants = {"honest": [base] * 4, "ts_skew": [base, base, skew, base], "g1_hash": [base, hmis, base, base],
                "g0_hash": [hmis, base, base, base], "oid_flip": [base, base, base, oflip],
                "longer": [base, longer, base, base], "all_skew": [base, skew, skew, skew]}
    certs = []
    for _ in range(40):  # enough certificates for several waves of k_grant_dedup lanes
        for gs in variants.values():
            certs.append([(gb, r, 0) for r, gb in enumerate(gs)])
    # two key slots in one certificate (k = 2), interleaved
    certs.append([(base, 0, 0), (skew, 0, 1), (base, 1, 0), (skew, 1, 1), (base, 2, 0), (skew, 2, 1)])
    b = _dedup_batch(pems, certs, shared_first)
    for strict in (True, False):
        g = ver4.verify(b, 4, strict)
        o = O.verify_batch(pool4.moduli, b, 4, strict, 2)
        assert_same(g, o, f"strict={strict}")
    ver4.set_small_batch(4096)
    assert (g.grant_flags & 1).all()  # every signature is valid
    reasons = {k: int(g.cert_reason[i]) for i, k in enumerate(variants)}
    assert reasons["honest"] == mh.ACCEPT and reasons["ts_skew"] == mh.REJECT_TS_MISMATCH
    assert reasons["g0_hash"] == mh.REJECT_HASH_MISMATCH


@pytest.mark.parametrize("shared_first", [False, True])
def test_grant_dedup_block_over_lds_and_third_slot(pool4, dedup_path, shared_first):
    """k_grant_prep_cert's edges: a block of 256 certificates holding more than
    kPrepBlockGrants (2048) grants stores its results lane by lane (no LDS staging, so
    no k_grant_match: byte compares in the certificate's lane), a second block within
    the bound is staged, and certificates with three key slots leave the third slot's
    grants to k_grant_prep_rare -- each with one-byte variants in every slot.  ==
    the oracle."""
    pems = W.load_keys(4)
    th = W.txn_hash_hex(9)
    g = [[W.encode_grant(f"DEMO_KEY_SLOT{j}", 1000 + 10 * j + d, th) for d in (0, 1)] for j in range(3)]
    certs = []
    for c in range(512):
        cert = []
        for r in range(4):
            for j in range(3 if c < 256 else 2):  # block 0: 256 x 12 grants > 2048; block 1: 256 x 8
                skew = (c + j) % 7 == 0 and r == 2  # one replica's grant of the slot differs in one byte
                cert.append((g[j][1 if skew else 0], r, j))
        certs.append(cert)
    b = _dedup_batch(pems, certs, shared_first)
    assert int(b.cert_grant_off[256]) > 2048 and int(b.cert_grant_off[512] - b.cert_grant_off[256]) <= 2048
    for strict in (True, False):
        got = dedup_path.verify(b, 4, strict)
        o = O.verify_batch(pool4.moduli, b, 4, strict, 4)
        assert_same(got, o, f"strict={strict}")
    assert (got.cert_reason == mh.REJECT_TS_MISMATCH).any() and (got.cert_reason == mh.ACCEPT).any()


@pytest.mark.parametrize("shared_first", [False, True])
def test_g0_hash_after_an_invalid_leader(pool4, dedup_path, shared_first):
    """g0 is not always its slot's first grant: with the first grant's signature
    invalid (absent, InMemoryDataStore.java:622-624) g0 is the next counted grant.
    When that grant differs from the first in its bytes its result is its own
    (k_grant_prep_rare), with no hash check from k_grant_prep_cert, and the lean
    k_tally compares its transactionHash itself, 16 bytes at a time -- equal (accept)
    and one byte off (REJECT_HASH_MISMATCH), at every alignment of the copy."""
    pems = W.load_keys(4)
    th = W.txn_hash_hex(9)
    oth = th[:-1] + ("0" if th[-1] != "0" else "1")
    base = W.encode_grant("DEMO_KEY_G0", 1000, th)
    longer = base + b"\x30\x01"  # same timestamp and hash, other bytes
    hmis = W.encode_grant("DEMO_KEY_G0", 1000, oth)
    hmis_longer = hmis + b"\x30\x01"
    variants = {"g0_ok": [base, longer, longer, longer], "g0_bad": [base, hmis, hmis, hmis],
                "g0_bad_tail": [base, hmis_longer, hmis_longer, longer],
                "g0_ok_lead_ok": [base, longer, base, base]}
    certs, bad = [], set()
    for rep in range(24):
        for name, gs in variants.items():
            if name != "g0_ok_lead_ok":
                bad.add((len(certs), 0))
            certs.append([(gb, r, 0) for r, gb in enumerate(gs)])
    b = _dedup_batch(pems, certs, shared_first, bad_sig=bad)
    for strict in (True, False):
        got = dedup_path.verify(b, 4, strict)
        o = O.verify_batch(pool4.moduli, b, 4, strict, 4)
        assert_same(got, o, f"strict={strict}")
    reasons = {k: int(got.cert_reason[i]) for i, k in enumerate(variants)}
    assert reasons["g0_ok"] == mh.ACCEPT and reasons["g0_ok_lead_ok"] == mh.ACCEPT
    assert reasons["g0_bad"] == mh.REJECT_HASH_MISMATCH and reasons["g0_bad_tail"] == mh.REJECT_HASH_MISMATCH


def test_grant_dedup_large_certificate(pool4, dedup_path):
    """A certificate of 300 grants (a 64-bit slot mask is not involved: one key; more
    grants than any wave) and a small one: results equal the oracle's."""
    ver4 = dedup_path
    pems = W.load_keys(4)
    th = W.txn_hash_hex(9)
    gs = [W.encode_grant("DEMO_KEY_BIG", 1000 + (i % 3 == 2), th) for i in range(300)]
    b = _dedup_batch(pems, [[(gb, i % 4, 0) for i, gb in enumerate(gs)], [(gs[0], r, 0) for r in range(4)]])
    g = ver4.verify(b, 4, True)
    o = O.verify_batch(pool4.moduli, b, 4, True, 2)
    assert_same(g, o)


def test_grant_prep_fast_path_shapes(pool4, ver4):
    """prep_dev.h grant_prep_fast takes the common Grant shape (0x0A L objectId 0x10 ts
    0x22 H hash, ASCII strings) from two 16-byte windows and checks the strings ASCII
    on the SHA-256 words; every other shape goes to the generic parse.  Shapes at and
    around its edges -- both sides of each bound -- give the oracle's flags,
    timestamps and verdicts."""
    pems = W.load_keys(4)
    th = W.txn_hash_hex(11)
    v = W._varint

    def g(oid: bytes, ts_bytes: bytes, hash_b: bytes, tail: bytes = b"", hlen: bytes = None) -> bytes:
        hl = v(len(hash_b)) if hlen is None else hlen
        return b"\x0a" + v(len(oid)) + oid + b"\x10" + ts_bytes + b"\x22" + hl + hash_b + tail

    H = th.encode()
    shapes = [
        g(b"K", v(1000), H),                        # the common shape
        g(b"", v(5), H),                            # empty objectId
        g(b"K" * 127, v(7), H),                     # L = 127 (one-byte length)
        g(b"K" * 128, v(7), H),                     # L = 128: generic
        g(b"K", v(0), H),                           # explicit zero timestamp
        g(b"K", v(2 ** 35 - 1), H),                 # 5-byte varint
        g(b"K", v(2 ** 35), H),                     # 6-byte varint: generic
        g(b"K", v(2 ** 63), H),                     # 10-byte varint: generic
        g(b"K", v(9), H[:127]),                     # 127-byte hash (one-byte length)
        g(b"K", v(9), b"h" * 200),                  # 2-byte hash length
        g(b"K", v(9), b""),                         # empty hash
        g(b"K", v(9), H, tail=b"\x28\x01"),         # a status after the hash: generic
        g("café".encode(), v(9), H),           # non-ASCII objectId (valid UTF-8): generic
        g(b"K", v(9), H[:-2] + "é".encode()),  # non-ASCII hash: generic
        g(b"K\xff", v(9), H),                       # invalid UTF-8 objectId: malformed
        g(b"K", v(9), H[:-1] + b"\x80"),            # invalid UTF-8 hash: malformed
        g(b"K", v(9), H)[:-1],                      # truncated: malformed
        g(b"K", b"\x80\x80\x80\x80\x80\x01", H),    # non-minimal 6-byte varint: generic
        g(b"K", b"\x85\x00", H),                    # non-minimal 2-byte varint (value 5): valid
        g(b"K", v(9), H, hlen=b"\x80\x01"[:1] + b"\x81"),  # hash length varint 3 bytes long: malformed
        b"\x10\x05" + g(b"K", v(9), H)[0:0] + b"\x0a\x01K\x22" + v(len(H)) + H,  # fields out of order
        b"\x0a\x01K\x18\x01\x22" + v(len(H)) + H,   # configstamp instead of a timestamp: generic
    ]
    n = len(shapes)
    blob = bytearray(b"\x00")
    offs = []
    for i, gb in enumerate(shapes):
        blob += b"\x55" * (i % 5)
        offs.append(len(blob))
        blob += gb
    sigs = [O.rsa_sign(pems[i % 4], gb) for i, gb in enumerate(shapes)]
    b = mh.Batch(grant_bytes=np.frombuffer(bytes(blob), np.uint8).copy(), grant_off=np.array(offs, np.uint64),
                 grant_len=np.array([len(x) for x in shapes], np.uint32),
                 sig=np.frombuffer(b"".join(sigs), np.uint8).reshape(n, 256).copy(),
                 signer=np.array([i % 4 for i in range(n)], np.uint16), grant_key=np.zeros(n, np.uint8),
                 cert_grant_off=np.arange(n + 1, dtype=np.uint32), cert_op_off=np.arange(n + 1, dtype=np.uint32),
                 op_key=np.zeros(n, np.uint8), op_flags=np.full(n, 3, np.uint8),
                 expected_hash=np.stack([np.frombuffer(H, np.uint8)] * n))
    for strict in (True, False):
        gv = ver4.verify(b, 4, strict)
        o = O.verify_batch(pool4.moduli, b, 4, strict, 2)
        assert_same(gv, o, f"strict={strict}")
    assert (gv.grant_flags & 1).all()  # every signature valid: only the parse differs
    assert not (gv.grant_flags[[14, 15, 16]] & mh.GRANT_PARSED).any()
    assert (gv.grant_flags[[0, 1, 2, 3, 5, 6, 12, 13, 18]] & mh.GRANT_PARSED).all()
