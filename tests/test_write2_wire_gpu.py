"""Write2ToServer wire path on the GPU (mochi_verify_write2 / mochi_write2_decode):
the device decoder agrees with the oracle decoder array for array, with the
golden protobuf vectors, and the wire path's verdicts equal the SoA path's."""
import numpy as np
import pytest

import mochi_hip as mh
import oracle_ffi as O
import workload as W
from test_write2_wire_cpu import _golden, check_decode_against_golden

pytestmark = pytest.mark.gpu

KEYS = ("grant_off", "grant_len", "sig", "signer", "grant_key", "cert_grant_off", "cert_op_off", "op_key",
        "op_flags", "msg_status", "cert_mg_off", "mg_grant_off", "op_key_off", "op_key_len")


@pytest.fixture(scope="module")
def pool4():
    return W.build_pool(R=4, k=1, P=512, P_f=64)


@pytest.fixture(scope="module")
def pool4k2_wire():
    return W.build_pool(R=4, k=2, P=256, P_f=64)


@pytest.fixture(scope="module")
def pool7k2():
    return W.build_pool(R=7, k=2, P=256, P_f=64)


def grant_ts_of_ops(s):
    """Per op: the timestamp of its certificate's first grant for the op's key slot
    (parsed by the oracle); stored-certificate timestamps are drawn around it."""
    b = s.batch
    out = np.zeros(b.n_ops, np.int64)
    for c in range(b.n_certs):
        g0, g1 = int(b.cert_grant_off[c]), int(b.cert_grant_off[c + 1])
        for o in range(int(b.cert_op_off[c]), int(b.cert_op_off[c + 1])):
            for g in range(g0, g1):
                if b.grant_key[g] == b.op_key[o]:
                    gb = b.grant_bytes[int(b.grant_off[g]):int(b.grant_off[g]) + int(b.grant_len[g])].tobytes()
                    out[o] = O.grant_parse(gb)["timestamp"]
                    break
    return out


def _ver(pool):
    v = mh.Verifier(pool.moduli, 0)
    v.set_server_ids(W.SERVER_IDS[:pool.R])
    return v


def _pack(msgs, pad=1):
    off, parts, pos = [], [], 0
    for i, m in enumerate(msgs):
        p = (i * pad) % 4
        parts.append(b"\x00" * p)
        pos += p
        off.append(pos)
        parts.append(m)
        pos += len(m)
    M = len(msgs)
    return W.WireBatch(wire=np.frombuffer(b"".join(parts) or b"\x00", np.uint8).copy(),
                       msg_off=np.array(off, np.uint64), msg_len=np.array([len(m) for m in msgs], np.uint32),
                       op_flags_off=None, op_flags=np.zeros(1, np.uint8),
                       expected_hash=np.zeros((M, 128), np.uint8))


def assert_decode_equal(a, b, what=""):
    for k in KEYS:
        np.testing.assert_array_equal(a[k], b[k], err_msg=f"{k} {what}")


def test_device_decode_golden_vectors(pool4):
    vecs, ids, blob, off = _golden()
    ver = mh.Verifier(pool4.moduli[:1] * len(ids), 0)
    ver.set_server_ids(ids)
    msgs = [bytes.fromhex(v["hex"]) for v in vecs]
    wb = _pack(msgs)
    d = ver.decode_write2(wb)
    o = O.w2_decode(wb, blob, off)
    assert_decode_equal(d, o, "golden batch")
    # and each vector on its own against its pinned expectations
    for v, m in zip(vecs, msgs):
        one = _pack([m])
        dd = ver.decode_write2(one)
        check_decode_against_golden(v, dd, m, ids)
    ver.close()


@pytest.mark.parametrize("strict", [True, False])
def test_wire_verdicts_equal_soa_verdicts(pool4, strict):
    ver = _ver(pool4)
    s = W.make_batch(pool4, 3000, first_cert=321)
    wb = W.encode_wire_batch(s, pad=5, client_id="client-7f3a", mg_hash=True)
    g, st = ver.verify_write2(wb, 4, strict)
    assert (st == 0).all()
    soa = ver.verify(s.batch, 4, strict)
    np.testing.assert_array_equal(g.cert_accept_bits, soa.cert_accept_bits)
    np.testing.assert_array_equal(g.cert_reason, soa.cert_reason)
    np.testing.assert_array_equal(g.cert_fail_op, soa.cert_fail_op)
    ids, off = W.server_id_table(4)
    o, ost = O.verify_write2(pool4.moduli, ids, off, wb, 4, strict)
    np.testing.assert_array_equal(g.cert_accept_bits, o.cert_accept_bits)
    np.testing.assert_array_equal(g.cert_reason, o.cert_reason)
    np.testing.assert_array_equal(st, ost)
    d = ver.decode_write2(wb)
    np.testing.assert_array_equal(d["signer"], s.batch.signer)
    np.testing.assert_array_equal(d["sig"], s.batch.sig)
    # per-op outputs: wire path == SoA path == oracle
    for k in ("op_decision", "op_g0", "op_ts"):
        np.testing.assert_array_equal(getattr(g, k), getattr(soa, k), err_msg=k)
        np.testing.assert_array_equal(getattr(g, k), getattr(o, k), err_msg=k)
    ver.close()


@pytest.mark.parametrize("chunk", [64, 0])
def test_wire_stored_state_and_per_op_outputs(pool4k2_wire, chunk):
    """SVOC state inputs through the wire path (op flags HAS_CURRENT_C / CURRENT_C_BAD /
    NOT_WRITE + op_object_ts): read vs apply branch, stored-certificate throws, per-op
    decisions / g0 / ts -- device == oracle, on the chunked host pipeline (64-grant
    chunks) and in one piece."""
    pool = pool4k2_wire
    ver = _ver(pool)
    if chunk:
        ver.set_chunk_grants(chunk)
    rng = np.random.default_rng(99)
    s = W.make_batch(pool, 1500, first_cert=77)
    wb = W.encode_wire_batch(s)
    O_ = int(wb.op_flags_off[-1])
    wb.op_flags = rng.choice(np.array([3, 7, 7, 7, 15, 1, 2, 23, 19, 11], np.uint8), O_)
    ts = np.zeros(O_, np.int64)
    # stored timestamps around each op's grant timestamp (read iff stored > g0.ts)
    base = grant_ts_of_ops(s)
    ts[:] = base + rng.integers(-2, 3, O_)
    wb.op_object_ts = ts
    ids, off = W.server_id_table(4)
    for strict in (True, False):
        g, st = ver.verify_write2(wb, 4, strict)
        o, ost = O.verify_write2(pool.moduli, ids, off, wb, 4, strict)
        np.testing.assert_array_equal(st, ost)
        np.testing.assert_array_equal(g.cert_reason, o.cert_reason)
        np.testing.assert_array_equal(g.cert_fail_op, o.cert_fail_op)
        np.testing.assert_array_equal(g.cert_accept_bits, o.cert_accept_bits)
        for k in ("op_decision", "op_g0", "op_ts"):
            np.testing.assert_array_equal(getattr(g, k), getattr(o, k), err_msg=k)
        assert {1, 2, 3, 4} <= set(np.unique(g.op_decision).tolist())
        assert {0, 9, 10} <= set(np.unique(g.cert_reason).tolist())
    ver.close()


def test_wire_r7_k2(pool7k2):
    ver = _ver(pool7k2)
    s = W.make_batch(pool7k2, 1500, first_cert=11)
    wb = W.encode_wire_batch(s)
    for strict in (True, False):
        g, st = ver.verify_write2(wb, 7, strict)
        soa = ver.verify(s.batch, 7, strict)
        np.testing.assert_array_equal(g.cert_reason, soa.cert_reason)
        np.testing.assert_array_equal(g.cert_accept_bits, soa.cert_accept_bits)
    ver.close()


def _mutate(rng, s, c, ids):
    """One certificate's message with a structural mutation (decode-semantics fuzz)."""
    b = s.batch
    g0, g1 = int(b.cert_grant_off[c]), int(b.cert_grant_off[c + 1])
    mgs = {}
    for g in range(g0, g1):
        gb = b.grant_bytes[int(b.grant_off[g]):int(b.grant_off[g]) + int(b.grant_len[g])].tobytes()
        mgs.setdefault(int(b.signer[g]), []).append((W.grant_object_id(gb), gb, b.sig[g].tobytes()))
    order = list(mgs)
    kind = int(rng.integers(0, 10))
    if kind == 1:
        rng.shuffle(order)  # MultiGrant wire order decides g0
    enc = []
    for r in order:
        items = mgs[r]
        sigs = [(o, sg) for o, _, sg in items]
        if kind == 2:
            sigs = sigs[1:]  # a grant without signature
        extra = b""
        if kind == 3:
            extra = b"\x48\x07" + W._ld(13, b"unknown")  # unknown fields
        enc.append((ids[r], W.encode_multigrant([(o, gb) for o, gb, _ in items], ids[r], "cl", "", sigs) + extra))
    if kind == 4 and len(enc) > 1:
        enc.append((enc[0][0], enc[-1][1]))  # repeated certificate key: first place, last value
    if kind == 5:
        enc.insert(0, (ids[order[0]], enc[0][1]))  # duplicate of the first entry
    ops = [W.encode_operation(2, o) for o, _, _ in mgs[order[0]]]
    if kind == 6:
        ops = ops + ops  # ops repeating a key (multiplicity)
    if kind == 9:  # READ / DELETE / unknown actions, an empty operand1 -> MOCHI_OP_NOT_WRITE or not
        ops = [W.encode_operation(int(rng.choice([0, 1, 2, 5])), o) for o, _, _ in mgs[order[0]]]
        ops.append(W.encode_operation(2, ""))
    m = W.encode_write2(enc, ops)
    if kind == 7 and len(m) > 8:
        i = int(rng.integers(0, len(m)))
        m = m[:i] + bytes([m[i] ^ (1 << int(rng.integers(0, 8)))]) + m[i + 1:]  # random bit flip
    if kind == 8:
        m = m[:int(rng.integers(0, len(m) + 1))]  # truncation
    return m


def test_wire_fuzz_device_equals_oracle(pool4):
    ver = _ver(pool4)
    rng = np.random.default_rng(2024)
    s = W.make_batch(pool4, 2000, first_cert=999)
    msgs = [_mutate(rng, s, c, W.SERVER_IDS) for c in range(s.batch.n_certs)]
    wb = _pack(msgs, pad=3)
    wb.expected_hash = s.batch.expected_hash.copy()
    ids, off = W.server_id_table(4)
    d = ver.decode_write2(wb)
    o = O.w2_decode(wb, ids, off)
    assert_decode_equal(d, o, "fuzz")
    assert len(set(d["msg_status"].tolist())) >= 2
    for strict in (True, False):
        g, st = ver.verify_write2(wb, 4, strict)
        ov, ost = O.verify_write2(pool4.moduli, ids, off, wb, 4, strict)
        np.testing.assert_array_equal(st, ost)
        np.testing.assert_array_equal(g.cert_reason, ov.cert_reason)
        np.testing.assert_array_equal(g.cert_fail_op, ov.cert_fail_op)
        np.testing.assert_array_equal(g.cert_accept_bits, ov.cert_accept_bits)
    ver.close()


def test_wire_edge_shapes(pool4):
    ver = _ver(pool4)
    # no messages
    g, st = ver.verify_write2(_pack([]), 4, True)
    assert st.size == 0
    # op_flags CSR disagreeing with the message -> OPS_MISMATCH / UNDECIDED
    s = W.make_batch(pool4, 40, faults=False)
    wb = W.encode_wire_batch(s)
    wb.op_flags_off = wb.op_flags_off.copy()
    wb.op_flags_off[5:] += 1
    wb.op_flags = np.concatenate([wb.op_flags, np.full(1, 3, np.uint8)])
    g, st = ver.verify_write2(wb, 4, True)
    assert st[4] == mh.MSG_OPS_MISMATCH and g.cert_reason[4] == mh.UNDECIDED and not g.cert_accept[4]
    assert (st[:4] == 0).all() and (st[5:] == 0).all()
    # op_flags from the caller: a non-local op is WRONG_SHARD, never checked
    wb2 = W.encode_wire_batch(s)
    wb2.op_flags[:] = 0
    g2, st2 = ver.verify_write2(wb2, 4, True)
    assert g2.cert_accept.all()
    ver.close()


@pytest.mark.parametrize("with_flags,n_ctx", [(False, 1), (True, 1), (False, 2)])
def test_batcher_concurrent_callers(pool4, with_flags, n_ctx):
    """mochi_batcher: 16 threads each block on their own messages; every caller
    gets exactly the verdict the oracle gives, and the requests were coalesced
    into far fewer GPU batches than messages (n_ctx contexts: that many batches
    in flight, mochi_batcher_create_multi)."""
    import threading

    vers = [_ver(pool4) for _ in range(n_ctx)]
    ver = vers[0]
    s = W.make_batch(pool4, 1200, first_cert=5000)
    wb = W.encode_wire_batch(s)
    if with_flags:
        wb.op_flags = wb.op_flags.copy()
        wb.op_flags[::7] = mh.OP_HAS_SVOC  # some ops not local -> WRONG_SHARD, never checked
    ids, off = W.server_id_table(4)
    ref, ref_st = O.verify_write2(pool4.moduli, ids, off, wb, 4, True)  # the oracle, not the library itself
    b = mh.Batcher(vers, 4, True, max_msgs=128, max_wait_us=2000, with_op_flags=with_flags)
    M = wb.n_msgs
    res = [None] * M
    msgs = [wb.wire[int(wb.msg_off[i]):int(wb.msg_off[i]) + int(wb.msg_len[i])].tobytes() for i in range(M)]
    hashes = [wb.expected_hash[i].tobytes() for i in range(M)]
    flags = [wb.op_flags[int(wb.op_flags_off[i]):int(wb.op_flags_off[i + 1])].tobytes() for i in range(M)]

    def worker(t):
        for i in range(t, M, 16):
            res[i] = b.verify(msgs[i], hashes[i], flags[i] if with_flags else None)

    th = [threading.Thread(target=worker, args=(t,)) for t in range(16)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    nb, nm = b.stats()
    b.close()
    assert nm == M and nb < M // 4
    acc = np.array([r[0] for r in res])
    np.testing.assert_array_equal(acc, ref.cert_accept)
    np.testing.assert_array_equal(np.array([r[1] for r in res], np.uint8), ref.cert_reason)
    np.testing.assert_array_equal(np.array([r[3] for r in res], np.uint8), ref_st)
    for v in vers:
        v.close()


def test_batcher_async_submit(pool4):
    """mochi_batcher_submit: one producer keeps every message in flight at once
    (the event-loop form); each completion callback carries the oracle's verdict
    and the batches grow far beyond what blocked threads would give."""
    import threading

    ver = _ver(pool4)
    s = W.make_batch(pool4, 1200, first_cert=9100)
    wb = W.encode_wire_batch(s)
    ids, off = W.server_id_table(4)
    ref, ref_st = O.verify_write2(pool4.moduli, ids, off, wb, 4, True)
    b = mh.Batcher(ver, 4, True, max_msgs=512, max_wait_us=500)
    M = wb.n_msgs
    res = [None] * M
    left = [M]
    cv = threading.Condition()

    def done_for(i):
        def done(rc, accepted, reason, fail_op, status):
            res[i] = (rc, accepted, reason, status)
            with cv:
                left[0] -= 1
                cv.notify()
        return done

    for i in range(M):
        msg = wb.wire[int(wb.msg_off[i]):int(wb.msg_off[i]) + int(wb.msg_len[i])].tobytes()
        b.submit(msg, wb.expected_hash[i].tobytes(), done_for(i))
    with cv:
        assert cv.wait_for(lambda: left[0] == 0, timeout=60)
    nb, nm = b.stats()
    b.close()
    assert nm == M and nb <= M // 64
    assert all(r[0] == mh.OK for r in res)
    np.testing.assert_array_equal(np.array([r[1] for r in res]), ref.cert_accept)
    np.testing.assert_array_equal(np.array([r[2] for r in res], np.uint8), ref.cert_reason)
    np.testing.assert_array_equal(np.array([r[3] for r in res], np.uint8), ref_st)
    ver.close()


def test_batcher_callback_reentry(pool4):
    """A completion callback may submit to the batcher that runs it (a Java
    CompletableFuture stage running inline submits the next request): a chain of
    submissions, each made from the previous one's callback, gets the oracle's
    verdicts; a blocking verify from a callback is refused with MOCHI_EINVAL; and
    mochi_batcher_destroy from a callback defers the teardown -- requests already
    queued still complete, new ones are refused, the last flusher frees it."""
    import threading

    ver = _ver(pool4)
    s = W.make_batch(pool4, 200, first_cert=9700)
    wb = W.encode_wire_batch(s)
    ids, off = W.server_id_table(4)
    ref, _ = O.verify_write2(pool4.moduli, ids, off, wb, 4, True)
    M = wb.n_msgs
    msgs = [wb.wire[int(wb.msg_off[i]):int(wb.msg_off[i]) + int(wb.msg_len[i])].tobytes() for i in range(M)]
    hashes = [wb.expected_hash[i].tobytes() for i in range(M)]
    b = mh.Batcher(ver, 4, True, max_msgs=64, max_wait_us=100)
    res, errs = [None] * M, []
    fin = threading.Event()

    def chain(i):
        def done(rc, accepted, reason, fail_op, status):
            res[i] = (rc, accepted, reason)
            if i == 0:
                try:  # blocking from the flusher's own thread: refused, not a deadlock
                    b.verify(msgs[0], hashes[0])
                    errs.append("blocking verify from a callback was accepted")
                except mh.MochiError:
                    pass
            try:
                if i + 1 < M:
                    b.submit(msgs[i + 1], hashes[i + 1], chain(i + 1))
                else:
                    fin.set()
            except Exception as e:  # noqa: BLE001 -- surfaced by the assert below
                errs.append(repr(e))
                fin.set()
        return done

    b.submit(msgs[0], hashes[0], chain(0))
    assert fin.wait(120), "callback chain stalled"
    assert not errs, errs
    assert all(r is not None and r[0] == mh.OK for r in res)
    np.testing.assert_array_equal(np.array([r[1] for r in res]), ref.cert_accept)
    np.testing.assert_array_equal(np.array([r[2] for r in res], np.uint8), ref.cert_reason)
    b.close()

    # destroy from inside a callback: 32 requests queued, the first callback destroys
    b2 = mh.Batcher(ver, 4, True, max_msgs=4, max_wait_us=50)
    got, left, refused = [], [32], []
    cv = threading.Condition()

    def cb(i):
        def done(rc, accepted, reason, fail_op, status):
            if i == 0:
                h = b2.h
                b2.close()  # deferred: this callback runs on one of b2's flushers
                # the library refuses a submission after the (deferred) destroy; the
                # batcher is alive at least until this callback returns
                rc2 = b2.lib.mochi_batcher_submit(h, msgs[40], len(msgs[40]), None, 0, hashes[40], b2._cb, 0)
                if rc2 == mh.EINVAL:
                    refused.append(True)
                try:
                    b2.submit(msgs[40], hashes[40], lambda *a: None)
                except mh.MochiError:
                    refused.append(True)
            with cv:
                got.append((i, rc, accepted))
                left[0] -= 1
                cv.notify()
        return done

    for i in range(32):
        b2.submit(msgs[i], hashes[i], cb(i))
    with cv:
        assert cv.wait_for(lambda: left[0] == 0, timeout=60), "queued requests lost after a deferred destroy"
    assert b2.h is None  # freed by its last flusher; close() dropped the handle
    b2.close()  # a second close is a no-op
    assert refused == [True, True]
    got.sort()
    assert [g[1] for g in got] == [mh.OK] * 32
    np.testing.assert_array_equal(np.array([g[2] for g in got]), ref.cert_accept[:32])
    ver.close()


def _fields(b):
    """(tag, raw field bytes) of a protobuf message with varint / length-delimited fields."""
    out, i = [], 0
    while i < len(b):
        j = i
        while b[j] & 0x80:
            j += 1
        tag = b[i]
        j += 1
        if tag & 7 == 0:
            while b[j] & 0x80:
                j += 1
            j += 1
        else:
            n, sh, k = 0, 0, j
            while True:
                n |= (b[k] & 0x7F) << sh
                sh += 7
                k += 1
                if not b[k - 1] & 0x80:
                    break
            j = k + n
        out.append((tag, b[i:j]))
        i = j
    return out


def _reorder(gb):
    """A canonical Grant with its fields written in reverse order (same parsed Grant)."""
    return b"".join(raw for _, raw in reversed(_fields(gb)))


def _fallback_forms(s, c, ids):
    """Certificate c of a synthetic batch re-encoded in legal forms the device fast path
    declines (MOCHI_MSG_FALLBACK); the library's host decoder must decide them."""
    b = s.batch
    g0, g1 = int(b.cert_grant_off[c]), int(b.cert_grant_off[c + 1])
    mgs = {}
    for g in range(g0, g1):
        gb = b.grant_bytes[int(b.grant_off[g]):int(b.grant_off[g]) + int(b.grant_len[g])].tobytes()
        mgs.setdefault(int(b.signer[g]), []).append((W.grant_object_id(gb), gb, b.sig[g].tobytes()))
    ent = [(ids[r], W.encode_multigrant([(o, gb) for o, gb, _ in it], ids[r], "cl", "", [(o, sg) for o, _, sg in it]))
           for r, it in mgs.items()]
    ops = [W.encode_operation(2, o) for o, _, _ in next(iter(mgs.values()))]
    canon = W.encode_write2(ent, ops)
    wc = b"".join(W.encode_map_entry(1, k.encode(), v) for k, v in ent)
    tx = b"".join(W._ld(1, o) for o in ops)
    oid, gb, _ = next(iter(mgs.values()))[0]
    forms = {
        "canonical": canon,
        "wc_split": W._ld(1, wc[:len(W.encode_map_entry(1, ent[0][0].encode(), ent[0][1]))]) + W._ld(2, tx) +
                    W._ld(1, wc[len(W.encode_map_entry(1, ent[0][0].encode(), ent[0][1])):]),
        "tx_twice": W._ld(1, wc) + W._ld(2, tx) + W._ld(2, b""),
        # 29 extra MultiGrants from unknown servers, unsigned, same grant: 33 MultiGrants in all
        "33_multigrants": W.encode_write2(ent + [(f"extra-{i}", W.encode_multigrant([(oid, gb)], f"extra-{i}"))
                                                 for i in range(29)], ops),
        # 33 certificate entries on the wire, 32 distinct keys (the first entry repeated
        # last): the fast path counts wire entries, so this leaves it too
        "33_entries_32_keys": W.encode_write2(ent + [(f"extra-{i}", W.encode_multigrant([(oid, gb)], f"extra-{i}"))
                                                     for i in range(28)] + [ent[0]], ops),
        # one MultiGrant repeating its grants / grantSignatures entries 65 times each
        "65_grant_entries": W.encode_write2(
            [(ids[r], W.encode_multigrant([(o, gb) for o, gb, _ in it] * 65, ids[r], "cl", "",
                                          [(o, sg) for o, _, sg in it] * 65)) for r, it in mgs.items()], ops),
        # every grant's fields out of canonical order: the signature covers the canonical
        # re-encoding (Grant.toByteArray()), so it still verifies
        "noncanonical_grants": W.encode_write2(
            [(ids[r], W.encode_multigrant([(o, _reorder(gb)) for o, gb, _ in it], ids[r], "cl", "",
                                          [(o, sg) for o, _, sg in it])) for r, it in mgs.items()], ops),
    }
    return forms


def test_wire_fallback_messages_decided_on_host(pool4):
    """Legal messages outside the device decoder's fast path are decoded on the host
    with full protobuf-java semantics and verified on the device (signatures are never
    skipped): same verdicts as their canonical form and as the oracle."""
    ver = _ver(pool4)
    s = W.make_batch(pool4, 64, first_cert=4242, faults=False)
    ids4 = W.SERVER_IDS[:4]
    msgs, kinds = [], []
    hashes = []
    for c in range(0, 64, 8):
        for k, m in _fallback_forms(s, c, ids4).items():
            msgs.append(m)
            kinds.append(k)
            hashes.append(s.batch.expected_hash[c])
    wb = _pack(msgs, pad=1)
    wb.expected_hash = np.stack(hashes)
    g, st = ver.verify_write2(wb, 4, True)
    ids, off = W.server_id_table(4)
    o, ost = O.verify_write2(pool4.moduli, ids, off, wb, 4, True)
    np.testing.assert_array_equal(st, ost)
    np.testing.assert_array_equal(g.cert_reason, o.cert_reason)
    np.testing.assert_array_equal(g.cert_accept_bits, o.cert_accept_bits)
    kinds = np.array(kinds)
    assert (st[kinds == "canonical"] == mh.MSG_OK).all()
    assert (st[np.isin(kinds, ["wc_split", "tx_twice", "33_multigrants", "33_entries_32_keys",
                               "65_grant_entries"])] == mh.MSG_FALLBACK).all()
    # decided, and like the canonical form: accepted (no faults in this stream)
    assert g.cert_accept.all(), list(zip(kinds, g.cert_reason))
    ver.close()


def test_unsigned_33_multigrant_certificate_not_accepted(pool4):
    """a client must not be able to skip signature checks by padding a
    certificate past the device fast path (33 MultiGrants): the host decoder decides it
    and, with no valid signature, it is rejected."""
    ver = _ver(pool4)
    s = W.make_batch(pool4, 4, first_cert=77, faults=False)
    b = s.batch
    gb = b.grant_bytes[int(b.grant_off[0]):int(b.grant_off[0]) + int(b.grant_len[0])].tobytes()
    oid = W.grant_object_id(gb)
    ids = W.SERVER_IDS[:4]
    ent = [(ids[i % 4] + ("" if i < 4 else f"-{i}"), W.encode_multigrant([(oid, gb)], ids[i % 4], "cl", "",
                                                                         [(oid, b"\x00" * 256)]))
           for i in range(33)]
    m = W.encode_write2(ent, [W.encode_operation(2, oid)])
    wb = _pack([m])
    wb.expected_hash = b.expected_hash[:1].copy()
    for strict in (True, False):
        g, st = ver.verify_write2(wb, 4, strict)
        assert st[0] == mh.MSG_FALLBACK
        assert not g.cert_accept[0] and g.cert_reason[0] == mh.REJECT_NO_GRANT
    ver.close()


def test_ten_byte_varint_garbage_is_not_canonical(pool4):
    """a negative timestamp is a 10-byte varint whose last byte carries
    bit 63 alone (0x01).  The same value with last byte 0x03 parses identically (bits
    past 64 are dropped) but is not Grant.toByteArray(): the device fast path must
    send it to FALLBACK like the oracle, which re-encodes and compares bytes."""
    ver = _ver(pool4)
    oid, th = "DEMO_KEY_NEG_TS", "ab" * 64
    canon = W.encode_grant(oid, -5, th)
    v = W._varint(-5)
    assert len(v) == 10 and v[-1] == 0x01
    bad = canon.replace(b"\x10" + v, b"\x10" + v[:-1] + b"\x03")
    assert bad != canon and len(bad) == len(canon)
    ids = W.SERVER_IDS[:4]
    msgs = []
    for gb in (canon, bad):
        ent = [(ids[r], W.encode_multigrant([(oid, gb)], ids[r], "cl", "", [(oid, b"\x00" * 256)])) for r in range(4)]
        msgs.append(W.encode_write2(ent, [W.encode_operation(2, oid)]))
    wb = _pack(msgs)
    wb.expected_hash = np.zeros((2, 128), np.uint8)
    g, st = ver.verify_write2(wb, 4, True)
    wids, woff = W.server_id_table(4)
    o, ost = O.verify_write2(pool4.moduli, wids, woff, wb, 4, True)
    np.testing.assert_array_equal(st, ost)
    assert st[0] == mh.MSG_OK and st[1] == mh.MSG_FALLBACK, st
    np.testing.assert_array_equal(g.cert_reason, o.cert_reason)
    ver.close()


def _bad_key_byte(m, oid):
    """m with the last byte of its first grants entry's key made 0xFF (invalid UTF-8)."""
    kb = oid.encode()
    pat = b"\x0a" + bytes([len(kb)]) + kb + b"\x12"
    assert pat in m
    return m.replace(pat, pat[:-2] + b"\xff\x12", 1)


def _matcher_forms(s, c, ids):
    """Certificate c re-encoded at and around the edges of k_w2_mg's layout matcher
    (mg_match: the reference encoder's one-grant MultiGrant, ASCII key and serverId
    <= 60 bytes, signature entry under the grant's key, Grant in its common canonical
    shape <= 192 bytes).  Each form is legal protobuf; the matcher either decodes it
    exactly as the walk does or leaves it to the walk."""
    b = s.batch
    g0, g1 = int(b.cert_grant_off[c]), int(b.cert_grant_off[c + 1])
    items = []
    for g in range(g0, g1):
        gb = b.grant_bytes[int(b.grant_off[g]):int(b.grant_off[g]) + int(b.grant_len[g])].tobytes()
        items.append((int(b.signer[g]), W.grant_object_id(gb), gb, b.sig[g].tobytes()))
    r0, oid, gb, _ = items[0]
    p = O.grant_parse(gb)
    ts, th = int(p["timestamp"]), p["transaction_hash"].decode()
    th_alt = th[:-1] + ("0" if th[-1] != "0" else "1")

    def msg(grant_of=lambda r, g: g, key_of=lambda r, o: o, sig_key_of=None, sid_of=lambda r: ids[r],
            sig_of=lambda r, sg: sg, extra_of=None, ops_of=None, cert_key_of=lambda r: ids[r], dup_entry=False):
        ent = []
        for r, o, g, sg in items:
            k = key_of(r, o)
            sk = sig_key_of(r, k) if sig_key_of else k
            gl = grant_of(r, g)
            grants = gl if isinstance(gl, list) else [(k, gl)]
            mg = W.encode_multigrant(grants, sid_of(r), "", "", [(sk, sig_of(r, sg))])
            ent.append((cert_key_of(r), mg + (extra_of(r) if extra_of else b"")))
        if dup_entry:
            ent.append(ent[0])  # a repeated certificate key: first position, last value
        key = key_of(r0, oid)
        return W.encode_write2(ent, ops_of(key) if ops_of else [W.encode_operation(2, key)])

    return {
        "plain": msg(),
        "sig_under_other_key": msg(sig_key_of=lambda r, k: k + "x"),
        "key_60": msg(key_of=lambda r, o: (o + "-" + "k" * 60)[:60]),
        "key_61": msg(key_of=lambda r, o: (o + "-" + "k" * 61)[:61]),
        "key_non_ascii": msg(key_of=lambda r, o: o + "é"),
        "sid_non_ascii": msg(sid_of=lambda r: ids[r] + "é"),
        "sid_61": msg(sid_of=lambda r: (ids[r] + "-" + "s" * 61)[:61]),
        "sig_255": msg(sig_of=lambda r, sg: sg[:255]),
        "trailing_unknown": msg(extra_of=lambda r: b"\x48\x07"),
        "short_grant": msg(grant_of=lambda r, g: W.encode_grant(oid, ts, "ab")),
        "grant_hash_127": msg(grant_of=lambda r, g: W.encode_grant(oid, ts, "c" * 127)),
        "grant_hash_128": msg(grant_of=lambda r, g: W.encode_grant(oid, ts, "c" * 128)),
        "grant_ts_1": msg(grant_of=lambda r, g: W.encode_grant(oid, 1, th)),
        "grant_ts_9_bytes": msg(grant_of=lambda r, g: W.encode_grant(oid, 1 << 62, th)),
        "grant_ts_negative": msg(grant_of=lambda r, g: W.encode_grant(oid, -7, th)),
        "grant_configstamp": msg(grant_of=lambda r, g: W.encode_grant(oid, ts, th, configstamp=3)),
        "grant_oid_non_ascii": msg(grant_of=lambda r, g: W.encode_grant(oid + "é", ts, th)),
        "grant_hash_non_ascii": msg(grant_of=lambda r, g: W.encode_grant(oid, ts, th[:-1] + "é")),
        "grant_reordered": msg(grant_of=lambda r, g: _reorder(g)),
        "grant_200_bytes": msg(grant_of=lambda r, g: W.encode_grant(oid + "o" * 40, ts, th)),
        "key_bad_utf8": _bad_key_byte(msg(), oid),
        # level-1 shapes: operations, certificate keys
        "op_no_action": msg(ops_of=lambda k: [W.encode_operation(0, k)]),
        "op_operand2": msg(ops_of=lambda k: [W.encode_operation(2, k, "v")]),
        "ops_4": msg(ops_of=lambda k: [W.encode_operation(2, k + str(i) if i else k) for i in range(4)]),
        "ops_5": msg(ops_of=lambda k: [W.encode_operation(2, k + str(i) if i else k) for i in range(5)]),
        "op_second_names_key": msg(ops_of=lambda k: [W.encode_operation(2, k + "z"), W.encode_operation(2, k)]),
        "op_key_57": msg(key_of=lambda r, o: (o + "-" + "q" * 57)[:57]),
        "cert_key_non_ascii": msg(cert_key_of=lambda r: ids[r] + "é"),
        "cert_key_57": msg(cert_key_of=lambda r: (ids[r] + "-" + "c" * 57)[:57]),
        "cert_key_repeated": msg(dup_entry=True),
        "cert_keys_equal_pairs": msg(cert_key_of=lambda r: ids[r % 2]),
        # the first MultiGrant names the grant key twice: LinkedHashMap keeps the first
        # position and the LAST value (a variant: another transaction hash), while every
        # other MultiGrant carries the first value's bytes -- they must not take the
        # variant's prep results
        "repeated_key_first_mg": msg(grant_of=lambda r, g: [(oid, g), (oid, W.encode_grant(oid, ts, th_alt))]
                                     if r == r0 else g),
    }


def test_wire_layout_matcher_edges(pool4):
    """Decode arrays and verdicts == oracle for every form around the layout matcher's
    edges (and the walk it falls back to), at every message alignment."""
    ver = _ver(pool4)
    s = W.make_batch(pool4, 16, first_cert=5150, faults=False)
    ids4 = W.SERVER_IDS[:4]
    msgs, kinds, hashes = [], [], []
    for c in range(0, 16, 4):
        forms = _matcher_forms(s, c, ids4)
        for kind, m in forms.items():
            msgs.append(m)
            kinds.append(kind)
            hashes.append(s.batch.expected_hash[c])
    ids, off = W.server_id_table(4)
    for pad in (1, 3):
        wb = _pack(msgs, pad=pad)
        wb.expected_hash = np.stack(hashes)
        d = ver.decode_write2(wb)
        o = O.w2_decode(wb, ids, off)
        assert_decode_equal(d, o, f"matcher forms pad={pad}")
        for strict in (True, False):
            g, st = ver.verify_write2(wb, 4, strict)
            ov, ost = O.verify_write2(pool4.moduli, ids, off, wb, 4, strict)
            np.testing.assert_array_equal(st, ost)
            np.testing.assert_array_equal(g.cert_reason, ov.cert_reason, err_msg=str(list(zip(kinds, g.cert_reason))))
            np.testing.assert_array_equal(g.cert_accept_bits, ov.cert_accept_bits)
    # (the last verify ran with strict = False: three valid grants of four are a quorum)
    kinds = np.array(kinds)
    acc = {k: g.cert_accept[kinds == k] for k in set(kinds.tolist())}
    for k in ("plain", "key_60", "key_61", "key_non_ascii", "trailing_unknown", "grant_reordered",
              "op_operand2", "op_key_57", "cert_key_non_ascii", "cert_key_57", "cert_key_repeated",
              "repeated_key_first_mg"):  # the last: the three other MultiGrants carry the signed bytes
        assert acc[k].all(), (k, g.cert_reason[kinds == k])
    for k in ("sig_under_other_key", "sig_255", "key_bad_utf8", "grant_200_bytes"):
        assert not acc[k].any(), k
    ver.close()


def test_context_closed_before_its_batcher(pool4):
    """Closing a Verifier while a Batcher on it is alive (explicit close, or __del__
    order in a host language) neither blocks nor frees the context under the
    batcher: mochi_ctx_destroy returns at once, the batcher keeps verifying with
    the oracle's verdicts, and the batcher's own teardown frees the context."""
    import time

    ver = _ver(pool4)
    s = W.make_batch(pool4, 64, first_cert=9900)
    wb = W.encode_wire_batch(s)
    ids, off = W.server_id_table(4)
    ref, _ = O.verify_write2(pool4.moduli, ids, off, wb, 4, True)
    b = mh.Batcher(ver, 4, True, max_msgs=64, max_wait_us=100)
    t0 = time.perf_counter()
    ver.close()
    assert time.perf_counter() - t0 < 5.0
    for i in range(wb.n_msgs):
        msg = wb.wire[int(wb.msg_off[i]):int(wb.msg_off[i]) + int(wb.msg_len[i])].tobytes()
        acc, reason, _, _ = b.verify(msg, wb.expected_hash[i].tobytes())
        assert acc == bool(ref.cert_accept[i]) and reason == ref.cert_reason[i]
    b.close()
