"""Write2ToServer wire path, CPU side: the oracle's protobuf-java-semantics
decoder (oracle/mochi_oracle.c) turns the encoded messages back into exactly
the SoA certificate batch they were built from, and the verdicts through the
wire equal the verdicts of the SoA batch."""
import numpy as np
import pytest

import oracle_ffi as O
import workload as W


@pytest.fixture(scope="module")
def pool4():
    return W.build_pool(R=4, k=1, P=64, P_f=32)


@pytest.fixture(scope="module")
def pool4k2():
    return W.build_pool(R=4, k=2, P=32, P_f=16)


@pytest.mark.parametrize("which", ["k1", "k2"])
def test_oracle_decode_roundtrip(pool4, pool4k2, which):
    pool = pool4 if which == "k1" else pool4k2
    s = W.make_batch(pool, 300, first_cert=41)
    wb = W.encode_wire_batch(s, pad=3, client_id="client-7f3a", mg_hash=True)
    ids, off = W.server_id_table(4)
    d = O.w2_decode(wb, ids, off)
    b = s.batch
    assert (d["msg_status"] == 0).all()
    np.testing.assert_array_equal(d["cert_grant_off"], b.cert_grant_off)
    np.testing.assert_array_equal(d["cert_op_off"], b.cert_op_off)
    np.testing.assert_array_equal(d["signer"], b.signer)
    np.testing.assert_array_equal(d["grant_key"], b.grant_key)
    np.testing.assert_array_equal(d["sig"], b.sig)
    np.testing.assert_array_equal(d["op_key"], b.op_key)
    np.testing.assert_array_equal(d["op_flags"], b.op_flags)
    # grant bytes are wire slices equal to the signed bytes
    for g in range(0, b.n_grants, 7):
        a = wb.wire[int(d["grant_off"][g]):int(d["grant_off"][g]) + int(d["grant_len"][g])]
        e = b.grant_bytes[int(b.grant_off[g]):int(b.grant_off[g]) + int(b.grant_len[g])]
        np.testing.assert_array_equal(a, e)


def test_oracle_wire_verdicts_equal_soa_verdicts(pool4):
    s = W.make_batch(pool4, 400, first_cert=7)
    wb = W.encode_wire_batch(s)
    ids, off = W.server_id_table(4)
    v, st = O.verify_write2(pool4.moduli, ids, off, wb, 4, True)
    o = O.verify_batch(pool4.moduli, s.batch, 4, True, 8)
    assert (st == 0).all()
    np.testing.assert_array_equal(v.cert_accept_bits, o.cert_accept_bits)
    np.testing.assert_array_equal(v.cert_reason, o.cert_reason)
    np.testing.assert_array_equal(v.cert_fail_op, o.cert_fail_op)


def _golden():
    import json
    import os

    d = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "write2_vectors.json")))
    ids = d["server_ids"]
    blob = "".join(ids).encode()
    off = np.zeros(len(ids) + 1, np.uint32)
    np.cumsum([len(x.encode()) for x in ids], out=off[1:])
    return d["vectors"], ids, np.frombuffer(blob, np.uint8).copy(), off


def _single(data: bytes, n_ops=None):
    return W.WireBatch(wire=np.frombuffer(data or b"\x00", np.uint8).copy(), msg_off=np.zeros(1, np.uint64),
                       msg_len=np.array([len(data)], np.uint32), op_flags_off=None, op_flags=np.zeros(1, np.uint8),
                       expected_hash=np.zeros((1, 128), np.uint8))


def check_decode_against_golden(v, d, wire, ids, full=False):
    """Decoded arrays of one golden message vs its pinned status / order / content.
    full=True: the full (host) decode -- v["full"] / v["full_status"], grant bytes in
    d["blob"] (re-serialized Grant.toByteArray())."""
    status, order = (v["full_status"], v["full"]) if full else (v["status"], v["order"])
    assert int(d["msg_status"][0]) == status, v["name"]
    if status != 0:
        return
    content = v["py_content"]
    java = v.get("java_grant_bytes", {})
    if full:
        wire = d["blob"]
    assert [o for o in order["ops"]] == content["ops"], v["name"]
    # op slots: ops naming the same operand1 share a slot
    exp_slots = [order["ops"].index(k) for k in order["ops"]]
    got_slots = d["op_key"].tolist()
    n = len(exp_slots)
    assert len(got_slots) == n, v["name"]
    assert all((got_slots[i] == got_slots[j]) == (exp_slots[i] == exp_slots[j]) for i in range(n) for j in range(n)), v["name"]
    # Operation.action (last value wins) / empty operand1 -> MOCHI_OP_NOT_WRITE; the op key slices
    for j, (k, act) in enumerate(zip(content["ops"], content["actions"])):
        notw = act not in (1, 2) or k == ""
        assert bool(d["op_flags"][j] & 0x10) == notw, (v["name"], j, act)
        o, n = int(d["op_key_off"][j]), int(d["op_key_len"][j])
        assert bytes(wire[o:o + n]).decode() == k, (v["name"], j)
    # MultiGrant boundaries: one per certificate entry (first occurrence), its grants
    assert d["cert_mg_off"].tolist() == [0, len(order["certs"])], v["name"]
    assert np.diff(d["mg_grant_off"]).tolist() == [len(x) for x in order["grants"]], v["name"]
    g = 0
    assert sum(len(x) for x in order["grants"]) == int(d["cert_grant_off"][1]), v["name"]
    for ci, ckey in enumerate(order["certs"]):
        c = content["certs"][ckey]
        sid = c["serverId"]
        exp_signer = ids.index(sid) if sid in ids else 0xFFFF
        for gkey in order["grants"][ci]:
            o, n = int(d["grant_off"][g]), int(d["grant_len"][g])
            exp = java.get(ckey, {}).get(gkey, c["grants"][gkey])
            assert bytes(wire[o:o + n]).hex() == exp, (v["name"], ckey, gkey)
            assert int(d["signer"][g]) == exp_signer, v["name"]
            s = c["sigs"].get(gkey)
            exp_sig = bytes.fromhex(s) if s is not None and len(s) == 512 else bytes(256)
            assert d["sig"][g].tobytes() == exp_sig, (v["name"], gkey)
            exp_key = order["ops"].index(gkey) if gkey in order["ops"] else None
            if exp_key is None:
                assert int(d["grant_key"][g]) == 0xFF, v["name"]
            else:
                assert int(d["grant_key"][g]) == got_slots[exp_key], v["name"]
            g += 1


def test_oracle_decode_matches_golden_vectors():
    vecs, ids, blob, off = _golden()
    assert len(vecs) >= 50
    for v in vecs:
        data = bytes.fromhex(v["hex"])
        d = O.w2_decode(_single(data), blob, off)
        check_decode_against_golden(v, d, data, ids)


def test_oracle_full_decode_matches_golden_vectors():
    """The oracle's full protobuf-java decode (what the library's host decoder must
    match for fast-path exits): merged repeated fields, merged map values, last-entry
    map values, re-serialized Grant bytes (python google.protobuf pins the values;
    protobuf-java's unknown-field order is written by hand), any MultiGrant count."""
    vecs, ids, blob, off = _golden()
    n_full = 0
    for v in vecs:
        data = bytes.fromhex(v["hex"])
        d = O.w2_decode_full(_single(data), blob, off)
        if v["status"] == 1:
            assert int(d["msg_status"][0]) == 1, v["name"]
            continue
        check_decode_against_golden(v, d, data, ids, full=True)
        n_full += v["status"] == 2 and v["full_status"] == 0
    assert n_full >= 14


def test_oracle_ops_mismatch_status():
    vecs, ids, blob, off = _golden()
    v = next(x for x in vecs if x["name"] == "canonical")
    data = bytes.fromhex(v["hex"])
    wb = _single(data)
    wb.op_flags_off = np.array([0, 3], np.uint32)  # message holds 2 ops
    wb.op_flags = np.full(3, 3, np.uint8)
    d = O.w2_decode(wb, blob, off)
    assert int(d["msg_status"][0]) == 3


def test_oracle_fast_path_counts_wire_entries():
    """The device fast path bounds its per-lane map resolution by counting entries
    on the wire, repeated keys included (w2_decode.hip k_w2_msg / k_w2_mg; restated in
    oracle/mochi_oracle.c decode_one): 32 certificate entries decode, 33 leave the fast
    path even when two share a key; a decoded MultiGrant with 65 grants or 65
    grantSignatures entries (one key repeated) leaves it too.  The full decode still
    yields the LinkedHashMap result for all of them."""
    ids, off = W.server_id_table(4)
    gb = W.encode_grant("obj-a", 7, "h" * 128, 1, 1)
    sig = b"\x01" * 256

    def mg(n_grants=1, n_sigs=1, sid=W.SERVER_IDS[0]):
        return W.encode_multigrant([("obj-a", gb)] * n_grants, sid, "cl", "", [("obj-a", sig)] * n_sigs)

    ops = [W.encode_operation(2, "obj-a")]
    cases = {
        "32_entries": (W.encode_write2([(f"k{i}", mg()) for i in range(32)], ops), 0, 32),
        "33_entries_32_keys": (W.encode_write2([(f"k{i}", mg()) for i in range(32)] + [("k0", mg())], ops), 2, 32),
        "64_grant_entries": (W.encode_write2([("k0", mg(n_grants=64))], ops), 0, 1),
        "65_grant_entries": (W.encode_write2([("k0", mg(n_grants=65))], ops), 2, 1),
        "65_sig_entries": (W.encode_write2([("k0", mg(n_sigs=65))], ops), 2, 1),
    }
    for name, (m, fast, n_mgs_full) in cases.items():
        d = O.w2_decode(_single(m), ids, off)
        assert int(d["msg_status"][0]) == fast, name
        f = O.w2_decode_full(_single(m), ids, off)
        assert int(f["msg_status"][0]) == 0, name
        assert int(f["cert_mg_off"][1]) == n_mgs_full, name
        assert int(f["cert_grant_off"][1]) == n_mgs_full, name  # one distinct grant per MultiGrant


def test_oracle_ten_byte_varint_garbage_not_canonical():
    """A negative timestamp's 10-byte varint ends in 0x01; with 0x03 instead the
    Grant parses to the same fields but is not Grant.toByteArray(), so the decoder's
    fast path declines it (FALLBACK, 2) while the canonical form decodes (OK, 0).
    The device twin is tests/test_write2_wire_gpu.py."""
    ids, off = W.server_id_table(4)
    oid = "DEMO_KEY_NEG_TS"
    canon = W.encode_grant(oid, -5, "ab" * 64)
    v = W._varint(-5)
    bad = canon.replace(b"\x10" + v, b"\x10" + v[:-1] + b"\x03")
    st = []
    for gb in (canon, bad):
        ent = [(W.SERVER_IDS[r], W.encode_multigrant([(oid, gb)], W.SERVER_IDS[r], "cl", "", [(oid, b"\x00" * 256)]))
               for r in range(4)]
        d = O.w2_decode(_single(W.encode_write2(ent, [W.encode_operation(2, oid)])), ids, off)
        st.append(int(d["msg_status"][0]))
    assert st == [0, 2], st
