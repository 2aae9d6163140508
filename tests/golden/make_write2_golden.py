#!/usr/bin/env python3
"""Generate tests/golden/write2_vectors.json: Write2ToServer wire messages and
what an independent protobuf implementation makes of them.

    python tests/golden/make_write2_golden.py

Each vector holds hand-encoded message bytes (hex) and
  py_ok       whether Python google.protobuf 7.35.1 parses it as a
              Write2ToServer (hand-built descriptor of MochiProtocol.proto:
              107-147 + MultiGrant.grantSignatures = 5) —
              malformed bytes / bad UTF-8 in a proto3 string fail it;
  py_content  for parseable messages: every certificate entry (by map key)
              with its MultiGrant.serverId, each grant's canonical bytes
              (SerializeToString of the parsed Grant) and each signature,
              plus the operations' operand1 — the value semantics (last value
              wins, repeated message fields merge) pinned independently;
  status      the expected enum mochi_msg_status of the device decoder's
              fast path (written by hand from include/mochi_hip.h);
  order       for status OK: the expected decode order — certificate map keys
              and per-MultiGrant grant keys in protobuf-java LinkedHashMap
              insertion order (first occurrence keeps its place), written by
              hand; Python's map iteration order is not insertion order, so
              this part is pinned by the restatement only.
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "mochi-db_amd"))

PKG = "edu.stanford.cs244b.mochi.server.messages"


def classes():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    T = descriptor_pb2.FieldDescriptorProto
    fdp = descriptor_pb2.FileDescriptorProto()
    fdp.name = "mochi_write2_golden.proto"
    fdp.package = PKG
    fdp.syntax = "proto3"
    e = fdp.enum_type.add()
    e.name = "OperationResultStatus"
    for nm, num in (("OK", 0), ("WRONG_SHARD", 1)):
        v = e.value.add()
        v.name, v.number = nm, num
    e = fdp.enum_type.add()
    e.name = "OperationAction"
    for nm, num in (("READ", 0), ("DELETE", 1), ("WRITE", 2)):
        v = e.value.add()
        v.name, v.number = nm, num

    def msg(name, fields, nested=()):
        m = fdp.message_type.add()
        m.name = name
        for nd in nested:
            m.nested_type.add().CopyFrom(nd)
        for nm, num, ty, tn, label in fields:
            f = m.field.add()
            f.name, f.number, f.type, f.label = nm, num, ty, label
            if tn:
                f.type_name = tn
        return m

    def entry(name, vty, vtn):
        d = descriptor_pb2.DescriptorProto()
        d.name = name
        d.options.map_entry = True
        k = d.field.add()
        k.name, k.number, k.type, k.label = "key", 1, T.TYPE_STRING, T.LABEL_OPTIONAL
        v = d.field.add()
        v.name, v.number, v.type, v.label = "value", 2, vty, T.LABEL_OPTIONAL
        if vtn:
            v.type_name = vtn
        return d

    O, R = T.LABEL_OPTIONAL, T.LABEL_REPEATED
    p = "." + PKG + "."
    msg("Operation", [("action", 1, T.TYPE_ENUM, p + "OperationAction", O), ("operand1", 2, T.TYPE_STRING, "", O),
                      ("operand2", 3, T.TYPE_STRING, "", O), ("operand3", 4, T.TYPE_STRING, "", O)])
    msg("Transaction", [("operations", 1, T.TYPE_MESSAGE, p + "Operation", R)])
    msg("Grant", [("objectId", 1, T.TYPE_STRING, "", O), ("timestamp", 2, T.TYPE_INT64, "", O),
                  ("configstamp", 3, T.TYPE_INT64, "", O), ("transactionHash", 4, T.TYPE_STRING, "", O),
                  ("status", 5, T.TYPE_ENUM, p + "OperationResultStatus", O)])
    msg("MultiGrant", [("grants", 1, T.TYPE_MESSAGE, p + "MultiGrant.GrantsEntry", R),
                       ("clientId", 2, T.TYPE_STRING, "", O), ("hash", 3, T.TYPE_STRING, "", O),
                       ("serverId", 4, T.TYPE_STRING, "", O),
                       ("grantSignatures", 5, T.TYPE_MESSAGE, p + "MultiGrant.GrantSignaturesEntry", R)],
        nested=[entry("GrantsEntry", T.TYPE_MESSAGE, p + "Grant"), entry("GrantSignaturesEntry", T.TYPE_BYTES, "")])
    msg("WriteCertificate", [("grants", 1, T.TYPE_MESSAGE, p + "WriteCertificate.GrantsEntry", R)],
        nested=[entry("GrantsEntry", T.TYPE_MESSAGE, p + "MultiGrant")])
    msg("Write2ToServer", [("writeCertificate", 1, T.TYPE_MESSAGE, p + "WriteCertificate", O),
                           ("transaction", 2, T.TYPE_MESSAGE, p + "Transaction", O)])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    get = lambda n: message_factory.GetMessageClass(pool.FindMessageTypeByName(PKG + "." + n))
    return get("Write2ToServer"), get("Grant")


def vectors():
    import workload as W

    ld, ent, var = W._ld, W.encode_map_entry, W._varint
    th = "ab" * 64
    g = lambda oid, ts, h=th: W.encode_grant(oid, ts, h)
    sig = lambda i: bytes(((i * 37 + j * 11) & 0xFF) for j in range(256))
    SID = W.SERVER_IDS

    def mg(sid, grants, sigs=None, cid="client-1", h=th, extra=b""):
        return W.encode_multigrant(grants, sid, cid, h, sigs) + extra

    def w2(mgs, ops, wc_extra=b"", tx_extra=b"", top_extra=b""):
        wc = b"".join(ent(1, k.encode(), v) for k, v in mgs) + wc_extra
        tx = b"".join(ld(1, o) for o in ops) + tx_extra
        return ld(1, wc) + ld(2, tx) + top_extra

    op = lambda k, v="val": W.encode_operation(2, k, v)
    A, B = "DEMO_KEY_A", "DEMO_KEY_B"
    gA = [g(A, 1000 + r) for r in range(3)]
    gB = [g(B, 2000 + r) for r in range(3)]

    def std(r, extra=b"", sids=None):
        return mg((sids or SID)[r], [(A, gA[r]), (B, gB[r])], [(A, sig(2 * r)), (B, sig(2 * r + 1))], extra=extra)

    base_mgs = [(SID[r], std(r)) for r in range(3)]
    base_ops = [op(A), op(B)]
    V = []

    def add(name, data, status, order=None, why="", full=None, full_status=0):
        # full / full_status: for fast-path exits (status 2), the order the library's host decoder
        # (full protobuf-java semantics) must produce, and whether it decides the message (0) or
        # leaves it undecided (2: more than 64 operations)
        V.append(dict(name=name, hex=data.hex(), status=status, order=order, why=why,
                      full=full if status == 2 else order, full_status=full_status if status == 2 else status))

    order3 = {"certs": [SID[0], SID[1], SID[2]], "grants": [[A, B]] * 3, "ops": [A, B]}
    add("canonical", w2(base_mgs, base_ops), 0, order3)
    add("empty_message", b"", 0, {"certs": [], "grants": [], "ops": []})
    add("no_transaction", ld(1, b"".join(ent(1, k.encode(), v) for k, v in base_mgs)), 0,
        {"certs": [SID[0], SID[1], SID[2]], "grants": [[A, B]] * 3, "ops": []})
    # repeated map keys: first position, last value
    dup_cert = [base_mgs[0], base_mgs[1], (SID[0], mg(SID[0], [(B, gB[0])], [(B, sig(1))])), base_mgs[2]]
    add("dup_cert_key", w2(dup_cert, base_ops), 0, {"certs": [SID[0], SID[1], SID[2]], "grants": [[B], [A, B], [A, B]], "ops": [A, B]},
        "LinkedHashMap.put keeps the first position, value of the last entry")
    dup_grant = mg(SID[1], [(A, gA[1]), (B, gB[1]), (A, g(A, 1001))], [(A, sig(2)), (B, sig(3))])
    add("dup_grant_key", w2([base_mgs[0], (SID[1], dup_grant), base_mgs[2]], base_ops), 0,
        {"certs": [SID[0], SID[1], SID[2]], "grants": [[A, B], [A, B], [A, B]], "ops": [A, B]})
    dup_sig = mg(SID[2], [(A, gA[2]), (B, gB[2])], [(A, sig(9)), (B, sig(5)), (A, sig(4))])
    add("dup_sig_key_last_wins", w2([base_mgs[0], base_mgs[1], (SID[2], dup_sig)], base_ops), 0, order3)
    # unknown fields at every level (varint, fixed64, fixed32, length-delimited, group)
    unk = var(9 << 3 | 0) + var(300) + var(10 << 3 | 1) + b"\x01" * 8 + var(11 << 3 | 5) + b"\x02" * 4 + \
        ld(12, b"zz") + var(13 << 3 | 3) + var(1 << 3 | 0) + b"\x05" + var(13 << 3 | 4)
    add("unknown_fields_everywhere", w2([(SID[0], std(0, extra=unk)), base_mgs[1], base_mgs[2]], [op(A) + unk, op(B)],
                                        wc_extra=unk, tx_extra=unk, top_extra=unk), 0, order3)
    # known field, wrong wire type -> unknown, skipped (serverId lost -> unknown signer)
    mg_wt = mg("", [(A, gA[0]), (B, gB[0])], [(A, sig(0)), (B, sig(1))]) + var(4 << 3 | 0) + var(7)
    add("serverid_wrong_wire_type", w2([(SID[0], mg_wt), base_mgs[1], base_mgs[2]], base_ops), 0, order3)
    add("unknown_server_id", w2([(SID[0], std(0, sids=["server-nobody"] * 3)), base_mgs[1], base_mgs[2]], base_ops), 0, order3)
    add("missing_signature", w2([(SID[0], mg(SID[0], [(A, gA[0]), (B, gB[0])], [(B, sig(1))])), base_mgs[1], base_mgs[2]],
                                base_ops), 0, order3)
    add("short_signature", w2([(SID[0], mg(SID[0], [(A, gA[0]), (B, gB[0])], [(A, sig(0)[:255]), (B, sig(1))])),
                               base_mgs[1], base_mgs[2]], base_ops), 0, order3)
    add("grant_key_not_an_op", w2(base_mgs, [op(A)]), 0, {"certs": [SID[0], SID[1], SID[2]], "grants": [[A, B]] * 3, "ops": [A]})
    add("ops_same_key", w2(base_mgs, [op(A), op(B), op(A, "again")]), 0,
        {"certs": [SID[0], SID[1], SID[2]], "grants": [[A, B]] * 3, "ops": [A, B, A]})
    add("entry_without_key_or_value", w2([("", b"")] + base_mgs, base_ops) , 0,
        {"certs": ["", SID[0], SID[1], SID[2]], "grants": [[], [A, B], [A, B], [A, B]], "ops": [A, B]})
    add("grant_entry_empty_value", w2([(SID[0], mg(SID[0], [(A, b""), (B, gB[0])], [(A, sig(0)), (B, sig(1))])),
                                       base_mgs[1], base_mgs[2]], base_ops), 0, order3)
    add("action_unknown_enum", w2(base_mgs, [W.encode_operation(9, A, "v"), op(B)]), 0, order3)
    # Operation.action / operand1 drive MOCHI_OP_NOT_WRITE (the read/apply step throws unless WRITE / DELETE
    # with a non-empty, hence write-locked, operand1: InMemoryDataStore.java:339-358, :529, :562)
    add("action_read_and_delete", w2(base_mgs, [W.encode_operation(0, A), W.encode_operation(1, B)]), 0, order3)
    add("action_given_twice_last_wins", w2(base_mgs, [b"\x08\x00" + op(A), op(B) + b"\x08\x00"]), 0, order3)
    add("operand1_empty", w2(base_mgs, [op(A), W.encode_operation(2, "", "v")]), 0,
        {"certs": [SID[0], SID[1], SID[2]], "grants": [[A, B]] * 3, "ops": [A, ""]})
    add("utf8_multibyte_keys", w2([(SID[0], mg(SID[0], [("clé-ü", g("clé-ü", 5))], [("clé-ü", sig(3))]))],
                                  [op("clé-ü")]), 0, {"certs": [SID[0]], "grants": [["clé-ü"]], "ops": ["clé-ü"]})
    # fast-path exits (legal protobuf, host fallback)
    wc_bytes = b"".join(ent(1, k.encode(), v) for k, v in base_mgs)
    tx_bytes = b"".join(ld(1, o) for o in base_ops)
    add("write_certificate_twice", ld(1, wc_bytes) + ld(2, tx_bytes) + ld(1, b""), 2,
        why="singular message field repeated: protobuf merges, fast path declines", full=order3)
    add("transaction_twice", ld(1, wc_bytes) + ld(2, tx_bytes) + ld(2, ld(1, op("C"))), 2,
        full={"certs": [SID[0], SID[1], SID[2]], "grants": [[A, B]] * 3, "ops": [A, B, "C"]})
    mg_twice = ld(1, ld(1, SID[0].encode()) + ld(2, std(0)) + ld(2, W.encode_multigrant([], "", "", "", None)))
    add("multigrant_value_twice", ld(1, mg_twice + b"".join(ent(1, k.encode(), v) for k, v in base_mgs[1:])) + ld(2, tx_bytes), 2,
        full=order3)
    g_twice = ld(1, ld(1, A.encode()) + ld(2, gA[0]) + ld(2, W.encode_grant("", 77, "")))
    add("grant_value_twice", w2([(SID[0], g_twice + ld(4, SID[0].encode())), base_mgs[1], base_mgs[2]], base_ops), 2,
        full={"certs": [SID[0], SID[1], SID[2]], "grants": [[A], [A, B], [A, B]], "ops": [A, B]})
    # the same key's MultiGrant given in two certificate entries AND merged: last entry wins, no merge across entries
    add("cert_key_twice_not_merged", w2([(SID[0], std(0)), (SID[0], mg(SID[0], [(B, gB[0])], [(B, sig(1))])),
                                         base_mgs[1]], base_ops) + ld(1, ent(1, SID[2].encode(), std(2))), 2,
        full={"certs": [SID[0], SID[1], SID[2]], "grants": [[B], [A, B], [A, B]], "ops": [A, B]})
    # unknown fields of several numbers / wire types inside a Grant: Grant.toByteArray() re-emits them
    # (UnknownFieldSet: ascending field number; per number varint, fixed32, fixed64, bytes, group)
    unk_g = g(A, 5) + ld(9, b"zz") + var(7 << 3 | 5) + b"\x01\x02\x03\x04" + var(9 << 3 | 0) + var(3) + \
        var(7 << 3 | 0) + var(8) + var(8 << 3 | 3) + var(2 << 3 | 0) + var(1) + var(8 << 3 | 4)
    add("grant_unknown_fields_reordered", w2([(SID[0], mg(SID[0], [(A, unk_g)], [(A, sig(0))]))], [op(A)]), 2,
        full={"certs": [SID[0]], "grants": [[A]], "ops": [A]},
        why="Python's serializer keeps unknown fields in arrival order; protobuf-java's UnknownFieldSet sorts "
            "them, so the Java bytes are written here by hand (java_grant_bytes)")
    V[-1]["java_grant_bytes"] = {SID[0]: {A: (g(A, 5) + var(7 << 3 | 0) + var(8) + var(7 << 3 | 5) +
                                              b"\x01\x02\x03\x04" + var(8 << 3 | 3) + var(2 << 3 | 0) + var(1) +
                                              var(8 << 3 | 4) + var(9 << 3 | 0) + var(3) + ld(9, b"zz")).hex()}}
    noncanon = [
        ("grant_ts_explicit_zero", b"\x0a\x0a" + A.encode() + b"\x10\x00" + ld(4, th.encode())),
        ("grant_fields_out_of_order", ld(4, th.encode()) + b"\x0a\x0a" + A.encode() + b"\x10\x05"),
        ("grant_nonminimal_varint", b"\x0a\x0a" + A.encode() + b"\x10\x85\x00" + ld(4, th.encode())),
        ("grant_unknown_field", g(A, 5) + b"\x30\x01"),
        ("grant_repeated_field", g(A, 5) + b"\x10\x06"),
        ("grant_nonminimal_length", b"\x0a\x8a\x00" + A.encode() + b"\x10\x05"),
    ]
    for name, gb in noncanon:
        add(name, w2([(SID[0], mg(SID[0], [(A, gb)], [(A, sig(0))]))], [op(A)]), 2,
            why="Grant bytes differ from Grant.toByteArray() of the parsed Grant",
            full={"certs": [SID[0]], "grants": [[A]], "ops": [A]})
    many = [(f"s{i}", mg(f"s{i}", [(A, gA[0])])) for i in range(33)]
    add("33_multigrants", w2(many, [op(A)]), 2, full={"certs": [f"s{i}" for i in range(33)], "grants": [[A]] * 33,
                                                       "ops": [A]})
    add("32_multigrants", w2(many[:32], [op(A)]), 0,
        {"certs": [f"s{i}" for i in range(32)], "grants": [[A]] * 32, "ops": [A]})
    add("65_operations", w2(base_mgs, [op(f"k{i}") for i in range(65)]), 2, full_status=2,
        why="op key slots are one byte (< 64): left undecided, never accepted")
    add("64_operations", w2(base_mgs, [op(f"k{i}") for i in range(64)]), 0,
        {"certs": [SID[0], SID[1], SID[2]], "grants": [[A, B]] * 3, "ops": [f"k{i}" for i in range(64)]})
    g65 = mg(SID[0], [(f"k{i}", g(f"k{i}", 3)) for i in range(65)])
    add("65_grants_in_multigrant", w2([(SID[0], g65)], [op("k0")]), 2,
        full={"certs": [SID[0]], "grants": [[f"k{i}" for i in range(65)]], "ops": ["k0"]})
    # malformed (the protobuf parser throws)
    canon = w2(base_mgs, base_ops)
    for cut in (1, 2, 5, 40, len(canon) // 2, len(canon) - 1):
        add(f"truncated_at_{cut}", canon[:cut], 1)
    bad = b"\xc3\x28"
    add("bad_utf8_cert_key", w2([(bad.decode("latin-1"), std(0))], base_ops).replace(bad.decode("latin-1").encode(), bad), 1)
    add("bad_utf8_server_id", w2([(SID[0], mg("x", [(A, gA[0])]).replace(b"\x22\x01x", b"\x22\x02" + bad))], base_ops), 1)
    add("bad_utf8_client_id", w2([(SID[0], mg(SID[0], [(A, gA[0])], cid="Q").replace(b"\x12\x01Q", b"\x12\x02" + bad))], base_ops), 1)
    add("bad_utf8_grant_key", w2([(SID[0], ld(1, ld(1, bad) + ld(2, gA[0])))], base_ops), 1)
    add("bad_utf8_sig_key", w2([(SID[0], ld(5, ld(1, bad) + ld(2, sig(0))))], base_ops), 1)
    add("bad_utf8_operand1", w2(base_mgs, [b"\x08\x02" + ld(2, bad)]), 1)
    add("bad_utf8_operand3", w2(base_mgs, [op(A) + ld(4, bad)]), 1)
    add("bad_utf8_inside_grant", w2([(SID[0], mg(SID[0], [(A, b"\x0a\x02" + bad)]))], base_ops), 1)
    add("malformed_grant_in_replaced_entry", w2([(SID[0], mg(SID[0], [(A, b"\x0f"), (A, gA[0])]))], [op(A)]), 1,
        why="the replaced value is parsed too before put() replaces it")
    add("tag_zero_in_multigrant", w2([(SID[0], std(0, extra=b"\x00"))], base_ops), 1)
    add("stray_end_group_in_operation", w2(base_mgs, [op(A) + b"\x0c"]), 1)
    add("wire_type_6_top", canon + b"\x0e", 1)
    add("negative_length", canon + b"\x1a\xff\xff\xff\xff\x0f", 1)
    add("unterminated_group", canon + var(14 << 3 | 3) + b"\x08\x01", 1)
    add("group_end_mismatch", canon + var(14 << 3 | 3) + var(15 << 3 | 4), 1)
    return V


def main():
    Write2, Grant = classes()
    vecs = vectors()
    for v in vecs:
        data = bytes.fromhex(v["hex"])
        try:
            m = Write2()
            m.ParseFromString(data)
            v["py_ok"] = True
            content = {}
            for key, mgv in m.writeCertificate.grants.items():
                content[key] = {
                    "serverId": mgv.serverId,
                    "grants": {gk: gv.SerializeToString(deterministic=True).hex() for gk, gv in mgv.grants.items()},
                    "sigs": {sk: sv.hex() for sk, sv in mgv.grantSignatures.items()},
                }
            v["py_content"] = {"certs": content, "ops": [o.operand1 for o in m.transaction.operations],
                               "actions": [int(o.action) for o in m.transaction.operations]}
        except Exception as ex:
            v["py_ok"] = False
            v["py_error"] = type(ex).__name__
        if v["status"] == 1:
            assert not v["py_ok"], v["name"]
        else:
            assert v["py_ok"], (v["name"], v.get("py_error"))
    out = {"source": "hand-encoded Write2ToServer bytes (workload.py encoders + literal edits); py_* from Python "
                     "google.protobuf 7.35.1 with a hand-built descriptor; status / order written from "
                     "include/mochi_hip.h and protobuf-java 3.16.3 MapField (LinkedHashMap) semantics",
           "server_ids": __import__("workload").SERVER_IDS, "vectors": vecs}
    with open(os.path.join(HERE, "write2_vectors.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(f"{len(vecs)} vectors")


if __name__ == "__main__":
    main()
