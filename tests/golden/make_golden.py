#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Run in the build container (needs Python google.protobuf and the openssl CLI;
neither is needed to *use* the fixtures):

    python tests/golden/make_golden.py

Outputs (all data, no code):
  sha256_vectors.json   NIST FIPS 180-4 / CAVP known answers (literal)
  grant_vectors.json    Grant proto3 bytes produced by Python google.protobuf
                        7.35.1 from a hand-built descriptor of
                        MochiProtocol.proto:107-113 (independent encoder)
  rsa_vectors.json      SHA256withRSA signatures made by `openssl dgst -sign`
                        over grant bytes, plus tampered variants; expected
                        verdicts from `openssl dgst -verify` (OpenSSL 3.0.2 CLI)
  cert_cases.json       hand-constructed certificates, one per verdict branch
                        of InMemoryDataStore.java:576-640, expected reason
                        codes written from the Java source (see `why` fields)
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
KEYS = os.path.join(HERE, "keys")


# ---------------------------------------------------------------------------
def sha256_vectors():
    # FIPS 180-4 examples / CAVP SHA256ShortMsg (literal known answers).
    vecs = [
        ("", "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"),
        ("616263", "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad"),
        ("6162636462636465636465666465666765666768666768696768696a68696a6b696a6b6c6a6b6c6d6b6c6d6e6c6d6e6f6d6e6f706e6f7071",
         "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1"),
        ("61626364656667686263646566676869636465666768696a6465666768696a6b65666768696a6b6c666768696a6b6c6d6768696a6b6c6d6e68696a6b6c6d6e6f696a6b6c6d6e6f706a6b6c6d6e6f70716b6c6d6e6f7071726c6d6e6f707172736d6e6f70717273746e6f707172737475",
         "cf5b16a778af8380036ce59e7b0492370b249b11e8f07a51afac45037afee9d1"),
        ("d3", "28969cdfa74a12c82f3bad960b0b000aca2ac329deea5c2328ebc6f2ba9802c1"),
        ("11af", "5ca7133fa735326081558ac312c620eeca9970d1e70a4b95533d956f072d1f98"),
    ]
    # self-check against hashlib, then add boundary lengths 55/56/63/64/119/120 bytes
    out = []
    for m, d in vecs:
        assert hashlib.sha256(bytes.fromhex(m)).hexdigest() == d, m
        out.append({"msg": m, "digest": d, "source": "FIPS 180-4 / CAVP SHA256ShortMsg"})
    for n in (55, 56, 63, 64, 65, 119, 120, 127, 128, 146, 170):
        m = bytes((i * 7 + 3) & 0xFF for i in range(n))
        out.append({"msg": m.hex(), "digest": hashlib.sha256(m).hexdigest(), "source": f"hashlib, {n} B padding boundary"})
    return out


# ---------------------------------------------------------------------------
def grant_message_class():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    fdp = descriptor_pb2.FileDescriptorProto()
    fdp.name = "mochi_golden.proto"
    fdp.package = "edu.stanford.cs244b.mochi.server.messages"
    fdp.syntax = "proto3"
    e = fdp.enum_type.add()
    e.name = "OperationResultStatus"
    for nm, num in (("OK", 0), ("WRONG_SHARD", 1)):
        v = e.value.add()
        v.name, v.number = nm, num
    m = fdp.message_type.add()
    m.name = "Grant"  # MochiProtocol.proto:107-113
    T = descriptor_pb2.FieldDescriptorProto
    for nm, num, ty in (("objectId", 1, T.TYPE_STRING), ("timestamp", 2, T.TYPE_INT64), ("configstamp", 3, T.TYPE_INT64),
                        ("transactionHash", 4, T.TYPE_STRING), ("status", 5, T.TYPE_ENUM)):
        f = m.field.add()
        f.name, f.number, f.type, f.label = nm, num, ty, T.LABEL_OPTIONAL
        if ty == T.TYPE_ENUM:
            f.type_name = ".edu.stanford.cs244b.mochi.server.messages.OperationResultStatus"
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    desc = pool.FindMessageTypeByName("edu.stanford.cs244b.mochi.server.messages.Grant")
    return message_factory.GetMessageClass(desc)


def grant_vectors():
    Grant = grant_message_class()
    h = hashlib.sha512(b"golden-txn").hexdigest()
    cases = [
        dict(objectId="DEMO_KEY_1", timestamp=1342, transactionHash="a" * 128),  # 146 B
        dict(objectId="DEMO_KEY_STRESS_TEST_199", timestamp=63999, transactionHash=h),
        dict(objectId="k", timestamp=0, transactionHash=h),  # ts default skipped
        dict(objectId="", timestamp=5, transactionHash=h),  # empty objectId skipped
        dict(objectId="neg", timestamp=-1, transactionHash=h),  # 10-byte varint
        dict(objectId="big", timestamp=(1 << 62) + 12345, transactionHash=h),
        dict(objectId="cfg", timestamp=1000, configstamp=7, transactionHash=h),
        dict(objectId="ws", timestamp=0, transactionHash=h, status=1),  # WRONG_SHARD
        dict(objectId="clé-ünï", timestamp=2024, transactionHash=h),  # UTF-8 objectId
        dict(objectId="x" * 200, timestamp=999, transactionHash=h),  # 2-byte length varint
        dict(objectId="nohash", timestamp=17),
    ]
    out = []
    for c in cases:
        g = Grant(**c)
        out.append({"fields": c, "bytes": g.SerializeToString(deterministic=True).hex(),
                    "source": "google.protobuf 7.35.1, hand-built descriptor of MochiProtocol.proto:107-113"})
    # parse-only vectors: decoded by google.protobuf (last-wins, unknown fields, errors)
    parse_cases = [
        ("dup_ts_last_wins", bytes.fromhex("0a016b1001100222" + "02" + "6868")),
        ("unknown_varint_field", bytes.fromhex("0a016b10053001") + b""),
        ("unknown_fixed64", bytes.fromhex("0a016b1005" + "39" + "0102030405060708")),
        ("unknown_len_field", bytes.fromhex("0a016b1005" + "52" + "03616263")),
        ("unknown_fixed32", bytes.fromhex("0a016b1005" + "5d" + "01020304")),
        ("group_skipped", bytes.fromhex("0a016b1005" + "5b" + "0801" + "5c")),
        ("truncated_string", bytes.fromhex("0a056b")),
        ("truncated_varint", bytes.fromhex("1085")),
        ("tag_zero", bytes.fromhex("00")),
        ("wire_type_7", bytes.fromhex("0f")),
        ("stray_end_group", bytes.fromhex("0a016b0c")),
        ("bad_utf8_objectid", bytes.fromhex("0a02c328")),
        ("bad_utf8_hash", bytes.fromhex("2201ff")),
        ("overlong_utf8", bytes.fromhex("0a02c0af")),
        ("surrogate_utf8", bytes.fromhex("0a03eda080")),
        ("mismatched_end_group", bytes.fromhex("5b" + "64")),
        ("empty", b""),
        ("varint_11_bytes", bytes.fromhex("10" + "ff" * 10 + "01")),
        ("neg_len", bytes.fromhex("0a" + "ffffffff0f")),
        # unknown groups nested 17 / 99 / 100 / 101 deep (CodedInputStream's recursion limit is 100)
        ("groups_nested_17", bytes.fromhex("0a016b1005" + "5b" * 17 + "5c" * 17)),
        ("groups_nested_99", bytes.fromhex("0a016b1005" + "5b" * 99 + "5c" * 99)),
        ("groups_nested_100", bytes.fromhex("0a016b1005" + "5b" * 100 + "5c" * 100)),
        ("groups_nested_101", bytes.fromhex("0a016b1005" + "5b" * 101 + "5c" * 101)),
    ]
    parse = []
    for name, data in parse_cases:
        try:
            g = Grant()
            g.ParseFromString(data)
            res = {"ok": True, "timestamp": g.timestamp, "transactionHash": g.transactionHash, "objectId": g.objectId}
        except Exception as ex:  # DecodeError
            res = {"ok": False, "error": type(ex).__name__}
        parse.append({"name": name, "bytes": data.hex(), "expect": res, "source": "google.protobuf 7.35.1 ParseFromString"})
    return out, parse


# ---------------------------------------------------------------------------
def openssl(*args, inp: bytes = b"") -> subprocess.CompletedProcess:
    return subprocess.run(["openssl", *args], input=inp, capture_output=True)


def rsa_vectors():
    from_pem = {}
    for i in range(7):
        p = os.path.join(KEYS, f"server{i}.pem")
        mod = openssl("rsa", "-in", p, "-noout", "-modulus").stdout.decode().strip().split("=", 1)[1]
        from_pem[i] = bytes.fromhex(mod)
    Grant = grant_message_class()
    vecs = []
    with tempfile.TemporaryDirectory() as td:
        def sign(key_i, msg):
            mp = os.path.join(td, "m")
            with open(mp, "wb") as f:
                f.write(msg)
            r = openssl("dgst", "-sha256", "-sign", os.path.join(KEYS, f"server{key_i}.pem"), mp)
            assert r.returncode == 0, r.stderr
            return r.stdout

        def verify(key_i, msg, sig):
            mp, sp, pub = os.path.join(td, "m"), os.path.join(td, "s"), os.path.join(td, f"pub{key_i}.pem")
            with open(mp, "wb") as f:
                f.write(msg)
            with open(sp, "wb") as f:
                f.write(sig)
            if not os.path.exists(pub):
                openssl("rsa", "-in", os.path.join(KEYS, f"server{key_i}.pem"), "-pubout", "-out", pub)
            r = openssl("dgst", "-sha256", "-verify", pub, "-signature", sp, mp)
            return r.returncode == 0 and b"Verified OK" in r.stdout

        h = hashlib.sha512(b"txn-rsa-golden").hexdigest()
        for i in range(7):
            for t in range(3):
                msg = Grant(objectId=f"DEMO_KEY_{i}_{t}", timestamp=1000 * t + 17 * i, transactionHash=h).SerializeToString()
                sig = sign(i, msg)
                n = from_pem[i]
                nint = int.from_bytes(n, "big")
                sint = int.from_bytes(sig, "big")
                variants = [("valid", msg, sig, i)]
                flipped = bytearray(sig)
                flipped[(37 * t + i) % 256] ^= 1 << (t % 8)
                variants.append(("flipped_sig_bit", msg, bytes(flipped), i))
                msg2 = bytearray(msg)
                msg2[-1] ^= 1
                variants.append(("tampered_msg", bytes(msg2), sig, i))
                variants.append(("wrong_key", msg, sig, (i + 1) % 7))
                if sint + nint < (1 << 2048):
                    variants.append(("sig_plus_n", msg, (sint + nint).to_bytes(256, "big"), i))
                variants.append(("sig_equals_n", msg, n, i))
                variants.append(("sig_zero", msg, bytes(256), i))
                variants.append(("sig_one", msg, (1).to_bytes(256, "big"), i))
                variants.append(("sig_n_minus_1", msg, (nint - 1).to_bytes(256, "big"), i))
                variants.append(("sig_all_ff", msg, b"\xff" * 256, i))
                for name, m, s, k in variants:
                    if t > 0 and name not in ("valid", "flipped_sig_bit"):
                        continue
                    vecs.append({"name": name, "key": k, "msg": m.hex(), "sig": s.hex(), "valid": verify(k, m, s),
                                 "source": "openssl 3.0.2 CLI dgst -sha256 -sign / -verify"})
    moduli = {str(i): from_pem[i].hex() for i in range(7)}
    return {"moduli": moduli, "vectors": vecs}


# ---------------------------------------------------------------------------
def cert_cases():
    """Hand-constructed certificates for every verdict branch.

    Grant spec: [server, key_slot, ts, hash ('good'|'evil'|'short'), sig ('ok'|'bad'), bytes ('ok'|'malformed'),
    optional extras {"mg": MultiGrant index, "oid": key slot written as Grant.objectId}], listed in certificate
    wire order (MultiGrant by MultiGrant).  Without "mg" every maximal run of one server's grants is one
    MultiGrant; a case may set "n_mgs" to add empty MultiGrants at the end.  Ops: [key_slot, flags, object_ts?]
    in txn order (flags: 1 = local shard, 2 = SVOC exists, 4 = SVOC holds a certificate whose timestamp is
    object_ts, 8 = that stored certificate throws, 16 = not a WRITE/DELETE).  quorum_mode: 0 = reference parity,
    1 = distinct signers, 2 = bind objectId / transactionHash.  Expected reason codes, failing ops, per-op
    decisions (0 skipped, 1 apply, 2 read, 3 wrong shard, 4 failed) and g0 (certificate-relative grant index,
    -1 none) are read off the Java source (InMemoryDataStore.java:521-640, StoreValueObjectContainer.java:175-198).
    """
    G, E = "good", "evil"
    ok4 = [[r, 0, 1000, G, "ok", "ok"] for r in range(4)]
    c = []

    def add(name, R, strict, grants, ops, reason, fail_op, decisions, g0, why, **kw):
        c.append(dict(name=name, R=R, strict=strict, grants=grants, ops=ops, reason=reason, fail_op=fail_op,
                      decisions=decisions, g0=g0, why=why, quorum_mode=kw.pop("quorum_mode", 0), **kw))

    add("accept_4of4_server", 4, 1, ok4, [[0, 3]], 0, 255, [1], [0],
        "4 grants, list.size()=4 > M=3 (InMemoryDataStore.java:590); g0 hash equal (:591); no stored "
        "certificate -> applyOperation (:597); every MultiGrant holds the key at ts 1000 (SVOC :186-194)")
    add("below_quorum_3of4_server", 4, 1, ok4[:3], [[0, 3]], 3, 0, [4], [0],
        "list.size()=3 > M=3 is false -> Utils.assertTrue throws IllegalStateException (:590)")
    add("client_predicate_3of4_accepts", 4, 0, ok4[:3], [[0, 3]], 0, 255, [1], [0],
        "client predicate count >= M (MochiDBClient.java:172,379): 3 >= 3")
    add("invalid_sig_counts_as_absent", 4, 1, [ok4[0], ok4[1], [2, 0, 1000, G, "bad", "ok"], ok4[3]], [[0, 3]], 3, 0,
        [4], [0], "bad signature => grant treated as absent (:622-624 null skip) -> 3 grants -> below quorum")
    add("ts_mismatch", 4, 1, [ok4[0], ok4[1], [2, 0, 1001, G, "ok", "ok"], ok4[3]], [[0, 3]], 1, 255, [0], [0],
        "valid grant with ts != first ts -> UnsupportedOperationException (:626-628)")
    add("ts_skew_on_invalid_sig_fails_apply", 4, 0, [ok4[0], ok4[1], [2, 0, 1001, G, "bad", "ok"], ok4[3]], [[0, 3]],
        8, 0, [4], [0],
        "the skewed grant has a bad signature, so the tally skips it (3 >= 3 passes), but applyOperation stores the "
        "certificate as received and getCurrentTimestampFromCurrentCertificate compares every MultiGrant: 1001 != "
        "1000 -> IllegalStateException (:533-534, StoreValueObjectContainer.java:192-194)")
    add("ts_skew_on_invalid_sig_read_branch_accepts", 4, 0,
        [ok4[0], ok4[1], [2, 0, 1001, G, "bad", "ok"], ok4[3]], [[0, 7, 5000]], 0, 255, [2], [0],
        "same certificate, but the SVOC's stored certificate has ts 5000 > g0.ts 1000 -> readOperation (:595-596), "
        "which never looks at the incoming certificate")
    add("g0_hash_mismatch", 4, 1, [[0, 0, 1000, E, "ok", "ok"]] + ok4[1:], [[0, 3]], 4, 0, [4], [0],
        "g0.transactionHash != txnHash -> UnsupportedOperationException (:591,605-607)")
    add("g1_hash_mismatch_accepted", 4, 1, [ok4[0], [1, 0, 1000, E, "ok", "ok"]] + ok4[2:], [[0, 3]], 0, 255, [1],
        [0], "only g0 = list.get(0) is compared (:588,591)")
    add("g0_invalid_then_g1_evil", 4, 0, [[0, 0, 1000, G, "bad", "ok"], [1, 0, 1000, E, "ok", "ok"]] + ok4[2:],
        [[0, 3]], 4, 0, [4], [1], "g0 absent (bad sig) so the first VALID grant (evil hash) becomes list.get(0)")
    add("hash_wrong_length", 4, 1, [[0, 0, 1000, "short", "ok", "ok"]] + ok4[1:], [[0, 3]], 4, 0, [4], [0],
        "String.equals fails on a 127-char hash")
    add("no_grant_for_key", 4, 1, ok4, [[0, 3], [1, 3]], 2, 1, [1, 4], [0, -1],
        "op 1's key has no grant: coalescedTxnGrantMap.get(key) == null -> NPE (:588); op 0 was already applied "
        "(the loop is not atomic)")
    add("wrong_shard_op_skipped", 4, 1, ok4, [[0, 3], [1, 2]], 0, 255, [1, 3], [0, -1],
        "op 1 not on this shard -> WRONG_SHARD result, no checks (:582-587)")
    add("no_svoc", 4, 1, ok4, [[0, 1]], 5, 0, [4], [0],
        "storeValueContainer == null -> op.getOperand1().equals(svoc.getKey()) NPE (:592-593)")
    add("duplicate_op_doubles_count", 4, 1, ok4[:2], [[0, 3], [0, 3]], 0, 255, [1, 1], [0, 0],
        "each op appends the grant again (:620-630): 2 grants x 2 ops = 4 > 3; op 1 sees currentC = wc (ts 1000, "
        "not > g0.ts) -> applies again")
    add("two_keys_accept", 4, 1, [[r, s, 1000 + 7 * s, G, "ok", "ok"] for r in range(4) for s in range(2)],
        [[0, 3], [1, 3]], 0, 255, [1, 1], [0, 1], "per-key lists, ts uniform per key only")
    add("two_keys_second_below_quorum", 4, 1,
        [[r, s, 1000, G, "ok" if (r, s) != (3, 1) else "bad", "ok"] for r in range(4) for s in range(2)],
        [[0, 3], [1, 3]], 3, 1, [1, 4], [0, 1], "key 1 has 3 valid grants; op 0 passes (and applies) first")
    add("ts_mismatch_beats_quorum", 4, 1, [[0, 0, 1000, G, "ok", "ok"], [1, 0, 1002, G, "ok", "ok"]], [[0, 3]], 1,
        255, [0], [0], "processMultiGrantsFromAllServers runs before write2apply (:646 vs :653)")
    add("malformed_grant_rejects", 4, 0, ok4[:3] + [[3, 0, 1000, G, "ok", "malformed"]], [[0, 3]], 6, 255, [0], [0],
        "unparseable Grant bytes: protobuf decode fails before the handler runs")
    add("grant_for_unnamed_key_ignored", 4, 1, [ok4[0], [0, 5, 77, E, "ok", "ok"]] + ok4[1:], [[0, 3]], 0, 255, [1],
        [0], "grants whose key no op names are never looked up (:621, SVOC :185 looks up only the op's key)")
    add("r7_server_6of7_accepts", 7, 1, [[r, 0, 5000, G, "ok", "ok"] for r in range(6)], [[0, 3]], 0, 255, [1], [0],
        "R=7: M=2*(7/3)+1=5 (ClusterConfiguration.java:264-267); 6 > 5")
    add("r7_server_5of7_rejects", 7, 1, [[r, 0, 5000, G, "ok", "ok"] for r in range(5)], [[0, 3]], 3, 0, [4], [0],
        "R=7: 5 > 5 is false under the server predicate")
    add("r7_client_5of7_accepts", 7, 0, [[r, 0, 5000, G, "ok", "ok"] for r in range(5)], [[0, 3]], 0, 255, [1], [0],
        "client predicate 5 >= 5 (the BASELINE '5-of-7 tally')")
    add("empty_certificate_no_ops", 4, 1, [], [], 0, 255, [], [], "no ops -> write2apply loop empty -> accepted")
    add("empty_certificate_with_op", 4, 1, [], [[0, 3]], 2, 0, [4], [-1],
        "no grants at all -> NPE on the first local op (:588)")
    # --- the read/apply step (InMemoryDataStore.java:594-599, :521-574) ---
    add("mg_without_key_fails_apply", 4, 1,
        [g + [{"mg": i}] for i, g in enumerate(ok4)] + [[0, 1, 1000, G, "ok", "ok", {"mg": 4}]], [[0, 3]], 8, 0, [4], [0],
        "a fifth MultiGrant carries only a grant for a key no op names: the tally never looks it up, but "
        "getCurrentTimestampFromCurrentCertificate does: grants.get(key) == null -> Utils.assertNotNull throws "
        "IllegalStateException (StoreValueObjectContainer.java:186)")
    add("empty_mg_fails_apply", 4, 1, [g + [{"mg": i}] for i, g in enumerate(ok4)],
        [[0, 3]], 8, 0, [4], [0], "an empty fifth MultiGrant: grants.get(key) == null (:186)", n_mgs=5)
    add("read_branch_stored_ts_newer", 4, 1, ok4, [[0, 7, 2000]], 0, 255, [2], [0],
        "objectTS 2000 > g0.ts 1000 -> readOperation (:595-596)")
    add("apply_branch_stored_ts_equal", 4, 1, ok4, [[0, 7, 1000]], 0, 255, [1], [0],
        "objectTS 1000 > 1000 is false -> applyOperation (:597)")
    add("apply_branch_stored_ts_older", 4, 1, ok4, [[0, 7, 999]], 0, 255, [1], [0],
        "objectTS 999 < g0.ts -> applyOperation")
    add("stored_cert_throws", 4, 1, ok4, [[0, 15, 0]], 9, 0, [4], [0],
        "the SVOC's stored certificate throws in getCurrentTimestampFromCurrentCertificate (:594)")
    add("not_write_op_apply_branch", 4, 1, ok4, [[0, 19]], 10, 0, [4], [0],
        "a READ op in a Write2 transaction: no write lock (:339-358) -> applyOperation throws (:525-526)")
    add("not_write_op_read_branch", 4, 1, ok4, [[0, 23, 2000]], 10, 0, [4], [0],
        "readOperation checks the lock / action too (:560-562, :572)")
    add("duplicate_op_read_then_read", 4, 1, ok4[:2], [[0, 7, 2000], [0, 7, 2000]], 0, 255, [2, 2], [0, 0],
        "readOperation leaves currentC alone, so the second op reads too")
    add("duplicate_op_apply_then_apply", 4, 1, ok4[:2], [[0, 7, 500], [0, 7, 5000]], 0, 255, [1, 1], [0, 0],
        "op 0 applies (500 < 1000) and stores wc; op 1's objectTS is then wc's 1000, not the stale 5000 -> applies")
    add("stored_cert_bad_replaced_by_apply", 4, 1, ok4, [[0, 3], [0, 11, 0]], 0, 255, [1, 1], [0, 0],
        "op 0 applies and replaces the bad stored certificate; op 1 sees wc")
    add("two_keys_second_fails_apply", 4, 0,
        [[r, s, 1000, G, "ok", "ok"] for r in range(4) for s in range(2) if (r, s) != (3, 1)],
        [[0, 3], [1, 3]], 8, 1, [1, 4], [0, 1],
        "key 1: 3 grants >= 3 (client predicate) but the fourth MultiGrant lacks it -> op 0 applied, op 1 throws "
        "in getCurrentTimestampFromCurrentCertificate (:186)")
    # --- quorum modes (the new signature layer as a Byzantine quorum; parity = mode 0) ---
    same_signer = [[0, 0, 1000, G, "ok", "ok", {"mg": i}] for i in range(4)]
    add("one_signer_four_map_keys_parity", 4, 1, same_signer, [[0, 3]], 0, 255, [1], [0],
        "parity: list.size() counts entries (:590), so 4 copies of server 0's MultiGrant under 4 certificate map "
        "keys reach 4 > 3")
    add("one_signer_four_map_keys_distinct", 4, 1, same_signer, [[0, 3]], 3, 0, [4], [0],
        "MOCHI_Q_DISTINCT_SIGNERS: server 0 counts once -> 1 > 3 fails", quorum_mode=1)
    add("distinct_signers_honest_accepts", 4, 1, ok4, [[0, 3]], 0, 255, [1], [0],
        "four different signers: unaffected by MOCHI_Q_DISTINCT_SIGNERS", quorum_mode=1)
    foreign = ok4[:3] + [[3, 0, 1000, G, "ok", "ok", {"oid": 7}]]
    add("foreign_object_grant_parity", 4, 1, foreign, [[0, 3]], 0, 255, [1], [0],
        "parity: server 3's grant for another object (objectId CASE_KEY_7) filed under key 0 still counts")
    add("foreign_object_grant_bind", 4, 1, foreign, [[0, 3]], 3, 0, [4], [0],
        "MOCHI_Q_BIND: objectId != map key -> not counted -> 3 > 3 fails", quorum_mode=2)
    add("foreign_txn_grant_bind", 4, 1, ok4[:3] + [[3, 0, 1000, E, "ok", "ok"]], [[0, 3]], 3, 0, [4], [0],
        "MOCHI_Q_BIND: transactionHash != expected -> not counted (parity only checks g0)", quorum_mode=2)
    add("bind_honest_accepts", 4, 1, ok4, [[0, 3]], 0, 255, [1], [0], "honest grants are bound", quorum_mode=2)
    add("bind_and_distinct", 4, 0, same_signer[:2] + [[1, 0, 1000, G, "ok", "ok", {"mg": 2}],
                                                      [2, 0, 1000, E, "ok", "ok", {"mg": 3}]], [[0, 3]], 3, 0, [4],
        [0], "mode 3: server 0 once, server 1 once, server 2's grant is for another txn -> 2 >= 3 fails",
        quorum_mode=3)
    return c


def main():
    if sys.argv[1:] == ["grant_vectors"]:  # regenerate only the google.protobuf Grant vectors
        gv, pv = grant_vectors()
        with open(os.path.join(HERE, "grant_vectors.json"), "w") as f:
            json.dump({"encode": gv, "parse": pv}, f, indent=1)
        return
    if sys.argv[1:] == ["cert_cases"]:  # regenerate only the hand-constructed verdict cases
        with open(os.path.join(HERE, "cert_cases.json"), "w") as f:
            json.dump(cert_cases(), f, indent=1)
        return
    with open(os.path.join(HERE, "sha256_vectors.json"), "w") as f:
        json.dump(sha256_vectors(), f, indent=1)
    gv, pv = grant_vectors()
    with open(os.path.join(HERE, "grant_vectors.json"), "w") as f:
        json.dump({"encode": gv, "parse": pv}, f, indent=1)
    with open(os.path.join(HERE, "rsa_vectors.json"), "w") as f:
        json.dump(rsa_vectors(), f, indent=1)
    with open(os.path.join(HERE, "cert_cases.json"), "w") as f:
        json.dump(cert_cases(), f, indent=1)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
