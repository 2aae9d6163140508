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

    Grant spec: [server, key_slot, ts, hash ('good'|'evil'|'short'), sig ('ok'|'bad'), bytes ('ok'|'malformed')],
    listed in certificate wire order (MultiGrant by MultiGrant).  Ops: [key_slot, flags] in txn order
    (flags: 1 = local shard, 2 = SVOC exists).  Expected reason codes are read off the Java source.
    """
    G, E = "good", "evil"
    ok4 = [[r, 0, 1000, G, "ok", "ok"] for r in range(4)]
    c = []
    c.append(dict(name="accept_4of4_server", R=4, strict=1, grants=ok4, ops=[[0, 3]], reason=0, fail_op=255,
                  why="4 grants, list.size()=4 > M=3 (InMemoryDataStore.java:590); g0 hash equal (:591)"))
    c.append(dict(name="below_quorum_3of4_server", R=4, strict=1, grants=ok4[:3], ops=[[0, 3]], reason=3, fail_op=0,
                  why="list.size()=3 > M=3 is false -> Utils.assertTrue throws IllegalStateException (:590)"))
    c.append(dict(name="client_predicate_3of4_accepts", R=4, strict=0, grants=ok4[:3], ops=[[0, 3]], reason=0,
                  fail_op=255, why="client predicate count >= M (MochiDBClient.java:172,379): 3 >= 3"))
    c.append(dict(name="invalid_sig_counts_as_absent", R=4, strict=1,
                  grants=[ok4[0], ok4[1], [2, 0, 1000, G, "bad", "ok"], ok4[3]], ops=[[0, 3]], reason=3, fail_op=0,
                  why="bad signature => grant treated as absent (:622-624 null skip) -> 3 grants -> below quorum"))
    c.append(dict(name="ts_mismatch", R=4, strict=1,
                  grants=[ok4[0], ok4[1], [2, 0, 1001, G, "ok", "ok"], ok4[3]], ops=[[0, 3]], reason=1, fail_op=255,
                  why="valid grant with ts != first ts -> UnsupportedOperationException (:626-628)"))
    c.append(dict(name="ts_mismatch_on_invalid_sig_ignored", R=4, strict=0,
                  grants=[ok4[0], ok4[1], [2, 0, 1001, G, "bad", "ok"], ok4[3]], ops=[[0, 3]], reason=0, fail_op=255,
                  why="the skewed grant has a bad signature, so it is absent; 3 >= 3 under the client predicate"))
    c.append(dict(name="g0_hash_mismatch", R=4, strict=1,
                  grants=[[0, 0, 1000, E, "ok", "ok"]] + ok4[1:], ops=[[0, 3]], reason=4, fail_op=0,
                  why="g0.transactionHash != txnHash -> UnsupportedOperationException (:591,605-607)"))
    c.append(dict(name="g1_hash_mismatch_accepted", R=4, strict=1,
                  grants=[ok4[0], [1, 0, 1000, E, "ok", "ok"]] + ok4[2:], ops=[[0, 3]], reason=0, fail_op=255,
                  why="only g0 = list.get(0) is compared (:588,591)"))
    c.append(dict(name="g0_invalid_then_g1_evil", R=4, strict=0,
                  grants=[[0, 0, 1000, G, "bad", "ok"], [1, 0, 1000, E, "ok", "ok"]] + ok4[2:], ops=[[0, 3]],
                  reason=4, fail_op=0, why="g0 absent (bad sig) so the first VALID grant (evil hash) becomes list.get(0)"))
    c.append(dict(name="hash_wrong_length", R=4, strict=1,
                  grants=[[0, 0, 1000, "short", "ok", "ok"]] + ok4[1:], ops=[[0, 3]], reason=4, fail_op=0,
                  why="String.equals fails on a 127-char hash"))
    c.append(dict(name="no_grant_for_key", R=4, strict=1, grants=ok4, ops=[[0, 3], [1, 3]], reason=2, fail_op=1,
                  why="op 1's key has no grant: coalescedTxnGrantMap.get(key) == null -> NPE (:588)"))
    c.append(dict(name="wrong_shard_op_skipped", R=4, strict=1, grants=ok4, ops=[[0, 3], [1, 2]], reason=0,
                  fail_op=255, why="op 1 not on this shard -> WRONG_SHARD result, no checks (:582-587)"))
    c.append(dict(name="no_svoc", R=4, strict=1, grants=ok4, ops=[[0, 1]], reason=5, fail_op=0,
                  why="storeValueContainer == null -> op.getOperand1().equals(svoc.getKey()) NPE (:592-593)"))
    c.append(dict(name="duplicate_op_doubles_count", R=4, strict=1, grants=ok4[:2], ops=[[0, 3], [0, 3]], reason=0,
                  fail_op=255, why="each op appends the grant again (:620-630): 2 grants x 2 ops = 4 > 3"))
    c.append(dict(name="two_keys_accept", R=4, strict=1,
                  grants=[[r, s, 1000 + 7 * s, G, "ok", "ok"] for r in range(4) for s in range(2)],
                  ops=[[0, 3], [1, 3]], reason=0, fail_op=255, why="per-key lists, ts uniform per key only"))
    c.append(dict(name="two_keys_second_below_quorum", R=4, strict=1,
                  grants=[[r, s, 1000, G, "ok" if (r, s) != (3, 1) else "bad", "ok"] for r in range(4) for s in range(2)],
                  ops=[[0, 3], [1, 3]], reason=3, fail_op=1, why="key 1 has 3 valid grants; op 0 passes first"))
    c.append(dict(name="ts_mismatch_beats_quorum", R=4, strict=1,
                  grants=[[0, 0, 1000, G, "ok", "ok"], [1, 0, 1002, G, "ok", "ok"]], ops=[[0, 3]], reason=1,
                  fail_op=255, why="processMultiGrantsFromAllServers runs before write2apply (:646 vs :653)"))
    c.append(dict(name="malformed_grant_rejects", R=4, strict=0,
                  grants=ok4[:3] + [[3, 0, 1000, G, "ok", "malformed"]], ops=[[0, 3]], reason=6, fail_op=255,
                  why="unparseable Grant bytes: protobuf decode fails before the handler runs"))
    c.append(dict(name="grant_for_unnamed_key_ignored", R=4, strict=1, grants=ok4 + [[0, 5, 77, E, "ok", "ok"]],
                  ops=[[0, 3]], reason=0, fail_op=255, why="grants whose key no op names are never looked up (:621)"))
    c.append(dict(name="r7_server_6of7_accepts", R=7, strict=1, grants=[[r, 0, 5000, G, "ok", "ok"] for r in range(6)],
                  ops=[[0, 3]], reason=0, fail_op=255, why="R=7: M=2*(7/3)+1=5 (ClusterConfiguration.java:264-267); 6 > 5"))
    c.append(dict(name="r7_server_5of7_rejects", R=7, strict=1, grants=[[r, 0, 5000, G, "ok", "ok"] for r in range(5)],
                  ops=[[0, 3]], reason=3, fail_op=0, why="R=7: 5 > 5 is false under the server predicate"))
    c.append(dict(name="r7_client_5of7_accepts", R=7, strict=0, grants=[[r, 0, 5000, G, "ok", "ok"] for r in range(5)],
                  ops=[[0, 3]], reason=0, fail_op=255, why="client predicate 5 >= 5 (the BASELINE '5-of-7 tally')"))
    c.append(dict(name="empty_certificate_no_ops", R=4, strict=1, grants=[], ops=[], reason=0, fail_op=255,
                  why="no ops -> write2apply loop empty -> accepted"))
    c.append(dict(name="empty_certificate_with_op", R=4, strict=1, grants=[], ops=[[0, 3]], reason=2, fail_op=0,
                  why="no grants at all -> NPE on the first local op (:588)"))
    return c


def main():
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
