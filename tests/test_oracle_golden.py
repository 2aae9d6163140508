"""Pin the CPU oracle against the committed golden fixtures (CPU only).

The oracle is test infrastructure (oracle/): these tests establish that it is
trustworthy before it is used to judge the HIP path.
"""
import json
import os

import numpy as np
import pytest

import oracle_ffi as O
from cases import build_case_batch, grouped_cases, load_cases, moduli_for
from workload import encode_grant, load_keys


def test_sha256_known_answers(golden_dir):
    vecs = json.load(open(os.path.join(golden_dir, "sha256_vectors.json")))
    assert len(vecs) >= 6
    for v in vecs:
        assert O.sha256(bytes.fromhex(v["msg"])).hex() == v["digest"], v


def test_grant_encoding_matches_google_protobuf(golden_dir):
    d = json.load(open(os.path.join(golden_dir, "grant_vectors.json")))
    for v in d["encode"]:
        f = v["fields"]
        oid = f.get("objectId", "").encode()
        th = f.get("transactionHash", "").encode()
        want = bytes.fromhex(v["bytes"])
        got = O.grant_encode(oid, f.get("timestamp", 0), th, f.get("configstamp", 0), f.get("status", 0))
        assert got == want, f
        # the producer-side encoder (workload.encode_grant) must agree too
        got2 = encode_grant(f.get("objectId", ""), f.get("timestamp", 0), f.get("transactionHash", ""),
                            f.get("configstamp", 0), f.get("status", 0))
        assert got2 == want, f
    # SURVEY §7.2 probe: 146 bytes for objectId=DEMO_KEY_1, ts=1342, hash=128*'a'
    assert len(bytes.fromhex(d["encode"][0]["bytes"])) == 146


def test_grant_parse_matches_google_protobuf(golden_dir):
    d = json.load(open(os.path.join(golden_dir, "grant_vectors.json")))
    for v in d["encode"]:
        data = bytes.fromhex(v["bytes"])
        g = O.grant_parse(data)
        assert g is not None
        assert g["timestamp"] == v["fields"].get("timestamp", 0)
        assert g["transaction_hash"] == v["fields"].get("transactionHash", "").encode()
    for v in d["parse"]:
        g = O.grant_parse(bytes.fromhex(v["bytes"]))
        e = v["expect"]
        assert (g is not None) == e["ok"], v["name"]
        if e["ok"]:
            assert g["timestamp"] == e["timestamp"], v["name"]
            assert g["transaction_hash"] == e["transactionHash"].encode(), v["name"]
            assert g["object_id"] == e["objectId"].encode(), v["name"]


def test_rsa_vectors_match_openssl_cli(golden_dir):
    d = json.load(open(os.path.join(golden_dir, "rsa_vectors.json")))
    moduli = {int(k): bytes.fromhex(v) for k, v in d["moduli"].items()}
    # the committed PEMs are the keys the fixtures were made with
    pems = load_keys(7)
    for i in range(7):
        assert O.pem_modulus(pems[i]) == moduli[i]
    n_valid = 0
    for v in d["vectors"]:
        got = O.rsa_verify(moduli[v["key"]], bytes.fromhex(v["msg"]), bytes.fromhex(v["sig"]))
        assert got == v["valid"], v["name"]
        n_valid += got
    assert n_valid == 21  # 7 keys x 3 valid grants
    names = {v["name"] for v in d["vectors"]}
    assert {"sig_plus_n", "sig_equals_n", "sig_zero", "wrong_key", "tampered_msg"} <= names


def test_oracle_sign_roundtrip():
    pems = load_keys(2)
    msg = encode_grant("DEMO_KEY_1", 1342, "a" * 128)
    s = O.rsa_sign(pems[0], msg)
    n0, n1 = O.pem_modulus(pems[0]), O.pem_modulus(pems[1])
    assert O.rsa_verify(n0, msg, s)
    assert not O.rsa_verify(n1, msg, s)


def test_server_majority_restatement():
    # ClusterConfiguration.java:264-267: 2*(R/3)+1
    assert [O.server_majority(r) for r in (4, 5, 6, 7, 10)] == [3, 3, 5, 5, 7]


def check_case_verdicts(v, cases, ex, what=""):
    """Verdicts (oracle or device) against the hand-derived expectations of cert_cases.json."""
    op = 0
    for i, c in enumerate(cases):
        n = len(c["ops"])
        assert v.cert_reason[i] == ex.reason[i], (what, c["name"], v.cert_reason[i], c["why"])
        assert v.cert_fail_op[i] == ex.fail_op[i], (what, c["name"], v.cert_fail_op[i])
        assert bool(v.cert_accept[i]) == (ex.reason[i] == 0), (what, c["name"])
        np.testing.assert_array_equal(v.op_decision[op:op + n], ex.decisions[op:op + n], err_msg=f"{what} {c['name']}")
        np.testing.assert_array_equal(v.op_g0[op:op + n], ex.g0[op:op + n], err_msg=f"{what} {c['name']} g0")
        np.testing.assert_array_equal(v.op_ts[op:op + n], ex.op_ts[op:op + n], err_msg=f"{what} {c['name']} ts")
        op += n
    assert op == v.op_decision.shape[0]


@pytest.mark.parametrize("explicit_mg", [True, False])
@pytest.mark.parametrize("key", sorted(grouped_cases().keys()))
def test_cert_branch_cases(key, explicit_mg):
    """Oracle restatement vs the per-branch expectations (reason, failing op, per-op
    read/apply decision, g0 and its timestamp), with MultiGrant boundaries given
    explicitly and -- where they are runs of one signer -- left to the default."""
    R, strict, qm = key
    cases = grouped_cases(explicit_mg).get(key)
    if not cases:
        pytest.skip("every case of this group needs explicit MultiGrants")
    batch, ex = build_case_batch(cases, load_keys(R), explicit_mg)
    v = O.verify_batch(moduli_for(R), batch, R, bool(strict), 2, quorum_mode=qm)
    check_case_verdicts(v, cases, ex, f"oracle mg={explicit_mg}")


def test_cert_cases_cover_every_reason_and_decision():
    cases = load_cases()
    reasons = {c["reason"] for c in cases}
    assert reasons == {0, 1, 2, 3, 4, 5, 6, 8, 9, 10}  # 7 (UNDECIDED) is wire-path only
    decisions = {d for c in cases for d in c["decisions"]}
    assert decisions == {0, 1, 2, 3, 4}
    assert {c.get("quorum_mode", 0) for c in cases} == {0, 1, 2, 3}


def test_write1_uniform_restatement():
    # MochiDBClient.java:195-219: per key, all ts equal
    assert O.write1_uniform([0, 0, 0, 0], [5, 5, 5, 5])
    assert not O.write1_uniform([0, 0, 0, 0], [5, 5, 6, 5])
    assert O.write1_uniform([0, 1, 0, 1], [5, 9, 5, 9])
    assert not O.write1_uniform([0, 1, 0, 1], [5, 9, 5, 8])
    assert O.write1_uniform([], [])
