"""The reference's own integration scenarios, replayed through libmochi_hip.

Each test restates one of MochiClientServerCommunicationTest.java's tests on a
fresh in-process 4-server-of-5 cluster built from the reference's
config/sample_config (tests/cluster_harness.py) and asserts exactly what that
test asserts.  Every Write1 grant is signed by its server, every Write2
certificate goes through the batcher's request API with the receiving server's
stored state, and the per-op apply/read decisions the library returns drive
the server model — so these outcomes (the only behavioural expectations the
reference holds for this path) pin the tally / apply semantics (SURVEY §8 a3,
a4, a7) end to end.

* CPU (`-m "not gpu"`): backend "host" — the library's host signing, Write1
  classification and response tally, with Write2 verdicts from the oracle.
* GPU (`-m gpu`): backend "device" — k_rsa_sign, the device classify / tally
  kernels and the batched Write2 verify, and the oracle re-checks every Write2
  verdict and per-op output on the same message and state.
"""
import pytest

import cluster_harness as H
import mochi_hip as mh

BACKENDS = [pytest.param("host", id="host"), pytest.param("device", id="device", marks=pytest.mark.gpu)]


@pytest.fixture(params=BACKENDS)
def make_cluster(request):
    made = []

    def mk(seed=1, **kw):
        c = H.Cluster(backend=request.param, check_oracle=request.param == "device", seed=seed, **kw)
        made.append(c)
        return c

    yield mk
    for c in made:
        if c.backend == "device":  # every verdict applied was re-checked (async: every submission)
            assert c.stats["oracle_checked"] == c.stats["write2"] + c.stats["resubmits"], c.stats
        c.close()


def check_in(v, *allowed):
    return v in allowed


def test_read_operation(make_cluster):
    """testReadOperation (MochiClientServerCommunicationTest.java:173-223)."""
    c = make_cluster()
    cl = c.new_client()
    r1 = c.execute_write(cl, H.write_ops(("DEMO_READ_KEY_1", "NEW_VALUE_FOR_KEY_1_TR_1"),
                                         ("DEMO_READ_KEY_2", "NEW_VALUE_FOR_KEY_2_TR_1")))
    assert len(r1) == 2
    assert r1[0].result == "NEW_VALUE_FOR_KEY_1_TR_1"
    assert r1[1].result == "NEW_VALUE_FOR_KEY_2_TR_1"
    assert r1[0].cert is not None and r1[1].cert is not None
    assert r1[0].existed and r1[1].existed
    r2 = c.execute_read(cl, H.read_ops("DEMO_READ_KEY_1", "DEMO_READ_KEY_2"))
    assert len(r2) == 2
    assert r2[0].result == "NEW_VALUE_FOR_KEY_1_TR_1"
    assert r2[1].result == "NEW_VALUE_FOR_KEY_2_TR_1"
    # every replica applied the certificate and moved the epoch past the grant
    for s in c.replica_idx:
        for k in ("DEMO_READ_KEY_1", "DEMO_READ_KEY_2"):
            sv = c.servers[s].store[k]
            assert sv.current_c is r1[0].cert and sv.epoch == 1000 and not sv.given


def test_demo(make_cluster):
    """testDemo (:225-255)."""
    c = make_cluster(seed=2)
    cl = c.new_client()
    c.execute_write(cl, H.write_ops(("KEY1", "Hello"), ("KE2", "World")))
    r = c.execute_read(cl, H.read_ops("KEY1", "KE2"))
    assert r[0].result == "Hello" and r[1].result == "World"


def test_delete_operation(make_cluster):
    """testDeleteOperation (:257-348).  The client sends every Write1 op as a
    WRITE without value (MochiDBClient.java:256-261), so the Write1 of a delete
    creates the container and the delete applies at Write2."""
    c = make_cluster(seed=3)
    cl = c.new_client()
    r1 = c.execute_write(cl, H.write_ops(("DEMO_READ_KEY_1", "NEW_VALUE_FOR_KEY_1_TR_1"),
                                         ("DEMO_READ_KEY_2", "NEW_VALUE_FOR_KEY_2_TR_1")))
    assert [x.result for x in r1] == ["NEW_VALUE_FOR_KEY_1_TR_1", "NEW_VALUE_FOR_KEY_2_TR_1"]
    assert all(x.cert is not None and x.existed for x in r1)
    r2 = c.execute_read(cl, H.read_ops("DEMO_READ_KEY_1", "DEMO_READ_KEY_2"))
    assert [x.result for x in r2] == ["NEW_VALUE_FOR_KEY_1_TR_1", "NEW_VALUE_FOR_KEY_2_TR_1"]
    r3 = c.execute_write(cl, H.delete_ops("DEMO_READ_KEY_1", "DEMO_READ_KEY_2"))
    assert len(r3) == 2
    assert r3[0].result == "" and r3[1].result == ""
    assert not r3[0].existed and not r3[1].existed
    r4 = c.execute_read(cl, H.read_ops("DEMO_READ_KEY_1", "DEMO_READ_KEY_2"))
    assert len(r4) == 2
    assert r4[0].result == "" and r4[1].result == ""
    assert not r4[0].existed and not r4[1].existed


def test_write_operation_overwrite(make_cluster):
    """testWriteOperation (:350-416): the second certificate's g0 timestamp is in
    the next epoch (StoreValueObjectContainer.java:83-88, Write1 issuance at
    InMemoryDataStore.java:127), so it lands on APPLY, not READ (:594-599)."""
    c = make_cluster(seed=4)
    cl = c.new_client()
    r1 = c.execute_write(cl, H.write_ops(("DEMO_KEY_1", "NEW_VALUE_FOR_KEY_1_TR_1"),
                                         ("DEMO_KEY_2", "NEW_VALUE_FOR_KEY_2_TR_1")))
    assert [x.result for x in r1] == ["NEW_VALUE_FOR_KEY_1_TR_1", "NEW_VALUE_FOR_KEY_2_TR_1"]
    assert all(x.cert is not None and x.existed for x in r1)
    ts1 = r1[0].cert.ts_for("DEMO_KEY_1")
    r2 = c.execute_write(cl, H.write_ops(("DEMO_KEY_1", "NEW_VALUE_FOR_KEY_1_TR_2"),
                                         ("DEMO_KEY_2", "NEW_VALUE_FOR_KEY_2_TR_2")))
    assert len(r2) == 2
    assert r2[0].result == "NEW_VALUE_FOR_KEY_1_TR_2" and r2[0].existed
    assert r2[1].result == "NEW_VALUE_FOR_KEY_2_TR_2" and r2[1].existed
    ts2 = r2[0].cert.ts_for("DEMO_KEY_1")
    assert ts1 < 1000 <= ts2 < 2000  # epoch 0 grant, then an epoch-1000 grant
    assert c.stats["read_branch"] == 0
    r3 = c.execute_read(cl, H.read_ops("DEMO_KEY_1", "DEMO_KEY_2"))
    assert [x.result for x in r3] == ["NEW_VALUE_FOR_KEY_1_TR_2", "NEW_VALUE_FOR_KEY_2_TR_2"]


def concurrent_runnable(cl):
    """MochiConcurrentTestRunnable.runTest (:499-595)."""
    r1 = yield ("write", H.write_ops(("DEMO_KEY_1", "NEW_VALUE_FOR_KEY_1_TR_1"),
                                     ("DEMO_KEY_2", "NEW_VALUE_FOR_KEY_2_TR_1")))
    assert isinstance(r1, list) and len(r1) == 2, r1
    assert check_in(r1[0].result, "NEW_VALUE_FOR_KEY_1_TR_1", "NEW_VALUE_FOR_KEY_1_TR_2")
    assert check_in(r1[1].result, "NEW_VALUE_FOR_KEY_2_TR_1", "NEW_VALUE_FOR_KEY_2_TR_2")
    assert r1[0].cert is not None and r1[1].cert is not None
    r2 = yield ("write", H.write_ops(("DEMO_KEY_1", "NEW_VALUE_FOR_KEY_1_TR_2"),
                                     ("DEMO_KEY_2", "NEW_VALUE_FOR_KEY_2_TR_2")))
    assert isinstance(r2, list) and len(r2) == 2, r2
    assert r2[0].existed and check_in(r2[0].result, "NEW_VALUE_FOR_KEY_1_TR_1", "NEW_VALUE_FOR_KEY_1_TR_2")
    assert r2[1].existed and check_in(r2[1].result, "NEW_VALUE_FOR_KEY_2_TR_1", "NEW_VALUE_FOR_KEY_2_TR_2")
    r3 = yield ("read", H.read_ops("DEMO_KEY_1", "DEMO_KEY_2"))
    assert isinstance(r3, list) and len(r3) == 2, r3
    assert check_in(r3[0].result, "NEW_VALUE_FOR_KEY_1_TR_1", "NEW_VALUE_FOR_KEY_1_TR_2")
    assert check_in(r3[1].result, "NEW_VALUE_FOR_KEY_2_TR_1", "NEW_VALUE_FOR_KEY_2_TR_2")
    r4 = yield ("write", H.write_ops(("DEMO_KEY_TEST_1", "1")))
    assert isinstance(r4, list), r4
    r5 = yield ("write", H.write_ops(("DEMO_KEY_TEST_2", "2")))
    assert isinstance(r5, list), r5


def test_write_operation_concurrent(make_cluster):
    """testWriteOperationConcurrent (:418-475): five clients run the runnable one
    by one, then all five concurrently (here: interleaved by the scheduler)."""
    c = make_cluster(seed=5)
    for _ in range(5):  # one by one
        cl = H.ScriptedClient(c, concurrent_runnable)
        H.run_clients(c, [cl])
        assert cl.error is None, cl.error
    clients = [H.ScriptedClient(c, concurrent_runnable) for _ in range(5)]  # concurrently
    H.run_clients(c, clients)
    for cl in clients:
        assert cl.error is None, cl.error
    # the interleaving really was concurrent: Write1 rounds saw mixed epochs and retried,
    # and late certificates took the READ branch
    assert c.stats["retries"] > 0 or c.stats["read_branch"] > 0, c.stats


def stress_runnable(start, n, seed):
    """MochiConcurrentStreeTestRunnable.runTest (:721-753)."""
    def script(cl):
        import random

        rng = random.Random(seed)
        nums = list(range(start, start + n))
        rng.shuffle(nums)
        for i in nums:
            key = f"DEMO_KEY_STRESS_TEST_{i}"
            r = yield ("write", H.write_ops((key, f"New Value for key {key}")))
            assert isinstance(r, list), r
        rng.shuffle(nums)
        for i in nums:
            key = f"DEMO_KEY_STRESS_TEST_{i}"
            r = yield ("read", H.read_ops(key))
            assert isinstance(r, list), r
            assert r[0].result == f"New Value for key {key}"
        for i in nums:
            key = f"DEMO_KEY_STRESS_TEST_{i}"
            r = yield ("write", H.delete_ops(key))
            assert isinstance(r, list), r
    return script


def test_write_operation_concurrent_stress(make_cluster):
    """testWriteOperationConcurrentStressTest (:636-685): 5 clients x 40 keys each
    (disjoint ranges): write all, read all back, delete all — concurrently."""
    c = make_cluster(seed=6)
    clients = [H.ScriptedClient(c, stress_runnable(40 * i, 40, 100 + i)) for i in range(5)]
    H.run_clients(c, clients)
    for cl in clients:
        assert cl.error is None, cl.error
    assert c.stats["write2"] == 5 * 80 * c.R


def test_java_collection_orders():
    """The orders the harness reproduces: String.hashCode / Server.hashCode and
    HashMap iteration (bucket = spread(hash) & 15, collisions in insertion order)."""
    assert H.java_string_hash("") == 0
    assert H.java_string_hash("a") == 97
    assert H.java_string_hash("hello") == 99162322
    assert H.java_string_hash("DEMO_KEY_1") == (0x0 + sum(ord(ch) * 31 ** (9 - i) for i, ch in enumerate("DEMO_KEY_1"))) % 2**32
    # two keys in one bucket keep insertion order; a lower bucket comes first
    ids = ["server-55a78d3f-783d-43ae-95c1-6d0f5f02fe0c", "server-6c023c90-87ed-40d9-8f38-48cb03fa2135",
           "server-ed25bc93-1047-4242-b87b-2246355b020b"]
    h = [H.java_string_hash(x) for x in ids]
    assert H.java_hash_order(ids, h) == [ids[2], ids[0], ids[1]]
    assert H.java_hash_order(ids[1::-1], h[1::-1]) == [ids[1], ids[0]]
    # resize past 12 entries keeps every key once
    keys = [f"k{i}" for i in range(40)]
    assert sorted(H.java_hash_order(keys, [H.java_string_hash(k) for k in keys])) == sorted(keys)


def test_rejected_certificate_hangs_the_client(make_cluster):
    """A tampered Write2 (a MultiGrant signature flipped on every replica's
    copy) is rejected by the servers; the reference throws inside
    processWrite2ToServer, sends no Write2Ans, and the client waits forever."""
    c = make_cluster(seed=7)
    cl = c.new_client()
    p = c.start_write(cl, H.write_ops(("DEMO_KEY_X", "v")))
    while p.kind == "W1":
        for q, out in c.step():
            assert q is not p, out
    # corrupt one grant signature of every MultiGrant before Write2 is delivered
    for _, mg in p.cert.mgs:
        g = mg.grants[0]
        g.sig = bytes([g.sig[0] ^ 1]) + g.sig[1:]
    import workload as W

    wc = b"".join(W.encode_map_entry(1, sid.encode(), mg.encode()) for sid, mg in p.cert.mgs)
    p.msg = W._ld(1, wc) + W._ld(2, H.encode_txn(p.ops))
    with pytest.raises(H.Hung):
        c.run(p)
    for s in c.replica_idx:  # nothing applied
        assert c.servers[s].store["DEMO_KEY_X"].current_c is None


def shared_keys_runnable(cid, keys, rounds, seed):
    """Clients hammering the same few keys: writes of one or two shared keys, read
    backs (the value is some client's write)."""
    def script(cl):
        import random

        rng = random.Random(seed)
        for j in range(rounds):
            ks = sorted(rng.sample(keys, rng.choice((1, 2))))
            r = yield ("write", H.write_ops(*[(k, f"c{cid}-{j}-{k}") for k in ks]))
            if isinstance(r, H.ClientError):
                continue  # a refused Write1 round (RequestRefused) is the reference's outcome too
            assert isinstance(r, list) and len(r) == len(ks), r
            r = yield ("read", H.read_ops(*ks))
            assert isinstance(r, list), r
            for k, x in zip(ks, r):
                assert x.result.startswith("c") and x.result.endswith(k), x
    return script


def test_async_handler_race_protocol(make_cluster):
    """INTEGRATION.md §4's asynchronous handler with Write2s on the
    same keys in flight together.  Each server snapshots the verifier's inputs,
    releases the locks and submits (mochi_batcher_submit_request); completions are
    applied at later steps after the sameWrite2State re-check, resubmitting when a
    Write2 on one of the keys landed meanwhile.  The reference's assertions hold,
    resubmissions happen, and every reply and the final per-key state equal a
    serial replay of the same events through the oracle (the reference holds the
    key write locks across validation and apply, InMemoryDataStore.java:641-666)."""
    c = make_cluster(seed=8, async_w2=True)
    clients = [H.ScriptedClient(c, concurrent_runnable) for _ in range(5)]
    keys = [f"SHARED_KEY_{i}" for i in range(3)]
    clients += [H.ScriptedClient(c, shared_keys_runnable(i, keys, 6, 300 + i)) for i in range(6)]
    H.run_clients(c, clients)
    for cl in clients:
        assert cl.error is None, cl.error
    assert c.stats["max_same_key_inflight"] >= 2, c.stats
    assert c.stats["resubmits"] > 0, c.stats
    assert not c.async_q
    n = H.replay_serial(c)
    assert n > 0 and c.stats["write2"] == sum(1 for e in c.log if e[1] == "W2")


def test_serial_replay_of_the_blocking_handler(make_cluster):
    """The replay check itself, on the blocking handler's stress run (no Write2 ever
    races there): replies and final state equal the serial oracle replay."""
    c = make_cluster(seed=9)
    keys = [f"SHARED_KEY_{i}" for i in range(3)]
    clients = [H.ScriptedClient(c, shared_keys_runnable(i, keys, 4, 400 + i)) for i in range(4)]
    H.run_clients(c, clients)
    for cl in clients:
        assert cl.error is None, cl.error
    assert c.stats["resubmits"] == 0
    assert H.replay_serial(c) > 0
