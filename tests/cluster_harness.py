"""In-process MochiDB cluster that drives libmochi_hip end to end (test-side).

The reference's integration tests (MochiClientServerCommunicationTest.java) run
a virtual cluster of MochiServers in one JVM (MochiVirtualCluster.java:35-73:
5 servers, R = 4) and assert what clients see.  No JVM exists here, so this
module replays those scenarios with:

* a **server model** that keeps only the state feeding the verifier — per key
  the StoreValueObjectContainer's epoch, the Write1 grants it has given, the
  stored certificate `currentC`, the value and `valueAvailble`
  (InMemoryDataStore.java:105-155, StoreValueObjectContainer.java:83-198);
* a **client model** of MochiDBClient's Write1 / Write2 / Read rounds
  (MochiDBClient.java:114-181, 236-387);

and every decision the hot path makes taken from the library:

* grant signing at the Write1 site (InMemoryDataStore.java:283-295, the TODO at
  MochiProtocol.proto:123): `mochi_sign_batch` (k_rsa_sign) per server;
* the client's Write1 round (:273-328): `mochi_write1_classify_device`;
* Write2 certificate validation + the apply/read decision per op
  (InMemoryDataStore.java:576-666): `mochi_batcher_submit_request`, with the
  op flags and stored-certificate timestamps taken from the server model — the
  per-op decisions are applied back into the model;
* the client's Write2 / Read aggregation (:148-175, 355-382):
  `mochi_tally_responses_device`.

`backend="host"` swaps the device calls for the library's host C++ paths
(OpenSSL signing, host classify / tally) and the CPU oracle for the Write2
verdicts, so the harness logic itself runs in the CPU test suite.  With
`check_oracle=True` (device backend) every Write2 verdict and per-op output is
compared with the oracle's (tests/oracle_ffi.py) on the same message + state.

Message delivery is a seeded deterministic scheduler: each step delivers a
random subset of the in-flight messages (never two Write2s for one key at one
server in the same step — the reference serialises them under the object's
write lock, InMemoryDataStore.java:369-383), so concurrent clients interleave
the way the reference's threads can.  Java collection orders that reach the
wire are reproduced: HashSet<Server> send order, HashMap<String,...> iteration
order of the certificate and grant maps (MochiDBClient.java:291-299, 333-338;
InMemoryDataStore.java:283-295).
"""
from __future__ import annotations

import hashlib
import os
import random
import sys
import threading
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for _p in (os.path.join(ROOT, "mochi-db_amd"), HERE):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import mochi_hip as mh  # noqa: E402
import workload as W  # noqa: E402

# MochiProtocol.proto enums
READ, DELETE, WRITE = 0, 1, 2
ST_OK, ST_WRONG_SHARD = 0, 1
SAMPLE_CONFIG = os.path.join(HERE, "golden", "sample_config")


# ---------------------------------------------------------------------------
# Java collection orders that reach the wire
# ---------------------------------------------------------------------------
def java_string_hash(s: str) -> int:
    """String.hashCode over UTF-16 code units, as an unsigned 32-bit value."""
    h = 0
    u = s.encode("utf-16-be")
    for i in range(0, len(u), 2):
        h = (31 * h + ((u[i] << 8) | u[i + 1])) & 0xFFFFFFFF
    return h


def java_server_hash(host: str, port: int) -> int:
    """Server.hashCode (messaging/Server.java:23-29)."""
    r = (31 * 1 + port) & 0xFFFFFFFF
    return (31 * r + java_string_hash(host)) & 0xFFFFFFFF


def java_hash_order(keys, hashes) -> list:
    """Iteration order of a java.util.HashMap / HashSet filled in `keys` order
    (default capacity 16, load factor 0.75, resize keeps relative order)."""
    cap, n = 16, 0
    buckets: List[list] = [[] for _ in range(cap)]
    for k, h in zip(keys, hashes):
        sp = (h ^ (h >> 16)) & 0xFFFFFFFF
        b = buckets[sp & (cap - 1)]
        if any(x == k for x, _ in b):
            continue
        b.append((k, sp))
        n += 1
        if n > cap * 3 // 4:
            cap *= 2
            nb: List[list] = [[] for _ in range(cap)]
            for bucket in buckets:
                for kk, hh in bucket:
                    nb[hh & (cap - 1)].append((kk, hh))
            buckets = nb
    return [k for b in buckets for k, _ in b]


# ---------------------------------------------------------------------------
# Protocol objects (the parts the path reads)
# ---------------------------------------------------------------------------
@dataclass
class Op:
    action: int
    key: str
    value: str = ""

    def encode(self) -> bytes:
        return W.encode_operation(self.action, self.key, self.value)


def encode_txn(ops: List[Op]) -> bytes:
    return b"".join(W._ld(1, op.encode()) for op in ops)


def txn_hash(ops: List[Op]) -> str:
    """Stand-in for Utils.objectSHA512(txn) (Utils.java:150-153): lowercase-hex
    SHA-512 of the Transaction's protobuf bytes (the Java-serialization envelope
    is not reproducible here; the hash enters the verifier as an opaque value)."""
    return hashlib.sha512(b"mochi-txn:" + encode_txn(ops)).hexdigest()


@dataclass
class GrantRec:
    object_id: str
    ts: int
    txn_hash: str
    status: int = ST_OK
    sig: Optional[bytes] = None

    def encode(self) -> bytes:
        return W.encode_grant(self.object_id, self.ts, self.txn_hash, 0, self.status)


@dataclass
class MultiGrantRec:
    server_id: str
    client_id: str
    grants: List[GrantRec]  # map insertion (= wire) order

    def encode(self) -> bytes:
        return W.encode_multigrant([(g.object_id, g.encode()) for g in self.grants], self.server_id, self.client_id,
                                   "", [(g.object_id, g.sig) for g in self.grants])

    def grant(self, key: str) -> Optional[GrantRec]:
        for g in self.grants:
            if g.object_id == key:
                return g
        return None


@dataclass
class Cert:
    """WriteCertificate: (serverId, MultiGrant) in wire order."""
    mgs: List[Tuple[str, MultiGrantRec]]

    def ts_for(self, key: str) -> int:
        """getCurrentTimestampFromCurrentCertificate (StoreValueObjectContainer.java:175-198)."""
        ts = None
        for _, mg in self.mgs:
            g = mg.grant(key)
            if g is None:
                raise IllegalState("grantForCurrentKey map should not be null")
            if ts is None:
                ts = g.ts
            elif ts != g.ts:
                raise IllegalState("Timestamp mismatch between grants from different servers")
        return ts


class IllegalState(Exception):
    pass


@dataclass
class OpResult:
    status: int = ST_OK
    result: str = ""
    existed: bool = False
    cert: Optional[Cert] = None


# ---------------------------------------------------------------------------
# Server model
# ---------------------------------------------------------------------------
@dataclass
class SVOC:
    """StoreValueObjectContainer: the per-key state the verifier depends on."""
    key: str
    value: Optional[str] = None
    available: bool = False
    current_c: Optional[Cert] = None
    epoch: int = 0
    given: Dict[int, GrantRec] = field(default_factory=dict)  # ts -> grant (epoch buckets folded)

    def move_to_next_epoch_if_necessary(self, ts: int):  # :83-88
        nxt = (ts // 1000 + 1) * 1000
        if self.epoch < nxt:
            self.epoch = nxt


class Server:
    def __init__(self, index: int, server_id: str, url: str, replicas: List[str]):
        self.index = index
        self.id = server_id
        self.host, port = url.split(":")
        self.port = int(port)
        self.replicas = replicas
        self.store: Dict[str, SVOC] = {}

    def local(self, key: str) -> bool:  # objectBelongsToCurrentShardServer (:63-72)
        return self.id in self.replicas

    # --- Write1 (InMemoryDataStore.processWrite / tryProcessWriteRegularly, :105-155, :233-310)
    def write1(self, ops: List[Op], seed: int, thash: str, client_id: str):
        """-> (kind, MultiGrantRec, new_grants_to_sign)"""
        granted, refused, new = {}, {}, []
        order = []
        all_ok = True
        for op in ops:
            if op.action not in (WRITE, DELETE):
                continue
            if not self.local(op.key):
                g = GrantRec(op.key, 0, thash, ST_WRONG_SHARD)
                granted[op.key] = g
                new.append(g)
                order.append(op.key)
                continue
            sv = self.store.get(op.key)
            if sv is None:  # getOrCreateStoreValue (the client sends every Write1 op as WRITE, :256-261)
                sv = self.store[op.key] = SVOC(op.key)
            ts = sv.epoch + seed
            g = sv.given.get(ts)
            if g is None:
                g = GrantRec(op.key, ts, thash)
                sv.given[ts] = g
                new.append(g)
                granted[op.key] = g
            elif g.txn_hash == thash:
                granted[op.key] = g  # a retry: the grant given before
            else:
                refused[op.key] = g  # someone else holds this timestamp
                all_ok = False
            order.append(op.key)
        src = granted if all_ok else refused
        keys = java_hash_order([k for k in order if k in src], [java_string_hash(k) for k in order if k in src])
        mg = MultiGrantRec(self.id, client_id, [src[k] for k in keys])
        return ("OK" if all_ok else "REFUSED"), mg, new

    # --- Write2: the state the verifier reads (op flags, stored certificate ts)
    def write2_state(self, ops: List[Op]):
        flags, ots = [], []
        applied = set()  # keys an earlier op of this transaction applies: the kernel tracks wc itself
        for op in ops:
            f = 0
            if self.local(op.key):
                f |= mh.OP_LOCAL
            sv = self.store.get(op.key)
            if sv is not None:
                f |= mh.OP_HAS_SVOC
                if sv.current_c is not None:
                    f |= mh.OP_HAS_CURRENT_C
                    try:
                        ots.append(sv.current_c.ts_for(op.key))
                    except IllegalState:
                        f |= mh.OP_CURRENT_C_BAD
                        ots.append(0)
                else:
                    ots.append(0)
            else:
                ots.append(0)
            if op.action not in (WRITE, DELETE):
                f |= mh.OP_NOT_WRITE
            flags.append(f)
            applied.add(op.key)
        return flags, ots

    # --- Write2 apply (write2apply / applyOperation / readOperation, :521-611)
    def write2_apply(self, ops: List[Op], cert: Cert, accepted: bool, per_op) -> Optional[List[OpResult]]:
        """Apply the library's per-op decisions.  Returns the Write2Ans results,
        or None when the reference throws (no reply is sent)."""
        results = []
        for op, (dec, g0, ts) in zip(ops, per_op):
            if dec == mh.OPD_WRONG_SHARD:
                results.append(OpResult(status=ST_WRONG_SHARD))
            elif dec == mh.OPD_READ:
                sv = self.store[op.key]
                results.append(OpResult(ST_OK, sv.value or "", True, sv.current_c))
            elif dec == mh.OPD_APPLY:
                sv = self.store[op.key]
                sv.current_c = cert
                t = cert.ts_for(op.key)
                assert t == ts, (t, ts)  # the library reports g0's timestamp = the certificate's
                sv.given.pop(t, None)
                sv.move_to_next_epoch_if_necessary(t)
                if op.action == WRITE:
                    sv.value, sv.available = op.value, True
                else:
                    sv.value, sv.available = None, False
                results.append(OpResult(ST_OK, op.value, sv.available, cert))
            else:  # FAILED / SKIPPED: the reference threw here (ops before stay applied)
                return None
        return results if accepted else None

    # --- Read (processReadRequest / processRead, :75-103, :201-231)
    def read(self, ops: List[Op]) -> Optional[List[OpResult]]:
        out = []
        for op in ops:
            if op.action != READ:
                return None  # checkAndFailOnReadOnly throws
            if not self.local(op.key):
                out.append(OpResult(status=ST_WRONG_SHARD))
                continue
            sv = self.store.get(op.key)
            if sv is None:
                return None  # keyStoreValue.isValueAvailble() on null: NPE, no reply
            out.append(OpResult(ST_OK, sv.value or "", sv.available, sv.current_c))
        return out


# ---------------------------------------------------------------------------
# Client exceptions (client/*Exception.java)
# ---------------------------------------------------------------------------
class ClientError(Exception):
    pass


class RequestRefused(ClientError):
    pass


class RequestFailed(ClientError):
    pass


class InconsistentWrite(ClientError):
    pass


class InconsistentRead(ClientError):
    pass


class Hung(ClientError):
    """A server threw on the request: the reference client waits forever
    (Utils.busyWaitForFutures has no timeout, Utils.java:65-93)."""


# ---------------------------------------------------------------------------
# The cluster
# ---------------------------------------------------------------------------
@dataclass
class Pending:
    """A client request in flight."""
    client: int
    kind: str  # "W1" | "W2" | "R"
    ops: List[Op]
    thash: str = ""
    seed: int = 0
    msg: bytes = b""
    cert: Optional[Cert] = None
    todo: List[int] = field(default_factory=list)  # servers not yet delivered
    replies: Dict[int, object] = field(default_factory=dict)
    dead: set = field(default_factory=set)  # servers that threw (no reply)
    t_start: float = 0.0
    outstanding: int = 0  # async Write2s delivered but not yet applied (async_w2 mode)


@dataclass
class AsyncW2:
    """A Write2 in the asynchronous handler: the state
    snapshot it was submitted with, and its verdict once the callback ran."""
    srv: "Server"
    p: Pending
    snap: Tuple[list, list]
    verdict: Optional[tuple] = None
    req: object = None
    submits: int = 0


class Cluster:
    def __init__(self, backend: str = "device", check_oracle: bool = False, seed: int = 1, device: int = 0,
                 config_path: str = SAMPLE_CONFIG, key_dir: str = W.DEFAULT_KEY_DIR, max_wait_us: int = 200,
                 async_w2: bool = False, p_apply: float = 0.35):
        """async_w2: Write2s go through INTEGRATION.md §4's asynchronous handler -- the
        server snapshots the verifier's inputs (op flags, stored-certificate
        timestamps) under the key locks, RELEASES them and submits; the verdict
        is applied at a later step (each ready completion with probability
        p_apply), after re-checking the state under the locks
        (sameWrite2State) and re-submitting when a Write2 on one of the keys
        landed meanwhile.  Several Write2s on one key at one server are then in
        flight together.  Every state change is logged (self.log) for
        replay_serial()."""
        assert backend in ("device", "host")
        self.async_w2 = async_w2
        self.p_apply = p_apply
        self.async_q: List[AsyncW2] = []
        self.log: List[tuple] = []
        self.backend = backend
        self.check_oracle = check_oracle
        self.rng = random.Random(seed)
        cfg = mh.ClusterConfig(config_path)
        self.R = cfg.replication_factor
        self.M = cfg.majority
        servers = cfg.servers()
        self.replica_idx = cfg.servers_for_key("")  # every key: tokens 0..R-1 (ClusterConfiguration.java:215)
        self.replica_ids = [servers[i][0] for i in self.replica_idx]
        cfg.close()
        self.servers = [Server(i, sid, url, self.replica_ids) for i, (sid, url) in enumerate(servers)]
        # relevantServers: a HashSet<Server> (MochiDBClient.java:238-243) -> send / response order
        rep = [self.servers[i] for i in self.replica_idx]
        self.send_order = java_hash_order([s.index for s in rep],
                                          [java_server_hash(s.host, s.port) for s in rep])
        # key i of the verifier = replica i (MultiGrant.serverId -> signer)
        self.pems = W.load_keys(self.R, key_dir)
        self.moduli = [mh.pem_modulus(p) for p in self.pems]
        self.ids_blob, self.ids_off = W.server_id_table(self.R, self.replica_ids)
        self.signer_of = {self.replica_idx[i]: i for i in range(self.R)}
        self.device = device
        self.verifier = self.batcher = None
        self.signers = []
        if backend == "device":
            self.verifier = mh.Verifier(self.moduli, device=device)
            self.verifier.set_server_ids(self.replica_ids)
            self.batcher = mh.Batcher(self.verifier, self.R, strict_gt=True, max_msgs=8192, max_wait_us=max_wait_us,
                                      with_op_flags=True)
            self.signers = [mh.DeviceSigner(p, device=device) for p in self.pems]
        self.inflight: List[Pending] = []
        self.n_clients = 0
        self.stats = {"write1": 0, "write2": 0, "reads": 0, "retries": 0, "oracle_checked": 0, "steps": 0,
                      "signed": 0, "read_branch": 0, "resubmits": 0, "max_same_key_inflight": 0}
        self.config_path = config_path

    def close(self):
        if self.batcher:
            self.batcher.close()
        for s in self.signers:
            s.close()
        if self.verifier:
            self.verifier.close()

    # --- library calls, batched per step -----------------------------------------
    def _sign(self, server: Server, grants: List[GrantRec]):
        if not grants:
            return
        enc = [g.encode() for g in grants]
        blob = np.frombuffer(b"".join(enc), np.uint8).copy()
        off = np.zeros(len(enc), np.uint64)
        off[1:] = np.cumsum([len(e) for e in enc])[:-1]
        ln = np.array([len(e) for e in enc], np.uint32)
        k = self.signer_of[server.index]
        if self.backend == "device":
            sig = self.signers[k].sign(blob, off, ln)
        else:
            sig = mh.sign_grants(self.pems[k], blob, off, ln)
        for g, s in zip(grants, sig):
            g.sig = s.tobytes()
        self.stats["signed"] += len(grants)

    def _classify(self, rounds):
        """rounds: [(Pending, [(kind, MultiGrantRec)] in response order)] -> decisions."""
        reqs = []
        for p, resps in rounds:
            slot = {}
            for op in p.ops:
                slot.setdefault(op.key, len(slot))
            rr = []
            for kind, mg in resps:
                k = {"OK": mh.W1_OK, "REFUSED": mh.W1_REFUSED}[kind]
                rr.append((k, self.replica_ids.index(mg.server_id),
                           [(slot.get(g.object_id, 0xFF), g.ts, g.status) for g in mg.grants]))
            reqs.append(rr)
        if self.backend == "device":
            return mh.write1_classify_device(reqs, self.device)
        return mh.write1_classify(reqs)

    def _tally(self, rounds):
        """rounds: [(Pending, [results per responding server])] -> (accept, chosen)."""
        responses = [[[r.status for r in res] for res in resps] for _, resps in rounds]
        n_ops = [len(p.ops) for p, _ in rounds]
        if self.backend == "device":
            acc, _, ch = mh.tally_responses_device(responses, n_ops, self.R, self.device)
        else:
            acc, _, ch = mh.tally_responses(responses, n_ops, self.R)
        return acc, ch

    def _verify_write2(self, jobs):
        """jobs: [(server, Pending, flags, ots)] -> [(accepted, reason, fail_op, per_op)]"""
        if not jobs:
            return []
        if self.backend == "device":
            reqs = [mh.Write2Request(p.msg, p.thash.encode(), flags, ots) for _, p, flags, ots in jobs]
            done = threading.Semaphore(0)
            for r in reqs:
                self.batcher.submit_request(r, lambda _r: done.release())
            for _ in reqs:
                done.acquire()
            out = []
            for r in reqs:
                rc, acc, reason, fail_op, _ = r.result
                assert rc == mh.OK, rc
                out.append((acc, reason, fail_op, r.ops()))
            if self.check_oracle:
                self._oracle_check(jobs, out)
            return out
        return self._oracle_verdicts(jobs)

    def _wire_batch(self, jobs):
        msgs = [p.msg for _, p, _, _ in jobs]
        off = np.zeros(len(msgs), np.uint64)
        off[1:] = np.cumsum([len(m) for m in msgs])[:-1]
        ofo = np.zeros(len(msgs) + 1, np.uint32)
        np.cumsum([len(f) for _, _, f, _ in jobs], out=ofo[1:])
        return W.WireBatch(wire=np.frombuffer(b"".join(msgs), np.uint8).copy(), msg_off=off,
                           msg_len=np.array([len(m) for m in msgs], np.uint32), op_flags_off=ofo,
                           op_flags=np.array([x for _, _, f, _ in jobs for x in f], np.uint8),
                           expected_hash=np.frombuffer(b"".join(p.thash.encode() for _, p, _, _ in jobs),
                                                       np.uint8).reshape(-1, 128).copy(),
                           op_object_ts=np.array([x for _, _, _, t in jobs for x in t], np.int64))

    def _oracle_verdicts(self, jobs):
        import oracle_ffi as O

        wb = self._wire_batch(jobs)
        v, _ = O.verify_write2(self.moduli, self.ids_blob, self.ids_off, wb, self.R, True, 4)
        out = []
        for i, (_, p, f, _) in enumerate(jobs):
            o0 = int(wb.op_flags_off[i])
            per_op = [(int(v.op_decision[o0 + j]), int(v.op_g0[o0 + j]), int(v.op_ts[o0 + j])) for j in range(len(f))]
            out.append((bool(v.cert_accept[i]), int(v.cert_reason[i]), int(v.cert_fail_op[i]), per_op))
        return out

    def _oracle_check(self, jobs, got):
        want = self._oracle_verdicts(jobs)
        for (s, p, f, t), g, w in zip(jobs, got, want):
            assert g == w, f"library {g} != oracle {w} (server {s.index}, flags {f}, ts {t})"
        self.stats["oracle_checked"] += len(jobs)

    # --- the asynchronous Write2 handler ------------------------
    def _async_submit(self, es: List[AsyncW2]):
        """Submit each entry with its snapshot; returns once every verdict is in
        (the callbacks ran), so the scheduler's choices stay deterministic."""
        if not es:
            return
        for e in es:
            e.submits += 1
            e.verdict = None
        if self.backend == "device":
            done = threading.Semaphore(0)
            for e in es:
                flags, ots = e.snap
                e.req = mh.Write2Request(e.p.msg, e.p.thash.encode(), flags, ots)
                self.batcher.submit_request(e.req, lambda _r: done.release())  # callback on a flusher thread
            for _ in es:
                done.acquire()
            for e in es:
                rc, acc, reason, fail_op, _ = e.req.result
                assert rc == mh.OK, rc
                e.verdict = (acc, reason, fail_op, e.req.ops())
            if self.check_oracle:
                self._oracle_check([(e.srv, e.p, e.snap[0], e.snap[1]) for e in es], [e.verdict for e in es])
        else:
            for e, v in zip(es, self._oracle_verdicts([(e.srv, e.p, e.snap[0], e.snap[1]) for e in es])):
                e.verdict = v

    def _async_complete(self):
        """The apply tasks of ready verdicts, a random subset per step, each under
        its keys' locks (atomic here): unchanged state -> apply the verdict and
        reply; changed -> verify again against the new state."""
        again = []
        ready = [e for e in self.async_q if e.verdict is not None]
        self.rng.shuffle(ready)
        for e in ready:
            if self.rng.random() >= self.p_apply:
                continue
            cur = e.srv.write2_state(e.p.ops)
            if cur != e.snap:  # sameWrite2State failed: a Write2 on one of the keys landed meanwhile
                e.snap = cur
                self.stats["resubmits"] += 1
                again.append(e)
                continue
            self.async_q.remove(e)
            self._apply_w2(e.srv, e.p, e.verdict)
            e.p.outstanding -= 1
        self._async_submit(again)

    def _apply_w2(self, srv, p, verdict):
        acc, reason, fail_op, per_op = verdict
        self.stats["write2"] += 1
        self.stats["read_branch"] += sum(1 for d, _, _ in per_op if d == mh.OPD_READ)
        res = srv.write2_apply(p.ops, p.cert, acc, per_op)
        self.log.append((srv.index, "W2", p, res))
        if res is None:
            p.dead.add(srv.index)
        else:
            p.replies[srv.index] = res

    # --- client API ------------------------------------------------------------------
    def new_client(self) -> int:
        self.n_clients += 1
        return self.n_clients - 1

    def start_write(self, client: int, ops: List[Op]) -> Pending:
        p = Pending(client, "W1", ops, thash=txn_hash(ops))
        self._send_write1(p)
        return p

    def start_read(self, client: int, ops: List[Op]) -> Pending:
        p = Pending(client, "R", ops)
        p.todo = list(self.send_order)
        self.inflight.append(p)
        return p

    def _send_write1(self, p: Pending):
        p.kind = "W1"
        p.seed = self.rng.randrange(1000)  # Random.nextInt(1000) (MochiDBClient.java:262)
        p.todo = list(self.send_order)
        p.replies = {}
        self.inflight.append(p)
        self.stats["write1"] += 1

    # --- the scheduler ---------------------------------------------------------------
    def step(self, p_deliver: float = 0.6):
        """Deliver a random subset of the in-flight messages, run the library on
        the batch they form, and advance the clients whose rounds completed.
        Returns the list of (Pending, outcome) finished this step, outcome =
        list of OpResult or a ClientError."""
        self.stats["steps"] += 1
        deliveries = []
        for p in self.inflight:
            for s in list(p.todo):
                if self.rng.random() < p_deliver:
                    deliveries.append((p, s))
        if not deliveries:  # always make progress
            p = next((q for q in self.inflight if q.todo), None)
            if p is not None:
                deliveries.append((p, p.todo[0]))
        self.rng.shuffle(deliveries)
        # one Write2 per (server, key) per step (the object's write lock serialises them)
        locked = set()
        w1_new: Dict[int, List[GrantRec]] = {}
        w2_jobs = []
        submit_now = []
        for p, s in deliveries:
            srv = self.servers[s]
            if p.kind == "W2" and self.async_w2:  # snapshot under the locks, release, submit
                e = AsyncW2(srv, p, srv.write2_state(p.ops))
                self.async_q.append(e)
                submit_now.append(e)
                p.outstanding += 1
                p.todo.remove(s)
                continue
            if p.kind == "W2":
                keys = {(s, op.key) for op in p.ops}
                if keys & locked:
                    continue
                locked |= keys
                flags, ots = srv.write2_state(p.ops)
                w2_jobs.append((srv, p, flags, ots))
            elif p.kind == "W1":
                if any((s, op.key) in locked for op in p.ops):
                    continue
                kind, mg, new = srv.write1(p.ops, p.seed, p.thash, "")
                w1_new.setdefault(s, []).extend(new)
                p.replies[s] = (kind, mg)
                self.log.append((s, "W1", p, (kind, [(g.object_id, g.ts, g.txn_hash, g.status) for g in mg.grants],
                                            p.seed)))
            else:
                if any((s, op.key) in locked for op in p.ops):
                    continue
                res = srv.read(p.ops)
                self.log.append((s, "R", p, res))
                if res is None:
                    p.dead.add(s)
                else:
                    p.replies[s] = res
            p.todo.remove(s)
        for s, grants in w1_new.items():  # the Write1 site signs every grant it issues
            self._sign(self.servers[s], grants)
        for (srv, p, flags, ots), v in zip(w2_jobs, self._verify_write2(w2_jobs)):
            self._apply_w2(srv, p, v)
        if self.async_w2:
            self._async_submit(submit_now)
            per_key: Dict[tuple, int] = {}
            for e in self.async_q:
                for k in {op.key for op in e.p.ops}:
                    per_key[(e.srv.index, k)] = per_key.get((e.srv.index, k), 0) + 1
            if per_key:
                self.stats["max_same_key_inflight"] = max(self.stats["max_same_key_inflight"], max(per_key.values()))
            self._async_complete()
        return self._advance()

    def _advance(self):
        finished = []
        w1_rounds, tallies = [], []
        for p in list(self.inflight):
            if p.todo or p.outstanding:
                continue
            self.inflight.remove(p)
            if p.dead:
                finished.append((p, Hung(f"{p.kind}: server(s) {sorted(p.dead)} threw; no reply")))
                continue
            if p.kind == "W1":
                w1_rounds.append((p, [p.replies[s] for s in self.send_order]))
            else:
                tallies.append((p, [p.replies[s] for s in self.send_order]))
        if w1_rounds:
            for (p, resps), dec in zip(w1_rounds, self._classify(w1_rounds)):
                if dec == mh.W1_RETRY:  # non-uniform timestamps: sleep 1 ms, resend (:310-318)
                    self.stats["retries"] += 1
                    self._send_write1(p)
                elif dec == mh.W1_PROCEED:
                    # WriteCertificate.putAllGrants(HashMap<serverId, MultiGrant>) (:291-299, :333-338)
                    by_id = {mg.server_id: mg for _, mg in resps}
                    order = java_hash_order([mg.server_id for _, mg in resps],
                                            [java_string_hash(mg.server_id) for _, mg in resps])
                    p.cert = Cert([(sid, by_id[sid]) for sid in order])
                    wc = b"".join(W.encode_map_entry(1, sid.encode(), mg.encode()) for sid, mg in p.cert.mgs)
                    p.msg = W._ld(1, wc) + W._ld(2, encode_txn(p.ops))
                    p.kind = "W2"
                    p.todo = list(self.send_order)
                    p.replies = {}
                    self.inflight.append(p)
                elif dec == mh.W1_THROW_REFUSED:
                    finished.append((p, RequestRefused("Write1 refused")))
                else:
                    finished.append((p, RequestFailed(f"Write1 decision {int(dec)}")))
        if tallies:
            acc, chosen = self._tally(tallies)
            for (p, resps), a, ch in zip(tallies, acc, chosen):
                if not a:
                    finished.append((p, InconsistentWrite() if p.kind == "W2" else InconsistentRead()))
                    continue
                res = [resps[int(ch[i])][i] for i in range(len(p.ops))]
                if any(r.status == ST_WRONG_SHARD for r in res):  # validateThatAllResponsesAreOk (:91-100)
                    finished.append((p, ClientError("wrong shard in merged result")))
                else:
                    finished.append((p, res))
                if p.kind == "R":
                    self.stats["reads"] += 1
        return finished

    def run(self, p: Pending, max_steps: int = 10000):
        """Drive the cluster until request p finishes (other requests advance too)."""
        for _ in range(max_steps):
            for q, out in self.step():
                if q is p:
                    if isinstance(out, Exception):
                        raise out
                    return out
        raise Hung("request did not finish")

    # the reference client's blocking calls (one client, nothing else in flight)
    def execute_write(self, client: int, ops: List[Op]) -> List[OpResult]:
        return self.run(self.start_write(client, ops))

    def execute_read(self, client: int, ops: List[Op]) -> List[OpResult]:
        return self.run(self.start_read(client, ops))


def _state(servers):
    return {(s.index, k): (sv.value, sv.available, id(sv.current_c) if sv.current_c is not None else None, sv.epoch,
                           tuple(sorted(sv.given)))
            for s in servers for k, sv in s.store.items()}


def replay_serial(c: Cluster) -> int:
    """Replay cluster c's logged server events (Write1 deliveries, Write2 applies,
    reads), in the order they changed state, on fresh servers with every Write2
    verified serially by the CPU oracle against the replayed state -- the
    reference's order of events, each Write2 validated and applied under its
    keys' write locks (InMemoryDataStore.java:641-666, StoreValueObjectContainer.java:229-251).
    Asserts every reply and the final per-key state (value, availability,
    currentC, epoch, given grants) equal c's.  Returns the events checked."""
    cfg = mh.ClusterConfig(c.config_path)
    servers = [Server(i, sid, url, c.replica_ids) for i, (sid, url) in enumerate(cfg.servers())]
    cfg.close()
    for n, (si, kind, p, got) in enumerate(c.log):
        srv = servers[si]
        if kind == "W1":
            k, mg, _ = srv.write1(p.ops, got[2], p.thash, "")
            want = (k, [(g.object_id, g.ts, g.txn_hash, g.status) for g in mg.grants], got[2])
        elif kind == "R":
            want = srv.read(p.ops)
        else:
            flags, ots = srv.write2_state(p.ops)
            acc, _, _, per_op = c._oracle_verdicts([(srv, p, flags, ots)])[0]
            want = srv.write2_apply(p.ops, p.cert, acc, per_op)
        assert want == got, f"event {n} ({kind} at server {si}): serial replay {want} != {got}"
    assert _state(servers) == _state(c.servers), "final per-key state differs from the serial replay"
    return len(c.log)


def write_ops(*kv) -> List[Op]:
    return [Op(WRITE, k, v) for k, v in kv]


def read_ops(*keys) -> List[Op]:
    return [Op(READ, k) for k in keys]


def delete_ops(*keys) -> List[Op]:
    return [Op(DELETE, k) for k in keys]


class ScriptedClient:
    """A client running a generator script: the script yields ("write"|"read",
    ops) and receives the results (or the exception) back — the reference's
    MochiConcurrentTestRunnable bodies as coroutines."""

    def __init__(self, cluster: Cluster, script):
        self.c = cluster
        self.id = cluster.new_client()
        self.gen = script(self)
        self.cur: Optional[Pending] = None
        self.done = False
        self.error: Optional[BaseException] = None
        self._send(None)

    def _send(self, value):
        try:
            if isinstance(value, Exception):
                kind, ops = self.gen.throw(value)
            else:
                kind, ops = self.gen.send(value)
        except StopIteration:
            self.done = True
            self.cur = None
            return
        except Exception as e:  # an assertion of the script failed
            self.done = True
            self.error = e
            self.cur = None
            return
        self.cur = self.c.start_write(self.id, ops) if kind == "write" else self.c.start_read(self.id, ops)

    def on_finished(self, p: Pending, out):
        if p is self.cur:
            self._send(out)


def run_clients(cluster: Cluster, clients: List[ScriptedClient], max_steps: int = 100000):
    for _ in range(max_steps):
        if all(c.done for c in clients):
            return
        for p, out in cluster.step():
            for c in clients:
                c.on_finished(p, out)
    raise Hung("clients did not finish")
