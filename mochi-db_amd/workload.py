"""Synthetic signed-grant workload.

Certificates look like the ones MochiDB's Write2 path receives
(InMemoryDataStore.java:641-666): R MultiGrants (one per replica, wire order
= server index), each holding one Grant per transaction op, every grant
signed by its server (SHA256withRSA).  Because CPU RSA signing is slow, a pool
of unique signed grant templates is signed once and batches are built by
seeded sampling from it; any certificate index regenerates independently
(splitmix64 of the seed and the index), so shards can be built per rank.

Fault mix per certificate (seeded): 1% one flipped signature bit, 0.5% one
replica with timestamp + 1 (validly signed), 0.5% a wrong transactionHash on
g0, 0.5% one replica missing, 0.25% a wrong hash on g1 (must still accept:
the reference checks only g0, InMemoryDataStore.java:588-591).
"""
from __future__ import annotations

import hashlib
import os
from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from mochi_hip import (OP_HAS_SVOC, OP_LOCAL, RSA_BYTES, TXN_HASH_BYTES, Batch, pem_modulus, sign_grants)

SEED = 0x4D4F434849  # "MOCHI"

# The cluster the synthetic certificates come from: the reference's own
# config/sample_config (copied to tests/golden/sample_config), read by the
# library's loader (mochi_config_load, ClusterConfiguration.java:138-187):
# R = 4 and the replica set every key maps to (tokens 0..R-1, because of
# ClusterConfiguration.java:215), plus three synthetic ids for R = 7.
SAMPLE_CONFIG = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                             "sample_config")


def _sample_replicas() -> List[str]:
    from mochi_hip import ClusterConfig

    cfg = ClusterConfig(SAMPLE_CONFIG)
    try:
        return cfg.replica_id_list()
    finally:
        cfg.close()


SERVER_IDS = _sample_replicas() + ["server-synthetic-r7-0004", "server-synthetic-r7-0005", "server-synthetic-r7-0006"]

DEFAULT_KEY_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "keys")

FAULT_NONE, FAULT_FLIP, FAULT_TS, FAULT_G0_HASH, FAULT_DROP, FAULT_G1_HASH = 0, 1, 2, 3, 4, 5
# cumulative thresholds out of 10000
_FAULT_TABLE = [(100, FAULT_FLIP), (150, FAULT_TS), (200, FAULT_G0_HASH), (250, FAULT_DROP), (275, FAULT_G1_HASH)]


# ---------------------------------------------------------------------------
# Grant encoding (producer side) — Grant.writeTo, MochiProtocol.java:7556-7574
# ---------------------------------------------------------------------------
def _varint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def encode_grant(object_id: str, timestamp: int, transaction_hash: str, configstamp: int = 0, status: int = 0) -> bytes:
    out = bytearray()
    oid = object_id.encode("utf-8")
    th = transaction_hash.encode("utf-8")
    if oid:
        out += b"\x0a" + _varint(len(oid)) + oid
    if timestamp:
        out += b"\x10" + _varint(timestamp)
    if configstamp:
        out += b"\x18" + _varint(configstamp)
    if th:
        out += b"\x22" + _varint(len(th)) + th
    if status:
        out += b"\x28" + _varint(status)
    return bytes(out)


def txn_hash_hex(p: int) -> str:
    """Stand-in for Utils.objectSHA512(txn) (Utils.java:150-153): lowercase hex SHA-512."""
    return hashlib.sha512(f"txn-{p}".encode()).hexdigest()


# ---------------------------------------------------------------------------
# splitmix64 (vectorized)
# ---------------------------------------------------------------------------
def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (np.asarray(x, dtype=np.uint64) + np.uint64(0x9E3779B97F4A7C15)).astype(np.uint64)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _h(seed: int, stream: int, idx: np.ndarray) -> np.ndarray:
    base = splitmix64(np.uint64((seed * 0x100000001B3 + stream) & 0xFFFFFFFFFFFFFFFF))
    with np.errstate(over="ignore"):
        return splitmix64(np.asarray(idx, np.uint64) ^ base)


def load_keys(n: int, key_dir: str = DEFAULT_KEY_DIR) -> List[bytes]:
    keys = []
    for i in range(n):
        with open(os.path.join(key_dir, f"server{i}.pem"), "rb") as f:
            keys.append(f.read())
    return keys


@dataclass
class Pool:
    """Signed grant templates: normal[P, k, R] and fault variants[P_f, k, R]."""

    R: int
    k: int
    P: int
    P_f: int
    blob: np.ndarray  # uint8
    off: np.ndarray  # uint64 [3, P, k, R]  (variant 0 normal, 1 ts+1, 2 evil hash; variants valid for p < P_f)
    length: np.ndarray  # uint32 [3, P, k, R]
    sig: np.ndarray  # uint8 [3, P, k, R, 256]
    expected_hash: np.ndarray  # uint8 [P, 128]
    moduli: List[bytes]
    key_pems: List[bytes]


def _template_fields(p: int, j: int, k: int, seed: int):
    oid = f"DEMO_KEY_STRESS_TEST_{(p * k + j) % 200}"
    hp = int(_h(seed, 7, np.array([p]))[0])
    ts = 1000 * ((p + j) % 64) + (hp % 1000)
    return oid, ts


def build_pool(R: int, k: int = 1, P: int = 4096, P_f: int = 256, seed: int = SEED, key_dir: str = DEFAULT_KEY_DIR,
               n_threads: Optional[int] = None, cache_dir: Optional[str] = None) -> Pool:
    if n_threads is None:
        n_threads = min(16, os.cpu_count() or 1)
    P_f = min(P_f, P)
    pems = load_keys(R, key_dir)
    cache = None
    if cache_dir:
        os.makedirs(cache_dir, exist_ok=True)
        tag = hashlib.sha256(b"".join(pems) + f"{R}/{k}/{P}/{P_f}/{seed}/v1".encode()).hexdigest()[:16]
        cache = os.path.join(cache_dir, f"pool_{tag}.npz")
        if os.path.exists(cache):
            z = np.load(cache)
            return Pool(R, k, P, P_f, z["blob"], z["off"], z["length"], z["sig"], z["expected_hash"],
                        [pem_modulus(p) for p in pems], pems)
    chunks: List[bytes] = []
    off = np.zeros((3, P, k, R), np.uint64)
    length = np.zeros((3, P, k, R), np.uint32)
    pos = 0
    expected = np.zeros((P, TXN_HASH_BYTES), np.uint8)
    for p in range(P):
        th = txn_hash_hex(p)
        expected[p] = np.frombuffer(th.encode(), np.uint8)
        evil = hashlib.sha512(f"txn-{p}-evil".encode()).hexdigest()
        for j in range(k):
            oid, ts = _template_fields(p, j, k, seed)
            variants = [encode_grant(oid, ts, th)]
            if p < P_f:
                variants += [encode_grant(oid, ts + 1, th), encode_grant(oid, ts, evil)]
            for v, g in enumerate(variants):
                # every replica signs the same grant bytes (one copy in the blob)
                off[v, p, j, :] = pos
                length[v, p, j, :] = len(g)
                chunks.append(g)
                pos += len(g)
    blob = np.frombuffer(b"".join(chunks), np.uint8).copy()
    sig = np.zeros((3, P, k, R, RSA_BYTES), np.uint8)
    nv = np.array([3 if p < P_f else 1 for p in range(P)])
    for r in range(R):
        sel = [(v, p, j) for p in range(P) for j in range(k) for v in range(nv[p])]
        vi = np.array([s[0] for s in sel]); pi = np.array([s[1] for s in sel]); ji = np.array([s[2] for s in sel])
        s = sign_grants(pems[r], blob, off[vi, pi, ji, r], length[vi, pi, ji, r], n_threads)
        sig[vi, pi, ji, r] = s
    pool = Pool(R, k, P, P_f, blob, off, length, sig, expected, [pem_modulus(p) for p in pems], pems)
    if cache:
        np.savez(cache, blob=blob, off=off, length=length, sig=sig, expected_hash=expected)
    return pool


@dataclass
class Synth:
    batch: Batch
    template: np.ndarray  # [C] pool template per certificate
    fault: np.ndarray  # [C] FAULT_*
    fault_replica: np.ndarray  # [C]
    expected_flags: np.ndarray  # [N] uint8 ground-truth MOCHI_GRANT_* bits


def make_batch(pool: Pool, n_certs: int, first_cert: int = 0, seed: int = SEED, faults: bool = True,
               local_flags: int = OP_LOCAL | OP_HAS_SVOC) -> Synth:
    """Certificates [first_cert, first_cert + n_certs) of the seeded stream."""
    R, k, P, P_f = pool.R, pool.k, pool.P, pool.P_f
    cidx = np.arange(first_cert, first_cert + n_certs, dtype=np.uint64)
    p = (_h(seed, 1, cidx) % np.uint64(P)).astype(np.int64)
    fault = np.zeros(n_certs, np.int64)
    if faults:
        u = (_h(seed, 2, cidx) % np.uint64(10000)).astype(np.int64)
        lo = 0
        for hi, f in _FAULT_TABLE:
            fault[(u >= lo) & (u < hi)] = f
            lo = hi
    rf = (_h(seed, 3, cidx) % np.uint64(R)).astype(np.int64)
    rf[fault == FAULT_G0_HASH] = 0
    rf[fault == FAULT_G1_HASH] = 1 % R
    p[fault != FAULT_NONE] %= P_f
    # grid [C, R, k]
    variant = np.zeros((n_certs, R, k), np.int64)
    rr = np.arange(R)[None, :, None]
    shape = (n_certs, R, k)
    is_rf = np.broadcast_to(rr == rf[:, None, None], shape)
    f3 = np.broadcast_to(fault[:, None, None], shape)
    variant[(f3 == FAULT_TS) & is_rf] = 1
    variant[((f3 == FAULT_G0_HASH) | (f3 == FAULT_G1_HASH)) & is_rf] = 2
    keep = np.ones(shape, bool)
    keep[(f3 == FAULT_DROP) & is_rf] = False
    P3 = np.broadcast_to(p[:, None, None], keep.shape)
    R3 = np.broadcast_to(rr, keep.shape)
    J3 = np.broadcast_to(np.arange(k)[None, None, :], keep.shape)
    sel = keep.reshape(-1)
    vv, pp, r_, jj = variant.reshape(-1)[sel], P3.reshape(-1)[sel], R3.reshape(-1)[sel], J3.reshape(-1)[sel]
    goff = pool.off[vv, pp, jj, r_]
    glen = pool.length[vv, pp, jj, r_]
    sig = pool.sig[vv, pp, jj, r_].copy()
    n = goff.shape[0]
    flags = np.full(n, 0x03, np.uint8)  # PARSED | SIG_OK
    per_cert = keep.reshape(n_certs, -1).sum(1)
    cert_grant_off = np.zeros(n_certs + 1, np.uint32)
    np.cumsum(per_cert, out=cert_grant_off[1:])
    # bit flip in replica rf's op-0 grant
    flip_c = np.nonzero(fault == FAULT_FLIP)[0]
    if flip_c.size:
        # position of (c, rf, j=0) within the flattened kept grants (no drops in flip certs)
        gi = cert_grant_off[flip_c].astype(np.int64) + rf[flip_c] * k
        bit = (_h(seed, 4, cidx[flip_c]) % np.uint64(2048)).astype(np.int64)
        sig[gi, bit // 8] ^= (1 << (bit % 8)).astype(np.uint8)
        flags[gi] = 0x02
    ops = np.tile(np.arange(k, dtype=np.uint8), n_certs)
    batch = Batch(
        grant_bytes=pool.blob,
        grant_off=goff.astype(np.uint64),
        grant_len=glen.astype(np.uint32),
        sig=sig,
        signer=r_.astype(np.uint16),
        grant_key=jj.astype(np.uint8),
        cert_grant_off=cert_grant_off,
        cert_op_off=(np.arange(n_certs + 1, dtype=np.uint64) * k).astype(np.uint32),
        op_key=ops,
        op_flags=np.full(n_certs * k, local_flags, np.uint8),
        expected_hash=pool.expected_hash[p],
    )
    return Synth(batch, p, fault, rf, flags)


def n_certs_for_grants(n_grants: int, R: int, k: int = 1) -> int:
    return max(1, n_grants // (R * k))


# ---------------------------------------------------------------------------
# Write2ToServer wire encoding (MochiProtocol.proto:107-147, proto3, field
# order and map-entry layout as protobuf-java writes them: every map entry
# carries its key and value, MapEntryLite.writeTo) with the grantSignatures
# map INTEGRATION.md adds to MultiGrant (field 5).
# ---------------------------------------------------------------------------
def _ld(field: int, payload: bytes) -> bytes:
    return _varint(field << 3 | 2) + _varint(len(payload)) + payload


def encode_map_entry(field: int, key: bytes, value: bytes) -> bytes:
    return _ld(field, _ld(1, key) + _ld(2, value))


def encode_multigrant(grants, server_id: str, client_id: str = "", mg_hash: str = "", sigs=None) -> bytes:
    """grants / sigs: lists of (objectId, bytes) in map insertion order."""
    out = bytearray()
    for oid, gb in grants:
        out += encode_map_entry(1, oid.encode(), gb)
    if client_id:
        out += _ld(2, client_id.encode())
    if mg_hash:
        out += _ld(3, mg_hash.encode())
    if server_id:
        out += _ld(4, server_id.encode())
    for oid, sig in sigs or []:
        out += encode_map_entry(5, oid.encode(), sig)
    return bytes(out)


def encode_operation(action: int, operand1: str, operand2: str = "") -> bytes:
    out = bytearray()
    if action:
        out += b"\x08" + _varint(action)
    if operand1:
        out += _ld(2, operand1.encode())
    if operand2:
        out += _ld(3, operand2.encode())
    return bytes(out)


def encode_write2(multigrants, operations) -> bytes:
    """multigrants: [(certificate map key = serverId, MultiGrant bytes)], operations: [Operation bytes]."""
    wc = b"".join(encode_map_entry(1, sid.encode(), mg) for sid, mg in multigrants)
    txn = b"".join(_ld(1, op) for op in operations)
    return (_ld(1, wc) if wc else b"") + (_ld(2, txn) if txn else b"")


def grant_object_id(gb: bytes) -> str:
    """objectId of a canonical Grant (field 1 first)."""
    if not gb or gb[0] != 0x0A:
        return ""
    n, i, shift = 0, 1, 0
    while True:
        c = gb[i]
        n |= (c & 0x7F) << shift
        i += 1
        if not c & 0x80:
            break
        shift += 7
    return gb[i:i + n].decode()


@dataclass
class WireBatch:
    """Write2ToServer messages + the host inputs of mochi_write2_batch."""

    wire: np.ndarray  # uint8 blob
    msg_off: np.ndarray  # uint64 [M]
    msg_len: np.ndarray  # uint32 [M]
    op_flags_off: Optional[np.ndarray]  # uint32 [M+1] or None
    op_flags: np.ndarray  # uint8
    expected_hash: np.ndarray  # uint8 [M, 128]
    op_object_ts: Optional[np.ndarray] = None  # int64, aligned with op_flags (stored currentC timestamps)

    @property
    def n_msgs(self) -> int:
        return int(self.msg_off.shape[0])


def encode_wire_batch(s: Synth, server_ids=None, client_id: str = "", pad: int = 0, mg_hash: bool = False) -> WireBatch:
    """The Write2ToServer messages a MochiDB server would receive for the
    synthetic certificates of `s`: one MultiGrant per replica in server order
    (certificate map key = MultiGrant.serverId), grants keyed by objectId with
    their signatures in grantSignatures, a WRITE operation per op key.  As the
    reference's producer builds them, MultiGrant.clientId is empty (it copies
    Write1ToServer.clientId, which MochiDBClient never sets:
    InMemoryDataStore.java:285, MochiDBClient.java:252-263) and MultiGrant.hash
    is unset; client_id / mg_hash=True add them (decoder coverage)."""
    b = s.batch
    ids = server_ids or SERVER_IDS
    C = b.n_certs
    msgs, ops_per = [], []
    for c in range(C):
        g0, g1 = int(b.cert_grant_off[c]), int(b.cert_grant_off[c + 1])
        o0, o1 = int(b.cert_op_off[c]), int(b.cert_op_off[c + 1])
        oids = {}
        mgs, cur, cur_r = [], [], None
        for g in range(g0, g1):
            gb = b.grant_bytes[int(b.grant_off[g]):int(b.grant_off[g]) + int(b.grant_len[g])].tobytes()
            oid = grant_object_id(gb)
            oids[int(b.grant_key[g])] = oid
            r = int(b.signer[g])
            if r != cur_r and cur:
                mgs.append((cur_r, cur))
                cur = []
            cur_r = r
            cur.append((oid, gb, b.sig[g].tobytes()))
        if cur:
            mgs.append((cur_r, cur))
        th = b.expected_hash[c].tobytes().decode()
        enc = []
        for r, items in mgs:
            sid = ids[r] if r < len(ids) else f"server-unknown-{r}"
            mg = encode_multigrant([(o, gb) for o, gb, _ in items], sid, client_id, th if mg_hash else "",
                                   [(o, sg) for o, _, sg in items])
            enc.append((sid, mg))
        ops = [encode_operation(2, oids.get(int(b.op_key[o]), f"key-{int(b.op_key[o])}"), f"value-{c}-{o - o0}")
               for o in range(o0, o1)]
        msgs.append(encode_write2(enc, ops))
        ops_per.append(o1 - o0)
    off = np.zeros(C, np.uint64)
    pos = 0
    parts = []
    for i, m in enumerate(msgs):
        pos += pad
        parts.append(b"\xee" * pad)
        off[i] = pos
        parts.append(m)
        pos += len(m)
    wire = np.frombuffer(b"".join(parts) or b"\x00", np.uint8).copy()
    ofo = np.zeros(C + 1, np.uint32)
    np.cumsum(ops_per, out=ofo[1:])
    return WireBatch(wire=wire, msg_off=off, msg_len=np.array([len(m) for m in msgs], np.uint32),
                     op_flags_off=ofo, op_flags=b.op_flags.copy(), expected_hash=b.expected_hash.copy())


def server_id_table(n: int, server_ids=None):
    ids = (server_ids or SERVER_IDS)[:n]
    blob = "".join(ids).encode()
    off = np.zeros(n + 1, np.uint32)
    np.cumsum([len(x.encode()) for x in ids], out=off[1:])
    return np.frombuffer(blob, np.uint8).copy(), off


def _txn_hashes(cidx: np.ndarray, suffix: str = "") -> np.ndarray:
    """[C, 128] lowercase-hex SHA-512 of "txn-{c}{suffix}" (the objectSHA512 stand-in)."""
    h = b"".join([hashlib.sha512(f"txn-{int(c)}{suffix}".encode()).hexdigest().encode() for c in cidx])
    return np.frombuffer(h, np.uint8).reshape(-1, TXN_HASH_BYTES) if len(cidx) else np.zeros((0, 128), np.uint8)


_OIDS = [f"DEMO_KEY_STRESS_TEST_{i}".encode() for i in range(200)]


def encode_grants_vec(oid_idx: np.ndarray, ts: np.ndarray, hashes: np.ndarray) -> tuple:
    """Vectorized Grant.toByteArray() (MochiProtocol.java:7556-7574) of n grants with
    objectId DEMO_KEY_STRESS_TEST_{oid_idx}, timestamp ts (0 <= ts < 2^21; 0 is
    omitted, proto3 default) and transactionHash = hashes[i] (128 ASCII bytes).
    Returns (blob, offsets, lengths): the grants concatenated in input order."""
    n = int(oid_idx.shape[0])
    ts = np.asarray(ts, np.int64)
    assert n == 0 or (ts.min() >= 0 and ts.max() < (1 << 21))
    lo = np.array([len(x) for x in _OIDS], np.int64)[oid_idx]
    lv = np.where(ts == 0, 0, np.where(ts < 128, 1, np.where(ts < 16384, 2, 3)))
    ln = 2 + lo + np.where(lv > 0, 1 + lv, 0) + 3 + TXN_HASH_BYTES
    W_ = int(ln.max()) if n else 0
    rows = np.zeros((n, W_), np.uint8)
    rows[:, 0] = 0x0A
    rows[:, 1] = lo
    otab = np.zeros((200, 24), np.uint8)
    for i, x in enumerate(_OIDS):
        otab[i, :len(x)] = np.frombuffer(x, np.uint8)
    for L in np.unique(lo):
        for v in np.unique(lv):
            sel = np.nonzero((lo == L) & (lv == v))[0]
            if not sel.size:
                continue
            L, v = int(L), int(v)
            rows[sel, 2:2 + L] = otab[oid_idx[sel], :L]
            p = 2 + L
            if v:
                t = ts[sel]
                rows[sel, p] = 0x10
                for b in range(v):
                    byte = (t >> (7 * b)) & 0x7F
                    rows[sel, p + 1 + b] = (byte | (0x80 if b + 1 < v else 0)).astype(np.uint8)
                p += 1 + v
            rows[sel, p] = 0x22
            rows[sel, p + 1] = 0x80
            rows[sel, p + 2] = 0x01
            rows[sel, p + 3:p + 3 + TXN_HASH_BYTES] = hashes[sel]
    blob = rows[np.arange(W_)[None, :] < ln[:, None]]
    off = np.zeros(n, np.uint64)
    if n:
        np.cumsum(ln[:-1], out=off[1:])
    return np.ascontiguousarray(blob), off, ln.astype(np.uint32)


# ---------------------------------------------------------------------------
# SURVEY.md §8d's per-certificate stream with UNIQUE grant bytes, signed on the
# device (k_rsa_sign, bit-identical to OpenSSL): certificate c has objectId
# DEMO_KEY_STRESS_TEST_{(c*k + j) mod 200} per op j, timestamp
# 1000*(c mod 64) + (h(c) mod 1000) and transactionHash = hex SHA-512 of
# "txn-{c}".  Every replica signs the same grant bytes (one copy in the blob,
# certificate order); fault variants get their own copy.  This is the bench
# workload: unlike the template pool, its grant bytes (~150 MB per 1M grants)
# do not sit in cache.
# ---------------------------------------------------------------------------
def make_batch_unique(R: int, n_certs: int, k: int = 1, first_cert: int = 0, seed: int = SEED, faults: bool = True,
                      device: int = 0, key_dir: str = DEFAULT_KEY_DIR,
                      local_flags: int = OP_LOCAL | OP_HAS_SVOC) -> Synth:
    import mochi_hip as mh

    pems = load_keys(R, key_dir)
    C = n_certs
    cidx = np.arange(first_cert, first_cert + C, dtype=np.uint64)
    fault = np.zeros(C, np.int64)
    if faults:
        u = (_h(seed, 2, cidx) % np.uint64(10000)).astype(np.int64)
        lo = 0
        for hi, f in _FAULT_TABLE:
            fault[(u >= lo) & (u < hi)] = f
            lo = hi
    rf = (_h(seed, 3, cidx) % np.uint64(R)).astype(np.int64)
    rf[fault == FAULT_G0_HASH] = 0
    rf[fault == FAULT_G1_HASH] = 1 % R
    hts = (_h(seed, 7, cidx) % np.uint64(1000)).astype(np.int64)
    ts_c = 1000 * (cidx % np.uint64(64)).astype(np.int64) + hts
    expected = _txn_hashes(cidx)
    # grant bytes, certificate order: per op j the normal grant, then the faulty replica's variant
    has_var = (fault == FAULT_TS) | (fault == FAULT_G0_HASH) | (fault == FAULT_G1_HASH)
    nv = np.where(has_var, 2, 1)  # grant copies per (cert, op)
    per_c = nv * k
    start = np.zeros(C + 1, np.int64)
    np.cumsum(per_c, out=start[1:])
    tot = int(start[-1])
    rep_c = np.repeat(np.arange(C), per_c)  # owning cert of each copy
    within = np.arange(tot) - start[rep_c]
    j_of = within // nv[rep_c]
    var_of = within % nv[rep_c]  # 0 normal, 1 fault variant
    oid_idx = ((cidx[rep_c].astype(np.int64) * k + j_of) % 200).astype(np.int64)
    tsv = ts_c[rep_c] + np.where((var_of == 1) & (fault[rep_c] == FAULT_TS), 1, 0)
    hashes = expected[rep_c]
    evil_c = np.nonzero((fault == FAULT_G0_HASH) | (fault == FAULT_G1_HASH))[0]
    if evil_c.size:
        evil = _txn_hashes(cidx[evil_c], "-evil")
        emap = np.full(C, -1, np.int64)
        emap[evil_c] = np.arange(evil_c.size)
        sel = np.nonzero((var_of == 1) & (emap[rep_c] >= 0))[0]
        hashes[sel] = evil[emap[rep_c[sel]]]
    blob, coff, clen = encode_grants_vec(oid_idx, tsv, hashes)
    copy_at = lambda c, j, v: start[c] + j * nv[c] + v  # index of a grant copy
    # grid [C, R, k] -> kept grants in (certificate, replica, op) order
    shape = (C, R, k)
    rr = np.arange(R)[None, :, None]
    is_rf = np.broadcast_to(rr == rf[:, None, None], shape)
    f3 = np.broadcast_to(fault[:, None, None], shape)
    use_var = (has_var[:, None, None] & is_rf)
    keep = np.ones(shape, bool)
    keep[(f3 == FAULT_DROP) & is_rf] = False
    C3 = np.broadcast_to(np.arange(C)[:, None, None], shape)
    J3 = np.broadcast_to(np.arange(k)[None, None, :], shape)
    sel = keep.reshape(-1)
    ci, ji, vi = C3.reshape(-1)[sel], J3.reshape(-1)[sel], use_var.reshape(-1)[sel].astype(np.int64)
    gi = copy_at(ci, ji, vi)
    goff = coff[gi]
    glen = clen[gi]
    signer = np.broadcast_to(rr, shape).reshape(-1)[sel].astype(np.uint16)
    gkey = ji.astype(np.uint8)
    n = goff.shape[0]
    sig = np.zeros((n, RSA_BYTES), np.uint8)
    for r in range(R):
        idx = np.nonzero(signer == r)[0]
        s = mh.DeviceSigner(pems[r], device)
        sig[idx] = s.sign(blob, goff[idx], glen[idx])
        s.close()
    per_cert = keep.reshape(C, -1).sum(1)
    cert_grant_off = np.zeros(C + 1, np.uint32)
    np.cumsum(per_cert, out=cert_grant_off[1:])
    flags = np.full(n, 0x03, np.uint8)
    flip_c = np.nonzero(fault == FAULT_FLIP)[0]
    if flip_c.size:
        gf = cert_grant_off[flip_c].astype(np.int64) + rf[flip_c] * k
        bit = (_h(seed, 4, cidx[flip_c]) % np.uint64(2048)).astype(np.int64)
        sig[gf, bit // 8] ^= (1 << (bit % 8)).astype(np.uint8)
        flags[gf] = 0x02
    batch = Batch(grant_bytes=blob, grant_off=goff, grant_len=glen, sig=sig, signer=signer, grant_key=gkey,
                  cert_grant_off=cert_grant_off,
                  cert_op_off=(np.arange(C + 1, dtype=np.uint64) * k).astype(np.uint32),
                  op_key=np.tile(np.arange(k, dtype=np.uint8), C), op_flags=np.full(C * k, local_flags, np.uint8),
                  expected_hash=expected)
    return Synth(batch, np.zeros(C, np.int64), fault, rf, flags)


def separate_copies(s: Synth, seed: int = SEED, chunk: int = 1 << 18) -> Synth:
    """The same certificates with every grant its OWN copy of its bytes, each
    after 0..15 bytes of filler (mixed alignments), in (certificate, MultiGrant)
    order -- the layout of grant slices of received Write2ToServer messages: in
    the reference every replica builds its own Grant (InMemoryDataStore.java:131-140)
    and the client ships all R MultiGrants (MochiDBClient.java:333-338).  Same
    bytes, signatures and ground truth as `s`; only grant_off and the blob differ,
    so grant prep must find equal grants by comparing bytes (no equal offsets)."""
    b = s.batch
    n = b.n_grants
    ln = np.ascontiguousarray(b.grant_len[:n], np.int64)
    pad = (_h(seed, 11, np.arange(n, dtype=np.uint64)) % np.uint64(16)).astype(np.int64)
    start = np.zeros(n + 1, np.int64)
    np.cumsum(pad + ln, out=start[1:])
    new_off = start[:-1] + pad
    out = np.full(int(start[-1]) or 1, 0xEE, np.uint8)
    src_all = np.ascontiguousarray(b.grant_off[:n], np.int64)
    W_ = int(ln.max()) if n else 0
    col = np.arange(W_, dtype=np.int64)[None, :]
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        m = col < ln[lo:hi, None]
        out[(new_off[lo:hi, None] + col)[m]] = b.grant_bytes[(src_all[lo:hi, None] + col)[m]]
    nb = Batch(grant_bytes=out, grant_off=new_off.astype(np.uint64), grant_len=b.grant_len[:n].copy(), sig=b.sig,
               signer=b.signer, grant_key=b.grant_key, cert_grant_off=b.cert_grant_off, cert_op_off=b.cert_op_off,
               op_key=b.op_key, op_flags=b.op_flags, expected_hash=b.expected_hash)
    return Synth(nb, s.template, s.fault, s.fault_replica, s.expected_flags)


def save_batch(path: str, s: Synth) -> None:
    b = s.batch
    np.savez(path, **{f: getattr(b, f) for f in ("grant_bytes", "grant_off", "grant_len", "sig", "signer",
                                                  "grant_key", "cert_grant_off", "cert_op_off", "op_key",
                                                  "op_flags", "expected_hash")},
             fault=s.fault, fault_replica=s.fault_replica, expected_flags=s.expected_flags)


def load_batch(path: str) -> Synth:
    z = np.load(path)
    b = Batch(**{f: z[f] for f in ("grant_bytes", "grant_off", "grant_len", "sig", "signer", "grant_key",
                                   "cert_grant_off", "cert_op_off", "op_key", "op_flags", "expected_hash")})
    return Synth(b, np.zeros(b.n_certs, np.int64), z["fault"], z["fault_replica"], z["expected_flags"])


def head_certs(s: Synth, n: int) -> Synth:
    """The first n certificates of a synthetic batch (grant blob shared)."""
    b = s.batch
    n = max(0, min(n, b.n_certs))
    g = int(b.cert_grant_off[n])
    o = int(b.cert_op_off[n])
    nb = Batch(grant_bytes=b.grant_bytes, grant_off=b.grant_off[:g], grant_len=b.grant_len[:g], sig=b.sig[:g],
               signer=b.signer[:g], grant_key=b.grant_key[:g], cert_grant_off=b.cert_grant_off[:n + 1],
               cert_op_off=b.cert_op_off[:n + 1], op_key=b.op_key[:o], op_flags=b.op_flags[:o],
               expected_hash=b.expected_hash[:n])
    return Synth(nb, s.template[:n], s.fault[:n], s.fault_replica[:n], s.expected_flags[:g])
