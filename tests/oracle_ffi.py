"""ctypes binding for the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg load this.  It is the checker, never the thing measured as
the product.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "liboracle.so")

_lib = None


def build_oracle() -> None:
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_LIB):
            build_oracle()
        L = ctypes.CDLL(ORACLE_LIB)
        vp, u32, i64, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int64, ctypes.c_size_t
        L.oracle_grant_encode.restype = ctypes.c_long
        L.oracle_grant_encode.argtypes = [ctypes.c_char_p, sz, i64, i64, ctypes.c_char_p, sz, ctypes.c_int32, vp, sz]
        L.oracle_grant_parse.argtypes = [vp, sz, vp]
        L.oracle_sha256.argtypes = [vp, sz, vp]
        L.oracle_rsa_verify.argtypes = [vp, vp, sz, vp]
        L.oracle_server_majority.restype = u32
        L.oracle_server_majority.argtypes = [u32]
        L.oracle_verify_batch.argtypes = [vp, u32, vp, vp, vp, ctypes.c_int]
        L.oracle_verify_grants.argtypes = [vp, u32, vp, u32, u32, vp, vp, ctypes.c_int]
        L.oracle_tally.argtypes = [vp, vp, vp, vp, vp]
        L.oracle_parse_grants.argtypes = [vp, u32, u32, vp, vp]
        L.oracle_tally_responses.argtypes = [u32, vp, vp, vp, vp, vp, vp, u32, vp, vp, vp]
        L.oracle_write1_uniform.argtypes = [u32, vp, vp]
        L.oracle_write1_classify.argtypes = [u32, vp, vp, vp, vp, vp, vp, vp, vp]
        L.oracle_w2_decode.argtypes = [vp, vp, vp, u32, vp]
        L.oracle_w2_free.argtypes = [vp]
        L.oracle_w2_decode_full.argtypes = [vp, vp, vp, u32, vp]
        L.oracle_verify_write2.argtypes = [vp, u32, vp, vp, vp, vp, vp, vp, ctypes.c_int]
        L.oracle_rsa_sign.argtypes = [ctypes.c_char_p, vp, sz, vp]
        L.oracle_pem_modulus.argtypes = [ctypes.c_char_p, vp]
        _lib = L
    return _lib


class GrantView(ctypes.Structure):
    _fields_ = [
        ("timestamp", ctypes.c_int64),
        ("configstamp", ctypes.c_int64),
        ("status", ctypes.c_int32),
        ("object_id_off", ctypes.c_uint32),
        ("object_id_len", ctypes.c_uint32),
        ("txn_hash_off", ctypes.c_uint32),
        ("txn_hash_len", ctypes.c_uint32),
    ]


def grant_encode(object_id: bytes, timestamp: int, txn_hash: bytes, configstamp: int = 0, status: int = 0) -> bytes:
    buf = ctypes.create_string_buffer(len(object_id) + len(txn_hash) + 64)
    n = lib().oracle_grant_encode(object_id, len(object_id), timestamp, configstamp, txn_hash, len(txn_hash), status,
                                  buf, len(buf))
    assert n >= 0
    return buf.raw[:n]


def grant_parse(data: bytes):
    v = GrantView()
    b = ctypes.create_string_buffer(data, len(data)) if data else ctypes.create_string_buffer(1)
    ok = lib().oracle_grant_parse(b, len(data), ctypes.byref(v))
    if not ok:
        return None
    return {
        "timestamp": v.timestamp,
        "configstamp": v.configstamp,
        "status": v.status,
        "object_id": data[v.object_id_off:v.object_id_off + v.object_id_len],
        "transaction_hash": data[v.txn_hash_off:v.txn_hash_off + v.txn_hash_len],
    }


def sha256(data: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    b = ctypes.create_string_buffer(data, len(data)) if data else ctypes.create_string_buffer(1)
    lib().oracle_sha256(b, len(data), out)
    return out.raw


def rsa_verify(n_be: bytes, msg: bytes, sig: bytes) -> bool:
    m = ctypes.create_string_buffer(msg, len(msg)) if msg else ctypes.create_string_buffer(1)
    return bool(lib().oracle_rsa_verify(n_be, m, len(msg), sig))


def rsa_sign(pem: bytes, msg: bytes) -> bytes:
    out = ctypes.create_string_buffer(256)
    m = ctypes.create_string_buffer(msg, len(msg)) if msg else ctypes.create_string_buffer(1)
    assert lib().oracle_rsa_sign(pem, m, len(msg), out) == 1
    return out.raw


def pem_modulus(pem: bytes) -> bytes:
    out = ctypes.create_string_buffer(256)
    assert lib().oracle_pem_modulus(pem, out) == 1
    return out.raw


def server_majority(R: int) -> int:
    return int(lib().oracle_server_majority(R))


def _moduli_buf(moduli):
    m = np.frombuffer(b"".join(moduli), np.uint8).copy()
    return m


def verify_batch(moduli, batch, replication_factor: int, strict_gt: bool = True, n_threads: int = 8,
                 quorum_mode: int = 0):
    """Oracle verdicts for a mochi_hip.Batch (host memory)."""
    import mochi_hip as mh

    b = batch.normalized()
    out = mh.Verdicts.alloc(b.n_grants, b.n_certs, b.n_ops)
    bc, vc = b.to_c(), out.to_c()
    p = mh.params(replication_factor, strict_gt, quorum_mode)
    m = _moduli_buf(moduli)
    rc = lib().oracle_verify_batch(m.ctypes.data, len(moduli), ctypes.byref(bc), ctypes.byref(p), ctypes.byref(vc),
                                   n_threads)
    assert rc == 0
    return out


def verify_grants(moduli, batch, begin: int, end: int, n_threads: int = 8):
    """Signature leg only (what the CPU baseline times): flags, ts for [begin, end)."""
    b = batch.normalized()
    bc = b.to_c()
    flags = np.zeros(b.n_grants, np.uint8)
    ts = np.zeros(b.n_grants, np.int64)
    m = _moduli_buf(moduli)
    rc = lib().oracle_verify_grants(m.ctypes.data, len(moduli), ctypes.byref(bc), begin, end, flags.ctypes.data,
                                    ts.ctypes.data, n_threads)
    assert rc == 0
    return flags, ts


def parse_grants(batch):
    """The oracle's own Grant parse of every grant: (PARSED flags, timestamps)."""
    b = batch.normalized()
    bc = b.to_c()
    flags = np.zeros(b.n_grants, np.uint8)
    ts = np.zeros(b.n_grants, np.int64)
    assert lib().oracle_parse_grants(ctypes.byref(bc), 0, b.n_grants, flags.ctypes.data, ts.ctypes.data) == 0
    return flags, ts


def tally(batch, grant_flags: np.ndarray, grant_ts: np.ndarray, replication_factor: int, strict_gt: bool = True,
          quorum_mode: int = 0):
    import mochi_hip as mh

    b = batch.normalized()
    out = mh.Verdicts.alloc(b.n_grants, b.n_certs, b.n_ops)
    bc, vc = b.to_c(), out.to_c()
    p = mh.params(replication_factor, strict_gt, quorum_mode)
    f = np.ascontiguousarray(grant_flags, np.uint8)
    t = np.ascontiguousarray(grant_ts, np.int64)
    rc = lib().oracle_tally(ctypes.byref(bc), ctypes.byref(p), f.ctypes.data, t.ctypes.data, ctypes.byref(vc))
    assert rc == 0
    return out


def write1_uniform(grant_key, ts) -> bool:
    k = np.ascontiguousarray(grant_key, np.uint8)
    t = np.ascontiguousarray(ts, np.int64)
    return bool(lib().oracle_write1_uniform(k.shape[0], k.ctypes.data, t.ctypes.data))


def tally_responses(responses, n_ops, replication_factor: int):
    nreq = len(responses)
    resp_off = np.zeros(nreq + 1, np.uint32)
    resp_n_ops, status_off, status = [], [], []
    chosen_off = np.zeros(max(nreq, 1), np.uint64)
    pos = cpos = 0
    for r, resps in enumerate(responses):
        resp_off[r + 1] = resp_off[r] + len(resps)
        chosen_off[r] = cpos
        cpos += n_ops[r]
        for st in resps:
            resp_n_ops.append(len(st))
            status_off.append(pos)
            status.extend(st)
            pos += len(st)
    n_ops_a = np.asarray(n_ops if n_ops else [0], np.uint32)
    rn = np.asarray(resp_n_ops if resp_n_ops else [0], np.uint32)
    so = np.asarray(status_off if status_off else [0], np.uint64)
    st = np.asarray(status if status else [0], np.uint8)
    chosen = np.full(max(cpos, 1), -1, np.int32)
    reason = np.zeros(max(nreq, 1), np.uint8)
    bits = np.zeros(max((nreq + 31) // 32, 1), np.uint32)
    rc = lib().oracle_tally_responses(nreq, resp_off.ctypes.data, n_ops_a.ctypes.data, rn.ctypes.data, so.ctypes.data,
                                      st.ctypes.data, chosen_off.ctypes.data, replication_factor, chosen.ctypes.data,
                                      reason.ctypes.data, bits.ctypes.data)
    assert rc == 0
    acc = np.unpackbits(bits.view(np.uint8), bitorder="little")[:nreq].astype(bool)
    ch = [chosen[int(chosen_off[r]):int(chosen_off[r]) + n_ops[r]].copy() for r in range(nreq)]
    return acc, reason[:nreq].copy(), ch


def write1_classify(requests):
    """Oracle restatement of the client Write1 round (same packing as mochi_hip.pack_write1)."""
    import mochi_hip as mh

    a = mh.pack_write1(requests)
    out = np.zeros(max(len(requests), 1), np.uint8)
    rc = lib().oracle_write1_classify(len(requests), *[x.ctypes.data for x in a], out.ctypes.data)
    assert rc == 0
    return out[:len(requests)].copy()


class W2Decoded_C(ctypes.Structure):
    pass


def _w2_c(wb):
    import mochi_hip as mh

    return mh.write2_batch_c(wb)


def _dec_struct():
    import mochi_hip as mh

    class Dec(ctypes.Structure):
        _fields_ = [("batch", mh.Batch_C), ("msg_status", ctypes.POINTER(ctypes.c_uint8)),
                    ("own_blob", ctypes.c_void_p)]

    return Dec


def _dec_arrays(d, wire=None):
    b = d.batch
    N, C, O = b.n_grants, b.n_certs, b.n_ops

    def arr(ptr, n, dt, shape=None):
        if n == 0:
            return np.zeros(shape or (0,), dt)
        a = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(np.ctypeslib.as_ctypes_type(dt))), shape=(n,))
        a = a.copy()
        return a.reshape(shape) if shape else a

    out = dict(
        grant_off=arr(b.grant_off, N, np.uint64), grant_len=arr(b.grant_len, N, np.uint32),
        sig=arr(b.sig, N * 256, np.uint8, (N, 256)), signer=arr(b.signer, N, np.uint16),
        grant_key=arr(b.grant_key, N, np.uint8), cert_grant_off=arr(b.cert_grant_off, C + 1, np.uint32),
        cert_op_off=arr(b.cert_op_off, C + 1, np.uint32), op_key=arr(b.op_key, O, np.uint8),
        op_flags=arr(b.op_flags, O, np.uint8), msg_status=arr(d.msg_status, C, np.uint8),
        cert_mg_off=arr(b.cert_mg_off, C + 1, np.uint32), mg_grant_off=arr(b.mg_grant_off, b.n_mgs + 1, np.uint32),
        op_key_off=arr(b.op_key_off, O, np.uint64), op_key_len=arr(b.op_key_len, O, np.uint32),
        op_object_ts=arr(b.op_object_ts, O, np.int64))
    if d.own_blob:
        out["blob"] = arr(d.own_blob, int(b.grant_bytes_len), np.uint8)
    return out


def w2_decode(wb, ids, id_off):
    """Oracle decode of a workload.WireBatch (the device fast path's semantics) -> dict
    of numpy arrays (grant_off, grant_len, sig, signer, grant_key, cert_grant_off,
    cert_op_off, op_key, op_flags, msg_status, MultiGrant CSR, op key slices)."""
    wc, keep = _w2_c(wb)
    d = _dec_struct()()
    rc = lib().oracle_w2_decode(ctypes.addressof(wc), ids.ctypes.data, id_off.ctypes.data, int(id_off.shape[0]) - 1,
                                ctypes.addressof(d))
    assert rc == 0
    out = _dec_arrays(d)
    lib().oracle_w2_free(ctypes.addressof(d))
    return out


def w2_decode_full(wb, ids, id_off):
    """Oracle FULL decode (no fast-path limits); grant_off / op_key_off index out["blob"],
    the re-serialized signed grant bytes."""
    wc, keep = _w2_c(wb)
    d = _dec_struct()()
    rc = lib().oracle_w2_decode_full(ctypes.addressof(wc), ids.ctypes.data, id_off.ctypes.data,
                                     int(id_off.shape[0]) - 1, ctypes.addressof(d))
    assert rc == 0
    out = _dec_arrays(d)
    lib().oracle_w2_free(ctypes.addressof(d))
    return out


def verify_write2(moduli, ids, id_off, wb, replication_factor: int, strict_gt: bool, n_threads: int = 8,
                  quorum_mode: int = 0):
    import mochi_hip as mh

    mod = np.frombuffer(b"".join(bytes(m) for m in moduli), np.uint8).copy()
    wc, keep = _w2_c(wb)
    M = wb.n_msgs
    O = int(wb.op_flags_off[-1]) if wb.op_flags_off is not None else 0
    out = mh.Verdicts.alloc(0, M, O)
    vc = out.to_c()
    vc.grant_valid_bits = vc.grant_flags = vc.grant_ts = None
    if wb.op_flags_off is None:
        vc.op_decision = vc.op_g0 = vc.op_ts = None
        out.op_decision = out.op_g0 = out.op_ts = None
    p = mh.params(replication_factor, strict_gt, quorum_mode)
    st = np.zeros(max(M, 1), np.uint8)
    rc = lib().oracle_verify_write2(mod.ctypes.data, len(moduli), ids.ctypes.data, id_off.ctypes.data,
                                    ctypes.addressof(wc), ctypes.addressof(p), ctypes.addressof(vc), st.ctypes.data,
                                    n_threads)
    assert rc == 0
    return out, st[:M].copy()

