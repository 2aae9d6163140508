"""ctypes binding for libmochi_hip (include/mochi_hip.h).

The host-side mirror of the reference's Write2 verification interface for
tests, the benchmark and Python callers.  The product path is the HIP
library; this module never falls back to a CPU implementation: if the shared
library is missing or no gfx950 device is visible, constructing a Verifier
raises.

Reference interface mirrored (tomisetsu/mochi-db):
  DataStore.processWrite2ToServer(Write2ToServer) -> Object
      server/datastrore/DataStore.java:12, InMemoryDataStore.java:641-666
  MochiDBClient read / Write2 aggregation
      client/MochiDBClient.java:148-175, 355-382
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# MOCHI_HIP_LIB: an alternative build of the same library (A/B measurements)
LIB_PATH = os.environ.get("MOCHI_HIP_LIB") or os.path.join(_HERE, "libmochi_hip.so")

RSA_BYTES = 256
RSA_E = 65537
TXN_HASH_BYTES = 128
MAX_OPS_PER_CERT = 64

# status codes
OK, EINVAL, EHIP, ENOMEM, ENODEV = 0, -1, -2, -3, -4

# reason codes (enum mochi_reason)
ACCEPT = 0
REJECT_TS_MISMATCH = 1
REJECT_NO_GRANT = 2
REJECT_BELOW_QUORUM = 3
REJECT_HASH_MISMATCH = 4
REJECT_NO_SVOC = 5
REJECT_MALFORMED = 6
REJECT_APPLY_STATE = 8
REJECT_STORED_CERT = 9
REJECT_NOT_WRITE = 10
REASON_NAMES = {
    ACCEPT: "ACCEPT",
    REJECT_TS_MISMATCH: "TS_MISMATCH",
    REJECT_NO_GRANT: "NO_GRANT",
    REJECT_BELOW_QUORUM: "BELOW_QUORUM",
    REJECT_HASH_MISMATCH: "HASH_MISMATCH",
    REJECT_NO_SVOC: "NO_SVOC",
    REJECT_MALFORMED: "MALFORMED",
    REJECT_APPLY_STATE: "APPLY_STATE",
    REJECT_STORED_CERT: "STORED_CERT",
    REJECT_NOT_WRITE: "NOT_WRITE",
}

OP_LOCAL = 0x01
OP_HAS_SVOC = 0x02
OP_HAS_CURRENT_C = 0x04
OP_CURRENT_C_BAD = 0x08
OP_NOT_WRITE = 0x10

# per-op decisions (enum mochi_op_decision)
OPD_SKIPPED, OPD_APPLY, OPD_READ, OPD_WRONG_SHARD, OPD_FAILED = 0, 1, 2, 3, 4

# mochi_params.quorum_mode bits
Q_DISTINCT_SIGNERS = 0x1
Q_BIND = 0x2
GRANT_SIG_OK = 0x01
GRANT_PARSED = 0x02


class MochiError(RuntimeError):
    pass


class Batch_C(ctypes.Structure):
    _fields_ = [
        ("n_grants", ctypes.c_uint32),
        ("n_certs", ctypes.c_uint32),
        ("n_ops", ctypes.c_uint32),
        ("n_mgs", ctypes.c_uint32),
        ("grant_bytes_len", ctypes.c_uint64),
        ("grant_bytes", ctypes.c_void_p),
        ("grant_off", ctypes.c_void_p),
        ("grant_len", ctypes.c_void_p),
        ("sig", ctypes.c_void_p),
        ("signer", ctypes.c_void_p),
        ("grant_key", ctypes.c_void_p),
        ("cert_grant_off", ctypes.c_void_p),
        ("cert_op_off", ctypes.c_void_p),
        ("op_key", ctypes.c_void_p),
        ("op_flags", ctypes.c_void_p),
        ("expected_hash", ctypes.c_void_p),
        ("cert_mg_off", ctypes.c_void_p),
        ("mg_grant_off", ctypes.c_void_p),
        ("op_object_ts", ctypes.c_void_p),
        ("op_key_off", ctypes.c_void_p),
        ("op_key_len", ctypes.c_void_p),
    ]


class Params_C(ctypes.Structure):
    _fields_ = [
        ("replication_factor", ctypes.c_uint32),
        ("strict_gt", ctypes.c_uint32),
        ("quorum_mode", ctypes.c_uint32),
        ("_pad", ctypes.c_uint32),
    ]


def params(replication_factor: int, strict_gt: bool = True, quorum_mode: int = 0) -> "Params_C":
    return Params_C(replication_factor=replication_factor, strict_gt=1 if strict_gt else 0, quorum_mode=quorum_mode)


class Verdicts_C(ctypes.Structure):
    _fields_ = [
        ("grant_valid_bits", ctypes.c_void_p),
        ("grant_flags", ctypes.c_void_p),
        ("grant_ts", ctypes.c_void_p),
        ("cert_accept_bits", ctypes.c_void_p),
        ("cert_reason", ctypes.c_void_p),
        ("cert_fail_op", ctypes.c_void_p),
        ("op_decision", ctypes.c_void_p),
        ("op_g0", ctypes.c_void_p),
        ("op_ts", ctypes.c_void_p),
    ]


_lib = None
ABI_VERSION = 3


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load libmochi_hip.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise MochiError(f"{path} not built: run `make -C mochi-db_amd` (or __graft_entry__.build())")
    # One HIP runtime per process: when PyTorch-ROCm is present, load it first so
    # that libmochi_hip's libamdhip64.so.7 dependency resolves (by SONAME) to the
    # runtime torch already mapped; device pointers and hipStream_t handles can
    # then cross the boundary.  Loading ours first would make torch map a second
    # runtime, which then sees no GPU.
    try:
        import torch  # noqa: F401  (plumbing only)
    except Exception:
        pass
    lib = ctypes.CDLL(path)
    vp, u32, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int32
    lib.mochi_abi_version.restype = ctypes.c_int
    lib.mochi_last_error.restype = ctypes.c_char_p
    lib.mochi_device_count.restype = ctypes.c_int
    lib.mochi_ctx_create.restype = vp
    lib.mochi_ctx_create.argtypes = [ctypes.c_int, vp, u32, u32, u32]
    lib.mochi_ctx_destroy.argtypes = [vp]
    lib.mochi_verify_batch.argtypes = [vp, ctypes.POINTER(Batch_C), ctypes.POINTER(Params_C), ctypes.POINTER(Verdicts_C)]
    lib.mochi_verify_batch_device.argtypes = [vp, ctypes.POINTER(Batch_C), ctypes.POINTER(Params_C),
                                              ctypes.POINTER(Verdicts_C), vp]
    lib.mochi_ctx_last_timing.argtypes = [vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float),
                                          ctypes.POINTER(ctypes.c_float)]
    lib.mochi_sign_grants.argtypes = [ctypes.c_char_p, u32, vp, vp, vp, vp, ctypes.c_int]
    lib.mochi_pem_modulus.argtypes = [ctypes.c_char_p, vp]
    lib.mochi_rsa_public_op.argtypes = [vp, u32, vp, vp, vp, vp]
    lib.mochi_fold_matrix.argtypes = [vp, vp, vp]
    lib.mochi_ctx_set_profiling.argtypes = [vp, ctypes.c_int]
    lib.mochi_ctx_read_profile.argtypes = [vp, vp, u32, vp]
    lib.mochi_tally_responses.argtypes = [u32, vp, vp, vp, vp, vp, vp, u32, vp, vp, vp]
    lib.mochi_write1_classify.argtypes = [u32, vp, vp, vp, vp, vp, vp, vp, vp]
    lib.mochi_tally_responses_device.argtypes = [u32, vp, vp, vp, vp, vp, vp, u32, vp, vp, vp, vp]
    lib.mochi_write1_classify_device.argtypes = [u32, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    lib.mochi_ctx_last_total_ms.argtypes = [vp, ctypes.POINTER(ctypes.c_float)]
    lib.mochi_ctx_set_chunk_grants.argtypes = [vp, u32]
    lib.mochi_ctx_set_small_batch.argtypes = [vp, u32]
    lib.mochi_ctx_set_server_ids.argtypes = [vp, vp, vp, u32]
    lib.mochi_verify_write2.argtypes = [vp, vp, vp, vp, vp]
    lib.mochi_verify_write2_device.argtypes = [vp, vp, vp, vp, vp, vp]
    lib.mochi_write2_decode.argtypes = [vp, vp, vp]
    lib.mochi_write2_decoded_free.argtypes = [vp]
    lib.mochi_signer_create.restype = vp
    lib.mochi_signer_create.argtypes = [ctypes.c_int, ctypes.c_char_p]
    lib.mochi_signer_destroy.argtypes = [vp]
    lib.mochi_sign_batch.argtypes = [vp, vp, ctypes.c_uint64, vp, vp, u32, vp]
    lib.mochi_sign_batch_device.argtypes = [vp, vp, vp, vp, u32, vp, vp]
    lib.mochi_signer_rejected.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64)]
    lib.mochi_signer_set_fault.argtypes = [vp, u32]
    lib.mochi_batcher_create.restype = vp
    lib.mochi_batcher_create.argtypes = [vp, vp, u32, u32, ctypes.c_int]
    lib.mochi_batcher_create_multi.restype = vp
    lib.mochi_batcher_create_multi.argtypes = [vp, u32, vp, u32, u32, ctypes.c_int]
    lib.mochi_batcher_verify.argtypes = [vp, vp, u32, vp, u32, vp, vp]
    lib.mochi_batcher_submit.argtypes = [vp, vp, u32, vp, u32, vp, VERDICT_CB, vp]
    lib.mochi_batcher_stats.argtypes = [vp, vp, vp]
    lib.mochi_batcher_destroy.argtypes = [vp]
    lib.mochi_shard_plan.argtypes = [u32, vp, u32, vp]
    lib.mochi_shard_words.restype = u32
    lib.mochi_shard_words.argtypes = [u32, vp]
    lib.mochi_bits_assemble.argtypes = [u32, vp, u32, vp, vp]
    lib.mochi_mctx_create.restype = vp
    lib.mochi_mctx_create.argtypes = [ctypes.c_uint64, vp, u32, u32, u32]
    lib.mochi_mctx_destroy.argtypes = [vp]
    lib.mochi_mctx_devices.argtypes = [vp, vp, ctypes.c_int]
    lib.mochi_mctx_context.restype = vp
    lib.mochi_mctx_context.argtypes = [vp, ctypes.c_int]
    lib.mochi_mctx_set_server_ids.argtypes = [vp, vp, vp, u32]
    lib.mochi_mverify_batch.argtypes = [vp, vp, vp, vp]
    lib.mochi_mverify_write2.argtypes = [vp, vp, vp, vp, vp]
    lib.mochi_mctx_gathered_bits.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p),
                                             ctypes.POINTER(ctypes.c_uint32)]
    lib.mochi_comm_unique_id.argtypes = [vp]
    lib.mochi_comm_init.restype = vp
    lib.mochi_comm_init.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.mochi_comm_allgather_bits.argtypes = [vp, vp, u32, vp, vp]
    lib.mochi_comm_destroy.argtypes = [vp]
    lib.mochi_test_gather_protocol.argtypes = [u32, u32, u32, u32, u32, ctypes.POINTER(u32), ctypes.POINTER(u32)]
    lib.mochi_host_alloc.restype = vp
    lib.mochi_host_alloc.argtypes = [ctypes.c_uint64]
    lib.mochi_host_free.argtypes = [vp]
    # ABI 3: per-request batcher calls with stored state + per-op outputs; cluster config
    lib.mochi_batcher_verify_request.argtypes = [vp, ctypes.POINTER(Write2Request_C), ctypes.POINTER(Verdict1_C)]
    lib.mochi_batcher_submit_request.argtypes = [vp, ctypes.POINTER(Write2Request_C), VERDICT_CB, vp]
    lib.mochi_config_load.restype = vp
    lib.mochi_config_load.argtypes = [ctypes.c_char_p]
    lib.mochi_config_parse.restype = vp
    lib.mochi_config_parse.argtypes = [ctypes.c_char_p, ctypes.c_uint64]
    lib.mochi_config_free.argtypes = [vp]
    lib.mochi_config_replication.restype = u32
    lib.mochi_config_replication.argtypes = [vp]
    lib.mochi_config_majority.restype = u32
    lib.mochi_config_majority.argtypes = [vp]
    lib.mochi_config_n_servers.restype = u32
    lib.mochi_config_n_servers.argtypes = [vp]
    lib.mochi_config_server_id.restype = ctypes.c_char_p
    lib.mochi_config_server_id.argtypes = [vp, u32]
    lib.mochi_config_server_url.restype = ctypes.c_char_p
    lib.mochi_config_server_url.argtypes = [vp, u32]
    lib.mochi_config_servers_for_key.argtypes = [vp, vp, u32, vp]
    lib.mochi_config_replica_ids.restype = ctypes.c_int64
    lib.mochi_config_replica_ids.argtypes = [vp, vp, u32, vp, ctypes.c_uint64, vp]
    if lib.mochi_abi_version() != ABI_VERSION:
        raise MochiError("libmochi_hip ABI mismatch")
    _lib = lib
    return lib


def _ptr(a: Optional[np.ndarray]) -> Optional[int]:
    if a is None:
        return None
    if not a.flags["C_CONTIGUOUS"]:
        raise ValueError("arrays must be C-contiguous")
    return a.ctypes.data


def _err(lib) -> str:
    return (lib.mochi_last_error() or b"").decode(errors="replace")


@dataclass
class Batch:
    """A batch of Write2 certificates, struct-of-arrays (see mochi_batch)."""

    grant_bytes: np.ndarray  # uint8 blob
    grant_off: np.ndarray  # uint64 [N]
    grant_len: np.ndarray  # uint32 [N]
    sig: np.ndarray  # uint8 [N, 256]
    signer: np.ndarray  # uint16 [N]
    grant_key: np.ndarray  # uint8 [N]
    cert_grant_off: np.ndarray  # uint32 [C+1]
    cert_op_off: np.ndarray  # uint32 [C+1]
    op_key: np.ndarray  # uint8 [O]
    op_flags: np.ndarray  # uint8 [O]
    expected_hash: np.ndarray  # uint8 [C, 128]
    # ABI 2 (optional): MultiGrant CSR, stored-certificate timestamps, op key slices
    cert_mg_off: Optional[np.ndarray] = None  # uint32 [C+1]
    mg_grant_off: Optional[np.ndarray] = None  # uint32 [n_mgs+1]
    op_object_ts: Optional[np.ndarray] = None  # int64 [O]
    op_key_off: Optional[np.ndarray] = None  # uint64 [O] into grant_bytes
    op_key_len: Optional[np.ndarray] = None  # uint32 [O]

    OPTIONAL = ("cert_mg_off", "mg_grant_off", "op_object_ts", "op_key_off", "op_key_len")
    OPT_DTYPES = {"cert_mg_off": np.uint32, "mg_grant_off": np.uint32, "op_object_ts": np.int64,
                  "op_key_off": np.uint64, "op_key_len": np.uint32}
    FIELDS = ("grant_bytes", "grant_off", "grant_len", "sig", "signer", "grant_key", "cert_grant_off",
              "cert_op_off", "op_key", "op_flags", "expected_hash")

    @property
    def n_mgs(self) -> int:
        return 0 if self.mg_grant_off is None else int(self.mg_grant_off.shape[0]) - 1

    @property
    def n_grants(self) -> int:
        return int(self.grant_off.shape[0])

    @property
    def n_certs(self) -> int:
        return int(self.cert_grant_off.shape[0]) - 1

    @property
    def n_ops(self) -> int:
        return int(self.op_key.shape[0])

    def normalized(self) -> "Batch":
        return Batch(
            grant_bytes=np.ascontiguousarray(self.grant_bytes, dtype=np.uint8),
            grant_off=np.ascontiguousarray(self.grant_off, dtype=np.uint64),
            grant_len=np.ascontiguousarray(self.grant_len, dtype=np.uint32),
            sig=np.ascontiguousarray(self.sig, dtype=np.uint8).reshape(-1, RSA_BYTES),
            signer=np.ascontiguousarray(self.signer, dtype=np.uint16),
            grant_key=np.ascontiguousarray(self.grant_key, dtype=np.uint8),
            cert_grant_off=np.ascontiguousarray(self.cert_grant_off, dtype=np.uint32),
            cert_op_off=np.ascontiguousarray(self.cert_op_off, dtype=np.uint32),
            op_key=np.ascontiguousarray(self.op_key, dtype=np.uint8),
            op_flags=np.ascontiguousarray(self.op_flags, dtype=np.uint8),
            expected_hash=np.ascontiguousarray(self.expected_hash, dtype=np.uint8).reshape(-1, TXN_HASH_BYTES),
            **{k: (None if getattr(self, k) is None else np.ascontiguousarray(getattr(self, k), dtype=self.OPT_DTYPES[k]))
               for k in self.OPTIONAL},
        )

    def pinned(self) -> "Batch":
        """A copy whose arrays live in one pinned host allocation (mochi_host_alloc):
        mochi_verify_batch DMAs such arrays in place instead of staging them."""
        b = self.normalized()
        names = self.FIELDS + tuple(k for k in self.OPTIONAL if getattr(b, k) is not None)
        arrs = [getattr(b, nm) for nm in names]
        offs, total = [], 0
        for a in arrs:
            offs.append(total)
            total = (total + a.nbytes + 255) // 256 * 256
        buf = PinnedHost(total)
        out = {}
        for nm, a, o in zip(names, arrs, offs):
            v = np.frombuffer(buf.view()[o:o + a.nbytes], dtype=a.dtype).reshape(a.shape)
            v[...] = a
            out[nm] = v
        pb = Batch(**out)
        pb._pinned = buf  # keep the allocation alive with the views
        return pb

    def to_c(self) -> Batch_C:
        b = Batch_C()
        b.n_grants, b.n_certs, b.n_ops = self.n_grants, self.n_certs, self.n_ops
        b.grant_bytes_len = int(self.grant_bytes.nbytes)
        b.grant_bytes = _ptr(self.grant_bytes)
        b.grant_off = _ptr(self.grant_off)
        b.grant_len = _ptr(self.grant_len)
        b.sig = _ptr(self.sig)
        b.signer = _ptr(self.signer)
        b.grant_key = _ptr(self.grant_key)
        b.cert_grant_off = _ptr(self.cert_grant_off)
        b.cert_op_off = _ptr(self.cert_op_off)
        b.op_key = _ptr(self.op_key)
        b.op_flags = _ptr(self.op_flags)
        b.expected_hash = _ptr(self.expected_hash)
        b.n_mgs = self.n_mgs
        for k in self.OPTIONAL:
            setattr(b, k, _ptr(getattr(self, k)))
        return b


class PinnedHost:
    """Pinned host allocation from libmochi_hip (mochi_host_alloc / mochi_host_free)."""

    def __init__(self, nbytes: int):
        self.lib = load_library()
        self.nbytes = max(int(nbytes), 1)
        self.ptr = self.lib.mochi_host_alloc(self.nbytes)
        if not self.ptr:
            raise MochiError(f"mochi_host_alloc: {_err(self.lib)}")

    def view(self) -> np.ndarray:
        return np.ctypeslib.as_array((ctypes.c_uint8 * self.nbytes).from_address(self.ptr))

    def __del__(self):  # pragma: no cover
        if getattr(self, "ptr", None):
            self.lib.mochi_host_free(self.ptr)
            self.ptr = None


@dataclass
class Verdicts:
    grant_valid_bits: np.ndarray
    grant_flags: np.ndarray
    grant_ts: np.ndarray
    cert_accept_bits: np.ndarray
    cert_reason: np.ndarray
    cert_fail_op: np.ndarray
    op_decision: Optional[np.ndarray] = None  # uint8 [O]
    op_g0: Optional[np.ndarray] = None  # uint32 [O]
    op_ts: Optional[np.ndarray] = None  # int64 [O]
    timing_ms: dict = field(default_factory=dict)

    @staticmethod
    def alloc(n_grants: int, n_certs: int, n_ops: int = 0) -> "Verdicts":
        return Verdicts(
            grant_valid_bits=np.zeros((n_grants + 31) // 32, np.uint32),
            grant_flags=np.zeros(n_grants, np.uint8),
            grant_ts=np.zeros(n_grants, np.int64),
            cert_accept_bits=np.zeros((n_certs + 31) // 32, np.uint32),
            cert_reason=np.zeros(n_certs, np.uint8),
            cert_fail_op=np.zeros(n_certs, np.uint8),
            op_decision=np.full(n_ops, 0xEE, np.uint8),
            op_g0=np.zeros(n_ops, np.uint32),
            op_ts=np.zeros(n_ops, np.int64),
        )

    def to_c(self) -> Verdicts_C:
        v = Verdicts_C()
        v.grant_valid_bits = _ptr(self.grant_valid_bits)
        v.grant_flags = _ptr(self.grant_flags)
        v.grant_ts = _ptr(self.grant_ts)
        v.cert_accept_bits = _ptr(self.cert_accept_bits)
        v.cert_reason = _ptr(self.cert_reason)
        v.cert_fail_op = _ptr(self.cert_fail_op)
        # zero-length op arrays still get a pointer (n_ops == 0 reads nothing)
        v.op_decision = _ptr(self.op_decision)
        v.op_g0 = _ptr(self.op_g0)
        v.op_ts = _ptr(self.op_ts)
        return v

    @property
    def grant_valid(self) -> np.ndarray:
        return unpack_bits(self.grant_valid_bits, self.grant_flags.shape[0])

    @property
    def cert_accept(self) -> np.ndarray:
        return unpack_bits(self.cert_accept_bits, self.cert_reason.shape[0])


def unpack_bits(words: np.ndarray, n: int) -> np.ndarray:
    """uint32 little-endian bitmap -> bool[n] (bit i of word i//32)."""
    b = np.unpackbits(np.ascontiguousarray(words, dtype="<u4").view(np.uint8), bitorder="little")
    return b[:n].astype(bool)


def majority(replication_factor: int) -> int:
    """ClusterConfiguration.getServerMajority (ClusterConfiguration.java:264-267)."""
    return 2 * (replication_factor // 3) + 1


class Verifier:
    """A libmochi_hip context: one device, one RSA public-key table.

    Key index i corresponds to the i-th server ID of the cluster (the
    MultiGrant.serverId that signed the grant).
    """

    def __init__(self, moduli_be: Sequence[bytes] | np.ndarray, device: int = 0):
        self.lib = load_library()
        mod = np.ascontiguousarray(
            np.frombuffer(b"".join(bytes(m) for m in moduli_be), np.uint8)
            if not isinstance(moduli_be, np.ndarray) else moduli_be.astype(np.uint8).reshape(-1)
        )
        if mod.size % RSA_BYTES:
            raise ValueError("moduli must be 256-byte big-endian values")
        self.n_keys = mod.size // RSA_BYTES
        self._moduli = mod
        self.ctx = self.lib.mochi_ctx_create(int(device), mod.ctypes.data, self.n_keys, RSA_BYTES, RSA_E)
        if not self.ctx:
            raise MochiError(f"mochi_ctx_create failed: {_err(self.lib)}")
        self.device = device

    def set_server_ids(self, server_ids) -> None:
        """Key i of the table belongs to MultiGrant.serverId == server_ids[i] (Write2 wire path)."""
        enc = [x.encode() if isinstance(x, str) else bytes(x) for x in server_ids]
        blob = np.frombuffer(b"".join(enc) or b"\x00", np.uint8).copy()
        off = np.zeros(len(enc) + 1, np.uint32)
        np.cumsum([len(x) for x in enc], out=off[1:])
        if self.lib.mochi_ctx_set_server_ids(self.ctx, _ptr(blob), _ptr(off), len(enc)) != OK:
            raise MochiError(f"mochi_ctx_set_server_ids: {_err(self.lib)}")

    def verify_write2(self, wb, replication_factor: int, strict_gt: bool = True, quorum_mode: int = 0):
        """Write2ToServer messages (workload.WireBatch, host memory) -> (Verdicts with
        certificate-level arrays -- and per-op arrays when wb.op_flags_off is set --,
        msg_status[M])."""
        wc, keep = write2_batch_c(wb)
        M = wb.n_msgs
        O = int(wb.op_flags_off[-1]) if wb.op_flags_off is not None else 0
        out = Verdicts.alloc(0, M, O)
        vc = out.to_c()
        vc.grant_valid_bits = vc.grant_flags = vc.grant_ts = None
        if wb.op_flags_off is None:
            vc.op_decision = vc.op_g0 = vc.op_ts = None
            out.op_decision = out.op_g0 = out.op_ts = None
        p = params(replication_factor, strict_gt, quorum_mode)
        st = np.zeros(max(M, 1), np.uint8)
        rc = self.lib.mochi_verify_write2(self.ctx, ctypes.addressof(wc), ctypes.addressof(p), ctypes.addressof(vc),
                                          _ptr(st))
        if rc != OK:
            raise MochiError(f"mochi_verify_write2 rc={rc}: {_err(self.lib)}")
        t = ctypes.c_float()
        self.lib.mochi_ctx_last_total_ms(self.ctx, ctypes.byref(t))
        out.timing_ms = {"total": t.value}
        return out, st[:M].copy()

    def verify_write2_device(self, dwb: "DeviceWireBatch", out: "DeviceVerdicts", replication_factor: int,
                             strict_gt: bool = True, stream: int = 0, quorum_mode: int = 0) -> None:
        """Device-resident Write2 wire messages -> certificate verdicts (async on `stream`,
        except for one wait on the decoded grant / op totals)."""
        wc = dwb.to_c()
        vc = out.to_c()
        vc.grant_valid_bits = vc.grant_flags = vc.grant_ts = None
        if dwb.op_flags_off is None:
            vc.op_decision = vc.op_g0 = vc.op_ts = None
        p = params(replication_factor, strict_gt, quorum_mode)
        rc = self.lib.mochi_verify_write2_device(self.ctx, ctypes.addressof(wc), ctypes.addressof(p),
                                                 ctypes.addressof(vc), dwb.status.data_ptr(), stream)
        if rc != OK:
            raise MochiError(f"mochi_verify_write2_device rc={rc}: {_err(self.lib)}")

    def decode_write2(self, wb) -> dict:
        """The device decoder's SoA view of the messages (inspection / tests)."""
        wc, keep = write2_batch_c(wb)
        d = Write2Decoded_C()
        rc = self.lib.mochi_write2_decode(self.ctx, ctypes.addressof(wc), ctypes.addressof(d))
        if rc != OK:
            raise MochiError(f"mochi_write2_decode rc={rc}: {_err(self.lib)}")
        N, M, O = d.n_grants, d.n_msgs, d.n_ops

        def arr(ptr, n, dt):
            if n == 0:
                return np.zeros(0, dt)
            return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(np.ctypeslib.as_ctypes_type(dt))),
                                         shape=(n,)).copy()

        out = dict(grant_off=arr(d.grant_off, N, np.uint64), grant_len=arr(d.grant_len, N, np.uint32),
                   sig=arr(d.sig, N * 256, np.uint8).reshape(N, 256), signer=arr(d.signer, N, np.uint16),
                   grant_key=arr(d.grant_key, N, np.uint8), cert_grant_off=arr(d.cert_grant_off, M + 1, np.uint32),
                   cert_op_off=arr(d.cert_op_off, M + 1, np.uint32), op_key=arr(d.op_key, O, np.uint8),
                   op_flags=arr(d.op_flags, O, np.uint8), msg_status=arr(d.msg_status, M, np.uint8),
                   cert_mg_off=arr(d.cert_mg_off, M + 1, np.uint32),
                   mg_grant_off=arr(d.mg_grant_off, d.n_mgs + 1, np.uint32),
                   op_key_off=arr(d.op_key_off, O, np.uint64), op_key_len=arr(d.op_key_len, O, np.uint32))
        self.lib.mochi_write2_decoded_free(ctypes.addressof(d))
        return out

    def set_small_batch(self, grants: int) -> None:
        """Batches of at most `grants` grants take the small-batch launch sequence
        (mochi_ctx_set_small_batch); 0 = never."""
        if self.lib.mochi_ctx_set_small_batch(self.ctx, int(grants)) != OK:
            raise MochiError(_err(self.lib))

    def set_chunk_grants(self, grants: int) -> None:
        """Host-path pipeline chunk target (grants); 0 restores the default."""
        if self.lib.mochi_ctx_set_chunk_grants(self.ctx, int(grants)) != OK:
            raise MochiError(_err(self.lib))

    def close(self) -> None:
        if getattr(self, "ctx", None):
            self.lib.mochi_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def verify(self, batch: Batch, replication_factor: int, strict_gt: bool = True, quorum_mode: int = 0) -> Verdicts:
        """Host-memory batch -> verdicts (pinned staging, synchronous)."""
        b = batch.normalized()
        out = Verdicts.alloc(b.n_grants, b.n_certs, b.n_ops)
        bc, vc = b.to_c(), out.to_c()
        p = params(replication_factor, strict_gt, quorum_mode)
        rc = self.lib.mochi_verify_batch(self.ctx, ctypes.byref(bc), ctypes.byref(p), ctypes.byref(vc))
        if rc != OK:
            raise MochiError(f"mochi_verify_batch rc={rc}: {_err(self.lib)}")
        h, k, d, t = ctypes.c_float(), ctypes.c_float(), ctypes.c_float(), ctypes.c_float()
        self.lib.mochi_ctx_last_timing(self.ctx, ctypes.byref(h), ctypes.byref(k), ctypes.byref(d))
        self.lib.mochi_ctx_last_total_ms(self.ctx, ctypes.byref(t))
        out.timing_ms = {"h2d": h.value, "kernels": k.value, "d2h": d.value, "total": t.value}
        return out

    STAGES = ("prep_sha256", "bucket", "rsa_pow", "rsa_final", "tally")

    def set_profiling(self, on: bool) -> None:
        self.lib.mochi_ctx_set_profiling(self.ctx, 1 if on else 0)

    def read_profile(self) -> dict:
        """Mean per-call stage times (ms) since the last read; waits for the device."""
        arr = (ctypes.c_float * len(self.STAGES))()
        n = ctypes.c_uint32()
        rc = self.lib.mochi_ctx_read_profile(self.ctx, arr, len(self.STAGES), ctypes.byref(n))
        if rc != OK:
            raise MochiError(f"mochi_ctx_read_profile rc={rc}: {_err(self.lib)}")
        calls = max(1, n.value)
        out = {name: arr[i] / calls for i, name in enumerate(self.STAGES)}
        out["calls"] = n.value
        return out

    def verify_device(self, dev: "DeviceBatch", out: "DeviceVerdicts", replication_factor: int,
                      strict_gt: bool = True, stream: int = 0, quorum_mode: int = 0) -> None:
        """Device-resident batch (torch tensors) -> device verdicts; async on `stream`."""
        p = params(replication_factor, strict_gt, quorum_mode)
        bc, vc = dev.to_c(), out.to_c()
        rc = self.lib.mochi_verify_batch_device(self.ctx, ctypes.byref(bc), ctypes.byref(p), ctypes.byref(vc),
                                                stream or None)
        if rc != OK:
            raise MochiError(f"mochi_verify_batch_device rc={rc}: {_err(self.lib)}")


def fold_matrix(modulus_be: bytes):
    """The k_rsa_pow fold matrix of one modulus (mochi_fold_matrix): int8 image
    [10 M-tiles][10 K-steps][64 lanes][16] and the bias correction cadd uint32[74]."""
    lib = load_library()
    m = np.frombuffer(bytes(modulus_be), np.uint8)
    img = np.zeros((10, 10, 64, 16), np.int8)
    cadd = np.zeros(74, np.uint32)
    rc = lib.mochi_fold_matrix(_ptr(m), _ptr(img), _ptr(cadd))
    if rc != OK:
        raise MochiError(f"mochi_fold_matrix rc={rc}: {_err(lib)}")
    return img, cadd


def rsa_public_op(verifier: "Verifier", sigs: np.ndarray, signer: np.ndarray, want_z: bool = False):
    """y = s^65537 mod n on the device (big-endian bytes); optionally the chain intermediate z."""
    lib = verifier.lib
    s = np.ascontiguousarray(sigs, np.uint8).reshape(-1, RSA_BYTES)
    sg = np.ascontiguousarray(signer, np.uint16)
    n = s.shape[0]
    out = np.zeros((n, RSA_BYTES), np.uint8)
    z = np.zeros((n, 74), np.uint32) if want_z else None
    rc = lib.mochi_rsa_public_op(verifier.ctx, n, _ptr(s), _ptr(sg), _ptr(out), _ptr(z) if want_z else None)
    if rc != OK:
        raise MochiError(f"mochi_rsa_public_op rc={rc}: {_err(lib)}")
    return (out, z) if want_z else out


class DeviceBatch:
    """A Batch copied into device memory with torch (plumbing only)."""

    def __init__(self, batch: Batch, device: int = 0):
        import torch

        b = batch.normalized()
        dev = torch.device("cuda", device)

        def t(a):
            return torch.from_numpy(np.ascontiguousarray(a)).to(dev)

        self.n_grants, self.n_certs, self.n_ops = b.n_grants, b.n_certs, b.n_ops
        self.grant_bytes = t(b.grant_bytes)
        self.grant_off = t(b.grant_off.view(np.int64))
        self.grant_len = t(b.grant_len.view(np.int32))
        self.sig = t(b.sig)
        self.signer = t(b.signer.view(np.int16))
        self.grant_key = t(b.grant_key)
        self.cert_grant_off = t(b.cert_grant_off.view(np.int32))
        self.cert_op_off = t(b.cert_op_off.view(np.int32))
        self.op_key = t(b.op_key)
        self.op_flags = t(b.op_flags)
        self.expected_hash = t(b.expected_hash)
        self.n_mgs = b.n_mgs
        sv = {np.uint32: np.int32, np.uint64: np.int64, np.int64: np.int64}
        for k in Batch.OPTIONAL:
            a = getattr(b, k)
            setattr(self, k, None if a is None else t(a.view(sv[Batch.OPT_DTYPES[k]])))

    def to_c(self) -> Batch_C:
        b = Batch_C()
        b.n_grants, b.n_certs, b.n_ops, b.n_mgs = self.n_grants, self.n_certs, self.n_ops, self.n_mgs
        b.grant_bytes_len = int(self.grant_bytes.numel())
        for name in Batch.FIELDS:
            setattr(b, name, getattr(self, name).data_ptr())
        for name in Batch.OPTIONAL:
            a = getattr(self, name)
            setattr(b, name, None if a is None else a.data_ptr())
        return b


class DeviceWireBatch:
    """A workload.WireBatch copied into device memory with torch (plumbing only)."""

    def __init__(self, wb, device: int = 0):
        import torch

        dev = torch.device("cuda", device)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        self.n_msgs = wb.n_msgs
        self.wire = t(wb.wire)
        self.msg_off = t(np.ascontiguousarray(wb.msg_off, np.uint64).view(np.int64))
        self.msg_len = t(np.ascontiguousarray(wb.msg_len, np.uint32).view(np.int32))
        self.op_flags_off = None if wb.op_flags_off is None else t(np.ascontiguousarray(wb.op_flags_off, np.uint32).view(np.int32))
        self.op_flags = t(wb.op_flags if wb.op_flags.size else np.zeros(1, np.uint8))
        self.expected_hash = t(np.ascontiguousarray(wb.expected_hash, np.uint8).reshape(-1))
        ots = getattr(wb, "op_object_ts", None)
        self.op_object_ts = None if ots is None or wb.op_flags_off is None else t(np.ascontiguousarray(ots, np.int64))
        self.status = torch.zeros(max(self.n_msgs, 1), dtype=torch.uint8, device=dev)

    def to_c(self) -> "Write2Batch_C":
        c = Write2Batch_C()
        c.n_msgs = self.n_msgs
        c.wire_len = int(self.wire.numel())
        c.wire, c.msg_off, c.msg_len = self.wire.data_ptr(), self.msg_off.data_ptr(), self.msg_len.data_ptr()
        c.op_flags_off = None if self.op_flags_off is None else self.op_flags_off.data_ptr()
        c.op_flags, c.expected_hash = self.op_flags.data_ptr(), self.expected_hash.data_ptr()
        c.op_object_ts = None if self.op_object_ts is None else self.op_object_ts.data_ptr()
        return c


class DeviceVerdicts:
    def __init__(self, n_grants: int, n_certs: int, device: int = 0, full: bool = True, n_ops: int = 0):
        import torch

        dev = torch.device("cuda", device)
        self.n_grants, self.n_certs = n_grants, n_certs
        self.cert_accept_bits = torch.zeros((n_certs + 31) // 32, dtype=torch.int32, device=dev)
        self.grant_valid_bits = torch.zeros((n_grants + 31) // 32, dtype=torch.int32, device=dev)
        self.grant_flags = torch.zeros(n_grants, dtype=torch.uint8, device=dev) if full else None
        self.grant_ts = torch.zeros(n_grants, dtype=torch.int64, device=dev) if full else None
        self.cert_reason = torch.zeros(n_certs, dtype=torch.uint8, device=dev) if full else None
        self.cert_fail_op = torch.zeros(n_certs, dtype=torch.uint8, device=dev) if full else None
        op = full and n_ops > 0
        self.op_decision = torch.zeros(n_ops, dtype=torch.uint8, device=dev) if op else None
        self.op_g0 = torch.zeros(n_ops, dtype=torch.int32, device=dev) if op else None
        self.op_ts = torch.zeros(n_ops, dtype=torch.int64, device=dev) if op else None

    NAMES = ("grant_valid_bits", "grant_flags", "grant_ts", "cert_accept_bits", "cert_reason", "cert_fail_op",
             "op_decision", "op_g0", "op_ts")

    def to_c(self) -> Verdicts_C:
        v = Verdicts_C()
        for name in self.NAMES:
            t = getattr(self, name)
            setattr(v, name, t.data_ptr() if t is not None else None)
        return v

    def to_host(self) -> Verdicts:
        def h(t, dt):
            return t.cpu().numpy().view(dt) if t is not None else None

        return Verdicts(
            grant_valid_bits=h(self.grant_valid_bits, np.uint32),
            grant_flags=h(self.grant_flags, np.uint8),
            grant_ts=h(self.grant_ts, np.int64),
            cert_accept_bits=h(self.cert_accept_bits, np.uint32),
            cert_reason=h(self.cert_reason, np.uint8),
            cert_fail_op=h(self.cert_fail_op, np.uint8),
            op_decision=h(self.op_decision, np.uint8),
            op_g0=h(self.op_g0, np.uint32),
            op_ts=h(self.op_ts, np.int64),
        )


def sign_grants(pem_private_key: bytes, grant_bytes: np.ndarray, grant_off: np.ndarray, grant_len: np.ndarray,
                n_threads: int = 8) -> np.ndarray:
    """Producer-side SHA256withRSA signing of grants (libmochi_hip, OpenSSL)."""
    lib = load_library()
    blob = np.ascontiguousarray(grant_bytes, np.uint8)
    off = np.ascontiguousarray(grant_off, np.uint64)
    ln = np.ascontiguousarray(grant_len, np.uint32)
    n = off.shape[0]
    out = np.zeros((n, RSA_BYTES), np.uint8)
    rc = lib.mochi_sign_grants(pem_private_key, n, _ptr(blob), _ptr(off), _ptr(ln), _ptr(out), int(n_threads))
    if rc != OK:
        raise MochiError(f"mochi_sign_grants rc={rc}")
    return out


def pem_modulus(pem: bytes) -> bytes:
    lib = load_library()
    out = np.zeros(RSA_BYTES, np.uint8)
    if lib.mochi_pem_modulus(pem, _ptr(out)) != OK:
        raise MochiError("not an RSA-2048 PEM key")
    return out.tobytes()


def tally_responses(responses: Sequence[Sequence[Sequence[int]]], n_ops: Sequence[int], replication_factor: int):
    """Client aggregation (MochiDBClient.java:148-175 / 355-382) via libmochi_hip.

    responses[r] = list of per-response status lists.  Returns (accept[bool],
    reason[uint8], chosen[list of int arrays]).
    """
    lib = load_library()
    nreq = len(responses)
    resp_off = np.zeros(nreq + 1, np.uint32)
    resp_n_ops, status_off, status, chosen_off = [], [], [], np.zeros(nreq, np.uint64)
    pos = 0
    cpos = 0
    for r, resps in enumerate(responses):
        resp_off[r + 1] = resp_off[r] + len(resps)
        chosen_off[r] = cpos
        cpos += n_ops[r]
        for st in resps:
            resp_n_ops.append(len(st))
            status_off.append(pos)
            status.extend(st)
            pos += len(st)
    n_ops_a = np.asarray(n_ops, np.uint32)
    resp_n_ops_a = np.asarray(resp_n_ops if resp_n_ops else [0], np.uint32)
    status_off_a = np.asarray(status_off if status_off else [0], np.uint64)
    status_a = np.asarray(status if status else [0], np.uint8)
    chosen = np.full(max(cpos, 1), -1, np.int32)
    reason = np.zeros(max(nreq, 1), np.uint8)
    bits = np.zeros(max((nreq + 31) // 32, 1), np.uint32)
    rc = lib.mochi_tally_responses(nreq, _ptr(resp_off), _ptr(n_ops_a), _ptr(resp_n_ops_a), _ptr(status_off_a),
                                   _ptr(status_a), _ptr(chosen_off), replication_factor, _ptr(chosen), _ptr(reason),
                                   _ptr(bits))
    if rc != OK:
        raise MochiError(f"mochi_tally_responses rc={rc}: {_err(lib)}")
    acc = unpack_bits(bits, nreq)
    ch = [chosen[int(chosen_off[r]):int(chosen_off[r]) + n_ops[r]].copy() for r in range(nreq)]
    return acc, reason[:nreq].copy(), ch


def _pack_responses(responses, n_ops):
    nreq = len(responses)
    resp_off = np.zeros(nreq + 1, np.uint32)
    resp_n_ops, status_off, status, chosen_off = [], [], [], np.zeros(max(nreq, 1), np.uint64)
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
    return (resp_off, np.asarray(n_ops if len(n_ops) else [0], np.uint32),
            np.asarray(resp_n_ops if resp_n_ops else [0], np.uint32),
            np.asarray(status_off if status_off else [0], np.uint64), np.asarray(status if status else [0], np.uint8),
            chosen_off, max(cpos, 1))


def tally_responses_device(responses, n_ops, replication_factor: int, device: int = 0):
    """Client aggregation on the device (mochi_tally_responses_device), batched over
    requests; same results as tally_responses.  torch moves the arrays (plumbing)."""
    import torch

    lib = load_library()
    nreq = len(responses)
    resp_off, n_ops_a, rn, so, st, co, nch = _pack_responses(responses, n_ops)
    d = torch.device("cuda", device)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view({1: np.uint8, 2: np.int16, 4: np.int32,
                                                                 8: np.int64}[a.dtype.itemsize])).to(d)
    ts = [t(x) for x in (resp_off, n_ops_a, rn, so, st, co)]
    chosen = torch.full((nch,), -1, dtype=torch.int32, device=d)
    reason = torch.zeros(max(nreq, 1), dtype=torch.uint8, device=d)
    bits = torch.zeros(max((nreq + 31) // 32, 1), dtype=torch.int32, device=d)
    rc = lib.mochi_tally_responses_device(nreq, *[x.data_ptr() for x in ts[:6]], replication_factor,
                                          chosen.data_ptr(), reason.data_ptr(), bits.data_ptr(),
                                          torch.cuda.current_stream(d).cuda_stream)
    if rc != OK:
        raise MochiError(f"mochi_tally_responses_device rc={rc}")
    torch.cuda.synchronize(d)
    acc = unpack_bits(bits.cpu().numpy().view(np.uint32), nreq)
    ch_h = chosen.cpu().numpy()
    ch = [ch_h[int(co[r]):int(co[r]) + n_ops[r]].copy() for r in range(nreq)]
    return acc, reason.cpu().numpy()[:nreq].copy(), ch


def write1_classify_device(requests, device: int = 0) -> np.ndarray:
    """Client Write1 round outcome per request on the device (mochi_write1_classify_device)."""
    import torch

    lib = load_library()
    a = pack_write1(requests)
    d = torch.device("cuda", device)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x).view({1: np.uint8, 4: np.int32,
                                                                 8: np.int64}[x.dtype.itemsize])).to(d)
    ts = [t(x) for x in a]
    out = torch.zeros(max(len(requests), 1), dtype=torch.uint8, device=d)
    rc = lib.mochi_write1_classify_device(len(requests), *[x.data_ptr() for x in ts], out.data_ptr(),
                                          torch.cuda.current_stream(d).cuda_stream)
    if rc != OK:
        raise MochiError(f"mochi_write1_classify_device rc={rc}")
    torch.cuda.synchronize(d)
    return out.cpu().numpy()[:len(requests)].copy()


# Write1 response kinds / round decisions (include/mochi_hip.h)
W1_OK, W1_REFUSED, W1_REQUEST_FAILED, W1_OTHER = 0, 1, 2, 3
W1_PROCEED, W1_RETRY, W1_THROW_REFUSED, W1_THROW_FAILED, W1_THROW_UNSUPPORTED = 0, 1, 2, 3, 4


def pack_write1(requests):
    """requests[r] = list of responses (kind, server_id, [(key_slot, ts, status), ...])
    -> the CSR arrays of mochi_write1_classify."""
    resp_off = np.zeros(len(requests) + 1, np.uint32)
    kinds, servers, goff, keys, tss, sts = [], [], [0], [], [], []
    for r, resps in enumerate(requests):
        resp_off[r + 1] = resp_off[r] + len(resps)
        for kind, sid, grants in resps:
            kinds.append(kind)
            servers.append(sid)
            for key, ts, st in grants:
                keys.append(key)
                tss.append(ts)
                sts.append(st)
            goff.append(len(keys))
    arr = lambda v, dt: np.asarray(v if v else [0], dt)
    return (resp_off, arr(kinds, np.uint8), arr(servers, np.uint32), np.asarray(goff, np.uint32),
            arr(keys, np.uint8), arr(tss, np.int64), arr(sts, np.uint8))


def write1_classify(requests) -> np.ndarray:
    """Client Write1 round outcome per request (MochiDBClient.java:236-332) via libmochi_hip."""
    lib = load_library()
    a = pack_write1(requests)
    out = np.zeros(max(len(requests), 1), np.uint8)
    rc = lib.mochi_write1_classify(len(requests), *[_ptr(x) for x in a], _ptr(out))
    if rc != OK:
        raise MochiError(f"mochi_write1_classify: {_err(lib)}")
    return out[:len(requests)].copy()


class Write2Batch_C(ctypes.Structure):
    _fields_ = [
        ("n_msgs", ctypes.c_uint32),
        ("_pad0", ctypes.c_uint32),
        ("wire_len", ctypes.c_uint64),
        ("wire", ctypes.c_void_p),
        ("msg_off", ctypes.c_void_p),
        ("msg_len", ctypes.c_void_p),
        ("op_flags_off", ctypes.c_void_p),
        ("op_flags", ctypes.c_void_p),
        ("expected_hash", ctypes.c_void_p),
        ("op_object_ts", ctypes.c_void_p),
    ]


MSG_OK, MSG_MALFORMED, MSG_FALLBACK, MSG_OPS_MISMATCH = 0, 1, 2, 3
UNDECIDED = 7
REASON_NAMES[UNDECIDED] = "UNDECIDED"


def write2_batch_c(wb):
    """workload.WireBatch (host arrays) -> (Write2Batch_C, keep-alive list)."""
    arrs = [np.ascontiguousarray(wb.wire, np.uint8), np.ascontiguousarray(wb.msg_off, np.uint64),
            np.ascontiguousarray(wb.msg_len, np.uint32),
            None if wb.op_flags_off is None else np.ascontiguousarray(wb.op_flags_off, np.uint32),
            np.ascontiguousarray(wb.op_flags if wb.op_flags.size else np.zeros(1, np.uint8), np.uint8),
            np.ascontiguousarray(wb.expected_hash, np.uint8).reshape(-1)]
    ots = getattr(wb, "op_object_ts", None)
    arrs.append(None if ots is None or wb.op_flags_off is None else np.ascontiguousarray(ots, np.int64))
    c = Write2Batch_C()
    c.n_msgs = int(arrs[1].shape[0])
    c.wire_len = int(arrs[0].nbytes)
    c.wire, c.msg_off, c.msg_len = _ptr(arrs[0]), _ptr(arrs[1]), _ptr(arrs[2])
    c.op_flags_off, c.op_flags, c.expected_hash = _ptr(arrs[3]), _ptr(arrs[4]), _ptr(arrs[5])
    c.op_object_ts = _ptr(arrs[6])
    return c, arrs


class Write2Decoded_C(ctypes.Structure):
    _fields_ = [("n_msgs", ctypes.c_uint32), ("n_grants", ctypes.c_uint32), ("n_ops", ctypes.c_uint32),
                ("n_mgs", ctypes.c_uint32), ("grant_off", ctypes.c_void_p), ("grant_len", ctypes.c_void_p),
                ("sig", ctypes.c_void_p), ("signer", ctypes.c_void_p), ("grant_key", ctypes.c_void_p),
                ("cert_grant_off", ctypes.c_void_p), ("cert_op_off", ctypes.c_void_p), ("op_key", ctypes.c_void_p),
                ("op_flags", ctypes.c_void_p), ("msg_status", ctypes.c_void_p), ("cert_mg_off", ctypes.c_void_p),
                ("mg_grant_off", ctypes.c_void_p), ("op_key_off", ctypes.c_void_p), ("op_key_len", ctypes.c_void_p)]


class Verdict1_C(ctypes.Structure):
    _fields_ = [("accepted", ctypes.c_uint8), ("reason", ctypes.c_uint8), ("fail_op", ctypes.c_uint8),
                ("msg_status", ctypes.c_uint8)]


VERDICT_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(Verdict1_C))


class Write2Request_C(ctypes.Structure):
    """mochi_write2_request (ABI 3)."""
    _fields_ = [("msg", ctypes.c_void_p), ("msg_len", ctypes.c_uint32), ("n_ops", ctypes.c_uint32),
                ("op_flags", ctypes.c_void_p), ("op_object_ts", ctypes.c_void_p), ("expected_hash", ctypes.c_void_p),
                ("op_decision", ctypes.c_void_p), ("op_g0", ctypes.c_void_p), ("op_ts", ctypes.c_void_p)]


class Write2Request:
    """One Write2ToServer as a server receives it, with its per-op state
    (MOCHI_OP_* flags, stored-certificate timestamps) and per-op outputs
    (decision, g0, g0's timestamp) — the buffers live as long as this object."""

    def __init__(self, msg: bytes, expected_hash: bytes, op_flags: Optional[Sequence[int]] = None,
                 op_object_ts: Optional[Sequence[int]] = None, want_ops: bool = True):
        self.msg = np.frombuffer(bytes(msg) or b"\x00", np.uint8).copy()
        self.msg_len = len(msg)
        self.expected_hash = np.frombuffer(bytes(expected_hash), np.uint8).copy()
        assert self.expected_hash.shape[0] == TXN_HASH_BYTES
        n = 0 if op_flags is None else len(op_flags)
        self.op_flags = None if op_flags is None else np.asarray(op_flags, np.uint8).copy()
        self.op_object_ts = None if op_object_ts is None else np.asarray(op_object_ts, np.int64).copy()
        if self.op_object_ts is not None:
            assert self.op_object_ts.shape[0] == n
        self.op_decision = np.zeros(max(n, 1), np.uint8) if want_ops and n else None
        self.op_g0 = np.zeros(max(n, 1), np.uint32) if want_ops and n else None
        self.op_ts = np.zeros(max(n, 1), np.int64) if want_ops and n else None
        self.c = Write2Request_C(_ptr(self.msg), self.msg_len, n, _ptr(self.op_flags), _ptr(self.op_object_ts),
                                 _ptr(self.expected_hash), _ptr(self.op_decision), _ptr(self.op_g0), _ptr(self.op_ts))
        self.result = None  # (rc, accepted, reason, fail_op, msg_status) once delivered

    def ops(self):
        """[(decision, g0, ts)] per op (after the verdict)."""
        if self.op_decision is None:
            return []
        n = self.c.n_ops
        return [(int(self.op_decision[i]), int(self.op_g0[i]), int(self.op_ts[i])) for i in range(n)]


class Batcher:
    """mochi_batcher: blocking per-request verify, coalesced across calling threads.
    (ctypes drops the GIL during the call, so Python threads block concurrently.)"""

    def __init__(self, verifier, replication_factor: int, strict_gt: bool = True, max_msgs: int = 4096,
                 max_wait_us: int = 200, with_op_flags: bool = False):
        # verifier: a Verifier, or a list of them (one flusher, i.e. one batch in
        # flight, per context: mochi_batcher_create_multi)
        vers = list(verifier) if isinstance(verifier, (list, tuple)) else [verifier]
        self.lib = vers[0].lib
        self._ver = vers
        self._p = params(replication_factor, strict_gt)
        self.with_op_flags = with_op_flags
        self._ctxs = (ctypes.c_void_p * len(vers))(*[v.ctx for v in vers])
        self.h = self.lib.mochi_batcher_create_multi(self._ctxs, len(vers), ctypes.addressof(self._p), max_msgs,
                                                     max_wait_us, 1 if with_op_flags else 0)
        if not self.h:
            raise MochiError("mochi_batcher_create failed")
        # mochi_batcher_submit: requests in flight keyed by the callback's user word
        import itertools

        self._seq = itertools.count(1)
        self._pending = {}
        self._cb = VERDICT_CB(self._on_done)

    def _on_done(self, user, rc, v):
        _, _, _, done = self._pending.pop(user)
        d = v.contents
        done(rc, bool(d.accepted), d.reason, d.fail_op, d.msg_status)

    def submit(self, msg: bytes, expected_hash: bytes, done, op_flags: Optional[bytes] = None):
        """Non-blocking (mochi_batcher_submit): done(rc, accepted, reason, fail_op,
        msg_status) runs on a flusher thread once the message's batch is verified."""
        if not self.h:
            raise MochiError("batcher closed")
        key = next(self._seq)
        self._pending[key] = (msg, expected_hash, op_flags, done)  # alive until the callback
        fl = op_flags if op_flags is not None else None
        rc = self.lib.mochi_batcher_submit(self.h, msg, len(msg), fl, len(fl) if fl else 0, expected_hash, self._cb,
                                           key)
        if rc != OK:
            self._pending.pop(key, None)
            raise MochiError(f"mochi_batcher_submit rc={rc}")

    def verify(self, msg: bytes, expected_hash: bytes, op_flags: Optional[bytes] = None):
        out = Verdict1_C()
        fl = op_flags if op_flags is not None else None
        rc = self.lib.mochi_batcher_verify(self.h, msg, len(msg), fl, len(fl) if fl else 0, expected_hash,
                                           ctypes.byref(out))
        if rc != OK:
            raise MochiError(f"mochi_batcher_verify rc={rc}: {_err(self.lib)}")
        return bool(out.accepted), out.reason, out.fail_op, out.msg_status

    def verify_request(self, req: "Write2Request"):
        """mochi_batcher_verify_request: blocks; fills req's per-op outputs."""
        out = Verdict1_C()
        rc = self.lib.mochi_batcher_verify_request(self.h, ctypes.byref(req.c), ctypes.byref(out))
        if rc != OK:
            raise MochiError(f"mochi_batcher_verify_request rc={rc}: {_err(self.lib)}")
        req.result = (rc, bool(out.accepted), out.reason, out.fail_op, out.msg_status)
        return req.result[1:]

    def submit_request(self, req: "Write2Request", done):
        """mochi_batcher_submit_request: done(req) runs on a flusher thread once
        req.result and its per-op outputs are set."""
        key = next(self._seq)

        def fin(rc, accepted, reason, fail_op, msg_status):
            req.result = (rc, accepted, reason, fail_op, msg_status)
            done(req)

        self._pending[key] = (req, None, None, fin)
        rc = self.lib.mochi_batcher_submit_request(self.h, ctypes.byref(req.c), self._cb, key)
        if rc != OK:
            self._pending.pop(key, None)
            raise MochiError(f"mochi_batcher_submit_request rc={rc}")

    def stats(self):
        b, m = ctypes.c_uint64(), ctypes.c_uint64()
        self.lib.mochi_batcher_stats(self.h, ctypes.byref(b), ctypes.byref(m))
        return b.value, m.value

    def close(self):
        """mochi_batcher_destroy, once.  From one of this batcher's callbacks the
        library defers the teardown (queued requests still complete; its last
        flusher frees it); the handle is dropped here either way, so a later
        close() / __del__ cannot free the batcher a second time.  The library
        holds the contexts until the batcher is freed (a mochi_ctx_destroy before that
        returns at once and the batcher's release frees the context)."""
        h, self.h = self.h, None
        if h:
            self.lib.mochi_batcher_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 -- interpreter teardown
            pass


class DeviceSigner:
    """Producer-side SHA256withRSA on the device with one server's private key
    (mochi_signer_*; bit-identical to sign_grants / OpenSSL)."""

    def __init__(self, pem_private_key: bytes, device: int = 0):
        self.lib = load_library()
        self.h = self.lib.mochi_signer_create(int(device), pem_private_key)
        if not self.h:
            raise MochiError(f"mochi_signer_create: {_err(self.lib)}")

    def sign(self, grant_bytes: np.ndarray, grant_off: np.ndarray, grant_len: np.ndarray) -> np.ndarray:
        blob = np.ascontiguousarray(grant_bytes, np.uint8)
        off = np.ascontiguousarray(grant_off, np.uint64)
        ln = np.ascontiguousarray(grant_len, np.uint32)
        n = int(off.shape[0])
        out = np.zeros((n, RSA_BYTES), np.uint8)
        rc = self.lib.mochi_sign_batch(self.h, _ptr(blob), blob.nbytes, _ptr(off), _ptr(ln), n, _ptr(out))
        if rc != OK:
            raise MochiError(f"mochi_sign_batch rc={rc}: {_err(self.lib)}")
        return out

    def sign_device(self, blob_t, off_t, len_t, n: int, sig_t, stream: int = 0) -> None:
        rc = self.lib.mochi_sign_batch_device(self.h, blob_t.data_ptr(), off_t.data_ptr(), len_t.data_ptr(), n,
                                              sig_t.data_ptr(), stream)
        if rc != OK:
            raise MochiError(f"mochi_sign_batch_device rc={rc}: {_err(self.lib)}")

    def rejected(self) -> int:
        """Signatures withheld by the public-key fault check since the last call."""
        v = ctypes.c_uint64()
        if self.lib.mochi_signer_rejected(self.h, ctypes.byref(v)) != OK:
            raise MochiError(f"mochi_signer_rejected: {_err(self.lib)}")
        return v.value

    def set_fault(self, grant_index: int) -> None:
        """Test hook: corrupt one CRT half of grant `grant_index` (-1 = off)."""
        self.lib.mochi_signer_set_fault(self.h, grant_index & 0xFFFFFFFF)

    def close(self):
        if self.h:
            self.lib.mochi_signer_destroy(self.h)
            self.h = None



# ---------------------------------------------------------------------------
# Multi-GPU (include/mochi_hip.h)
# ---------------------------------------------------------------------------
def shard_plan(n_certs: int, n_shards: int, cert_grant_off: Optional[np.ndarray] = None) -> np.ndarray:
    """Contiguous 32-aligned certificate shards (mochi_shard_plan): cert_lo[n_shards+1]."""
    lib = load_library()
    out = np.zeros(n_shards + 1, np.uint32)
    cgo = None if cert_grant_off is None else np.ascontiguousarray(cert_grant_off, np.uint32)
    if lib.mochi_shard_plan(n_certs, _ptr(cgo), n_shards, _ptr(out)) != OK:
        raise MochiError("mochi_shard_plan failed")
    return out


def shard_words(cert_lo: np.ndarray) -> int:
    lo = np.ascontiguousarray(cert_lo, np.uint32)
    return int(load_library().mochi_shard_words(lo.shape[0] - 1, _ptr(lo)))


def bits_assemble(cert_lo: np.ndarray, gathered: np.ndarray) -> np.ndarray:
    """The batch's accept bitmap from the all-gathered per-shard slots (mochi_bits_assemble)."""
    lo = np.ascontiguousarray(cert_lo, np.uint32)
    g = np.ascontiguousarray(gathered, np.uint32)
    n = lo.shape[0] - 1
    out = np.zeros(max(1, (int(lo[-1]) + 31) // 32), np.uint32)
    if load_library().mochi_bits_assemble(n, _ptr(lo), g.shape[0] // n, _ptr(g), _ptr(out)) != OK:
        raise MochiError("mochi_bits_assemble failed")
    return out[:(int(lo[-1]) + 31) // 32]


class MultiVerifier:
    """mochi_mctx: one process, the GPUs of device_mask, one context + host thread
    each, RCCL all-gather of the verdict bitmaps."""

    def __init__(self, moduli_be, device_mask: int):
        self.lib = load_library()
        mod = np.ascontiguousarray(np.frombuffer(b"".join(bytes(m) for m in moduli_be), np.uint8))
        self._mod = mod
        self.h = self.lib.mochi_mctx_create(device_mask, mod.ctypes.data, mod.size // RSA_BYTES, RSA_BYTES, RSA_E)
        if not self.h:
            raise MochiError(f"mochi_mctx_create: {_err(self.lib)}")
        devs = (ctypes.c_int * 64)()
        self.devices = list(devs)[:self.lib.mochi_mctx_devices(self.h, devs, 64)]

    def set_server_ids(self, server_ids) -> None:
        enc = [x.encode() if isinstance(x, str) else bytes(x) for x in server_ids]
        blob = np.frombuffer(b"".join(enc) or b"\x00", np.uint8).copy()
        off = np.zeros(len(enc) + 1, np.uint32)
        np.cumsum([len(x) for x in enc], out=off[1:])
        if self.lib.mochi_mctx_set_server_ids(self.h, _ptr(blob), _ptr(off), len(enc)) != OK:
            raise MochiError(_err(self.lib))

    def verify(self, batch: Batch, replication_factor: int, strict_gt: bool = True, quorum_mode: int = 0) -> Verdicts:
        b = batch.normalized()
        out = Verdicts.alloc(b.n_grants, b.n_certs, b.n_ops)
        bc, vc = b.to_c(), out.to_c()
        vc.grant_valid_bits = None
        p = params(replication_factor, strict_gt, quorum_mode)
        rc = self.lib.mochi_mverify_batch(self.h, ctypes.byref(bc), ctypes.byref(p), ctypes.byref(vc))
        if rc != OK:
            raise MochiError(f"mochi_mverify_batch rc={rc}: {_err(self.lib)}")
        out.grant_valid_bits = np.zeros_like(out.grant_valid_bits)
        return out

    def verify_write2(self, wb, replication_factor: int, strict_gt: bool = True, quorum_mode: int = 0):
        wc, keep = write2_batch_c(wb)
        M = wb.n_msgs
        O = int(wb.op_flags_off[-1]) if wb.op_flags_off is not None else 0
        out = Verdicts.alloc(0, M, O)
        vc = out.to_c()
        vc.grant_valid_bits = vc.grant_flags = vc.grant_ts = None
        if wb.op_flags_off is None:
            vc.op_decision = vc.op_g0 = vc.op_ts = None
        p = params(replication_factor, strict_gt, quorum_mode)
        st = np.zeros(max(M, 1), np.uint8)
        rc = self.lib.mochi_mverify_write2(self.h, ctypes.addressof(wc), ctypes.addressof(p), ctypes.addressof(vc),
                                           _ptr(st))
        if rc != OK:
            raise MochiError(f"mochi_mverify_write2 rc={rc}: {_err(self.lib)}")
        return out, st[:M].copy()

    def gathered_bits(self, i: int):
        """(device pointer, words per device slot) of device i's all-gathered buffer."""
        p, w = ctypes.c_void_p(), ctypes.c_uint32()
        if self.lib.mochi_mctx_gathered_bits(self.h, i, ctypes.byref(p), ctypes.byref(w)) != OK:
            raise MochiError(_err(self.lib))
        return p.value, w.value

    def close(self):
        if self.h:
            self.lib.mochi_mctx_destroy(self.h)
            self.h = None


class Comm:
    """mochi_comm: one process per GPU; the verdict-bitmap all-gather through librccl."""

    def __init__(self, unique_id: bytes, n_ranks: int, rank: int, device: int):
        self.lib = load_library()
        idb = ctypes.create_string_buffer(bytes(unique_id), 128)
        self.h = self.lib.mochi_comm_init(idb, n_ranks, rank, device)
        if not self.h:
            raise MochiError(f"mochi_comm_init: {_err(self.lib)}")
        self.n_ranks = n_ranks

    @staticmethod
    def unique_id() -> bytes:
        lib = load_library()
        b = ctypes.create_string_buffer(128)
        if lib.mochi_comm_unique_id(b) != OK:
            raise MochiError(f"mochi_comm_unique_id: {_err(lib)}")
        return b.raw

    def allgather_bits(self, local_t, out_t, stream: int = 0) -> None:
        """int32 torch tensors: local [W] -> out [n_ranks * W] (async on `stream`)."""
        rc = self.lib.mochi_comm_allgather_bits(self.h, local_t.data_ptr(), local_t.numel(), out_t.data_ptr(), stream)
        if rc != OK:
            raise MochiError(f"mochi_comm_allgather_bits: {_err(self.lib)}")

    def close(self):
        if self.h:
            self.lib.mochi_comm_destroy(self.h)
            self.h = None


def properties_bytes(text: str) -> bytes:
    """A str as the bytes of a properties file Properties.load(InputStream) reads
    back as that str: ISO-8859-1 for U+0000..U+00FF, a \\uXXXX escape per UTF-16
    code unit above (a supplementary character becomes its surrogate pair)."""
    out = bytearray()
    for ch in text:
        cp = ord(ch)
        if cp <= 0xFF:
            out.append(cp)
        else:
            u = ch.encode("utf-16-be", "surrogatepass")
            for i in range(0, len(u), 2):
                out += b"\\u%04X" % int.from_bytes(u[i:i + 2], "big")
    return bytes(out)


class ClusterConfig:
    """The reference's cluster properties file (mochi_config_*;
    ClusterConfiguration.loadInitialConfigurationFromProperties,
    ClusterConfiguration.java:138-187)."""

    def __init__(self, path: Optional[str] = None, text=None):
        # text: the file's bytes (read as ISO-8859-1, like Properties.load(InputStream)),
        # or a str, written the way Properties.store would: ISO-8859-1, every
        # character above U+00FF as a \\uXXXX escape (UTF-16 units), so an id given
        # as a str reads back as that same str (not its UTF-8 bytes re-read as Latin-1)
        self.lib = load_library()
        if path is not None:
            self.h = self.lib.mochi_config_load(path.encode())
        else:
            raw = text if isinstance(text, (bytes, bytearray)) else properties_bytes(text or "")
            self.h = self.lib.mochi_config_parse(raw, len(raw))
        if not self.h:
            raise MochiError(f"mochi_config: {_err(self.lib)}")

    @property
    def replication_factor(self) -> int:
        return int(self.lib.mochi_config_replication(self.h))

    @property
    def majority(self) -> int:
        return int(self.lib.mochi_config_majority(self.h))

    def servers(self):
        n = self.lib.mochi_config_n_servers(self.h)
        return [(self.lib.mochi_config_server_id(self.h, i).decode(), self.lib.mochi_config_server_url(self.h, i).decode())
                for i in range(n)]

    def servers_for_key(self, key: str):
        """getServersForObject(key): indices into servers(), replica order."""
        kb = key.encode()
        out = np.zeros(self.replication_factor, np.uint32)
        rc = self.lib.mochi_config_servers_for_key(self.h, kb, len(kb), _ptr(out))
        if rc != OK:
            raise MochiError(f"mochi_config_servers_for_key: {_err(self.lib)}")
        return [int(i) for i in out]

    def replica_ids(self, key: Optional[str] = None):
        """(ids blob, id_off[R+1]) for mochi_ctx_set_server_ids."""
        kb = key.encode() if key is not None else None
        off = np.zeros(self.replication_factor + 1, np.uint32)
        need = self.lib.mochi_config_replica_ids(self.h, kb, len(kb) if kb else 0, None, 0, _ptr(off))
        if need < 0:
            raise MochiError(f"mochi_config_replica_ids: {_err(self.lib)}")
        blob = np.zeros(max(int(need), 1), np.uint8)
        self.lib.mochi_config_replica_ids(self.h, kb, len(kb) if kb else 0, _ptr(blob), int(need), _ptr(off))
        return blob[:int(need)], off

    def replica_id_list(self, key: Optional[str] = None):
        blob, off = self.replica_ids(key)
        b = blob.tobytes()
        return [b[off[i]:off[i + 1]].decode() for i in range(len(off) - 1)]

    def close(self):
        if getattr(self, "h", None):
            self.lib.mochi_config_free(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass
