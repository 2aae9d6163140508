"""Build mochi_hip.Batch objects from tests/golden/cert_cases.json specs."""
from __future__ import annotations

import hashlib
import json
import os
from dataclasses import dataclass
from typing import Dict, List, Tuple

import numpy as np

import oracle_ffi as O
from mochi_hip import Batch
from workload import encode_grant, load_keys

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_cases() -> List[dict]:
    with open(os.path.join(GOLDEN, "cert_cases.json")) as f:
        return json.load(f)


def case_hashes(name: str) -> Dict[str, str]:
    good = hashlib.sha512(f"case-{name}".encode()).hexdigest()
    evil = hashlib.sha512(f"case-{name}-evil".encode()).hexdigest()
    return {"good": good, "evil": evil, "short": good[:127]}


def uses_explicit_mgs(case: dict) -> bool:
    return "n_mgs" in case or any(len(g) > 6 and "mg" in g[6] for g in case["grants"])


def case_multigrants(case: dict) -> List[int]:
    """Grants per MultiGrant: explicit "mg" indices / "n_mgs", else maximal runs of one server."""
    grants = case["grants"]
    if uses_explicit_mgs(case):
        n = case.get("n_mgs", 0)
        idx = [g[6]["mg"] for g in grants]
        n = max([n] + [i + 1 for i in idx])
        assert idx == sorted(idx), "MultiGrants must be contiguous in wire order"
        return [idx.count(m) for m in range(n)]
    runs: List[int] = []
    for i, g in enumerate(grants):
        if i == 0 or g[0] != grants[i - 1][0]:
            runs.append(0)
        runs[-1] += 1
    return runs


@dataclass
class Expect:
    reason: np.ndarray  # [C]
    fail_op: np.ndarray  # [C]
    decisions: np.ndarray  # [O]
    g0: np.ndarray  # [O] uint32 (0xFFFFFFFF none)
    op_ts: np.ndarray  # [O]


def build_case_batch(cases: List[dict], pems: List[bytes], explicit_mg: bool = True) -> Tuple[Batch, Expect]:
    """Concatenate cases into one batch.  explicit_mg=False leaves cert_mg_off / mg_grant_off NULL
    (the library then takes each run of one signer as a MultiGrant)."""
    blob = bytearray()
    goff, glen, sigs, signer, gkey = [], [], [], [], []
    cgo, coo, opk, opf, ots, exp = [0], [0], [], [], [], []
    cmo, mgo = [0], [0]
    key_slices = []  # (op index, slot) -> op key bytes appended after the grants
    for c in cases:
        h = case_hashes(c["name"])
        for spec in c["grants"]:
            server, slot, ts, hname, sigq, bq = spec[:6]
            extra = spec[6] if len(spec) > 6 else {}
            g = encode_grant(f"CASE_KEY_{extra.get('oid', slot)}", ts, h[hname])
            if bq == "malformed":
                g = g + b"\x0f"  # wire type 7: DecodeError
            # misalign every other grant on purpose (zero-copy slices are unaligned)
            if len(blob) % 2 == 0:
                blob += b"\xee"
            goff.append(len(blob))
            glen.append(len(g))
            blob += g
            s = bytearray(O.rsa_sign(pems[server], g))
            if sigq == "bad":
                s[100] ^= 0x10
            sigs.append(bytes(s))
            signer.append(server)
            gkey.append(slot)
        cgo.append(len(goff))
        for n in case_multigrants(c):
            mgo.append(mgo[-1] + n)
        cmo.append(len(mgo) - 1)
        for op in c["ops"]:
            key_slices.append((len(opk), op[0]))
            opk.append(op[0])
            opf.append(op[1])
            ots.append(op[2] if len(op) > 2 else 0)
        coo.append(len(opk))
        exp.append(np.frombuffer(h["good"].encode(), np.uint8))
    okoff, oklen = [], []
    for _, slot in key_slices:
        k = f"CASE_KEY_{slot}".encode()
        okoff.append(len(blob))
        oklen.append(len(k))
        blob += k
    batch = Batch(
        grant_bytes=np.frombuffer(bytes(blob) if blob else b"\0", np.uint8).copy(),
        grant_off=np.asarray(goff, np.uint64),
        grant_len=np.asarray(glen, np.uint32),
        sig=np.frombuffer(b"".join(sigs), np.uint8).reshape(-1, 256).copy() if sigs else np.zeros((0, 256), np.uint8),
        signer=np.asarray(signer, np.uint16),
        grant_key=np.asarray(gkey, np.uint8),
        cert_grant_off=np.asarray(cgo, np.uint32),
        cert_op_off=np.asarray(coo, np.uint32),
        op_key=np.asarray(opk, np.uint8),
        op_flags=np.asarray(opf, np.uint8),
        expected_hash=np.stack(exp) if exp else np.zeros((0, 128), np.uint8),
        cert_mg_off=np.asarray(cmo, np.uint32) if explicit_mg else None,
        mg_grant_off=np.asarray(mgo, np.uint32) if explicit_mg else None,
        op_object_ts=np.asarray(ots, np.int64),
        op_key_off=np.asarray(okoff, np.uint64),
        op_key_len=np.asarray(oklen, np.uint32),
    )
    dec, g0, ts = [], [], []
    for c in cases:
        dec += c["decisions"]
        for x in c["g0"]:
            g0.append(0xFFFFFFFF if x < 0 else x)
            ts.append(0 if x < 0 else c["grants"][x][2])
    ex = Expect(reason=np.asarray([c["reason"] for c in cases], np.uint8),
                fail_op=np.asarray([c["fail_op"] for c in cases], np.uint8),
                decisions=np.asarray(dec, np.uint8), g0=np.asarray(g0, np.uint32), op_ts=np.asarray(ts, np.int64))
    return batch, ex


def grouped_cases(explicit_mg: bool = True):
    """Cases grouped by (R, strict, quorum_mode) since params are per batch; explicit_mg=False keeps only
    the cases whose MultiGrants are runs of one signer (the library's default when the CSR is NULL)."""
    groups: Dict[Tuple[int, int, int], List[dict]] = {}
    for c in load_cases():
        if not explicit_mg and uses_explicit_mgs(c):
            continue
        groups.setdefault((c["R"], c["strict"], c.get("quorum_mode", 0)), []).append(c)
    return groups


def moduli_for(R: int) -> List[bytes]:
    return [O.pem_modulus(p) for p in load_keys(R)]
