"""Build mochi_hip.Batch objects from tests/golden/cert_cases.json specs."""
from __future__ import annotations

import hashlib
import json
import os
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


def build_case_batch(cases: List[dict], pems: List[bytes]) -> Tuple[Batch, np.ndarray, np.ndarray]:
    """Concatenate cases into one batch; returns (batch, expected_reason, expected_fail_op)."""
    blob = bytearray()
    goff, glen, sigs, signer, gkey = [], [], [], [], []
    cgo, coo, opk, opf, exp = [0], [0], [], [], []
    for c in cases:
        h = case_hashes(c["name"])
        for (server, slot, ts, hname, sigq, bq) in c["grants"]:
            g = encode_grant(f"CASE_KEY_{slot}", ts, h[hname])
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
        for slot, fl in c["ops"]:
            opk.append(slot)
            opf.append(fl)
        coo.append(len(opk))
        exp.append(np.frombuffer(h["good"].encode(), np.uint8))
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
    )
    return batch, np.asarray([c["reason"] for c in cases], np.uint8), np.asarray([c["fail_op"] for c in cases], np.uint8)


def grouped_cases():
    """Cases grouped by (R, strict) since params are per batch."""
    groups: Dict[Tuple[int, int], List[dict]] = {}
    for c in load_cases():
        groups.setdefault((c["R"], c["strict"]), []).append(c)
    return groups


def moduli_for(R: int) -> List[bytes]:
    return [O.pem_modulus(p) for p in load_keys(R)]
