"""CPU model of k_rsa_final's check (mochi-db_amd/csrc/rsa_final.hip).

The kernel never forms s^65537 mod n: the matrix-core fold of t = z*s yields
    D = x + (n - Cpad) - H,   x == s^65537 (mod n),  0 <= x < 2^2064
(x is whatever representative the fold leaves), and the grant is valid iff
s < n and D == 0 (mod n).  One Montgomery step by 2^28,
    D' = (D + m n) / 2^28,  m = D * (-n^-1) mod 2^28,
lands in (0, 2n), so valid <=> D' == n exactly.  This test replays that limb
schedule (radix 2^28, 64-bit unsigned accumulator) in Python integers over every
OpenSSL golden vector (tests/golden/rsa_vectors.json), for the smallest, the
largest and random representatives x < 2^2064, and checks the verdict equals
OpenSSL's.  (The fold itself is pinned by tests/test_fold_cpu.py.)
"""
import hashlib
import json
import os
import random

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B, L = 28, 74
MASK = (1 << B) - 1
DIGEST_INFO = bytes.fromhex("3031300d060960864801650304020105000420")
CPAD = int.from_bytes(b"\x00\x01" + b"\xff" * 202 + b"\x00" + DIGEST_INFO + b"\x00" * 32, "big")
XMAX = 1 << 2064  # the fold's output bound (mochi-db_amd/csrc/fold.h)


def limbs(v, n=L):
    assert 0 <= v < 1 << (B * n)
    return [(v >> (B * j)) & MASK for j in range(n)]


def final_check(n, s, x_rep, h_int):
    """Limb-exact replay of k_rsa_final after the fold (x given)."""
    n0inv = (-pow(n, -1, 1 << B)) % (1 << B)
    D = x_rep + (n - CPAD) - h_int
    assert 0 < D < XMAX + n
    Dl, N = limbs(D), limbs(n)
    m = ((Dl[0] * n0inv) & 0xFFFFFFFF) & MASK
    acc = m * N[0] + Dl[0]
    assert acc & MASK == 0 and acc < 1 << 64
    c, diff = acc >> B, 0
    for k in range(1, L):
        acc = m * N[k] + Dl[k] + c
        assert acc < 1 << 64
        diff |= (acc & MASK) ^ N[k - 1]
        c = acc >> B
    diff |= int(c != N[L - 1])
    # the bound the kernel relies on: D' in (0, 2n)
    Dp = (D + m * n) >> B
    assert 0 < Dp < 2 * n
    return s < n and diff == 0


def vectors():
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "rsa_vectors.json")))
    return d["moduli"], d["vectors"]


@pytest.mark.parametrize("rep", ["min", "max", "random"])
def test_final_check_matches_openssl(rep):
    moduli, vecs = vectors()
    rng = random.Random(7)
    seen = 0
    for v in vecs:
        n = int(moduli[str(v["key"])], 16)
        sig = bytes.fromhex(v["sig"])
        if len(sig) != 256:
            continue
        s = int.from_bytes(sig, "big")
        h = int.from_bytes(hashlib.sha256(bytes.fromhex(v["msg"])).digest(), "big")
        y = pow(s, 65537, n)
        top = (XMAX - 1 - y) // n
        j = {"min": 0, "max": top, "random": rng.randrange(top + 1)}[rep]
        got = final_check(n, s, y + j * n, h)
        assert got == (v["valid"] in (True, "True")), v["name"]
        seen += 1
    assert seen > 50
