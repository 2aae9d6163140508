"""CPU model of k_rsa_final's single-multiply verify (mochi-db_amd/csrc/rsa_final.hip).

The kernel never forms s^65537 mod n: it checks A2 + H*Q - MontMul(z, s) == 0
(mod n) with one 10-limb Montgomery reduction and a limb compare against n.
This test replays that exact limb schedule (radix 2^28, signed 64-bit column
accumulator, two's-complement wrap) in Python integers over every OpenSSL
golden vector (tests/golden/rsa_vectors.json), with both representatives of z
and u in [0, 2n) the kernel may see, and checks the verdict equals OpenSSL's.
"""
import hashlib
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B, L, HL = 28, 74, 10
MASK = (1 << B) - 1
R = 1 << (B * L)
DIGEST_INFO = bytes.fromhex("3031300d060960864801650304020105000420")


def limbs(v, n=L):
    return [(v >> (B * j)) & MASK for j in range(n)]


def wrap64(v):
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >> 63 else v


def key_consts(n):
    q = pow(pow(R, 1 << 16, n), -1, n)
    cpad = int.from_bytes(b"\x00\x01" + b"\xff" * 202 + b"\x00" + DIGEST_INFO + b"\x00" * 32, "big")
    a2 = cpad * q % n + 2 * n
    n0inv = (-pow(n, -1, 1 << B)) % (1 << B)
    return q, a2, n0inv


def final_check(n, s, u_rep, h_int):
    """Limb-exact replay of k_rsa_final after the MontMul (u given)."""
    q, a2, n0inv = key_consts(n)
    N, Q, A2, U, H = limbs(n), limbs(q), limbs(a2), limbs(u_rep), limbs(h_int, HL)
    m = [0] * HL
    carry, diff = 0, 0
    for k in range(L + HL - 1):
        lo = max(0, k - (L - 1))
        acc = carry + (A2[k] - U[k] if k < L else 0)
        for i in range(lo, min(k, HL - 1) + 1):
            acc += H[i] * Q[k - i]
        for i in range(lo, min(k - 1, HL - 1) + 1):
            acc += m[i] * N[k - i]
        acc = wrap64(acc)
        assert -(1 << 62) < acc < (1 << 62)
        if k < HL:
            m[k] = ((acc & 0xFFFFFFFF) * n0inv) & MASK
            acc = wrap64(acc + m[k] * N[0])
        else:
            diff |= (acc & MASK) ^ N[k - HL]
        carry = acc >> B
    diff |= int(carry != N[L - 1])
    return s < n and diff == 0


def vectors():
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "rsa_vectors.json")))
    return d["moduli"], d["vectors"]


@pytest.mark.parametrize("bump", [0, 1])
def test_final_check_matches_openssl(bump):
    moduli, vecs = vectors()
    seen = 0
    for v in vecs:
        n = int(moduli[str(v["key"])], 16)
        sig = bytes.fromhex(v["sig"])
        if len(sig) != 256:
            continue
        s = int.from_bytes(sig, "big")
        h = int.from_bytes(hashlib.sha256(bytes.fromhex(v["msg"])).digest(), "big")
        z = pow(s, 1 << 16, n) * pow(pow(R, (1 << 16) - 1, n), -1, n) % n
        u = z * s * pow(R, -1, n) % n
        u_rep = u + n * bump  # MontMul leaves u anywhere in [0, 2n)
        got = final_check(n, s, u_rep, h)
        assert got == (v["valid"] in (True, "True")), v["name"]
        seen += 1
    assert seen > 50
