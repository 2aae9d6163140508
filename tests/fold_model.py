"""Test infrastructure: Python model of k_rsa_pow's fold squaring
(mochi-db_amd/csrc/rsa_pow.hip, csrc/fold.h; prototype microbench/fold_pow.hip).

One squaring step for a value x < 2^2064 held as 74 limbs of 28 bits:

    t = x^2                                   (148 limbs, VALU product scanning)
    x' = t_lo + sum_{j,b} byte_b(t_hi_j) * R_{j,b}     R_{j,b} = 2^(28*(73+j)+8b) mod n

t_lo = limbs 0..72, t_hi = limbs 73..147.  The sum over the 300 bytes of t_hi is a
[signature x 300] x [300 x 296] int8 GEMM on the matrix cores: the weights are the
balanced mixed-radix digits of every R_{j,b} (three signed bytes and a signed
nibble per 28-bit limb), the signature side is the raw bytes biased by -128.
Bound: fold < 75 * (3*255 + 15) * n < 2^15.84 * 2^2048, so x' < 2^2064 again.

This module builds the weight image in the exact per-lane MFMA fragment order
and replays the arithmetic with Python ints.  Checked against the library's
mochi_fold_matrix and against pow() in tests/test_fold_cpu.py.
"""
# Round 3: the product is one level of Karatsuba (kara_terms) and leaves the
# limbs 37..111 signed and unnormalised; the fold takes each t_hi limb as an
# int32 whose low three bytes are biased (XOR 0x80) and whose top byte is a
# signed digit, and cadd carries 128 * sum_{j, b<3} R_{j,b} + 2401 n (the
# multiple of n keeps x' > 0 whatever the signs).
import numpy as np

L = 74          # limbs of x (2072 bits)
F = 73          # fold point: t_lo = limbs [0, 73)
NH = 75         # t_hi limbs 73..147
KSTEPS = 10     # 8 limbs (32 bytes) per K-step, 80 limb slots >= 75
MTILES = 10     # 8 output limbs per M-tile, 80 >= 74
M28 = (1 << 28) - 1


def balanced_digits(v):
    """v (>= 0, < 2^2052) -> digits d[q][s] (q < 74 limbs, s < 4 slots) with
    v = sum d[q][s] * 2^(28q + 8s), d in [-128,127] (s<3) / [-8,7] (s=3)."""
    d = np.zeros((L, 4), np.int64)
    for q in range(L):
        for s, w in enumerate((8, 8, 8, 4)):
            r = v & ((1 << w) - 1)
            if r >= 1 << (w - 1):
                r -= 1 << w
            d[q, s] = r
            v = (v - r) >> w
    assert v == 0
    return d


HALF = 37        # Karatsuba split: x = x_lo + 2^(28*37) x_hi
BIAS_MASK = 0x00808080  # t_hi bytes 0..2 biased to signed, byte 3 a signed digit
OFF_N = 2401     # cadd's multiple of n: top digits >= -32 (|t_j| < 2^29) and t_lo > -n


def cadd_value(n):
    """sum_{j, b<3} 128 R_{j,b} + OFF_N n: the bias of bytes 0..2 added back, plus
    a multiple of n that keeps x' positive whatever the signed limbs."""
    return 128 * sum(pow(2, 28 * (F + j) + 8 * b, n) for j in range(NH) for b in range(3)) + OFF_N * n


def make_weights(n):
    """Weight image int8 [MTILES][KSTEPS][64 lanes][16], cadd uint32 [74], W."""
    W = np.zeros((L * 4, NH * 4), np.int64)  # [out row (q,s)][k (j,b)]
    for j in range(NH):
        for b in range(4):
            R = pow(2, 28 * (F + j) + 8 * b, n)
            W[:, 4 * j + b] = balanced_digits(R).reshape(-1)
    img = np.zeros((MTILES, KSTEPS, 64, 16), np.int8)
    for mt in range(MTILES):
        for ks in range(KSTEPS):
            for lane in range(64):
                r, h = lane & 31, lane >> 5
                row = mt * 32 + r
                for jj in range(16):
                    limb = 8 * ks + 4 * h + jj // 4
                    if row < L * 4 and limb < NH:
                        img[mt, ks, lane, jj] = W[row, 4 * limb + jj % 4]
    ctot = cadd_value(n)
    assert ctot < 1 << (28 * L)
    cadd = np.array(to_limbs(ctot), np.uint32)
    return img, cadd, W


def _columns(a, b, sqr):
    """Product-scanning column sums of a*b (a*a with the cross products counted
    once and doubled when sqr), normalised through the kernel's 64-bit carry chain."""
    na = len(a)
    out, carry = [], 0
    for k in range(2 * na - 1):
        lo, hi = max(0, k - na + 1), min(k, na - 1)
        if sqr:
            # kara_dev.h half_square: the lower index of every cross product is
            # read doubled (a_i is doubled in place after column 2i), the square
            # term joins the chain; every operand fits 32 bits, every partial
            # sum 64 bits (the chain only grows, so the final check covers it)
            acc = carry
            for i in range(lo, (k - 1) // 2 + 1):
                if i < k - i:
                    assert 2 * a[i] < 1 << 32 and a[k - i] < 1 << 32
                    acc += (2 * a[i]) * a[k - i]
            if k % 2 == 0:
                acc += a[k // 2] * a[k // 2]
        else:
            acc = carry + sum(a[i] * b[k - i] for i in range(lo, hi + 1))
        assert acc < 1 << 64, "column sum overflows the 64-bit accumulator"
        out.append(acc & M28)
        carry = acc >> 28
    out.append(carry & M28)
    out.append(carry >> 28)
    return out  # 2 na + 1 limbs (the last one is zero unless the operands exceed 28 bits)


def kara_terms(a, b=None):
    """t = a*b (a*a if b is None), 74-limb operands, as 148 signed limbs: the
    kernel's one-level Karatsuba with its order of operations (M into t[37..111],
    then the L and H chains in lockstep, t_k = Q_k + M_(k-37) - Q_(k-37) with
    Q = L - 2^(28*37) H) and no normalisation of the combination, t[37..111] in
    (-2^29, 2^29)."""
    sqr = b is None
    a0, a1 = list(a[:HALF]), list(a[HALF:])
    if sqr:
        S = [a0[i] + a1[i] for i in range(HALF)]
        M = _columns(S, None, True)
        Lw = _columns(a0, None, True)
        Hw = _columns(a1, None, True)
    else:
        b0, b1 = list(b[:HALF]), list(b[HALF:])
        M = _columns([a0[i] + a1[i] for i in range(HALF)], [b0[i] + b1[i] for i in range(HALF)], False)
        Lw = _columns(a0, b0, False)
        Hw = _columns(a1, b1, False)
    assert len(M) == 75 and Lw[74] == 0 and Hw[74] == 0
    t = [0] * (2 * L)
    for k in range(75):          # M_k -> t[37 + k]
        t[HALF + k] = M[k]
    for c in range(3 * HALF):    # step c: L column c beside H column c - 37
        if c < HALF:             # Q_c = L_c
            t[c] = Lw[c]
            t[HALF + c] -= Lw[c]
        elif c < L:              # Q_c = L_c - H_(c-37), used twice
            q = Lw[c] - Hw[c - HALF]
            t[c] += q
            t[HALF + c] -= q
        else:                    # Q_c = -H_(c-37); t_(c+37) = H_(c-37)
            m = c - HALF
            t[c] -= Hw[m]
            if m == HALF:
                t[HALF + c] += Hw[m]
            else:
                t[HALF + c] = Hw[m]
    assert all(-(1 << 29) < v < (1 << 29) for v in t)
    av, bv = from_limbs(a), from_limbs(a if sqr else b)
    assert sum(v << (28 * k) for k, v in enumerate(t)) == av * bv
    return t


def fold_signed(t, W, cadd, sub_h=None):
    """x' = t_lo + fold(t_hi) + cadd (- h): the kernel's fold of signed limbs."""
    t_lo, t_hi = t[:F], t[F:]
    kb = []
    for j in range(NH):
        v = t_hi[j] & 0xFFFFFFFF
        for bb in range(4):
            byte = (v >> (8 * bb)) & 0xFF
            kb.append(byte - 128 if bb < 3 else (byte - 256 if byte >= 128 else byte))
    c = (W @ np.array(kb, np.int64)).reshape(L, 4)
    assert np.abs(c).max() < 2 ** 31
    out, carry = [], 0
    for q in range(L):
        p = int(c[q, 0]) + (int(c[q, 1]) << 8) + (t_lo[q] if q < F else 0) + int(cadd[q]) \
            - (sub_h[q] if sub_h and q < len(sub_h) else 0)
        h = int(c[q, 2]) + (int(c[q, 3]) << 8)
        assert -2 ** 31 <= p < 2 ** 31 and -2 ** 31 <= h < 2 ** 31  # the kernel's int32 halves
        v = (h << 16) + p + carry
        out.append(v & M28)
        carry = v >> 28
    assert carry == 0
    return out


def to_limbs(v, n=L):
    return [(v >> (28 * i)) & M28 for i in range(n)]


def from_limbs(x):
    return sum(int(l) << (28 * i) for i, l in enumerate(x))


def fold_square(x, W, cadd):
    """One step on limbs, the kernel's arithmetic exactly (Karatsuba x^2, signed
    limbs, int8 bias of bytes 0..2 included)."""
    return fold_signed(kara_terms(x), W, cadd)


def self_check(seed=1, iters=16):
    import random
    rnd = random.Random(seed)
    n = rnd.getrandbits(2048) | (1 << 2047) | 1
    _, cadd, W = make_weights(n)
    s = rnd.randrange(n)
    x = to_limbs(s)
    for _ in range(iters):
        x = fold_square(x, W, cadd)
        assert from_limbs(x) < 1 << 2064
    assert from_limbs(x) % n == pow(s, 1 << iters, n)
    return True


if __name__ == "__main__":
    print(self_check())
