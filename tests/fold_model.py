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
    # bias correction: sum_k 128 * R_k, added once as a normalised 74-limb number
    # (the -128 bias of every t_hi byte removes exactly 128 * R_k per k)
    ctot = 128 * sum(pow(2, 28 * (F + j) + 8 * b, n) for j in range(NH) for b in range(4))
    assert ctot < 1 << (28 * L)
    cadd = np.array(to_limbs(ctot), np.uint32)
    return img, cadd, W


def to_limbs(v, n=L):
    return [(v >> (28 * i)) & M28 for i in range(n)]


def from_limbs(x):
    return sum(int(l) << (28 * i) for i, l in enumerate(x))


def fold_square(x, W, cadd):
    """One step on limbs, the kernel's arithmetic exactly (int8 bias included)."""
    xv = from_limbs(x)
    t = to_limbs(xv * xv, 2 * L)
    t_lo, t_hi = t[:F], t[F:]
    kb = np.array([((t_hi[j] >> (8 * b)) & 0xFF) - 128 for j in range(NH) for b in range(4)], np.int64)
    c = (W @ kb).reshape(L, 4)  # raw MFMA columns
    assert np.abs(c).max() < 2 ** 31
    out, carry = [], 0
    for q in range(L):
        p = int(c[q, 0]) + (int(c[q, 1]) << 8) + (t_lo[q] if q < F else 0) + int(cadd[q])
        h = int(c[q, 2]) + (int(c[q, 3]) << 8)
        assert -2 ** 31 <= p < 2 ** 31 and -2 ** 31 <= h < 2 ** 31  # the kernel's int32 halves
        v = (h << 16) + p + carry
        out.append(v & M28)
        carry = v >> 28
    assert carry == 0
    return out


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
