"""k_rsa_pow's fold squaring (csrc/fold.h) on the CPU: the library's fold matrix
(mochi_fold_matrix, the one every context uploads) equals the Python model's,
and the model's exact arithmetic -- int8 bias, balanced digits, int32 column
sums, carry chain -- computes s^(2^16) mod n while staying below 2^2064, also
from the worst-case input 2^2064 - 1."""
import random

import numpy as np
import pytest

import fold_model as FM
import mochi_hip as mh


def _moduli():
    rnd = random.Random(2024)
    out = [rnd.getrandbits(2048) | (1 << 2047) | 1 for _ in range(2)]
    out.append((1 << 2048) - 1)               # all-ones modulus
    out.append((1 << 2047) | 1)               # smallest 2048-bit odd modulus
    return out


@pytest.mark.parametrize("idx", range(4))
def test_fold_matrix_matches_model(idx):
    n = _moduli()[idx]
    img, cadd = mh.fold_matrix(n.to_bytes(256, "big"))
    img_m, cadd_m, W = FM.make_weights(n)
    np.testing.assert_array_equal(img, img_m)
    np.testing.assert_array_equal(cadd, cadd_m)
    assert np.abs(W).max() <= 128 and np.abs(W.reshape(74, 4, -1)[:, 3]).max() <= 8


@pytest.mark.parametrize("idx", range(4))
def test_fold_chain_is_s_pow_2_16(idx):
    n = _moduli()[idx]
    _, cadd, W = FM.make_weights(n)
    rnd = random.Random(idx)
    for s in (0, 1, n - 1, rnd.randrange(n), (1 << 2048) - 1):  # s >= n still runs (verdict rejects it)
        x = FM.to_limbs(s)
        for _ in range(16):
            x = FM.fold_square(x, W, cadd)
            assert FM.from_limbs(x) < 1 << 2064 and max(x) < 1 << 28
        assert FM.from_limbs(x) % n == pow(s, 1 << 16, n)


def test_fold_worst_case_input():
    n = _moduli()[0]
    _, cadd, W = FM.make_weights(n)
    x = FM.to_limbs((1 << 2064) - 1)
    y = FM.fold_square(x, W, cadd)
    assert FM.from_limbs(y) < 1 << 2064
    assert FM.from_limbs(y) % n == pow((1 << 2064) - 1, 2, n)


def test_fold_matrix_rejects_bad_modulus():
    with pytest.raises(mh.MochiError):
        mh.fold_matrix(((1 << 2047) + 2).to_bytes(256, "big"))  # even
    with pytest.raises(mh.MochiError):
        mh.fold_matrix((12345).to_bytes(256, "big"))             # not 2048 bits
