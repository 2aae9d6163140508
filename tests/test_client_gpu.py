"""Client-side aggregation on the device: MochiDBClient's Read /
Write2 response tally (MochiDBClient.java:148-175, 355-382) and Write1 round
classification (:195-219, 236-332), batched across thousands of in-flight
transactions -- bit-exact with the oracle restatement (and with the host C++)."""
import numpy as np
import pytest

import mochi_hip as mh
import oracle_ffi as O
from test_capi_cpu import _random_responses, _random_write1

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("R", [4, 5, 7])
def test_tally_responses_device_matches_oracle(R):
    rng = np.random.default_rng(4321 + R)
    resps, n_ops = _random_responses(rng, 20000)
    a1, r1, c1 = mh.tally_responses_device(resps, n_ops, R)
    a2, r2, c2 = O.tally_responses(resps, n_ops, R)
    np.testing.assert_array_equal(a1, a2)
    np.testing.assert_array_equal(r1, r2)
    for x, y in zip(c1, c2):
        np.testing.assert_array_equal(x, y)
    assert set(np.unique(r1).tolist()) == {0, 1, 2}


def test_tally_responses_device_reference_semantics():
    acc, why, ch = mh.tally_responses_device([[[0], [0], [0], [0]], [[0], [1], [0], [1]], [[0, 0], [0]]], [1, 1, 2], 4)
    assert acc.tolist() == [True, False, False]
    assert why.tolist() == [0, 2, 1]
    assert ch[0][0] == 3 and ch[1][0] == 2


def test_write1_classify_device_matches_oracle():
    rng = np.random.default_rng(78)
    reqs = _random_write1(rng, 20000)
    got = mh.write1_classify_device(reqs)
    np.testing.assert_array_equal(got, O.write1_classify(reqs))
    np.testing.assert_array_equal(got, mh.write1_classify(reqs))
    assert set(np.unique(got).tolist()) == {0, 1, 2, 3, 4}


def test_client_device_empty():
    acc, why, ch = mh.tally_responses_device([], [], 4)
    assert acc.size == 0
    assert mh.write1_classify_device([]).size == 0
