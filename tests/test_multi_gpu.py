"""The multi-GPU entry points of libmochi_hip on the GPU box (which has one GPU):
mochi_mctx over device_mask = every visible device, and mochi_comm with one rank.
With one device the RCCL all-gather is the identity, but the whole path runs --
shard plan, per-device worker thread, ncclCommInitAll / ncclCommInitRank,
ncclAllGather, bitmap assembly -- and must give exactly the single-context
verdicts (which test_gpu_parity pins to the oracle)."""
import numpy as np
import pytest

import mochi_hip as mh
import oracle_ffi as O
import workload as W

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pool4():
    return W.build_pool(R=4, k=1, P=512, P_f=64)


def _mask():
    import torch

    return (1 << torch.cuda.device_count()) - 1


def test_mctx_batch_equals_single_context(pool4):
    s = W.make_batch(pool4, 5000, first_cert=31)
    mv = mh.MultiVerifier(pool4.moduli, _mask())
    assert mv.devices
    g = mv.verify(s.batch, 4, True)
    one = mh.Verifier(pool4.moduli, 0)
    r = one.verify(s.batch, 4, True)
    for k in ("grant_flags", "grant_ts", "cert_accept_bits", "cert_reason", "cert_fail_op", "op_decision", "op_g0",
              "op_ts"):
        np.testing.assert_array_equal(getattr(g, k), getattr(r, k), err_msg=k)
    o = O.verify_batch(pool4.moduli, s.batch, 4, True, 8)
    np.testing.assert_array_equal(g.cert_accept_bits, o.cert_accept_bits)
    # every device holds the gathered bitmap
    import torch

    ptr, words = mv.gathered_bits(0)
    assert ptr and words * len(mv.devices) >= (5000 + 31) // 32
    mv.close()
    one.close()


def test_mctx_write2_equals_single_context(pool4):
    s = W.make_batch(pool4, 1500, first_cert=901)
    wb = W.encode_wire_batch(s)
    mv = mh.MultiVerifier(pool4.moduli, _mask())
    mv.set_server_ids(W.SERVER_IDS[:4])
    g, st = mv.verify_write2(wb, 4, False)
    ids, off = W.server_id_table(4)
    o, ost = O.verify_write2(pool4.moduli, ids, off, wb, 4, False)
    np.testing.assert_array_equal(st, ost)
    np.testing.assert_array_equal(g.cert_accept_bits, o.cert_accept_bits)
    np.testing.assert_array_equal(g.cert_reason, o.cert_reason)
    np.testing.assert_array_equal(g.op_decision, o.op_decision)
    mv.close()


def test_comm_single_rank_allgather():
    import torch

    uid = mh.Comm.unique_id()
    assert len(uid) == 128
    c = mh.Comm(uid, 1, 0, 0)
    src = torch.arange(37, dtype=torch.int32, device="cuda") * 7 + 3
    dst = torch.zeros(37, dtype=torch.int32, device="cuda")
    c.allgather_bits(src, dst, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(src, dst)
    c.close()
