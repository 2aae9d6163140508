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


def test_mverify_write2_rejects_grant_level_outputs(pool4):
    """Like mochi_verify_write2 (check_write2_header), the multi-device wire path
    produces no grant-level outputs and says so instead of leaving them unwritten."""
    import ctypes

    s = W.make_batch(pool4, 64, first_cert=77)
    wb = W.encode_wire_batch(s)
    mv = mh.MultiVerifier(pool4.moduli, _mask())
    mv.set_server_ids(W.SERVER_IDS[:4])
    wc, keep = mh.write2_batch_c(wb)
    out = mh.Verdicts.alloc(s.batch.n_grants, wb.n_msgs, int(wb.op_flags_off[-1]))
    vc = out.to_c()  # grant_flags / grant_ts / grant_valid_bits set
    p = mh.params(4, True)
    st = np.zeros(wb.n_msgs, np.uint8)
    rc = mv.lib.mochi_mverify_write2(mv.h, ctypes.addressof(wc), ctypes.addressof(p), ctypes.addressof(vc),
                                     st.ctypes.data)
    assert rc == mh.EINVAL
    assert b"grant-level" in mv.lib.mochi_last_error()
    mv.close()


def test_mctx_gathered_bits_are_the_verdicts(pool4):
    """The all-gather reads each device's accept bitmap where the verify left it.
    Device 0's gathered buffer, assembled by the shard plan, is checked against
    verdicts computed WITHOUT it: the oracle's bitmap and a single-context verify
    of the same batch (not the mctx's own output bits, which gather_bits derives
    from that same buffer).  Ragged tail: 4,141 certificates."""
    s = W.make_batch(pool4, 4096 + 45, first_cert=5)
    mv = mh.MultiVerifier(pool4.moduli, _mask())
    mv.verify(s.batch, 4, True)
    ptr, words = mv.gathered_bits(0)
    n = len(mv.devices)
    plan = mh.shard_plan(s.batch.n_certs, n, s.batch.cert_grant_off)
    got = mh.bits_assemble(plan, _d2h(ptr, n * words))
    o = O.verify_batch(pool4.moduli, s.batch, 4, True, 8)
    nw = o.cert_accept_bits.shape[0]
    np.testing.assert_array_equal(got[:nw], o.cert_accept_bits)
    one = mh.Verifier(pool4.moduli, 0)
    np.testing.assert_array_equal(got[:nw], one.verify(s.batch, 4, True).cert_accept_bits)
    one.close()
    mv.close()


def test_mctx_write2_gathered_bits_are_the_verdicts(pool4):
    """The same for mochi_mverify_write2: the gathered device bitmap after a
    wire-path verify equals the oracle's decode + verify of the messages."""
    s = W.make_batch(pool4, 1500 + 13, first_cert=1201)
    wb = W.encode_wire_batch(s)
    mv = mh.MultiVerifier(pool4.moduli, _mask())
    mv.set_server_ids(W.SERVER_IDS[:4])
    mv.verify_write2(wb, 4, True)
    ptr, words = mv.gathered_bits(0)
    n = len(mv.devices)
    pb = np.concatenate([[0], np.cumsum(wb.msg_len.astype(np.uint64))])  # mochi_mverify_write2's byte prefix
    plan = mh.shard_plan(wb.n_msgs, n, (pb // (int(pb[-1]) // 0xFFFFFFFF + 1)).astype(np.uint32))
    got = mh.bits_assemble(plan, _d2h(ptr, n * words))
    ids, off = W.server_id_table(4)
    o, _ = O.verify_write2(pool4.moduli, ids, off, wb, 4, True)
    nw = o.cert_accept_bits.shape[0]
    np.testing.assert_array_equal(got[:nw], o.cert_accept_bits)
    mv.close()


def _d2h(dev_ptr, words):
    """Copy `words` uint32 from a raw device pointer with the HIP runtime this
    process already mapped (torch's and the library's)."""
    import ctypes

    import torch

    torch.cuda.synchronize()
    path = next(line.split()[-1] for line in open("/proc/self/maps") if "libamdhip64.so" in line)
    hip = ctypes.CDLL(path)
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    out = np.zeros(words, np.uint32)
    assert hip.hipMemcpy(out.ctypes.data, dev_ptr, 4 * words, 2) == 0  # hipMemcpyDeviceToHost
    return out

