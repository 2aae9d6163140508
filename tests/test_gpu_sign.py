"""Producer-side signing on the device (k_rsa_sign, CRT): every signature is
byte-identical to OpenSSL's (PKCS#1 v1.5 is deterministic) and verifies."""
import numpy as np
import pytest

import mochi_hip as mh
import oracle_ffi as O
import workload as W

pytestmark = pytest.mark.gpu


def _grants(n, seed=3):
    rng = np.random.default_rng(seed)
    th = W.txn_hash_hex(seed)
    gs = [W.encode_grant(f"DEMO_KEY_STRESS_TEST_{int(rng.integers(0, 200))}", int(rng.integers(0, 64000)), th)
          for _ in range(n)]
    gs[0] = b""  # empty grant (all defaults)
    gs[1] = W.encode_grant("K" * 3000, 7, th)  # many SHA blocks
    blob, off = bytearray(b"\x05"), []
    for g in gs:
        off.append(len(blob))
        blob += g
    return (np.frombuffer(bytes(blob), np.uint8).copy(), np.array(off, np.uint64),
            np.array([len(g) for g in gs], np.uint32))


@pytest.mark.parametrize("key", range(7))
def test_device_signatures_equal_openssl(key):
    pem = W.load_keys(7)[key]
    blob, off, ln = _grants(700, seed=key)
    s = mh.DeviceSigner(pem, 0)
    got = s.sign(blob, off, ln)
    s.close()
    ref = mh.sign_grants(pem, blob, off, ln, 8)
    np.testing.assert_array_equal(got, ref)
    n = mh.pem_modulus(pem)
    for i in (0, 1, 2, 699):
        assert O.rsa_verify(n, blob[int(off[i]):int(off[i]) + int(ln[i])].tobytes(), got[i].tobytes())


def test_device_signed_grants_verify_on_device():
    pems = W.load_keys(4)
    blob, off, ln = _grants(4096, seed=9)
    sig = np.zeros((4096, 256), np.uint8)
    signer = np.arange(4096) % 4
    for k in range(4):
        s = mh.DeviceSigner(pems[k], 0)
        idx = np.nonzero(signer == k)[0]
        sig[idx] = s.sign(blob, off[idx], ln[idx])
        s.close()
    ver = mh.Verifier([mh.pem_modulus(p) for p in pems], 0)
    C = 1024
    b = mh.Batch(grant_bytes=blob, grant_off=off, grant_len=ln, sig=sig, signer=signer.astype(np.uint16),
                 grant_key=np.zeros(4096, np.uint8), cert_grant_off=(np.arange(C + 1) * 4).astype(np.uint32),
                 cert_op_off=np.arange(C + 1, dtype=np.uint32), op_key=np.zeros(C, np.uint8),
                 op_flags=np.full(C, 3, np.uint8), expected_hash=np.zeros((C, 128), np.uint8))
    g = ver.verify(b, 4, True)
    assert (g.grant_flags & 1).all()
    ver.close()


def test_crt_fault_is_withheld():
    """A fault in one RSA-CRT half (injected into grant 5's m_p) must never reach the
    caller: the public-key check after k_rsa_sign zeroes that signature and counts it;
    every other signature is still OpenSSL's.  Host and device entry points."""
    import torch

    pem = W.load_keys(2)[1]
    blob, off, ln = _grants(300, seed=21)
    ref = mh.sign_grants(pem, blob, off, ln, 8)
    s = mh.DeviceSigner(pem, 0)
    assert s.rejected() == 0
    s.set_fault(5)
    got = s.sign(blob, off, ln)
    assert s.rejected() == 1
    assert not got[5].any()
    keep = np.arange(300) != 5
    np.testing.assert_array_equal(got[keep], ref[keep])
    # device entry point, fault at the last grant
    s.set_fault(299)
    d = torch.device("cuda", 0)
    bt = torch.from_numpy(blob).to(d)
    ot = torch.from_numpy(off.view(np.int64)).to(d)
    lt = torch.from_numpy(ln.view(np.int32)).to(d)
    st = torch.empty((300, 256), dtype=torch.uint8, device=d)
    s.sign_device(bt, ot, lt, 300, st, torch.cuda.current_stream().cuda_stream)
    assert s.rejected() == 1
    g2 = st.cpu().numpy()
    assert not g2[299].any()
    np.testing.assert_array_equal(g2[:299], ref[:299])
    s.set_fault(-1)
    np.testing.assert_array_equal(s.sign(blob, off, ln), ref)
    assert s.rejected() == 0
    s.close()
