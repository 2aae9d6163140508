// multi.cpp — the batch verifier across the GPUs of one node.
//
// Certificates are independent: a batch is cut into contiguous certificate
// ranges, one per GPU, with every boundary on a multiple of 32 certificates so
// the per-GPU accept bitmaps concatenate word by word.  Each GPU verifies its
// range through its own context (its own host thread, streams and chunked
// PCIe pipeline).  The only collective is ONE RCCL all-gather of the per-GPU
// certificate-verdict bitmaps over xGMI, after which every GPU of the context
// holds the verdicts of the whole batch (device-resident, for a consumer on any
// GPU).  The reference's only "collective" is the client's TCP fan-out/fan-in
// (Utils.java:113-123, 65-93); nothing here has a reference counterpart.
//
// Two ways in:
//   * mochi_mctx_*  one process owns several GPUs (a JVM server with 8 GPUs):
//                   ncclCommInitAll over the device_mask;
//   * mochi_comm_*  one process per GPU (torchrun / MPI style): the caller moves
//                   the 128-byte unique id between processes (any transport),
//                   ncclCommInitRank, and calls the all-gather on its stream.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mochi_hip.h"

namespace mochi {
int set_error(int code, const std::string& msg);  // capi.cpp: the text mochi_last_error() returns
// capi.cpp: the accept bitmap of the context's last host-path call, on its device
uint64_t ctx_call_gen();  // capi.cpp: generation of this thread's last context call
int ctx_copy_accept_dev(mochi_ctx* c, uint64_t gen, int device, uint32_t* dst, uint32_t need, hipStream_t st);
}

namespace {

int mfail(int code, const std::string& msg) { return mochi::set_error(code, msg); }

const char* nccl_str(ncclResult_t r) { return ncclGetErrorString(r); }

uint32_t words(uint32_t bits) { return (bits + 31) / 32; }

}  // namespace

extern "C" {

int mochi_shard_plan(uint32_t n_certs, const uint32_t* cert_grant_off, uint32_t n_shards, uint32_t* cert_lo) {
  if (!cert_lo || n_shards == 0) return MOCHI_EINVAL;
  cert_lo[0] = 0;
  const uint64_t total = cert_grant_off ? cert_grant_off[n_certs] : n_certs;
  uint32_t c = 0;
  for (uint32_t s = 1; s < n_shards; s++) {
    // the first 32-aligned boundary whose prefix reaches s/n of the work
    const uint64_t want = total * s / n_shards;
    uint32_t lo = c, hi = n_certs;
    while (lo < hi) {  // smallest boundary b with work(b) >= want
      const uint32_t mid = lo + (hi - lo) / 2;
      const uint64_t w = cert_grant_off ? cert_grant_off[mid] : mid;
      if (w >= want) hi = mid;
      else lo = mid + 1;
    }
    uint32_t b = (lo + 31) / 32 * 32;
    if (b > n_certs) b = n_certs;
    if (b < c) b = c;
    cert_lo[s] = c = b;
  }
  cert_lo[n_shards] = n_certs;
  return MOCHI_OK;
}

uint32_t mochi_shard_words(uint32_t n_shards, const uint32_t* cert_lo) {
  uint32_t w = 1;
  for (uint32_t s = 0; s < n_shards; s++) {
    const uint32_t k = words(cert_lo[s + 1] - cert_lo[s]);
    w = k > w ? k : w;
  }
  return w;
}

int mochi_bits_assemble(uint32_t n_shards, const uint32_t* cert_lo, uint32_t words_per_shard, const uint32_t* gathered,
                        uint32_t* bits_out) {
  if (!cert_lo || !gathered || !bits_out) return MOCHI_EINVAL;
  const uint32_t n = cert_lo[n_shards];
  memset(bits_out, 0, 4 * (size_t)words(n));
  for (uint32_t s = 0; s < n_shards; s++) {
    const uint32_t lo = cert_lo[s], len = cert_lo[s + 1] - lo;
    if (lo % 32 != 0 && len) return MOCHI_EINVAL;  // plans from mochi_shard_plan are 32-aligned
    const uint32_t* src = gathered + (size_t)s * words_per_shard;
    for (uint32_t w = 0; w < words(len); w++) {
      uint32_t v = src[w];
      const uint32_t valid = len - 32 * w;
      if (valid < 32) v &= (1u << valid) - 1u;
      bits_out[lo / 32 + w] |= v;
    }
  }
  return MOCHI_OK;
}

// ---- one process per GPU -------------------------------------------------------
struct mochi_comm {
  ncclComm_t comm = nullptr;
  int device = 0;
};

int mochi_comm_unique_id(uint8_t* id_out) {
  if (!id_out) return MOCHI_EINVAL;
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  if (r != ncclSuccess) return mfail(MOCHI_EHIP, std::string("ncclGetUniqueId: ") + nccl_str(r));
  memcpy(id_out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return MOCHI_OK;
}

mochi_comm* mochi_comm_init(const uint8_t* id, int n_ranks, int rank, int device) {
  if (!id || n_ranks < 1 || rank < 0 || rank >= n_ranks) {
    mfail(MOCHI_EINVAL, "bad communicator arguments");
    return nullptr;
  }
  int save = 0;
  (void)hipGetDevice(&save);
  if (hipSetDevice(device) != hipSuccess) {
    mfail(MOCHI_ENODEV, "hipSetDevice failed");
    return nullptr;
  }
  ncclUniqueId uid;
  memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
  mochi_comm* c = new mochi_comm;
  c->device = device;
  const ncclResult_t r = ncclCommInitRank(&c->comm, n_ranks, uid, rank);
  (void)hipSetDevice(save);
  if (r != ncclSuccess) {
    mfail(MOCHI_EHIP, std::string("ncclCommInitRank: ") + nccl_str(r));
    delete c;
    return nullptr;
  }
  return c;
}

int mochi_comm_allgather_bits(mochi_comm* c, const uint32_t* d_send, uint32_t words_per_rank, uint32_t* d_recv,
                              void* stream) {
  if (!c || !d_send || !d_recv) return MOCHI_EINVAL;
  int save = 0;
  (void)hipGetDevice(&save);
  if (hipSetDevice(c->device) != hipSuccess) return mfail(MOCHI_EHIP, "hipSetDevice failed");
  const ncclResult_t r = ncclAllGather(d_send, d_recv, words_per_rank, ncclUint32, c->comm, (hipStream_t)stream);
  (void)hipSetDevice(save);
  return r == ncclSuccess ? MOCHI_OK : mfail(MOCHI_EHIP, std::string("ncclAllGather: ") + nccl_str(r));
}

void mochi_comm_destroy(mochi_comm* c) {
  if (!c) return;
  if (c->comm) (void)ncclCommDestroy(c->comm);
  delete c;
}

// ---- one process, several GPUs -------------------------------------------------
struct mochi_mctx {
  std::vector<int> devices;
  std::vector<mochi_ctx*> ctx;
  std::vector<ncclComm_t> comm;
  std::vector<hipStream_t> stream;
  std::vector<uint32_t*> gathered;  // per device: n_dev * words_per_shard words (device memory)
  std::vector<size_t> gathered_cap;
  uint32_t last_words = 0;
  bool comm_aborted = false;  // a gather aborted the communicators: rebuilt by the next gather
};

mochi_mctx* mochi_mctx_create(uint64_t device_mask, const uint8_t* moduli_be, uint32_t n_keys, uint32_t key_bytes,
                              uint32_t public_exponent) {
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    mfail(MOCHI_ENODEV, "no HIP device visible");
    return nullptr;
  }
  mochi_mctx* m = new mochi_mctx;
  for (int d = 0; d < 64 && d < ndev; d++)
    if ((device_mask >> d) & 1) m->devices.push_back(d);
  if (m->devices.empty() || (ndev < 64 && (device_mask >> ndev) != 0)) {
    mfail(MOCHI_ENODEV, "device_mask names no visible device, or a device that is not visible");
    delete m;
    return nullptr;
  }
  for (int d : m->devices) {
    mochi_ctx* c = mochi_ctx_create(d, moduli_be, n_keys, key_bytes, public_exponent);
    if (!c) {
      mfail(MOCHI_ENODEV, mochi_last_error());
      mochi_mctx_destroy(m);
      return nullptr;
    }
    m->ctx.push_back(c);
  }
  const int n = (int)m->devices.size();
  m->comm.assign(n, nullptr);
  m->stream.assign(n, nullptr);
  m->gathered.assign(n, nullptr);
  m->gathered_cap.assign(n, 0);
  int save = 0;
  (void)hipGetDevice(&save);
  for (int i = 0; i < n; i++) {
    if (hipSetDevice(m->devices[i]) != hipSuccess ||
        hipStreamCreateWithFlags(&m->stream[i], hipStreamNonBlocking) != hipSuccess) {
      (void)hipSetDevice(save);
      mfail(MOCHI_EHIP, "stream creation failed");
      mochi_mctx_destroy(m);
      return nullptr;
    }
  }
  (void)hipSetDevice(save);
  const ncclResult_t r = ncclCommInitAll(m->comm.data(), n, m->devices.data());
  if (r != ncclSuccess) {
    mfail(MOCHI_EHIP, std::string("ncclCommInitAll: ") + nccl_str(r));
    mochi_mctx_destroy(m);
    return nullptr;
  }
  return m;
}

void mochi_mctx_destroy(mochi_mctx* m) {
  if (!m) return;
  int save = 0;
  (void)hipGetDevice(&save);
  for (size_t i = 0; i < m->comm.size(); i++)
    if (m->comm[i]) (void)ncclCommDestroy(m->comm[i]);
  for (size_t i = 0; i < m->stream.size(); i++) {
    (void)hipSetDevice(m->devices[i]);
    if (m->gathered[i]) (void)hipFree(m->gathered[i]);
    if (m->stream[i]) (void)hipStreamDestroy(m->stream[i]);
  }
  (void)hipSetDevice(save);
  for (mochi_ctx* c : m->ctx) mochi_ctx_destroy(c);
  delete m;
}

int mochi_mctx_devices(mochi_mctx* m, int* devices, int max) {
  if (!m) return MOCHI_EINVAL;
  for (int i = 0; i < (int)m->devices.size() && i < max; i++) devices[i] = m->devices[i];
  return (int)m->devices.size();
}

mochi_ctx* mochi_mctx_context(mochi_mctx* m, int i) {
  return m && i >= 0 && i < (int)m->ctx.size() ? m->ctx[i] : nullptr;
}

int mochi_mctx_set_server_ids(mochi_mctx* m, const uint8_t* ids, const uint32_t* id_off, uint32_t n_ids) {
  if (!m) return MOCHI_EINVAL;
  for (mochi_ctx* c : m->ctx) {
    const int rc = mochi_ctx_set_server_ids(c, ids, id_off, n_ids);
    if (rc) return rc;
  }
  return MOCHI_OK;
}

}  // extern "C"

namespace {

// Certificate range [c0, c1) of a host batch as a batch of its own (pointers
// offset, CSR offsets rebased into `csr`).  Grant byte offsets stay absolute.
struct SubBatch {
  mochi_batch b;
  std::vector<uint32_t> cg, co, cm, mg;
};

void slice_batch(const mochi_batch* B, uint32_t c0, uint32_t c1, SubBatch& s) {
  const uint32_t g0 = B->cert_grant_off[c0], g1 = B->cert_grant_off[c1];
  const uint32_t o0 = B->cert_op_off[c0], o1 = B->cert_op_off[c1];
  s.b = *B;
  s.b.n_certs = c1 - c0;
  s.b.n_grants = g1 - g0;
  s.b.n_ops = o1 - o0;
  s.cg.resize(c1 - c0 + 1);
  s.co.resize(c1 - c0 + 1);
  for (uint32_t c = c0; c <= c1; c++) {
    s.cg[c - c0] = B->cert_grant_off[c] - g0;
    s.co[c - c0] = B->cert_op_off[c] - o0;
  }
  s.b.grant_off = B->grant_off + g0;
  s.b.grant_len = B->grant_len + g0;
  s.b.sig = B->sig + (size_t)MOCHI_RSA_BYTES * g0;
  s.b.signer = B->signer + g0;
  s.b.grant_key = B->grant_key + g0;
  s.b.cert_grant_off = s.cg.data();
  s.b.cert_op_off = s.co.data();
  s.b.op_key = B->op_key + o0;
  s.b.op_flags = B->op_flags + o0;
  s.b.expected_hash = B->expected_hash + (size_t)MOCHI_TXN_HASH_BYTES * c0;
  if (B->op_object_ts) s.b.op_object_ts = B->op_object_ts + o0;
  if (B->op_key_off) s.b.op_key_off = B->op_key_off + o0, s.b.op_key_len = B->op_key_len + o0;
  if (B->cert_mg_off) {
    const uint32_t m0 = B->cert_mg_off[c0], m1 = B->cert_mg_off[c1];
    s.cm.resize(c1 - c0 + 1);
    s.mg.resize(m1 - m0 + 1);
    for (uint32_t c = c0; c <= c1; c++) s.cm[c - c0] = B->cert_mg_off[c] - m0;
    for (uint32_t x = m0; x <= m1; x++) s.mg[x - m0] = B->mg_grant_off[x] - g0;
    s.b.n_mgs = m1 - m0;
    s.b.cert_mg_off = s.cm.data();
    s.b.mg_grant_off = s.mg.data();
  }
}

// The all-gather protocol, one host thread per device (multi.cpp's gather_bits
// and the CPU test hook mochi_test_gather_protocol drive the same code):
//   1. select the device (once: every later step runs on this thread) and make
//      its gather buffer;
//   -- barrier: a failure in 1 on ANY device is seen by all of them here, and
//      then no device enters the collective (no peer is left waiting in it);
//   2. fill the device's slot; a local failure is recorded, and the device still
//      enqueues its part of the collective so its peers complete;
//   3. enqueue the collective;
//   -- barrier: if ANY device failed to enqueue, every device aborts its
//      communicator (which ends the peers' pending collective kernels) instead
//      of waiting on its stream; the communicators are rebuilt on the next call;
//   4. wait for the device's stream.
// Returns the first error of any device, after every thread has joined.
struct GatherOps {
  std::function<int(int)> select, prep, fill, enqueue, finish, abort;
};

class Barrier {
 public:
  explicit Barrier(int n) : n_(n) {}
  void arrive_and_wait() {
    std::unique_lock<std::mutex> lk(mu_);
    const uint64_t gen = gen_;
    if (++count_ == n_) {
      count_ = 0;
      gen_++;
      cv_.notify_all();
    } else {
      cv_.wait(lk, [&] { return gen_ != gen; });
    }
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  int n_, count_ = 0;
  uint64_t gen_ = 0;
};

int run_gather(int n, const GatherOps& ops, std::string* what) {
  std::vector<int> rc_setup(n, MOCHI_OK), rc_fill(n, MOCHI_OK), rc_enq(n, MOCHI_OK), rc_fin(n, MOCHI_OK);
  Barrier bar(n);
  std::atomic<bool> setup_failed{false}, enq_failed{false};
  auto dev = [&](int i) {
    int r = ops.select(i);
    if (r == MOCHI_OK) r = ops.prep(i);
    rc_setup[i] = r;
    if (r) setup_failed = true;
    bar.arrive_and_wait();
    if (setup_failed) return;
    rc_fill[i] = ops.fill(i);
    rc_enq[i] = ops.enqueue(i);
    if (rc_enq[i]) enq_failed = true;
    bar.arrive_and_wait();
    if (enq_failed) {
      ops.abort(i);
      return;
    }
    rc_fin[i] = ops.finish(i);
  };
  std::vector<std::thread> th;
  for (int i = 0; i < n; i++) th.emplace_back(dev, i);
  for (auto& t : th) t.join();
  const std::vector<int>* stages[4] = {&rc_setup, &rc_fill, &rc_enq, &rc_fin};
  const char* names[4] = {"device selection / gather buffer", "slot fill", "all-gather enqueue (communicators aborted)",
                          "all-gather completion"};
  for (int s = 0; s < 4; s++)
    for (int i = 0; i < n; i++)
      if ((*stages[s])[i]) {
        if (what) *what = std::string(names[s]) + " failed on device slot " + std::to_string(i);
        return (*stages[s])[i];
      }
  return MOCHI_OK;
}

// Each device's shard verdicts are already on that device: the accept bitmap
// of the context call that just returned (a slice of its output buffer).  Per
// device it is copied device to device into the device's slot of its gather
// buffer (zero-padded to W words), then one ncclAllGather fills every device's
// buffer, and bits_out comes from ONE device-to-host copy of device 0's.  A
// context whose device bitmap is not the final verdict (messages decided by the
// host fallback decoder) uploads its host bits into its slot instead.
int gather_bits(mochi_mctx* m, const std::vector<uint32_t>& cert_lo, const std::vector<std::vector<uint32_t>>& shard_bits,
                const std::vector<uint64_t>& gen, uint32_t* bits_out) {
  const int n = (int)m->devices.size();
  const uint32_t W = mochi_shard_words((uint32_t)n, cert_lo.data());
  if (m->comm_aborted) {  // a previous call aborted the communicators: rebuild them
    for (auto& c : m->comm)
      if (c) (void)ncclCommDestroy(c), c = nullptr;
    const ncclResult_t r = ncclCommInitAll(m->comm.data(), n, m->devices.data());
    if (r != ncclSuccess) return mfail(MOCHI_EHIP, std::string("ncclCommInitAll (rebuild): ") + nccl_str(r));
    m->comm_aborted = false;
  }
  GatherOps ops;
  ops.select = [&](int i) { return hipSetDevice(m->devices[i]) == hipSuccess ? MOCHI_OK : MOCHI_EHIP; };
  ops.prep = [&](int i) {
    const size_t bytes = 4 * (size_t)W * n;
    if (bytes <= m->gathered_cap[i]) return MOCHI_OK;
    if (m->gathered[i]) (void)hipFree(m->gathered[i]);
    m->gathered[i] = nullptr;
    m->gathered_cap[i] = 0;
    if (hipMalloc(&m->gathered[i], bytes) != hipSuccess) return MOCHI_ENOMEM;
    m->gathered_cap[i] = bytes;
    return MOCHI_OK;
  };
  ops.fill = [&](int i) {
    uint32_t* slot = m->gathered[i] + (size_t)W * i;
    const uint32_t need = words(cert_lo[i + 1] - cert_lo[i]);  // <= W
    hipError_t e = hipMemsetAsync(slot, 0, 4 * (size_t)W, m->stream[i]);
    if (e == hipSuccess && need) {
      // the shard's bitmap where its verify left it, if no later call on the
      // context has touched its buffers since (checked and copied under the
      // context's lock); otherwise the host bits the verify returned
      const int d = mochi::ctx_copy_accept_dev(m->ctx[i], gen[i], m->devices[i], slot, need, m->stream[i]);
      if (d == MOCHI_EHIP) e = hipErrorUnknown;
      else if (d != MOCHI_OK) {
        const size_t have = shard_bits[i].size() < need ? shard_bits[i].size() : need;
        e = hipMemcpyAsync(slot, shard_bits[i].data(), 4 * have, hipMemcpyHostToDevice, m->stream[i]);
      }
    }
    return e == hipSuccess ? MOCHI_OK : MOCHI_EHIP;
  };
  ops.enqueue = [&](int i) {
    uint32_t* slot = m->gathered[i] + (size_t)W * i;
    return ncclAllGather(slot, m->gathered[i], W, ncclUint32, m->comm[i], m->stream[i]) == ncclSuccess ? MOCHI_OK
                                                                                                       : MOCHI_EHIP;
  };
  ops.finish = [&](int i) { return hipStreamSynchronize(m->stream[i]) == hipSuccess ? MOCHI_OK : MOCHI_EHIP; };
  std::atomic<bool> aborted{false};
  ops.abort = [&](int i) {
    (void)ncclCommAbort(m->comm[i]);
    m->comm[i] = nullptr;
    aborted = true;
    return MOCHI_OK;
  };
  int save = 0;
  (void)hipGetDevice(&save);
  std::string what;
  const int rc = run_gather(n, ops, &what);
  if (aborted) m->comm_aborted = true;
  (void)hipSetDevice(save);
  if (rc) return mfail(rc, "bitmap all-gather: " + what);
  m->last_words = W;
  std::vector<uint32_t> all((size_t)W * n);
  (void)hipSetDevice(m->devices[0]);
  const hipError_t e = hipMemcpy(all.data(), m->gathered[0], 4 * all.size(), hipMemcpyDeviceToHost);
  (void)hipSetDevice(save);
  if (e != hipSuccess) return mfail(MOCHI_EHIP, "gathered bitmap copy failed");
  return mochi_bits_assemble((uint32_t)n, cert_lo.data(), W, all.data(), bits_out);
}

}  // namespace

extern "C" {

int mochi_mverify_batch(mochi_mctx* m, const mochi_batch* b, const mochi_params* p, mochi_verdicts* o) {
  if (!m || !b || !p || !o || (!o->cert_accept_bits && b->n_certs)) return mfail(MOCHI_EINVAL, "null argument");
  if (o->grant_valid_bits) return mfail(MOCHI_EINVAL, "grant_valid_bits is not produced across devices (use grant_flags)");
  const int n = (int)m->devices.size();
  std::vector<uint32_t> lo(n + 1);
  mochi_shard_plan(b->n_certs, b->cert_grant_off, (uint32_t)n, lo.data());
  std::vector<std::vector<uint32_t>> bits(n);
  std::vector<uint64_t> gen(n, 0);
  std::vector<int> rc(n, MOCHI_OK);
  std::vector<std::string> err(n);
  auto work = [&](int i) {
    SubBatch s;
    slice_batch(b, lo[i], lo[i + 1], s);
    const uint32_t g0 = b->cert_grant_off[lo[i]], o0 = b->cert_op_off[lo[i]];
    bits[i].assign(words(lo[i + 1] - lo[i]) + 1, 0u);  // +1: a non-empty vector for empty shards
    mochi_verdicts v;
    memset(&v, 0, sizeof v);
    v.grant_flags = o->grant_flags ? o->grant_flags + g0 : nullptr;
    v.grant_ts = o->grant_ts ? o->grant_ts + g0 : nullptr;
    v.cert_accept_bits = bits[i].data();
    v.cert_reason = o->cert_reason ? o->cert_reason + lo[i] : nullptr;
    v.cert_fail_op = o->cert_fail_op ? o->cert_fail_op + lo[i] : nullptr;
    v.op_decision = o->op_decision ? o->op_decision + o0 : nullptr;
    v.op_g0 = o->op_g0 ? o->op_g0 + o0 : nullptr;
    v.op_ts = o->op_ts ? o->op_ts + o0 : nullptr;
    rc[i] = mochi_verify_batch(m->ctx[i], &s.b, p, &v);
    gen[i] = mochi::ctx_call_gen();
    if (rc[i]) err[i] = mochi_last_error();
  };
  std::vector<std::thread> th;
  for (int i = 0; i < n; i++) th.emplace_back(work, i);
  for (auto& t : th) t.join();
  for (int i = 0; i < n; i++)
    if (rc[i]) return mfail(rc[i], "device " + std::to_string(m->devices[i]) + ": " + err[i]);
  return b->n_certs ? gather_bits(m, lo, bits, gen, o->cert_accept_bits) : MOCHI_OK;
}

int mochi_mverify_write2(mochi_mctx* m, const mochi_write2_batch* w, const mochi_params* p, mochi_verdicts* o,
                         uint8_t* msg_status) {
  if (!m || !w || !p || !o || (!o->cert_accept_bits && w->n_msgs)) return mfail(MOCHI_EINVAL, "null argument");
  if (o->grant_flags || o->grant_ts || o->grant_valid_bits)  // as mochi_verify_write2 (check_write2_header)
    return mfail(MOCHI_EINVAL, "grant-level outputs are not produced on the wire path (must be NULL)");
  const int n = (int)m->devices.size();
  // shard by wire bytes (a proxy for grants: the messages are not decoded yet)
  std::vector<uint32_t> prefix(w->n_msgs + 1, 0);
  std::vector<uint64_t> pb(w->n_msgs + 1, 0);
  for (uint32_t i = 0; i < w->n_msgs; i++) pb[i + 1] = pb[i] + w->msg_len[i];
  const uint64_t scale = pb[w->n_msgs] / 0xFFFFFFFFull + 1;  // keep the prefix in 32 bits
  for (uint32_t i = 0; i <= w->n_msgs; i++) prefix[i] = (uint32_t)(pb[i] / scale);
  std::vector<uint32_t> lo(n + 1);
  mochi_shard_plan(w->n_msgs, prefix.data(), (uint32_t)n, lo.data());
  std::vector<std::vector<uint32_t>> bits(n);
  std::vector<uint64_t> gen(n, 0);
  std::vector<int> rc(n, MOCHI_OK);
  std::vector<std::string> err(n);
  auto work = [&](int i) {
    const uint32_t m0 = lo[i], m1 = lo[i + 1];
    mochi_write2_batch s = *w;
    s.n_msgs = m1 - m0;
    s.msg_off = w->msg_off + m0;
    s.msg_len = w->msg_len + m0;
    s.expected_hash = w->expected_hash + (size_t)MOCHI_TXN_HASH_BYTES * m0;
    std::vector<uint32_t> ofo;
    uint32_t o0 = 0;
    if (w->op_flags_off) {
      o0 = w->op_flags_off[m0];
      ofo.resize(m1 - m0 + 1);
      for (uint32_t x = m0; x <= m1; x++) ofo[x - m0] = w->op_flags_off[x] - o0;
      s.op_flags_off = ofo.data();
      s.op_flags = w->op_flags + o0;
      if (w->op_object_ts) s.op_object_ts = w->op_object_ts + o0;
    }
    bits[i].assign(words(m1 - m0) + 1, 0u);  // +1: a non-empty vector for empty shards
    mochi_verdicts v;
    memset(&v, 0, sizeof v);
    v.cert_accept_bits = bits[i].data();
    v.cert_reason = o->cert_reason ? o->cert_reason + m0 : nullptr;
    v.cert_fail_op = o->cert_fail_op ? o->cert_fail_op + m0 : nullptr;
    v.op_decision = o->op_decision ? o->op_decision + o0 : nullptr;
    v.op_g0 = o->op_g0 ? o->op_g0 + o0 : nullptr;
    v.op_ts = o->op_ts ? o->op_ts + o0 : nullptr;
    rc[i] = mochi_verify_write2(m->ctx[i], &s, p, &v, msg_status ? msg_status + m0 : nullptr);
    gen[i] = mochi::ctx_call_gen();
    if (rc[i]) err[i] = mochi_last_error();
  };
  std::vector<std::thread> th;
  for (int i = 0; i < n; i++) th.emplace_back(work, i);
  for (auto& t : th) t.join();
  for (int i = 0; i < n; i++)
    if (rc[i]) return mfail(rc[i], "device " + std::to_string(m->devices[i]) + ": " + err[i]);
  return w->n_msgs ? gather_bits(m, lo, bits, gen, o->cert_accept_bits) : MOCHI_OK;
}

int mochi_mctx_gathered_bits(mochi_mctx* m, int i, const uint32_t** d_bits, uint32_t* words_per_device) {
  if (!m || i < 0 || i >= (int)m->devices.size() || !d_bits) return MOCHI_EINVAL;
  *d_bits = m->gathered[i];
  if (words_per_device) *words_per_device = m->last_words;
  return MOCHI_OK;
}

// CPU test hook for the all-gather protocol (run_gather): n device threads with
// no GPU, the collective a host rendezvous that only completes when all n
// threads enqueued (or one aborted); a thread that never arrives makes the
// others time out after `timeout_ms` -- the hang the protocol must prevent.
int mochi_test_gather_protocol(uint32_t n, uint32_t fail_select, uint32_t fail_fill, uint32_t fail_enqueue,
                               uint32_t timeout_ms, uint32_t* entered_collective, uint32_t* timed_out) {
  if (n == 0 || n > 32) return MOCHI_EINVAL;
  std::mutex mu;
  std::condition_variable cv;
  uint32_t arrived = 0, timeouts = 0;
  bool aborted = false;
  GatherOps ops;
  ops.select = [&](int i) { return (fail_select >> i) & 1 ? MOCHI_EHIP : MOCHI_OK; };
  ops.prep = [&](int) { return MOCHI_OK; };
  ops.fill = [&](int i) { return (fail_fill >> i) & 1 ? MOCHI_EHIP : MOCHI_OK; };
  ops.enqueue = [&](int i) {
    if ((fail_enqueue >> i) & 1) return MOCHI_EHIP;
    std::lock_guard<std::mutex> lk(mu);
    arrived++;
    cv.notify_all();
    return MOCHI_OK;
  };
  ops.finish = [&](int) {
    std::unique_lock<std::mutex> lk(mu);
    if (!cv.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return arrived == n || aborted; })) {
      timeouts++;
      return MOCHI_EHIP;
    }
    return aborted ? MOCHI_EHIP : MOCHI_OK;
  };
  ops.abort = [&](int) {
    std::lock_guard<std::mutex> lk(mu);
    aborted = true;
    cv.notify_all();
    return MOCHI_OK;
  };
  std::string what;
  const int rc = run_gather((int)n, ops, &what);
  if (entered_collective) *entered_collective = arrived;
  if (timed_out) *timed_out = timeouts;
  if (rc) mfail(rc, what);
  return rc;
}

}  // extern "C"
