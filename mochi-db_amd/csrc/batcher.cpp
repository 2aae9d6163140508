// batcher.cpp — the micro-batcher in front of mochi_verify_write2.
//
// The reference validates one Write2ToServer per worker-thread call
// (Write2ToServerRequestHandler.handle -> InMemoryDataStore.processWrite2ToServer,
// Write2ToServerRequestHandler.java:25-31, InMemoryDataStore.java:641-666) on a
// ThreadPoolExecutor of core 2 / max 20 threads (MochiServer.java:36-40).  One
// certificate is far too little work for a GPU launch, so the drop-in keeps
// that blocking per-request call and coalesces the requests of all threads:
// callers enqueue their message and sleep; a flusher thread takes up to
// max_msgs pending messages (or whatever is pending once the oldest has waited
// max_wait_us), verifies them with ONE mochi_verify_write2 call, and wakes each
// caller with its own verdict.  While a batch is on the GPU the next one
// accumulates, so the batch size follows the offered load; with several
// contexts (mochi_batcher_create_multi) several batches are in flight at once.
//
// Each flusher assembles its batch straight into pinned host memory
// (mochi_host_alloc), which mochi_verify_write2 DMAs in place: a request's
// bytes are copied once, from the caller's buffer into the batch.
//
// Built only on the public C ABI (include/mochi_hip.h).
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mochi_hip.h"

namespace mochi {
int set_error(int code, const std::string& msg);  // capi.cpp: the text mochi_last_error() returns
void ctx_hold(mochi_ctx* c);                      // capi.cpp: mochi_ctx_destroy waits for the batchers
void ctx_release(mochi_ctx* c);                   // that hold the context
}

namespace {

struct Request {
  mochi_write2_request r;  // caller's buffers (valid until completion)
  std::chrono::steady_clock::time_point t_enq;
  mochi_verdict1* out;  // blocking call: the caller's verdict slot
  mochi_verdict_cb cb;  // submit: completion callback (heap request)
  void* user;
  int rc = 0;
  bool done = false;
};

// A grow-only pinned host array (mochi_host_alloc), reused across batches.
template <typename T>
struct Pinned {
  T* p = nullptr;
  size_t cap = 0;
  ~Pinned() { mochi_host_free(p); }
  bool reserve(size_t n) {
    if (n <= cap) return true;
    size_t c = cap ? cap : 256;
    while (c < n) c *= 2;
    T* q = (T*)mochi_host_alloc(sizeof(T) * c);
    if (!q) return false;
    mochi_host_free(p);
    p = q;
    cap = c;
    return true;
  }
};

// One flusher per context: with n contexts, n batches are in flight at once
// (one assembling/decoding while another's k_rsa_pow runs), so a request that
// arrives while a batch is on the GPU need not wait for it to come back.
struct Flusher {
  mochi_ctx* ctx;
  std::thread th;
  // batch assembly (this flusher's thread only): inputs pinned, outputs host
  Pinned<uint8_t> wire, flags, hashes;
  Pinned<uint64_t> off;
  Pinned<uint32_t> len, flags_off;
  Pinned<int64_t> ots;
  std::vector<uint8_t> status, reason, fail_op, op_dec;
  std::vector<uint32_t> accept, op_g0;
  std::vector<int64_t> op_ts;
  // when this flusher's last batch completed (under the batcher's mu, before its
  // callers were woken): the batcher's arrival count then and the batch's size
  uint64_t arr_at_done = 0, last_n = 0;
  std::chrono::steady_clock::time_point t_done;
};

// the batcher whose flusher runs on this thread (a callback re-entering the
// batcher it runs on would deadlock a single-context batcher)
thread_local const void* t_flushing = nullptr;

}  // namespace

struct mochi_batcher {
  mochi_params params;
  uint32_t max_msgs, max_wait_us;
  bool with_op_flags;
  std::mutex mu;
  std::condition_variable cv_work, cv_done;
  std::deque<Request*> q;
  bool stop = false;
  bool deferred_delete = false;  // destroyed from one of its own callbacks: the last flusher out frees it
  uint32_t live = 0;             // flusher threads still in run()
  uint32_t waiters = 0;          // blocking callers not yet out of their wait (mu is theirs until then)
  uint64_t n_batches = 0, n_msgs = 0;
  uint64_t n_arrived = 0;  // requests ever enqueued (take(): arrivals since a flusher's last completion)
  uint32_t collecting = 0;  // flushers waiting for the callers their last batch released
  uint32_t in_flight = 0;   // batches taken and not yet completed
  static constexpr size_t kConcurrentMin = 64;
  std::vector<Flusher> fl;

  // Frees the flushers' pinned buffers, then lets the contexts go: however the
  // batcher ends (joined, or freed by its last flusher after a deferred
  // destroy), mochi_ctx_destroy on one of its contexts returns only after this.
  ~mochi_batcher() {
    std::vector<mochi_ctx*> cs;
    for (auto& f : fl) cs.push_back(f.ctx);
    fl.clear();
    for (mochi_ctx* c : cs) mochi::ctx_release(c);
  }

  // Takes the next batch.  Waits for work; then, if this flusher has just
  // completed a batch, until the callers that batch released are back (as many
  // requests arrived since the completion as the batch held, whichever flusher
  // they went to) or max_wait_us after the completion: blocking callers resubmit within
  // microseconds of their verdicts, and taking the first of them alone would
  // split them into alternating batches that each wait for the other's flight
  // (2 blocking workers on one context: every request paid two GPU round
  // trips).  An idle flusher takes what is queued at once; a full batch
  // (max_msgs) is taken at once.  Returns false when stopped and drained.
  bool take(Flusher& f, std::vector<Request*>& batch) {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      // Small batches go to the GPU one at a time: two in flight at once on one
      // GPU took about twice as long each (2 blocking workers on 2 contexts: p50
      // 945 us vs 555 us on one), so a flusher takes work while a sibling's batch
      // is in flight only once kConcurrentMin requests wait (load that fills
      // several contexts), and an idle flusher leaves arrivals to a sibling that
      // is collecting the callers its batch released.
      auto may_take = [&] { return in_flight == 0 || q.size() >= kConcurrentMin || q.size() >= max_msgs; };
      cv_work.wait(lk, [&] {
        return stop || (!q.empty() && (f.last_n || collecting == 0 || q.size() >= max_msgs) && may_take());
      });
      if (q.empty()) {  // stopped and drained
        if (f.last_n) collecting--, f.last_n = 0;
        return false;
      }
      if (f.last_n) {  // a collector since its batch completed (run(): collecting++ under mu)
        const auto deadline = f.t_done + std::chrono::microseconds(max_wait_us);
        while (!stop && !q.empty() && q.size() < max_msgs && n_arrived - f.arr_at_done < f.last_n) {
          if (std::chrono::steady_clock::now() >= deadline) break;
          cv_work.wait_until(lk, deadline);
        }
        collecting--;
        f.last_n = 0;
        if (collecting == 0) cv_work.notify_all();  // idle siblings may take what this batch leaves
      }
      if (q.empty() || !may_take()) continue;  // a sibling took it (never verify M = 0), or one is in flight
      const size_t n = q.size() < max_msgs ? q.size() : max_msgs;
      batch.assign(q.begin(), q.begin() + n);
      q.erase(q.begin(), q.begin() + n);
      in_flight++;
      if (!q.empty()) cv_work.notify_one();  // leave the rest to an idle sibling now
      return true;
    }
  }

  void run(Flusher& f) {
    t_flushing = this;
    std::vector<Request*> batch, owned;
    while (take(f, batch)) {
      verify(f, batch);  // fills the blocking callers' slots, runs the submitters' callbacks
      // the submitted (heap) requests are freed here; a blocking caller's request
      // lives on its stack and may be gone the moment it sees `done`, so it is
      // not touched again after that
      owned.clear();
      for (Request* r : batch)
        if (r->cb) owned.push_back(r);
      {
        std::lock_guard<std::mutex> lk(mu);
        // the callers this batch releases: its blocking ones (a completion
        // callback that resubmits has done so already, above)
        size_t blocking = 0;
        for (Request* r : batch) blocking += r->cb ? 0 : 1;
        for (Request* r : batch)
          if (!r->cb) r->done = true;
        n_batches++;
        n_msgs += batch.size();
        f.arr_at_done = n_arrived;
        f.last_n = blocking;
        in_flight--;
        if (blocking) collecting++;  // until take() has collected them: idle siblings hold back
        f.t_done = std::chrono::steady_clock::now();
      }
      cv_done.notify_all();
      cv_work.notify_all();  // siblings holding back while this batch was in flight
      for (Request* r : owned) delete r;
    }
    bool last;
    {
      std::unique_lock<std::mutex> lk(mu);
      last = --live == 0 && deferred_delete;
      if (last) cv_done.wait(lk, [&] { return waiters == 0; });
    }
    if (last) {  // mochi_batcher_destroy ran inside a callback: nobody will join us
      t_flushing = nullptr;
      for (auto& g : fl) g.th.detach();
      delete this;
    }
  }

  void verify(Flusher& f, const std::vector<Request*>& batch) {
    const uint32_t M = (uint32_t)batch.size();
    size_t total = 0, n_ops = 0;
    bool any_ts = false, any_op_out = false;
    for (Request* q : batch) {
      total += q->r.msg_len;
      n_ops += q->r.n_ops;
      any_ts |= q->r.op_object_ts != nullptr;
      any_op_out |= q->r.op_decision || q->r.op_g0 || q->r.op_ts;
    }
    const bool flags_in = with_op_flags;
    int rc = MOCHI_OK;
    if (!f.wire.reserve(total ? total : 1) || !f.off.reserve(M) || !f.len.reserve(M) ||
        !f.hashes.reserve((size_t)M * MOCHI_TXN_HASH_BYTES) || !f.flags_off.reserve(M + 1) ||
        !f.flags.reserve(n_ops ? n_ops : 1) || (any_ts && !f.ots.reserve(n_ops ? n_ops : 1)))
      rc = MOCHI_ENOMEM;
    if (rc == MOCHI_OK) {
      size_t pos = 0, op = 0;
      for (uint32_t i = 0; i < M; i++) {
        const mochi_write2_request& r = batch[i]->r;
        memcpy(f.wire.p + pos, r.msg, r.msg_len);
        f.off.p[i] = pos;
        f.len.p[i] = r.msg_len;
        pos += r.msg_len;
        memcpy(f.hashes.p + (size_t)i * MOCHI_TXN_HASH_BYTES, r.expected_hash, MOCHI_TXN_HASH_BYTES);
        f.flags_off.p[i] = (uint32_t)op;
        for (uint32_t j = 0; j < r.n_ops; j++) {
          f.flags.p[op + j] = r.op_flags ? r.op_flags[j] : (uint8_t)(MOCHI_OP_LOCAL | MOCHI_OP_HAS_SVOC);
          if (any_ts) f.ots.p[op + j] = r.op_object_ts ? r.op_object_ts[j] : 0;
        }
        op += r.n_ops;
      }
      f.flags_off.p[M] = (uint32_t)op;
      mochi_write2_batch w;
      memset(&w, 0, sizeof w);
      w.n_msgs = M;
      w.wire_len = total;
      w.wire = f.wire.p;
      w.msg_off = f.off.p;
      w.msg_len = f.len.p;
      // without per-op flags the decoder's default (LOCAL|HAS_SVOC) applies
      w.op_flags_off = flags_in ? f.flags_off.p : nullptr;
      w.op_flags = flags_in ? f.flags.p : nullptr;
      w.op_object_ts = flags_in && any_ts ? f.ots.p : nullptr;
      w.expected_hash = f.hashes.p;
      f.accept.assign((M + 31) / 32, 0);
      f.reason.resize(M);
      f.fail_op.resize(M);
      f.status.resize(M);
      const bool op_out = flags_in && any_op_out;
      if (op_out) {
        f.op_dec.resize(n_ops ? n_ops : 1);
        f.op_g0.resize(n_ops ? n_ops : 1);
        f.op_ts.resize(n_ops ? n_ops : 1);
      }
      mochi_verdicts v;
      memset(&v, 0, sizeof v);
      v.cert_accept_bits = f.accept.data();
      v.cert_reason = f.reason.data();
      v.cert_fail_op = f.fail_op.data();
      v.op_decision = op_out ? f.op_dec.data() : nullptr;
      v.op_g0 = op_out ? f.op_g0.data() : nullptr;
      v.op_ts = op_out ? f.op_ts.data() : nullptr;
      rc = mochi_verify_write2(f.ctx, &w, &params, &v, f.status.data());
      if (rc == MOCHI_OK && op_out)
        for (uint32_t i = 0; i < M; i++) {
          const mochi_write2_request& r = batch[i]->r;
          const size_t o0 = f.flags_off.p[i];
          for (uint32_t j = 0; j < r.n_ops; j++) {
            if (r.op_decision) r.op_decision[j] = f.op_dec[o0 + j];
            if (r.op_g0) r.op_g0[j] = f.op_g0[o0 + j];
            if (r.op_ts) r.op_ts[j] = f.op_ts[o0 + j];
          }
        }
    }
    for (uint32_t i = 0; i < M; i++) {
      Request* r = batch[i];
      r->rc = rc;
      mochi_verdict1 v{};
      if (rc == MOCHI_OK) {
        v.accepted = (uint8_t)((f.accept[i >> 5] >> (i & 31)) & 1u);
        v.reason = f.reason[i];
        v.fail_op = f.fail_op[i];
        v.msg_status = f.status[i];
      }
      if (r->cb) r->cb(r->user, rc, &v);
      else if (rc == MOCHI_OK) *r->out = v;
    }
  }

  int check(const mochi_write2_request* r) const {
    if (!r || (!r->msg && r->msg_len) || !r->expected_hash) return MOCHI_EINVAL;
    if (with_op_flags ? (r->op_flags == nullptr && r->n_ops != 0)
                      : (r->op_flags != nullptr || r->n_ops != 0 || r->op_object_ts || r->op_decision || r->op_g0 ||
                         r->op_ts))
      return MOCHI_EINVAL;
    return MOCHI_OK;
  }

  void enqueue(Request* r) {  // mu held
    q.push_back(r);
    n_arrived++;
    // every waiting flusher re-checks: a collecting one counts the arrival, an idle
    // one takes the queue (notify_one could wake only the idle one, which takes
    // the request, while the collector sleeps on to its deadline)
    cv_work.notify_all();
  }
};

extern "C" {

mochi_batcher* mochi_batcher_create_multi(mochi_ctx* const* ctxs, uint32_t n_ctx, const mochi_params* params,
                                          uint32_t max_msgs, uint32_t max_wait_us, int with_op_flags) {
  if (!ctxs || n_ctx == 0 || !params || max_msgs == 0) return nullptr;
  for (uint32_t i = 0; i < n_ctx; i++)
    if (!ctxs[i]) return nullptr;
  mochi_batcher* b = new mochi_batcher();
  b->with_op_flags = with_op_flags != 0;
  b->params = *params;
  b->max_msgs = max_msgs;
  b->max_wait_us = max_wait_us;
  b->fl.resize(n_ctx);
  b->live = n_ctx;
  for (uint32_t i = 0; i < n_ctx; i++) {
    b->fl[i].ctx = ctxs[i];
    mochi::ctx_hold(ctxs[i]);
  }
  for (auto& f : b->fl) {
    Flusher* fp = &f;
    f.th = std::thread([b, fp] { b->run(*fp); });
  }
  return b;
}

mochi_batcher* mochi_batcher_create(mochi_ctx* ctx, const mochi_params* params, uint32_t max_msgs,
                                    uint32_t max_wait_us, int with_op_flags) {
  return mochi_batcher_create_multi(&ctx, 1, params, max_msgs, max_wait_us, with_op_flags);
}

int mochi_batcher_verify_request(mochi_batcher* b, const mochi_write2_request* req, mochi_verdict1* out) {
  if (!b || !out) return MOCHI_EINVAL;
  int rc = b->check(req);
  if (rc) return rc;
  // a callback blocking on the batcher that runs it would wait for itself
  // (one flusher) or stall a flusher the others may be counting on; submitting
  // from a callback is fine (enqueue only takes mu, which verify() has released)
  if (t_flushing == b)
    return mochi::set_error(MOCHI_EINVAL, "mochi_batcher_verify*: called from a completion callback of the same batcher; "
                                          "use mochi_batcher_submit* there");
  Request r;
  r.r = *req;
  r.out = out;
  r.cb = nullptr;
  r.user = nullptr;
  r.t_enq = std::chrono::steady_clock::now();
  std::unique_lock<std::mutex> lk(b->mu);
  if (b->stop) return MOCHI_EINVAL;
  b->enqueue(&r);
  b->waiters++;
  b->cv_done.wait(lk, [&] { return r.done; });
  if (--b->waiters == 0 && b->stop) b->cv_done.notify_all();  // a destroy may be waiting for us
  return r.rc;
}

int mochi_batcher_submit_request(mochi_batcher* b, const mochi_write2_request* req, mochi_verdict_cb cb, void* user) {
  if (!b || !cb) return MOCHI_EINVAL;
  int rc = b->check(req);
  if (rc) return rc;
  Request* r = new Request();
  r->r = *req;
  r->out = nullptr;
  r->cb = cb;
  r->user = user;
  r->t_enq = std::chrono::steady_clock::now();
  std::lock_guard<std::mutex> lk(b->mu);
  if (b->stop) {
    delete r;
    return MOCHI_EINVAL;
  }
  b->enqueue(r);
  return MOCHI_OK;
}

int mochi_batcher_verify(mochi_batcher* b, const uint8_t* msg, uint32_t msg_len, const uint8_t* op_flags,
                         uint32_t n_ops, const uint8_t* expected_hash, mochi_verdict1* out) {
  mochi_write2_request r;
  memset(&r, 0, sizeof r);
  r.msg = msg;
  r.msg_len = msg_len;
  r.op_flags = op_flags;
  r.n_ops = n_ops;
  r.expected_hash = expected_hash;
  return mochi_batcher_verify_request(b, &r, out);
}

int mochi_batcher_submit(mochi_batcher* b, const uint8_t* msg, uint32_t msg_len, const uint8_t* op_flags,
                         uint32_t n_ops, const uint8_t* expected_hash, mochi_verdict_cb cb, void* user) {
  mochi_write2_request r;
  memset(&r, 0, sizeof r);
  r.msg = msg;
  r.msg_len = msg_len;
  r.op_flags = op_flags;
  r.n_ops = n_ops;
  r.expected_hash = expected_hash;
  return mochi_batcher_submit_request(b, &r, cb, user);
}

int mochi_batcher_stats(mochi_batcher* b, uint64_t* batches, uint64_t* msgs) {
  if (!b) return MOCHI_EINVAL;
  std::lock_guard<std::mutex> lk(b->mu);
  if (batches) *batches = b->n_batches;
  if (msgs) *msgs = b->n_msgs;
  return MOCHI_OK;
}

void mochi_batcher_destroy(mochi_batcher* b) {
  if (!b) return;
  if (t_flushing == b) {
    // from one of its own callbacks: the flusher cannot join itself, so the
    // teardown is deferred -- new submissions are refused from now on, the
    // queue drains as usual, and the last flusher to leave frees the batcher
    {
      std::lock_guard<std::mutex> lk(b->mu);
      b->stop = true;
      b->deferred_delete = true;
    }
    b->cv_work.notify_all();
    return;
  }
  {
    std::lock_guard<std::mutex> lk(b->mu);
    b->stop = true;
  }
  b->cv_work.notify_all();
  for (auto& f : b->fl)
    if (f.th.joinable()) f.th.join();
  {
    std::unique_lock<std::mutex> lk(b->mu);
    b->cv_done.wait(lk, [&] { return b->waiters == 0; });  // served callers still leaving their wait
  }
  delete b;
}

}  // extern "C"
