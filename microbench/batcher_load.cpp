// batcher_load — native load driver for the drop-in micro-batcher.
//
// What a Netty/JNI MochiDB server would see of libmochi_hip: T native threads
// (the reference's Write2 worker pool is core 2 / max 20, MochiServer.java:36-40)
// each calling mochi_batcher_verify on one Write2ToServer body at a time
// (mode "sync"), or T event-loop threads keeping up to `window` bodies in
// flight through mochi_batcher_submit with a completion callback ("async").
// No Python anywhere on the request path, so the numbers are the library's.
//
//   batcher_load <input.bin> <requests> <max_msgs> <max_wait_us> <mode:threads:contexts[:window[:requests]]>...
//
// e.g. `... sync:2:1 sync:20:2 sync:64:2 async:4:2:8192`: one JSON line per
// configuration.  If input.bin does not exist yet the driver waits for it (up
// to 10 minutes): bench.py starts the driver before it touches the GPU itself
// and writes the input once its workload exists, then waits for the driver.
//
// input.bin (written by bench.py / tests, little-endian):
//   "MOCHIW2\0", u32 R, u32 M, R x 256 B moduli (big-endian),
//   u32 ids_len, ids blob, (R+1) x u32 id_off,
//   u64 wire_len, wire, M x u64 msg_off, M x u32 msg_len, M x 128 B expected hash,
//   M x u8 expected reason, M x u8 expected accept
// Request i sends message i % M; every verdict is checked against the expected
// one.  Prints one JSON line.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../include/mochi_hip.h"

namespace {

using Clock = std::chrono::steady_clock;

struct Input {
  uint32_t R = 0, M = 0;
  std::vector<uint8_t> moduli, ids, wire, hashes, reason, accept;
  std::vector<uint32_t> id_off, len;
  std::vector<uint64_t> off;
};

bool rd(FILE* f, void* p, size_t n) { return fread(p, 1, n, f) == n; }

bool load(const char* path, Input& in) {
  FILE* f = fopen(path, "rb");
  if (!f) return false;
  char magic[8];
  bool ok = rd(f, magic, 8) && memcmp(magic, "MOCHIW2", 8) == 0 && rd(f, &in.R, 4) && rd(f, &in.M, 4);
  if (ok) {
    in.moduli.resize((size_t)in.R * 256);
    uint32_t ids_len = 0;
    ok = rd(f, in.moduli.data(), in.moduli.size()) && rd(f, &ids_len, 4);
    in.ids.resize(ids_len);
    in.id_off.resize(in.R + 1);
    ok = ok && rd(f, in.ids.data(), ids_len) && rd(f, in.id_off.data(), 4 * (in.R + 1));
    uint64_t wl = 0;
    ok = ok && rd(f, &wl, 8);
    in.wire.resize(wl);
    in.off.resize(in.M);
    in.len.resize(in.M);
    in.hashes.resize((size_t)in.M * MOCHI_TXN_HASH_BYTES);
    in.reason.resize(in.M);
    in.accept.resize(in.M);
    ok = ok && rd(f, in.wire.data(), wl) && rd(f, in.off.data(), 8 * (size_t)in.M) &&
         rd(f, in.len.data(), 4 * (size_t)in.M) && rd(f, in.hashes.data(), in.hashes.size()) &&
         rd(f, in.reason.data(), in.M) && rd(f, in.accept.data(), in.M);
  }
  fclose(f);
  return ok && in.M > 0;
}

double pct(std::vector<double>& v, double p) {
  if (v.empty()) return 0;
  const size_t i = std::min(v.size() - 1, (size_t)(p / 100.0 * (double)(v.size() - 1) + 0.5));
  std::nth_element(v.begin(), v.begin() + i, v.end());
  return v[i];
}

// async mode: a shared window of in-flight requests
struct Window {
  std::mutex mu;
  std::condition_variable cv;
  uint32_t free;
  uint64_t left;
};

struct Slot {
  Clock::time_point t0;
  uint32_t msg;
  double* lat;
  std::atomic<uint64_t>* bad;
  const Input* in;
  Window* w;
};

void on_done(void* user, int rc, const mochi_verdict1* v) {
  Slot* s = (Slot*)user;
  *s->lat = std::chrono::duration<double, std::micro>(Clock::now() - s->t0).count();
  if (rc != MOCHI_OK || v->reason != s->in->reason[s->msg] || v->accepted != s->in->accept[s->msg]) (*s->bad)++;
  Window* w = s->w;
  std::lock_guard<std::mutex> lk(w->mu);  // notify under the lock: the waiter may free w once left == 0
  w->free++;
  w->left--;
  w->cv.notify_all();
}

}  // namespace

// One configuration: T threads, NC contexts; prints one JSON line.
int run(const Input& in, bool async, uint32_t T, uint32_t NC, uint64_t N, uint32_t window, uint32_t max_msgs,
        uint32_t max_wait) {
  std::vector<mochi_ctx*> ctx(NC);
  for (uint32_t i = 0; i < NC; i++) {
    ctx[i] = mochi_ctx_create(0, in.moduli.data(), in.R, 256, 65537);
    if (!ctx[i] || mochi_ctx_set_server_ids(ctx[i], in.ids.data(), in.id_off.data(), in.R) != MOCHI_OK) {
      fprintf(stderr, "context: %s\n", mochi_last_error());
      return 1;
    }
  }
  mochi_params p;
  memset(&p, 0, sizeof p);
  p.replication_factor = in.R;
  p.strict_gt = 1;
  mochi_batcher* b = mochi_batcher_create_multi(ctx.data(), NC, &p, max_msgs, max_wait, 0);
  if (!b) {
    fprintf(stderr, "batcher creation failed\n");
    return 1;
  }
  const uint8_t* wire = in.wire.data();
  auto msg = [&](uint64_t i) { return (uint32_t)(i % in.M); };
  // warm-up: every context sizes its buffers on its first batches
  {
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < std::max<uint32_t>(T, 2 * NC); t++)
      th.emplace_back([&, t] {
        for (uint32_t i = t; i < std::min<uint32_t>(in.M, 1024); i += std::max<uint32_t>(T, 2 * NC)) {
          mochi_verdict1 v;
          (void)mochi_batcher_verify(b, wire + in.off[i], in.len[i], nullptr, 0, in.hashes.data() + (size_t)i * 128,
                                     &v);
        }
      });
    for (auto& x : th) x.join();
  }
  uint64_t nb0 = 0, nm0 = 0;
  mochi_batcher_stats(b, &nb0, &nm0);
  std::vector<double> lat(N);
  std::atomic<uint64_t> bad{0};
  const auto t0 = Clock::now();
  if (!async) {
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < T; t++)
      th.emplace_back([&, t] {
        for (uint64_t i = t; i < N; i += T) {
          const uint32_t m = msg(i);
          mochi_verdict1 v;
          const auto s = Clock::now();
          const int rc = mochi_batcher_verify(b, wire + in.off[m], in.len[m], nullptr, 0,
                                              in.hashes.data() + (size_t)m * 128, &v);
          lat[i] = std::chrono::duration<double, std::micro>(Clock::now() - s).count();
          if (rc != MOCHI_OK || v.reason != in.reason[m] || v.accepted != in.accept[m]) bad++;
        }
      });
    for (auto& x : th) x.join();
  } else {
    Window w;
    w.free = window;
    w.left = N;
    std::vector<Slot> slots(N);
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < T; t++)
      th.emplace_back([&, t] {
        for (uint64_t i = t; i < N; i += T) {
          {
            std::unique_lock<std::mutex> lk(w.mu);
            w.cv.wait(lk, [&] { return w.free > 0; });
            w.free--;
          }
          const uint32_t m = msg(i);
          Slot& s = slots[i];
          s.msg = m;
          s.lat = &lat[i];
          s.bad = &bad;
          s.in = &in;
          s.w = &w;
          s.t0 = Clock::now();
          if (mochi_batcher_submit(b, wire + in.off[m], in.len[m], nullptr, 0, in.hashes.data() + (size_t)m * 128,
                                   on_done, &s) != MOCHI_OK) {
            bad++;
            std::lock_guard<std::mutex> lk(w.mu);
            w.free++;
            w.left--;
            w.cv.notify_all();
          }
        }
      });
    for (auto& x : th) x.join();
    std::unique_lock<std::mutex> lk(w.mu);
    w.cv.wait(lk, [&] { return w.left == 0; });
  }
  const double wall = std::chrono::duration<double>(Clock::now() - t0).count();
  uint64_t nb = 0, nm = 0;
  mochi_batcher_stats(b, &nb, &nm);
  mochi_batcher_destroy(b);
  for (auto* c : ctx) mochi_ctx_destroy(c);
  const double mx = *std::max_element(lat.begin(), lat.end());
  printf("{\"mode\": \"%s\", \"threads\": %u, \"contexts\": %u, \"requests\": %llu, \"window\": %u, "
         "\"requests_per_s\": %.1f, \"latency_us\": {\"p50\": %.1f, \"p99\": %.1f, \"max\": %.1f}, "
         "\"gpu_batches\": %llu, \"mean_batch_msgs\": %.2f, \"verdict_mismatches\": %llu, \"wall_s\": %.3f}\n",
         async ? "async" : "sync", T, NC, (unsigned long long)N, async ? window : 0, (double)N / wall, pct(lat, 50),
         pct(lat, 99), mx, (unsigned long long)(nb - nb0), (double)(nm - nm0) / (double)std::max<uint64_t>(1, nb - nb0),
         (unsigned long long)bad.load(), wall);
  fflush(stdout);
  return bad.load() ? 3 : 0;
}

int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: %s input.bin requests max_msgs max_wait_us mode:threads:contexts[:window]...\n", argv[0]);
    return 2;
  }
  for (int i = 0; i < 12000; i++) {  // wait for the input (written once the caller's workload exists)
    FILE* f = fopen(argv[1], "rb");
    if (f) {
      fclose(f);
      break;
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
  }
  Input in;
  if (!load(argv[1], in)) {
    fprintf(stderr, "cannot read %s\n", argv[1]);
    return 2;
  }
  const uint64_t N = strtoull(argv[2], nullptr, 10);
  const uint32_t max_msgs = (uint32_t)atoi(argv[3]), max_wait = (uint32_t)atoi(argv[4]);
  int worst = 0;
  for (int a = 5; a < argc; a++) {
    char mode[16] = {0};
    unsigned T = 0, NC = 0, W = 8192;
    unsigned long long n = N;
    if (sscanf(argv[a], "%15[a-z]:%u:%u:%u:%llu", mode, &T, &NC, &W, &n) < 3 || T == 0 || NC == 0 || n == 0) {
      fprintf(stderr, "bad configuration %s\n", argv[a]);
      return 2;
    }
    const int rc = run(in, strcmp(mode, "async") == 0, T, NC, n, W, max_msgs, max_wait);
    if (rc == 1) return 1;
    worst = std::max(worst, rc);
  }
  return worst;
}
