// ThreadSanitizer harness of the engine's host scheduling (grandine_amd/csrc/gbls_sched.h):
// the per-device context pool and the cross-caller coalescer, instantiated with stub
// contexts and a stub verifier (no GPU), driven by 32+ threads that mix block-import and
// gossip calls of random sizes, key kinds and segment counts.  Every caller checks that it
// got back exactly its own verdicts and signature statuses.  Built by
// tests/test_host_sanitizers.py with -fsanitize=thread; exits nonzero on any mismatch, and
// TSan reports data races on stderr (halt_on_error=1).
//
// Reference callers: p2p/src/attestation_verifier.rs:68,142-163 (gossip batches from the
// verifier tasks), p2p/src/block_verification_pool.rs:39-49,103-128 (block batches).
// GCC 11's TSan runtime does not intercept pthread_cond_clockwait, which libstdc++ uses for
// condition_variable::wait_until on steady_clock: TSan would then believe a waiter still holds
// the mutex ("double lock").  This test build makes libstdc++ use the intercepted
// pthread_cond_timedwait instead; the engine build is unchanged.
#include <bits/c++config.h>
#undef _GLIBCXX_USE_PTHREAD_COND_CLOCKWAIT

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <future>
#include <random>
#include <thread>

#include "gbls_sched.h"

using namespace gbls;

namespace {

int g_fail = 0;
std::mutex g_fail_mu;
#define CHECK(cond, ...)                          \
  do {                                            \
    if (!(cond)) {                                \
      std::lock_guard<std::mutex> lk(g_fail_mu);  \
      std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      std::fprintf(stderr, __VA_ARGS__);          \
      std::fprintf(stderr, "\n");                 \
      g_fail++;                                   \
    }                                             \
  } while (0)

// ------------------------------------------------------------------ context pool
struct StubCtx {
  int cls = -1;
  bool used = false;
  const void *last_stream = nullptr;
  int polls = 0;                       // guarded by the pool mutex (idle_on_gpu runs under it)
  std::atomic<int> holders{0};         // leases currently holding this context
  bool idle_on_gpu() { return (++polls % 3) != 0; }
};

// (pools and coalescers live on the heap: libstdc++'s std::mutex has a trivial destructor, so a
// new mutex at a reused stack address looks to TSan like the old one)
void pool_stress() {
  auto owner = std::make_unique<sched::CtxPool<StubCtx>>();
  auto &pool = *owner;
  std::atomic<int> live[2] = {{0}, {0}};
  std::vector<std::thread> ths;
  for (int t = 0; t < 48; t++)
    ths.emplace_back([&, t] {
      std::mt19937 rng(1000 + t);
      const void *stream = reinterpret_cast<const void *>((uintptr_t)(t % 5 + 1) * 64);
      for (int k = 0; k < 400; k++) {
        const int cls = rng() % 8 == 0 ? 1 : 0;
        bool fresh = false;
        StubCtx *c = pool.acquire(rng() % 2 == 0, stream, cls, &fresh);
        CHECK(c->cls == cls, "leased class %d for %d", c->cls, cls);
        CHECK(c->holders.fetch_add(1) == 0, "context leased twice");
        CHECK(live[cls].fetch_add(1) + 1 <= sched::kMaxCtx[cls], "more live leases than the cap");
        if (rng() % 4 == 0) std::this_thread::yield();
        c->used = true;  // exclusive while leased
        c->last_stream = stream;
        live[cls].fetch_sub(1);
        c->holders.fetch_sub(1);
        pool.release(c);
      }
    });
  for (auto &th : ths) th.join();
  int n0 = 0, n1 = 0;
  for (auto &c : pool.all) (c->cls ? n1 : n0)++;
  CHECK(n0 <= sched::kMaxCtx[0] && n1 <= sched::kMaxCtx[1], "pool grew past a cap: %d %d", n0, n1);
  std::printf("pool: 48 threads x 400 leases, %d normal + %d block contexts\n", n0, n1);
}

// with every normal slot leased, a block-import lease must still succeed
void pool_block_not_starved() {
  auto owner = std::make_unique<sched::CtxPool<StubCtx>>();
  auto &pool = *owner;
  std::vector<StubCtx *> held;
  bool fresh = false;
  for (int i = 0; i < sched::kMaxCtx[0]; i++) held.push_back(pool.acquire(false, nullptr, 0, &fresh));
  auto block = std::async(std::launch::async, [&] {
    bool f = false;
    StubCtx *c = pool.acquire(false, nullptr, 1, &f);
    const int cls = c->cls;
    pool.release(c);
    return cls;
  });
  if (block.wait_for(std::chrono::seconds(10)) != std::future_status::ready) {
    std::fprintf(stderr, "FAIL: block-import lease starved by %d normal leases\n", sched::kMaxCtx[0]);
    std::fflush(stderr);
    std::_Exit(3);
  }
  CHECK(block.get() == 1, "block lease got a normal context");
  // and the reverse: every block slot leased, a normal lease still succeeds
  for (StubCtx *c : held) pool.release(c);
  std::vector<StubCtx *> bheld;
  for (int i = 0; i < sched::kMaxCtx[1]; i++) bheld.push_back(pool.acquire(false, nullptr, 1, &fresh));
  auto normal = std::async(std::launch::async, [&] {
    bool f = false;
    StubCtx *c = pool.acquire(false, nullptr, 0, &f);
    pool.release(c);
    return 0;
  });
  if (normal.wait_for(std::chrono::seconds(10)) != std::future_status::ready) {
    std::fprintf(stderr, "FAIL: normal lease starved by block leases\n");
    std::_Exit(3);
  }
  for (StubCtx *c : bheld) pool.release(c);
  std::printf("pool: block lease with %d normal leases held, normal lease with %d block leases held\n",
              sched::kMaxCtx[0], sched::kMaxCtx[1]);
}

// ------------------------------------------------------------------ coalescer
struct P1 {
  uint8_t b[96];
};
struct P2 {
  uint8_t b[192];
};
using Req = sched::Request<P1, P2>;

constexpr int32_t kOk = 0, kFail = 5;
constexpr uint8_t kPoison = 0xEE;  // a message starting with it makes the stub verifier fail

// the stub "pipeline": a segment verifies iff the sum of its sets' (message byte 0 + key byte
// 0 + signature byte 0) is even; a compressed signature decodes iff its byte 0 is not a
// multiple of 7 (else status 1).  Key bytes come from points, or from a fake registry by index.
uint8_t reg_byte(uint32_t idx) { return (uint8_t)(idx * 2654435761u >> 24); }

int32_t expected_segment(const Req &r, size_t b, size_t e) {
  unsigned sum = 0;
  for (size_t i = b; i < e; i++) {
    sum += r.msgs[32 * i];
    if (r.sigs_c) {
      if (r.sigs_c[96 * i] % 7 == 0) return kFail;  // a bad signature fails its segment
      sum += r.sigs_c[96 * i];
    } else {
      sum += r.sigs[i].b[0];
    }
    const size_t kb = r.src.off ? r.src.off[i] : i, ke = r.src.off ? r.src.off[i + 1] : i + 1;
    for (size_t k = kb; k < ke; k++) sum += r.src.pts ? r.src.pts[k].b[0] : reg_byte(r.src.idx[k]);
  }
  return sum % 2 == 0 ? kOk : kFail;
}

std::atomic<int> g_in_verify{0}, g_max_in_verify{0};

void stub_verify(Req &m) {
  const int now = g_in_verify.fetch_add(1) + 1;
  int prev = g_max_in_verify.load();
  while (now > prev && !g_max_in_verify.compare_exchange_weak(prev, now)) {
  }
  bool poison = false;
  for (size_t i = 0; i < m.n; i++) poison |= m.msgs[32 * i] == kPoison;
  for (size_t s = 0; s < m.nseg; s++) m.verdicts[s] = expected_segment(m, m.seg_off[s], m.seg_off[s + 1]);
  if (m.sigs_c)
    for (size_t i = 0; i < m.n; i++) m.sig_status[i] = m.sigs_c[96 * i] % 7 == 0 ? 1 : 0;
  std::this_thread::sleep_for(std::chrono::microseconds(50 + (m.n % 7) * 40));  // "GPU time"
  m.ok = !poison;
  m.err = poison ? 101 : 0;
  g_in_verify.fetch_sub(1);
}

void coalescer_stress() {
  auto owner = std::make_unique<sched::Coalescer<Req>>();
  auto &co = *owner;
  sched::Config cfg;
  cfg.devices = 2;
  cfg.leaders = 2;
  cfg.max_merged = 2048;
  cfg.max_merged_block = 512;
  std::atomic<int> hold{0};  // block calls hold new normal submissions while they run
  cfg.hold = &hold;
  cfg.hold_max_us = 2000;
  std::atomic<long> sets{0}, calls{0}, merged_ok{0};
  std::vector<std::thread> ths;
  const int kThreads = 32, kCalls = 150;
  for (int t = 0; t < kThreads; t++)
    ths.emplace_back([&, t] {
      std::mt19937 rng(77 + t);
      for (int k = 0; k < kCalls; k++) {
        const size_t n = 1 + rng() % 160;
        const size_t nseg = 1 + rng() % std::min<size_t>(4, n);
        std::vector<uint32_t> seg(nseg + 1, 0);
        for (size_t s = 1; s < nseg; s++) seg[s] = (uint32_t)(rng() % (n + 1));
        seg[nseg] = (uint32_t)n;
        std::sort(seg.begin(), seg.end());
        std::vector<uint8_t> msgs(32 * n);
        for (auto &x : msgs) x = (uint8_t)rng();
        for (size_t i = 0; i < n; i++)
          if (msgs[32 * i] == kPoison) msgs[32 * i] = 0;
        const bool poison = rng() % 100 == 0;
        if (poison) msgs[32 * (rng() % n)] = kPoison;
        const int kind = rng() % 4;  // 0: points, 1: indices, 2: aggregated indices, 3: compressed
        const bool block = rng() % 8 == 0;
        std::vector<P2> sigs(kind == 3 ? 0 : n);
        for (auto &s : sigs) s.b[0] = (uint8_t)rng();
        std::vector<uint8_t> sigc(kind == 3 ? 96 * n : 0);
        for (size_t i = 0; i < sigc.size(); i += 96) sigc[i] = (uint8_t)(rng() % 50 == 0 ? 14 : 1 + rng() % 6);
        std::vector<P1> pts;
        std::vector<uint32_t> idx, off;
        if (kind == 0 || kind == 3) {
          pts.resize(n);
          for (auto &p : pts) p.b[0] = (uint8_t)rng();
        } else if (kind == 1) {
          idx.resize(n);
          for (auto &x : idx) x = rng();
        } else {
          off.push_back(0);
          for (size_t i = 0; i < n; i++) {
            const size_t c = 1 + rng() % 5;
            for (size_t j = 0; j < c; j++) idx.push_back(rng());
            off.push_back((uint32_t)idx.size());
          }
        }
        std::vector<uint64_t> rands(n, 1);
        std::vector<int32_t> v(nseg, -1), st(kind == 3 ? n : 0, -1);
        Req r{msgs.data(), kind == 3 ? nullptr : sigs.data(), sched::KeySource<P1>(), rands.data(), n,
              seg.data(), nseg, v.data()};
        if (!pts.empty()) r.src.pts = pts.data();
        else r.src.idx = idx.data();
        if (!off.empty()) r.src.off = off.data();
        if (kind == 3) {
          r.sigs_c = sigc.data();
          r.sig_status = st.data();
        }
        r.prio = block ? 1 : 0;
        if (block) hold.fetch_add(1);
        const bool ok = co.submit(r, cfg, stub_verify);
        if (block && hold.fetch_sub(1) == 1) co.wake();
        calls++;
        sets += (long)n;
        CHECK(r.done, "returned before done");
        if (poison) CHECK(!ok && r.err == 101, "poisoned call not failed");
        if (!ok) {
          CHECK(r.err == 101, "failure without the verifier's error code (%d)", r.err);
          continue;  // a call merged with a poisoned one fails closed with the error code
        }
        merged_ok++;
        CHECK(r.err == 0, "stale error code %d", r.err);
        for (size_t s = 0; s < nseg; s++)
          CHECK(v[s] == expected_segment(r, seg[s], seg[s + 1]), "thread %d call %d segment %zu: verdict %d",
                t, k, s, v[s]);
        for (size_t i = 0; i < st.size(); i++)
          CHECK(st[i] == (sigc[96 * i] % 7 == 0 ? 1 : 0), "thread %d call %d set %zu: status %d", t, k, i, st[i]);
      }
    });
  for (auto &th : ths) th.join();
  const int bound = cfg.leaders * cfg.devices + cfg.devices;  // normal + block leaders
  CHECK(g_max_in_verify.load() <= bound, "%d concurrent submissions > %d leaders", g_max_in_verify.load(), bound);
  std::printf("coalescer: %d threads, %ld calls (%ld sets; %ld with a verdict), at most %d submissions in flight\n",
              kThreads, calls.load(), sets.load(), merged_ok.load(), g_max_in_verify.load());
}

}  // namespace

int main() {
  pool_block_not_starved();
  pool_stress();
  coalescer_stress();
  if (g_fail) {
    std::fprintf(stderr, "%d failures\n", g_fail);
    return 1;
  }
  std::printf("sched_tsan: OK\n");
  return 0;
}
