// Host-side scheduling of the engine: the per-device context pool and the cross-caller
// coalescer (f3).  Host-only C++ (no HIP): gbls_capi.hip instantiates it with its HIP
// contexts and its verification pipeline; tests/native/sched_tsan.cpp instantiates it with
// stub contexts and a stub verifier and runs it under ThreadSanitizer with 32 threads.
//
// Callers arrive concurrently from rayon workers, the de-low executor, the block
// verification pool and fork-choice workers (reference p2p/src/attestation_verifier.rs:68,
// 142-163; p2p/src/block_verification_pool.rs:39-49,103-128).
#pragma once

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <memory>
#include <mutex>
#include <vector>

namespace gbls {
namespace sched {

// ---------------------------------------------------------------- context pool
// Two classes of contexts: 0 = normal, 1 = block import (every stream at the highest
// priority).  Each class has its own cap, so a burst of normal calls (e.g. signature
// decompressions from every rayon worker) can never use up the slots block import needs, and
// the reverse.
constexpr int kClasses = 2;
constexpr int kMaxCtx[kClasses] = {64, 16};

// Ctx needs: int cls; bool used; <stream> last_stream; bool idle_on_gpu() (called under the
// pool mutex).
template <class Ctx>
struct CtxPool {
  std::mutex mu;
  std::condition_variable cv;
  std::vector<Ctx *> idle;
  std::vector<std::unique_ptr<Ctx>> all;
  int count[kClasses] = {0, 0};

  // A context of class `cls`: the idle one last used on `stream` (affine: stream order makes
  // its reuse free), else an idle one whose previous call has finished on the GPU, else a new
  // one (up to the class cap; *fresh = true, the caller initialises it), else the least
  // recently released idle one of the class (its reuse is ordered behind its previous call on
  // the GPU), else wait until one of the class comes back.
  template <class Stream>
  Ctx *acquire(bool affine, Stream stream, int cls, bool *fresh) {
    cls = cls ? 1 : 0;
    *fresh = false;
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      Ctx *c = nullptr;
      for (size_t i = 0; affine && !c && i < idle.size(); i++)
        if (idle[i]->cls == cls && idle[i]->used && idle[i]->last_stream == stream) c = take(i);
      for (size_t i = 0; !c && i < idle.size(); i++)
        if (idle[i]->cls == cls && idle[i]->idle_on_gpu()) c = take(i);
      if (!c && count[cls] < kMaxCtx[cls]) {
        all.emplace_back(new Ctx());
        c = all.back().get();
        c->cls = cls;
        count[cls]++;
        *fresh = true;
      }
      for (size_t i = 0; !c && i < idle.size(); i++)
        if (idle[i]->cls == cls) c = take(i);
      if (c) return c;
      cv.wait(lk);  // every context of this class is leased: wait for one to come back
    }
  }
  // a new idle context of class cls, initialised by init(ctx) before any caller can lease it
  // (engine start: the first concurrent calls then find contexts instead of creating them)
  template <class Init>
  bool prewarm(int cls, Init &&init) {
    cls = cls ? 1 : 0;
    std::unique_ptr<Ctx> c(new Ctx());
    c->cls = cls;
    if (!init(*c)) return false;
    std::lock_guard<std::mutex> lk(mu);
    if (count[cls] >= kMaxCtx[cls]) return false;
    count[cls]++;
    idle.push_back(c.get());
    all.push_back(std::move(c));
    return true;
  }
  void release(Ctx *c) {
    {
      std::lock_guard<std::mutex> lk(mu);
      idle.push_back(c);
    }
    cv.notify_all();  // waiters of either class
  }
  size_t size() {
    std::lock_guard<std::mutex> lk(mu);
    return all.size();
  }
  // f(ctx) for every context, leased or idle (under the pool mutex: f must not block)
  template <class F>
  void for_each(F &&f) {
    std::lock_guard<std::mutex> lk(mu);
    for (auto &c : all) f(*c);
  }

 private:
  Ctx *take(size_t i) {
    Ctx *c = idle[i];
    idle.erase(idle.begin() + (std::ptrdiff_t)i);
    return c;
  }
};

// ---------------------------------------------------------------- coalescer
template <class G1>
struct KeySource {
  const G1 *pts = nullptr;        // points: one per set (off == nullptr) or summed per set
  const uint32_t *idx = nullptr;  // registry indices: one per set (off == nullptr) or summed
  const uint32_t *off = nullptr;  // per-set ranges [off[i], off[i+1]) of pts / idx
};

// One caller's batch (host pointers, borrowed for the call).  rands == nullptr: independent
// single checks (Signature::verify / fast_aggregate_verify semantics: r_i = 1, the
// signature's subgroup check, one segment per set), merged only with other single checks.
template <class G1, class G2>
struct Request {
  using g1_type = G1;
  using g2_type = G2;
  const uint8_t *msgs;
  const G2 *sigs;
  KeySource<G1> src;
  const uint64_t *rands;
  size_t n;
  const uint32_t *seg_off;
  size_t nseg;
  int32_t *verdicts;
  const uint8_t *sigs_c = nullptr;  // compressed signatures instead of sigs (96 B each)
  int32_t *sig_status = nullptr;    // their decompression statuses (with sigs_c)
  int prio = 0;                     // 1: block import
  bool done = false, ok = false;
  int err = 0;                      // the verifier's side-channel error code
  int kind() const {
    return (src.pts ? 1 : 0) | (src.off ? 2 : 0) | (sigs_c ? 4 : 0) | (rands ? 0 : 8);
  }
  size_t nkeys() const { return src.off ? src.off[n] : n; }
};

struct Config {
  bool coalesce = true;
  int devices = 1;
  int leaders = 2;                  // normal leaders per device (block import: 1 per device)
  size_t max_merged = 1 << 16;      // merged normal submissions stay below one C2 step
  size_t max_merged_block = 8192;   // block import: the latency cap
  size_t merge_target = 768;        // a new leader's collection window ends at this many sets
  int merge_window_us = 300;        // ... or after this long (only while another is in flight)
  // while *hold > 0 (a block import in progress), a normal request does not start a new
  // submission for up to hold_max_us: the block shares the GPU only with the normal
  // submissions already running (null: never hold)
  const std::atomic<int> *hold = nullptr;
  int hold_max_us = 4000;
};

// Runs the requests of `batch` (all of one kind) as ONE segmented verification: the merged
// request is handed to verify(Req &) (which sets ok and err), then every caller's verdicts and
// signature statuses are copied back from its own range.
template <class Req, class Verify>
void run_merged(std::vector<Req *> &batch, Verify &&verify) {
  if (batch.size() == 1) {
    verify(*batch[0]);
    return;
  }
  using G1 = typename Req::g1_type;
  using G2 = typename Req::g2_type;
  size_t n = 0, nseg = 0, nk = 0;
  for (Req *r : batch) {
    n += r->n;
    nseg += r->nseg;
    nk += r->nkeys();
  }
  const Req &r0 = *batch[0];
  const bool comp = r0.sigs_c != nullptr, single = r0.rands == nullptr;
  std::vector<uint8_t> msgs(32 * n), sigc(comp ? 96 * n : 0);
  std::vector<G2> sigs(comp ? 0 : n);
  std::vector<int32_t> sst(comp ? n : 0, 1 /* BAD_ENCODING until decoded */);
  std::vector<uint64_t> rands(single ? 0 : n);
  std::vector<G1> pts;
  std::vector<uint32_t> idx, off, seg(nseg + 1);
  if (r0.src.pts)
    pts.resize(nk);
  else
    idx.resize(nk);
  if (r0.src.off) off.resize(n + 1);
  std::vector<int32_t> v(nseg, 5 /* VERIFY_FAIL */);
  size_t at = 0, sat = 0, kat = 0;
  seg[0] = 0;
  for (Req *r : batch) {
    std::memcpy(&msgs[32 * at], r->msgs, 32 * r->n);
    if (comp)
      std::memcpy(&sigc[96 * at], r->sigs_c, 96 * r->n);
    else
      std::memcpy(&sigs[at], r->sigs, r->n * sizeof(G2));
    if (!single) std::memcpy(&rands[at], r->rands, r->n * 8);
    const size_t k = r->nkeys();
    if (r0.src.pts)
      std::memcpy(&pts[kat], r->src.pts, k * sizeof(G1));
    else
      std::memcpy(&idx[kat], r->src.idx, k * 4);
    if (r0.src.off)
      for (size_t i = 0; i <= r->n; i++) off[at + i] = (uint32_t)(kat + r->src.off[i]);
    for (size_t s = 1; s <= r->nseg; s++) seg[sat + s] = (uint32_t)(at + r->seg_off[s]);
    at += r->n;
    sat += r->nseg;
    kat += k;
  }
  Req m{msgs.data(), comp ? nullptr : sigs.data(), KeySource<G1>(), single ? nullptr : rands.data(),
        n, seg.data(), nseg, v.data()};
  if (r0.src.pts)
    m.src.pts = pts.data();
  else
    m.src.idx = idx.data();
  if (r0.src.off) m.src.off = off.data();
  if (comp) {
    m.sigs_c = sigc.data();
    m.sig_status = sst.data();
  }
  m.prio = r0.prio;
  verify(m);
  sat = 0;
  at = 0;
  for (Req *r : batch) {
    std::memcpy(r->verdicts, &v[sat], r->nseg * 4);
    if (comp) std::memcpy(r->sig_status, &sst[at], r->n * 4);
    sat += r->nseg;
    at += r->n;
    r->ok = m.ok;
    r->err = m.err;
  }
}

// Concurrent batch verifications queue here; a caller that finds fewer than
// leaders x devices submissions in flight becomes a leader and verifies every queued request
// with the same key-source kind as ONE segmented submission (each keeping its own segments
// and verdicts), up to max_merged sets.  Block import (prio) has its own queue and leader
// slot per device, is merged only with other block requests (up to max_merged_block sets) and
// never waits in a collection window.
template <class Req>
class Coalescer {
 public:
  template <class Verify>
  bool submit(Req &r, const Config &cfg, Verify &&verify) {
    if (!cfg.coalesce) {
      verify(r);
      return r.ok;
    }
    const int max_leaders = (r.prio ? 1 : cfg.leaders) * std::max(1, cfg.devices);
    const size_t cap = r.prio ? cfg.max_merged_block : cfg.max_merged;
    std::vector<Req *> &q = r.prio ? pq_ : q_;
    int &leaders = r.prio ? pleaders_ : leaders_;
    std::unique_lock<std::mutex> lk(mu_);
    q.push_back(&r);
    cv_.notify_all();  // a leader collecting a batch (below) sees the new request at once
    bool waited = false, held = false;
    while (!r.done) {
      if (!r.prio && !held && cfg.hold && cfg.hold->load() > 0) {
        held = true;  // a block import is being verified: leave it the GPU for a while
        const auto deadline =
            std::chrono::steady_clock::now() + std::chrono::microseconds(cfg.hold_max_us);
        cv_.wait_until(lk, deadline, [&] { return r.done || cfg.hold->load() == 0; });
        continue;
      }
      if (leaders < max_leaders && !q.empty()) {
        // Another submission is already in flight: the GPU is busy, so a short collection
        // window costs little latency and lets the callers that return from that submission
        // join this one (without it the first of them leads a batch of one).  Never for block
        // import, never on an idle engine.
        auto queued = [&q]() {
          size_t t = 0;
          for (const Req *x : q) t += x->n;
          return t;
        };
        if (!r.prio && leaders > 0 && !waited && queued() < cfg.merge_target) {
          waited = true;
          const auto deadline =
              std::chrono::steady_clock::now() + std::chrono::microseconds(cfg.merge_window_us);
          cv_.wait_until(lk, deadline, [&] { return r.done || queued() >= cfg.merge_target; });
          continue;
        }
        leaders++;
        std::vector<Req *> batch;
        auto mine = std::find(q.begin(), q.end(), &r);
        const int kind = mine != q.end() ? r.kind() : q.front()->kind();
        size_t sets = 0;
        if (mine != q.end()) {
          batch.push_back(&r);
          sets = r.n;
          q.erase(mine);
        }
        for (auto it = q.begin(); it != q.end();) {
          if ((*it)->kind() == kind && (batch.empty() || sets + (*it)->n <= cap)) {
            sets += (*it)->n;
            batch.push_back(*it);
            it = q.erase(it);
          } else {
            ++it;
          }
        }
        lk.unlock();
        run_merged(batch, verify);  // writes verdicts, ok, err; `done` is published under mu_
        lk.lock();
        for (Req *b : batch) b->done = true;
        leaders--;
        cv_.notify_all();
      } else {
        cv_.wait(lk);
      }
    }
    return r.ok;
  }
  // wake waiting callers (e.g. when the hold of Config::hold is released)
  void wake() {
    std::lock_guard<std::mutex> lk(mu_);
    cv_.notify_all();
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<Req *> q_, pq_;  // normal and block-import queues
  int leaders_ = 0, pleaders_ = 0;
};

}  // namespace sched
}  // namespace gbls
