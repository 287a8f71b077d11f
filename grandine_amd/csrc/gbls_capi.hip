// C ABI of the MI355X BLS12-381 engine: host-side orchestration of the gfx950 kernels
// (k_*.hip).  Entry points, their reference counterparts and semantics are documented
// in include/grandine_bls_gpu.h.
//
// Concurrency model (rayon workers, the de-low executor, the block
// verification pool and fork-choice workers all call in concurrently):
//   * one Device per GPU of gbls_init's device mask (optionally several engines per
//     GPU, for tests of the multi-device paths on one card);
//   * every call leases a Ctx -- streams, events, grow-only workspaces, a pinned
//     staging buffer -- from its device's pool, so concurrent callers run side by side
//     on separate streams with no shared scratch;
//   * a Ctx is handed to the next caller only behind a GPU-side wait on the completion
//     event of its previous call (device-pointer calls return before their kernels
//     finish), and its buffers are only regrown after a host wait on that event;
//   * host-pointer calls shard big batches over the devices: whole segments per device,
//     or, for one large batch, per-device Miller partials combined by one final
//     exponentiation.
// Every failure is fail-closed: GBLS_VERIFY_FAIL (verdict arrays filled with it first)
// plus a thread-local gbls_last_error code.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <chrono>
#include <cerrno>
#include <sys/random.h>
#include <mutex>
#include <shared_mutex>
#include <vector>

#include "../../include/grandine_bls_gpu.h"
#include "gbls_common.h"
#include "gbls_sched.h"
#include "gbls_tables.h"

using namespace gbls;

static_assert(gbls::kTableWave == (uint32_t)gbls::WG, "k_ml_group wave");

static_assert(sizeof(g1a) == sizeof(gbls_p1_affine), "p1 layout");
static_assert(sizeof(g2a) == sizeof(gbls_p2_affine), "p2 layout");
static_assert(sizeof(fp12) == sizeof(gbls_fp12), "fp12 layout");

uint32_t gbls::g_row_clear_max = gbls::kRowClearMax;
uint32_t gbls::g_ml_r28 = 1;
uint32_t gbls::g_msm_k = 0;  // chosen per plan (msm_plan) unless GBLS_MSM_K is set
uint32_t gbls::g_msm_r28 = 1;
uint32_t gbls::g_ml_xcd = 1;
uint32_t gbls::g_ml_dma = 0;
uint32_t gbls::g_ml_prefetch = 1;
uint32_t gbls::g_ml_kara = 0;
uint32_t gbls::g_lane_r28 = 1;
uint32_t gbls::g_lane_min = gbls::kLaneRegimeSets;
uint32_t gbls::g_clear_staged = 0;
uint32_t gbls::g_map_rows_max = 2048;

namespace {

constexpr int FAILED = GBLS_VERIFY_FAIL;  // engine/driver failure return (fail closed)
constexpr size_t kShardMinSets = 1024;     // per device, before a batch is split
// contexts per device created by gbls_init (normal, block import).  Measured r06
// (profiles/r06/README.md, tools/gpu/ab_c2c4.sh): HIP binds every stream to a hardware queue of
// its priority when the stream is created (up to GPU_MAX_HW_QUEUES per priority), and the set of
// queues a process holds moves the default bench by several per cent.  Two normal contexts (two
// submissions in flight) plus the registry's high-priority update stream, created here in that
// order, measured best on every leg in one box: C2 4.37-4.40M sets/s, a single 4096-set batch
// 779-790k, C4 525-537k.  With the block context as well (3 more high-priority queues) the single
// batch drops to ~690k; with one more normal-priority queue (the registry's retire stream, now
// created by the first table growth) to ~685k; without the third high-priority queue C2 varies
// 4.20-4.35M; and creating contexts inside a timed loop costs C4 a third (350-390k).
// Block-import contexts are created by the first block import.
constexpr int kPrewarmCtx[2] = {2, 0};
// submissions of at least this many Miller pairs read normalized points (k_ml_pcols)
constexpr uint32_t kPcnMinPairs = 32768;

thread_local int t_last_error = GBLS_ERR_NONE;

bool fail(int code) {
  t_last_error = code;
  return false;
}

#define HIPCHK(x)                  \
  do {                             \
    if ((x) != hipSuccess) {       \
      t_last_error = GBLS_ERR_HIP; \
      return false;                \
    }                              \
  } while (0)

// the byte size a buffer grows to for `bytes`
inline size_t grow_size(size_t bytes) { return bytes < 4096 ? 4096 : bytes + bytes / 4; }

struct Buf {
  void *p = nullptr;
  size_t cap = 0;
  bool pooled = false;  // p from hipMallocAsync (freed by hipFreeAsync)
  // synchronous allocation (devices without stream-ordered allocation; scratch outside a lease)
  bool ensure(size_t bytes) {
    if (bytes <= cap) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    pooled = false;
    size_t want = grow_size(bytes);
    if (hipMalloc(&p, want) != hipSuccess) return false;
    cap = want;
    return true;
  }
  template <class T>
  T *as() const {
    return reinterpret_cast<T *>(p);
  }
};

// ---- optional per-stage timing (HIP events on the launch stream), for bench.py
enum Stage {
  S_H2C_FIELD, S_H2C_MAP, S_H2C_CLEAR, S_G1MUL, S_G2MUL, S_G2SUM, S_LINES, S_LINES_S, S_ML_LEAF,
  S_ML_REDUCE, S_ML_HORNER, S_FINAL, S_PK_GATHER, S_MSM, S_COUNT
};
const char *kStageNames[S_COUNT] = {"k_h2c_field", "k_h2c_map",   "k_h2c_clear", "k_mv_g1mul",
                                    "k_mv_g2mul",  "k_g2sum",      "k_lines",     "k_lines_S",
                                    "k_ml_group",  "k_ml_reduce",  "k_ml_horner", "k_final_verdict",
                                    "k_pk_resolve", "k_msm"};

// GBLS_TRACE_STALLS=1: report host waits inside device entry points (diagnostics); every line
// carries the call index (leases since gbls_init) and whether the lease created its context
static bool trace_stalls() {
  static const bool on = [] {
    const char *e = std::getenv("GBLS_TRACE_STALLS");
    return e && *e == '1';
  }();
  return on;
}
std::atomic<unsigned long long> g_lease_calls{0};

// Workspaces grow by stream-ordered allocation (hipMallocAsync / hipFreeAsync from the device's
// default pool) when the device supports it: a growth never waits on the host and never frees
// through hipFree, which synchronises the whole device (every other caller's work included).
// Set once by engine_init.
bool g_stream_alloc = false;

struct Prof {
  std::mutex mu;
  std::atomic<bool> on{false};
  struct Rec {
    int stage;
    hipEvent_t a, b;
  };
  std::vector<Rec> pending;
  // timing events are reused (gbls_profile_read returns them here) and a batch is created when
  // profiling is switched on, so that no hipEventCreate runs inside a profiled call: creating
  // events while kernels run took milliseconds at times (r05 C4 enqueue stalls)
  std::vector<hipEvent_t> free_ev;
  double ms[S_COUNT] = {0};
  uint32_t calls[S_COUNT] = {0};
  bool take(hipEvent_t &a, hipEvent_t &b) {
    {
      std::lock_guard<std::mutex> lk(mu);
      if (free_ev.size() >= 2) {
        a = free_ev.back();
        free_ev.pop_back();
        b = free_ev.back();
        free_ev.pop_back();
        return true;
      }
    }
    if (hipEventCreate(&a) != hipSuccess) return false;
    if (hipEventCreate(&b) != hipSuccess) {
      (void)hipEventDestroy(a);
      return false;
    }
    return true;
  }
} prof;

struct StageTimer {  // RAII: events around one stage's launches when profiling
  hipEvent_t a = nullptr, b = nullptr;
  hipStream_t st;
  int stage;
  StageTimer(int s, hipStream_t stream) : st(stream), stage(s) {
    if (!prof.on.load(std::memory_order_relaxed)) return;
    if (!prof.take(a, b)) {
      a = b = nullptr;
      return;
    }
    (void)hipEventRecord(a, st);
  }
  ~StageTimer() {
    if (!a || !b) return;
    (void)hipEventRecord(b, st);
    std::lock_guard<std::mutex> lk(prof.mu);
    prof.pending.push_back({stage, a, b});
  }
};

// ---------------------------------------------------------------- per-call context
struct Ctx {
  int hipdev = -1;
  hipStream_t own = nullptr, side1 = nullptr, side2 = nullptr;
  // latency-regime streams on disjoint CU sets (created on first use, see cu_split): the
  // main chain's waves never share a SIMD with the side streams' waves
  hipStream_t own_m = nullptr, side1_m = nullptr, side2_m = nullptr;
  // normal-class streams kept off the CUs reserved for block import while a block is being
  // verified (created on first use, see Engine::block_reserve)
  hipStream_t own_g = nullptr, side1_g = nullptr, side2_g = nullptr;
  const uint32_t *line_col = nullptr;  // the last pipeline's line columns (LineCols), in tab
  uint32_t line_ncol = 0;
  hipEvent_t ev_fork = nullptr, ev_side1 = nullptr, ev_side2 = nullptr, ev_pks = nullptr,
             ev_done = nullptr, ev_in = nullptr, ev_out = nullptr;
  bool done_pending = false;
  // buffer growth: old buffers are freed and new ones allocated on `own`, ordered (GPU-side, by
  // ev_grow) behind every other stream of the context and ahead of their later work
  hipEvent_t ev_grow = nullptr;
  // pinned staging buffers replaced by bigger ones: hipHostFree synchronises the device, so they
  // are kept (growth doubles, so they total less than the live ring) instead of freed mid-call
  std::vector<void *> retired_host;
  unsigned long long call_id = 0;  // diagnostics: the lease's call index, and whether it
  bool fresh = false;              // created this context
  // recorded behind this context's last kernel that read the validator registry (written under
  // the shared registry lock, read by gbls_registry_set under the exclusive one): a grown
  // registry's old table is freed only after every such reader
  hipEvent_t ev_reg = nullptr;
  bool reg_read = false;
  int cls = 0;                        // 0: normal, 1: block import (every stream high priority)
  bool active = false;                // a call holds the lease and has begun
  hipStream_t cur = nullptr;          // its main stream (nullptr = the legacy default stream)
  bool used = false;                  // last_stream is meaningful
  hipStream_t last_stream = nullptr;  // main stream of the previous call
  Buf in0, in1, in2, in3, in4, in5, U, Q, H, P, Pc, R, Sj, gpart, lines, Ts, V0, V1, V28, hparts, tab, part, err, out0,
      out1, pks, pre, pre2, msm, sigd, sigst, rnd, ng1, gerr, gv, redo, rtab;
  // per-call option of the next pipeline_partials on this lease: compressed signatures
  // (96 B each, device) to decompress on the signature-side stream into `sigs`, with their
  // BLST_ERROR statuses (device) failing their segments (consumed and reset by the pipeline)
  const uint8_t *sig_c = nullptr;
  int32_t *sig_st = nullptr;
  // Pinned staging for host tables and host inputs: a ring of kStageRing buffers, one per call,
  // each recycled only once the uploads of the call that used it have landed.  (One buffer made
  // every call wait on the host for the previous call's uploads, which are queued behind that
  // call's predecessor on the GPU: a device entry point ran at most ~2 calls ahead of the GPU.)
  static constexpr int kStageRing = 4;
  struct Stage {
    void *p = nullptr;
    size_t cap = 0;
    hipEvent_t ev = nullptr;  // after this buffer's last upload
    bool pending = false;
  } ring[kStageRing];
  int stage_at = 0;
  size_t stage_used = 0;
  std::vector<uint32_t> host_tab;  // table assembly, reused across calls

  bool init(int dev, bool side2_high, int prio_mode, int klass) {
    hipdev = dev;
    cls = klass;
    HIPCHK(hipSetDevice(dev));
    // the hash_to_G2 -> lines chain is the critical path: its stream gets the highest
    // priority, the key-side and signature-side streams (slack of several ms) the lowest
    int least = 0, greatest = 0;
    HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    // prio_mode (GBLS_PRIO_MODE, experiments): 1 = every stream high, 2 = every stream low
    // a block-import context (klass 1) runs all three streams at the highest priority
    const int pm = klass ? 1 : prio_mode, hi = pm == 2 ? least : greatest,
              lo = pm == 1 ? greatest : least;
    HIPCHK(hipStreamCreateWithPriority(&own, hipStreamNonBlocking, hi));
    HIPCHK(hipStreamCreateWithPriority(&side1, hipStreamNonBlocking, lo));
    HIPCHK(hipStreamCreateWithPriority(&side2, hipStreamNonBlocking, side2_high ? hi : lo));
    HIPCHK(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&ev_side1, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&ev_side2, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&ev_pks, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&ev_in, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&ev_out, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&ev_done, hipEventDisableTiming));
    for (Stage &r : ring) HIPCHK(hipEventCreateWithFlags(&r.ev, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&ev_reg, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&ev_grow, hipEventDisableTiming));
    return true;
  }
  // CU-masked stream triple: mode 1 = main chain on the first `main_cus` CUs, sides on the
  // rest; mode 2 = the same split over interleaved CUs (CU i to the main chain when
  // i % 4 != 3)
  bool init_masked(int mode, int ncu) {
    if (own_m) return true;
    std::vector<uint32_t> mm((ncu + 31) / 32, 0), ms((ncu + 31) / 32, 0);
    for (int i = 0; i < ncu; i++) {
      bool main = mode == 1 ? i < ncu * 3 / 4 : (i % 4) != 3;
      (main ? mm : ms)[i / 32] |= 1u << (i % 32);
    }
    HIPCHK(hipExtStreamCreateWithCUMask(&own_m, (uint32_t)mm.size(), mm.data()));
    HIPCHK(hipExtStreamCreateWithCUMask(&side1_m, (uint32_t)ms.size(), ms.data()));
    HIPCHK(hipExtStreamCreateWithCUMask(&side2_m, (uint32_t)ms.size(), ms.data()));
    return true;
  }
  // streams on every CU except one in `reserve` (CU i with i % reserve == reserve - 1): a normal
  // submission's kernels cannot occupy those, so a block import's waves always find SIMDs there
  bool init_gossip_masked(int reserve, int ncu) {
    if (own_g) return true;
    std::vector<uint32_t> m((ncu + 31) / 32, 0);
    for (int i = 0; i < ncu; i++)
      if (i % reserve != reserve - 1) m[i / 32] |= 1u << (i % 32);
    HIPCHK(hipExtStreamCreateWithCUMask(&own_g, (uint32_t)m.size(), m.data()));
    HIPCHK(hipExtStreamCreateWithCUMask(&side1_g, (uint32_t)m.size(), m.data()));
    HIPCHK(hipExtStreamCreateWithCUMask(&side2_g, (uint32_t)m.size(), m.data()));
    return true;
  }
  // the call's main stream waits (on the GPU) for the previous call on this context;
  // the staging buffer is recycled once the previous call's uploads have landed
  bool begin(hipStream_t st) {
    cur = st;
    active = true;
    stage_at = (stage_at + 1) % kStageRing;  // this call's staging buffer
    Stage &r = ring[stage_at];
    if (r.pending && hipEventQuery(r.ev) == hipSuccess) r.pending = false;  // landed already
    if (r.pending) {  // only when kStageRing calls of this context are still uploading
      if (trace_stalls())
        fprintf(stderr, "gbls: call %llu ctx %p%s waits for staging slot %d\n", call_id, (void *)this,
                fresh ? " (fresh)" : "", stage_at);
      HIPCHK(hipEventSynchronize(r.ev));
      r.pending = false;
    }
    stage_used = 0;
    if (done_pending) HIPCHK(hipStreamWaitEvent(st, ev_done, 0));
    return true;
  }
  // true when the previous call on this context has finished on the GPU
  bool idle_on_gpu() {
    if (!done_pending) return true;
    if (hipEventQuery(ev_done) != hipSuccess) return false;
    done_pending = false;
    return true;
  }
  // host wait for the previous call (before buffers are reallocated)
  bool drain() {
    if (done_pending) {
      HIPCHK(hipEventSynchronize(ev_done));
      done_pending = false;
    }
    return true;
  }
  // every stream other than `own` this context's work may be on (the caller's stream when a call
  // is active; it may be the legacy default stream, nullptr)
  int other_streams(hipStream_t (&ss)[10]) {
    int n = 0;
    if (active && cur != own) ss[n++] = cur;
    for (hipStream_t s : {side1, side2, own_m, side1_m, side2_m, own_g, side1_g, side2_g})
      if (s && !(active && s == cur)) ss[n++] = s;
    return n;
  }
  bool ensure(Buf &b, size_t bytes) {
    if (bytes <= b.cap) return true;
    if (trace_stalls())
      fprintf(stderr, "gbls: call %llu ctx %p%s grows a buffer %zu -> %zu bytes (%s)\n", call_id, (void *)this,
              fresh ? " (fresh)" : "", b.cap, bytes, g_stream_alloc ? "stream-ordered" : "host wait");
    if (g_stream_alloc) return grow_async(b, bytes) || fail(GBLS_ERR_HIP);
    if (!drain()) return false;
    // an in-flight stage of THIS call may still read the old buffer
    if (active) HIPCHK(hipStreamSynchronize(cur));
    return b.ensure(bytes) || fail(GBLS_ERR_HIP);
  }
  // Growth without a host wait: the old buffer is freed on `own` behind the previous call on this
  // context (ev_done) and behind everything this call has enqueued so far on its other streams;
  // the new one is allocated on `own`, and every other stream waits for that before its next
  // work.  (Growth happens on a context's first calls of a size; the cross-stream waits cost
  // overlap only then.)  No stream of its own: HIP maps streams onto a few hardware queues, and
  // every extra stream makes two streams' packets share one more often.
  bool grow_async(Buf &b, size_t bytes) {
    hipStream_t ss[10];
    const int ns = other_streams(ss);
    if (b.p) {
      if (done_pending) HIPCHK(hipStreamWaitEvent(own, ev_done, 0));
      for (int i = 0; i < ns; i++) {  // one event, re-recorded: each wait takes its current record
        HIPCHK(hipEventRecord(ev_grow, ss[i]));
        HIPCHK(hipStreamWaitEvent(own, ev_grow, 0));
      }
      if (b.pooled) {
        HIPCHK(hipFreeAsync(b.p, own));
      } else {  // allocated before stream-ordered allocation was switched on
        HIPCHK(hipStreamSynchronize(own));
        HIPCHK(hipFree(b.p));
      }
      b.p = nullptr;
      b.cap = 0;
    }
    const size_t want = grow_size(bytes);
    HIPCHK(hipMallocAsync(&b.p, want, own));
    b.cap = want;
    b.pooled = true;
    HIPCHK(hipEventRecord(ev_grow, own));
    for (int i = 0; i < ns; i++) HIPCHK(hipStreamWaitEvent(ss[i], ev_grow, 0));
    return true;
  }
  // bump allocation in the pinned staging buffer (per call); regrowing waits for the
  // uploads of this call that still read it
  void *staging(size_t bytes) {
    Stage &r = ring[stage_at];
    size_t need = (bytes + 255) & ~(size_t)255;
    if (stage_used + need > r.cap) {
      if (r.pending) {
        if (trace_stalls())
          fprintf(stderr, "gbls: call %llu ctx %p%s waits for staging slot %d to grow it\n", call_id,
                  (void *)this, fresh ? " (fresh)" : "", stage_at);
        if (hipEventSynchronize(r.ev) != hipSuccess) return nullptr;
        r.pending = false;
      }
      if (need > r.cap) {
        const size_t want = std::max<size_t>(need * 2, 1 << 20);
        // every idle slot of the ring grows with it (up to kStageShared bytes): the next calls'
        // slots are then sized by the first call of a size (a warm-up), not by the first call
        // that reaches them (pinning pages takes milliseconds).  Above that only this call's
        // slot grows, so a one-off huge upload pins one buffer, not the whole ring.  Replaced
        // buffers are retired, not freed (hipHostFree synchronises the device).
        constexpr size_t kStageShared = 64u << 20;
        for (int q = 0; q < kStageRing; q++) {
          Stage &o = ring[q];
          if (o.cap >= want || (q != stage_at && (o.pending || want > kStageShared))) continue;
          if (trace_stalls())
            fprintf(stderr, "gbls: call %llu ctx %p%s grows staging slot %d %zu -> %zu bytes\n", call_id,
                    (void *)this, fresh ? " (fresh)" : "", q, o.cap, want);
          if (o.p) retired_host.push_back(o.p);
          o.p = nullptr;
          o.cap = 0;
          if (hipHostMalloc(&o.p, want, hipHostMallocDefault) != hipSuccess) return nullptr;
          o.cap = want;
        }
      }
      stage_used = 0;
    }
    void *p = static_cast<uint8_t *>(r.p) + stage_used;
    stage_used += need;
    return p;
  }
  bool upload_staged(Buf &dst, const void *host, size_t bytes, hipStream_t st) {
    if (!ensure(dst, bytes + 16)) return false;
    if (!bytes) return true;
    void *s = staging(bytes);
    if (!s) return fail(GBLS_ERR_HIP);
    std::memcpy(s, host, bytes);
    HIPCHK(hipMemcpyAsync(dst.p, s, bytes, hipMemcpyHostToDevice, st));
    HIPCHK(hipEventRecord(ring[stage_at].ev, st));
    ring[stage_at].pending = true;
    return true;
  }
};

// k_ml_group launches of more than this many waves per SIMD pick G to fill whole rounds
constexpr uint32_t kMlRounds = 2;

struct Device {
  int hipdev = -1;
  uint32_t nsimd = 1024;  // 4 SIMDs per CU
  int ncu = 256;
  sched::CtxPool<Ctx> pool;  // per-class capped context pool (gbls_sched.h)
  // validator registry (replica), guarded by Engine::reg_mu.  Every write (growth, zeroing,
  // decompression, replica copies) is stream-ordered on reg_st; reg_ev follows the last one and
  // every registry reader's stream waits on it (GPU-side) before its gather.  A grown table's
  // old buffer is freed on retire_st behind its readers (Ctx::ev_reg), never by a host wait.
  Buf reg;
  bool reg_pooled = false;  // reg.p from hipMallocAsync (freed by hipFreeAsync)
  // old tables when stream-ordered allocation is missing: each freed (hipFree) by a later growth
  // once its event, recorded on retire_st behind the table's readers, has completed
  struct Kept {
    void *p;
    hipEvent_t ev;
  };
  std::vector<Kept> reg_kept;
  hipStream_t reg_st = nullptr, retire_st = nullptr;
  hipEvent_t reg_ev = nullptr, reg_tmp = nullptr;
  bool reg_ev_set = false;
};

struct Engine {
  std::mutex mu;
  std::atomic<bool> ready{false};
  std::vector<std::unique_ptr<Device>> devs;
  std::atomic<uint32_t> rr{0};
  std::shared_mutex reg_mu;
  size_t reg_n = 0;
  std::atomic<bool> coalesce{true};
  std::atomic<bool> per_check{false};  // GBLS_INIT_PER_CHECK: no grouped single checks
  size_t msm_min = kMsmMinPerSeg;  // segments at least this large use the bucket MSM
  size_t line_budget = kLineBudget; // line-coefficient buffer bound per submission (bytes)
  uint32_t ml_g = 0;                // forced k_ml_group group size (0: chosen per launch)
  uint32_t ml_rounds = kMlRounds;   // k_ml_group waves per SIMD for large launches
  bool side2_high = false;          // signature-side stream (MSM) at the main stream's priority
  int prio_mode = 0;                // 0: main high, sides low; 1: all high; 2: all low
  int cu_split = 0;                 // latency-regime submissions on CU-masked streams (0: off)
  uint32_t cu_split_max = 1024;     // ... up to this many sets
  int leaders = 2;                  // coalescer leaders per device
  size_t merge_target = 768;        // a new gossip leader's collection target (gbls_sched.h)
  int merge_window_us = 300;        // ... and its longest wait
  // Block import under load (f3): while a GBLS_CALL_BLOCK call is in progress, normal-class
  // submissions run on streams masked off one CU in block_reserve (0: off), so the block's
  // waves never wait for SIMDs held by gossip kernels launched meanwhile.
  int block_reserve = 0;
  // ... and normal requests do not start new submissions meanwhile (up to 4 ms, gbls_sched.h
  // Config::hold): the block shares the GPU only with the submissions already running
  bool block_hold = true;
  bool ml_pcn = true;         // the Miller kernel reads normalized points by column (GBLS_ML_PCN)
  uint32_t g2sum_ch = WGR;    // sets per level-1 chunk of the signature sum (GBLS_G2SUM_CH)
  bool lines_s_main = false;  // experiments: the MSM pairs' lines on the main stream after the join,
  bool lines_s_lane = false;  // ... in the one-lane form
  std::atomic<int> block_active{0};
} g;

// RAII lease of a context of one device (sched::CtxPool::acquire: the idle context last
// used on the caller's stream, else one idle on the GPU, else a new one up to the class cap,
// else the least recently used idle one of the class, else wait).
class Lease {
 public:
  Lease(Device &d, bool affine, hipStream_t stream, int cls = 0) : d_(d) {
    c_ = d.pool.acquire(affine, stream, cls, &fresh_);
    c_->call_id = g_lease_calls.fetch_add(1);
    c_->fresh = fresh_ || !c_->used;  // created now, or created by gbls_init and never used
    if (fresh_ && trace_stalls())
      fprintf(stderr, "gbls: call %llu creates ctx %p (class %d, %zu contexts)\n", c_->call_id, (void *)c_,
              c_->cls, d.pool.size());
    ok_ = fresh_ ? c_->init(d.hipdev, g.side2_high, g.prio_mode, c_->cls)
                 : (hipSetDevice(d.hipdev) == hipSuccess || fail(GBLS_ERR_HIP));
  }
  explicit Lease(Device &d, int cls = 0) : Lease(d, false, nullptr, cls) {}
  ~Lease() {
    if (c_->active) {
      if (hipEventRecord(c_->ev_done, c_->cur) == hipSuccess) c_->done_pending = true;
      c_->last_stream = c_->cur;
      c_->used = true;
      c_->active = false;
      c_->cur = nullptr;
    }
    d_.pool.release(c_);
  }
  bool ok() const { return ok_; }
  Ctx &operator*() { return *c_; }
  Ctx *operator->() { return c_; }

 private:
  Device &d_;
  Ctx *c_ = nullptr;
  bool fresh_ = false, ok_ = false;
};

bool registry_streams(Device &d);

bool engine_init(uint32_t device_mask, uint32_t flags) {
  std::lock_guard<std::mutex> lk(g.mu);
  // policy flags are sticky: a gbls_init that names one turns it on, also on an engine that is
  // already open, and no later gbls_init turns it off (a library's lazy gbls_init(mask, 0) must
  // not undo an operator's or a spec-test harness's choice); gbls_set_policy sets them outright
  if (flags & GBLS_INIT_NO_COALESCE) g.coalesce.store(false);
  if (flags & GBLS_INIT_PER_CHECK) g.per_check.store(true);
  if (g.ready.load()) return true;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(GBLS_ERR_NO_DEVICE);
  std::vector<int> ids;
  if (device_mask) {
    for (int d = 0; d < 32 && d < ndev; d++)
      if ((device_mask >> d) & 1) ids.push_back(d);
  } else {
    int cur = 0;
    (void)hipGetDevice(&cur);
    ids.push_back(cur);
  }
  if (ids.empty()) return fail(GBLS_ERR_NO_DEVICE);
  // tuning knobs: only for tests and sweeps that ask for them (GBLS_INIT_TUNING); a node
  // embedding the library runs the measured defaults whatever its environment holds
  if (flags & GBLS_INIT_TUNING) {
    if (const char *e = std::getenv("GBLS_MSM_MIN")) g.msm_min = std::strtoull(e, nullptr, 10);
    if (const char *e = std::getenv("GBLS_LINE_BUDGET_MB"))
      g.line_budget = (size_t)std::strtoull(e, nullptr, 10) << 20;
    if (const char *e = std::getenv("GBLS_ML_G")) g.ml_g = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char *e = std::getenv("GBLS_ML_ROUNDS"))
      g.ml_rounds = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char *e = std::getenv("GBLS_SIDE2_HIGH")) g.side2_high = std::atoi(e) != 0;
    if (const char *e = std::getenv("GBLS_PRIO_MODE")) g.prio_mode = std::atoi(e);
    if (const char *e = std::getenv("GBLS_G2SUM_CH")) g.g2sum_ch = std::max(16u, (uint32_t)std::strtoul(e, nullptr, 10));
    if (const char *e = std::getenv("GBLS_ROW_CLEAR_MAX"))
      g_row_clear_max = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char *e = std::getenv("GBLS_CU_SPLIT")) g.cu_split = std::atoi(e);
    if (const char *e = std::getenv("GBLS_MSM_K")) g_msm_k = std::max(1u, (uint32_t)std::strtoul(e, nullptr, 10));
    if (const char *e = std::getenv("GBLS_MSM_R28")) g_msm_r28 = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char *e = std::getenv("GBLS_ML_XCD")) g_ml_xcd = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char *e = std::getenv("GBLS_LANE_R28")) g_lane_r28 = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char *e = std::getenv("GBLS_CLEAR_STAGED")) g_clear_staged = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char *e = std::getenv("GBLS_MAP_ROWS_MAX")) g_map_rows_max = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char *e = std::getenv("GBLS_LANE_MIN")) g_lane_min = std::max(1u, (uint32_t)std::strtoul(e, nullptr, 10));
    if (const char *e = std::getenv("GBLS_CU_SPLIT_MAX"))
      g.cu_split_max = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char *e = std::getenv("GBLS_LEADERS")) g.leaders = std::max(1, std::atoi(e));
    if (const char *e = std::getenv("GBLS_MERGE_TARGET")) g.merge_target = std::strtoull(e, nullptr, 10);
    if (const char *e = std::getenv("GBLS_MERGE_WINDOW_US")) g.merge_window_us = std::atoi(e);
    if (const char *e = std::getenv("GBLS_BLOCK_RESERVE")) g.block_reserve = std::atoi(e);
    if (const char *e = std::getenv("GBLS_BLOCK_HOLD")) g.block_hold = std::atoi(e) != 0;
    if (const char *e = std::getenv("GBLS_ML_R28")) g_ml_r28 = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char *e = std::getenv("GBLS_ML_DMA")) g_ml_dma = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char *e = std::getenv("GBLS_ML_PREFETCH")) g_ml_prefetch = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char *e = std::getenv("GBLS_ML_KARA")) g_ml_kara = (uint32_t)std::strtoul(e, nullptr, 10);
    if (const char *e = std::getenv("GBLS_LINES_S_MAIN")) g.lines_s_main = std::atoi(e) != 0;
    if (const char *e = std::getenv("GBLS_ML_PCN")) g.ml_pcn = std::atoi(e) != 0;
    if (const char *e = std::getenv("GBLS_LINES_S_LANE")) g.lines_s_lane = std::atoi(e) != 0;
  }
  int replicas = (int)(flags & 0xffu);
  if (replicas < 1) replicas = 1;
  bool stream_alloc = true;
  for (int id : ids) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, id) != hipSuccess) return fail(GBLS_ERR_NO_DEVICE);
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return fail(GBLS_ERR_NO_DEVICE);
    // stream-ordered allocation for the workspaces (Ctx::grow_async): the default pool keeps
    // freed memory (no release at synchronisation points), never makes one stream's allocation
    // wait for another stream's pending free (contexts stay independent), and is readable by
    // the other engine devices (partials and registry slices cross devices by peer copies)
    int pools = 0;
    hipMemPool_t pool = nullptr;
    if (hipDeviceGetAttribute(&pools, hipDeviceAttributeMemoryPoolsSupported, id) != hipSuccess || !pools ||
        hipDeviceGetDefaultMemPool(&pool, id) != hipSuccess) {
      stream_alloc = false;
    } else {
      uint64_t keep = UINT64_MAX;
      int no = 0;
      (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
      (void)hipMemPoolSetAttribute(pool, hipMemPoolReuseAllowInternalDependencies, &no);
      for (int peer : ids) {
        if (peer == id) continue;
        hipMemAccessDesc acc{};
        acc.location.type = hipMemLocationTypeDevice;
        acc.location.id = peer;
        acc.flags = hipMemAccessFlagsProtReadWrite;
        (void)hipMemPoolSetAccess(pool, &acc, 1);
      }
    }
    for (int r = 0; r < replicas; r++) {
      g.devs.emplace_back(new Device());
      g.devs.back()->hipdev = id;
      g.devs.back()->nsimd = 4u * (uint32_t)prop.multiProcessorCount;
      g.devs.back()->ncu = prop.multiProcessorCount;
    }
  }
  (void)hipGetLastError();
  g_stream_alloc = stream_alloc && !(flags & GBLS_INIT_TUNING && std::getenv("GBLS_SYNC_ALLOC"));
  // contexts created up front (streams and events; workspaces grow on first use): the first
  // concurrent callers, e.g. two submissions in flight, lease instead of creating
  int prewarm[2] = {kPrewarmCtx[0], kPrewarmCtx[1]};
  if (flags & GBLS_INIT_TUNING)
    if (const char *e = std::getenv("GBLS_PREWARM")) {  // "normal[,block]"
      prewarm[0] = prewarm[1] = std::atoi(e);
      if (const char *c = std::strchr(e, ',')) prewarm[1] = std::atoi(c + 1);
    }
  // experiments (tuning only): GBLS_PREWARM_BLOCK_FIRST=1 creates the block-class contexts
  // first; GBLS_DUMMY_STREAMS=n,prio creates n idle streams of priority prio (0 high, 1 low,
  // 2 default) after the contexts (HIP maps streams onto hardware queues per priority)
  const bool block_first = (flags & GBLS_INIT_TUNING) && std::getenv("GBLS_PREWARM_BLOCK_FIRST");
  for (auto &dp : g.devs) {
    Device &d = *dp;
    for (int k = 0; k < prewarm[0] + prewarm[1]; k++) {
      const int cls = block_first ? (k < prewarm[1] ? 1 : 0) : (k < prewarm[0] ? 0 : 1);
      if (!d.pool.prewarm(cls, [&](Ctx &c) { return c.init(d.hipdev, g.side2_high, g.prio_mode, cls); }))
        return fail(GBLS_ERR_HIP);
    }
    // the registry's streams at start as well (one high-priority stream for its updates, one for
    // retiring old tables), not at the first gbls_registry_set; the update stream is touched
    // here so that it holds its hardware queue from the start (HIP binds a stream's queue at
    // its first use), which is the queue set measured best above
    const bool reg_at_init = !((flags & GBLS_INIT_TUNING) && std::getenv("GBLS_REG_AT_INIT") &&
                               std::atoi(std::getenv("GBLS_REG_AT_INIT")) == 0);
    if (reg_at_init && (!registry_streams(d) || hipStreamQuery(d.reg_st) != hipSuccess))
      return fail(GBLS_ERR_HIP);
    if (const char *e = (flags & GBLS_INIT_TUNING) ? std::getenv("GBLS_DUMMY_STREAMS") : nullptr) {
      int least = 0, greatest = 0;
      (void)hipSetDevice(d.hipdev);
      (void)hipDeviceGetStreamPriorityRange(&least, &greatest);
      const char *c = std::strchr(e, ',');
      const int pr = c ? std::atoi(c + 1) : 0;
      for (int k = std::atoi(e); k > 0; k--) {
        hipStream_t s = nullptr;
        if (pr == 2)
          (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
        else
          (void)hipStreamCreateWithPriority(&s, hipStreamNonBlocking, pr == 0 ? greatest : least);
        if (s) (void)hipStreamQuery(s);
      }
    }
  }
  // direct xGMI peer access between the engine's devices (partials gathered device-to-device,
  // registry replicas); without it hipMemcpyPeerAsync still works, staged by the runtime
  for (int a : ids)
    for (int b : ids) {
      int can = 0;
      if (a != b && hipDeviceCanAccessPeer(&can, a, b) == hipSuccess && can && hipSetDevice(a) == hipSuccess)
        (void)hipDeviceEnablePeerAccess(b, 0);  // "already enabled" is fine
    }
  (void)hipGetLastError();
  g.ready.store(true);
  return true;
}

bool ensure_ready() { return g.ready.load() || engine_init(0, 0); }

// the engine device(s) of the calling thread's current HIP device (device-pointer calls)
Device *current_device() {
  int id = 0;
  if (hipGetDevice(&id) != hipSuccess) return nullptr;
  std::vector<Device *> cand;
  for (auto &d : g.devs)
    if (d->hipdev == id) cand.push_back(d.get());
  if (cand.empty()) return nullptr;
  return cand[g.rr.fetch_add(1) % cand.size()];
}
Device &pick_device() { return *g.devs[g.rr.fetch_add(1) % g.devs.size()]; }

bool valid_offsets(const uint32_t *off, size_t nseg, size_t n) {
  if (!off || off[0] != 0 || off[nseg] != n) return false;
  for (size_t s = 0; s < nseg; s++)
    if (off[s + 1] < off[s]) return false;
  return true;
}

// ----- where a batch's public keys come from (device pointers inside the pipeline, host
// pointers in a coalescer request)
using PkSource = sched::KeySource<g1a>;

// A kernel reading the registry on stream st: first wait (on the GPU) for the registry's
// pending writes, afterwards mark the read so that a growth retires the old table behind it.
// Both under the shared registry lock.
bool registry_read_begin(Ctx &c, Device &d, hipStream_t st) {
  (void)c;
  if (d.reg_ev_set) HIPCHK(hipStreamWaitEvent(st, d.reg_ev, 0));
  return true;
}
bool registry_read_end(Ctx &c, hipStream_t st) {
  HIPCHK(hipEventRecord(c.ev_reg, st));
  c.reg_read = true;
  return true;
}

// Resolve a DEVICE key source into per-set affine keys on stream st; *pre = per-set
// status (nonzero = reject: empty aggregate, index out of range) or nullptr.  The caller
// holds the registry lock (shared) while it enqueues.
bool resolve_pks(Ctx &c, Device &d, const PkSource &src, size_t n, hipStream_t st,
                 const g1a **pks, const int32_t **pre) {
  *pre = nullptr;
  if ((src.pts && !src.off) || n == 0) {
    *pks = src.pts;
    return true;
  }
  if (!src.pts && !src.idx) return fail(GBLS_ERR_ARG);
  if (!c.ensure(c.pks, n * sizeof(g1a)) || !c.ensure(c.pre, n * sizeof(int32_t))) return false;
  StageTimer t(S_PK_GATHER, st);
  const g1a *reg = d.reg.as<g1a>();
  if (src.idx && !registry_read_begin(c, d, st)) return false;
  if (src.pts)
    launch_g1_aggregate_seg(st, src.pts, src.off, (uint32_t)n, c.pks.as<g1a>(),
                            c.pre.as<int32_t>());
  else if (src.off)
    launch_g1_aggregate_idx(st, reg, (uint32_t)g.reg_n, src.idx, src.off, (uint32_t)n,
                            c.pks.as<g1a>(), c.pre.as<int32_t>());
  else
    launch_g1_gather_idx(st, reg, (uint32_t)g.reg_n, src.idx, (uint32_t)n, c.pks.as<g1a>(),
                         c.pre.as<int32_t>());
  if (src.idx && !registry_read_end(c, st)) return false;
  *pks = c.pks.as<g1a>();
  *pre = c.pre.as<int32_t>();
  return true;
}

// the reduction levels and the Horner step after k_ml_group (products in c.V0)
// submissions up to this many sets split their Horner chains (latency regime: blocks, gossip
// merges, single C2 batches, a C4 epoch); larger ones (many batches) keep one chain
constexpr size_t kSplitHornerMaxSets = 8192;

void ml_tail(Ctx &c, hipStream_t st, const MlTables &mt, const uint32_t *T, uint32_t nms,
             fp12 *partials, bool split) {
  fp12 *cur = c.V0.as<fp12>(), *other = c.V1.as<fp12>();
  {
    StageTimer t(S_ML_REDUCE, st);
    for (const MlTables::Level &L : mt.levels) {
      launch_ml_reduce(st, cur, (uint32_t)L.nin, T + L.tab_off, (uint32_t)L.nout, other);
      std::swap(cur, other);
    }
  }
  StageTimer t(S_ML_HORNER, st);
  // latency regime: the Horner chain split in 4 parts (their values in a buffer of their own,
  // ensured with the workspaces); throughput regime: one chain (the parts' extra squarings
  // only cost there, where another submission fills the chip during the tail)
  fp12 *tmp = split && nms <= 64 ? c.hparts.as<fp12>() : nullptr;
  launch_ml_horner(st, cur, nms, partials, nullptr, 0, tmp);
}

// ----- the verification pipeline on device pointers.
// Sets [0, n) grouped in segments by seg_off (HOST array, nseg + 1 entries); per segment
// a Miller partial (no final exponentiation) and an error flag.  rands == nullptr
// means r_i = 1 (single checks); sig_groupcheck adds the G2 subgroup check of every
// signature (verify / fast_aggregate_verify, signature.rs:51,86).  Streams:
//   side 1: key resolution (gather / aggregation) -> r_i pk_i
//   side 2: signature group check, then S = sum r_i sig_i (waits for the keys' flags),
//           then the lines of the (-g1, S) pairs (or of the MSM's weighted bucket sums)
//   main:   hash_to_G2 -> the sets' lines;  join -> Miller product tree -> partials
bool pipeline_partials(Ctx &c, Device &d, const uint8_t *msgs, const uint32_t *msg_off,
                       const g2a *sigs, const PkSource &src, const uint64_t *rands,
                       bool sig_groupcheck, size_t n, const uint32_t *seg_off, size_t nseg,
                       int empty_is_error, fp12 *partials, int32_t *seg_err,
                       hipStream_t caller, uint32_t grp = 0, const uint64_t *grp_r = nullptr,
                       size_t *nms_out = nullptr) {
  // The main chain runs on the context's high-priority stream; a caller stream (device
  // entry points) hands over to it and waits for it at the end.  Small submissions may run
  // on CU-masked streams (g.cu_split), the main chain apart from the side streams.
  hipStream_t own = c.own, side1 = c.side1, side2 = c.side2;
  if (g.cu_split && n <= g.cu_split_max) {
    if (!c.init_masked(g.cu_split, d.ncu)) return false;
    own = c.own_m;
    side1 = c.side1_m;
    side2 = c.side2_m;
  } else if (c.cls == 0 && g.block_reserve > 1 && g.block_active.load(std::memory_order_relaxed) > 0) {
    if (!c.init_gossip_masked(g.block_reserve, d.ncu)) return false;
    own = c.own_g;
    side1 = c.side1_g;
    side2 = c.side2_g;
  }
  hipStream_t st = caller;
  if (caller != own) {
    HIPCHK(hipEventRecord(c.ev_in, caller));
    HIPCHK(hipStreamWaitEvent(own, c.ev_in, 0));
    st = own;
  }
  bool single = !rands && n == nseg;  // one set per segment, r = 1
  for (size_t s = 0; single && s <= nseg; s++) single = seg_off[s] == s;
  // bucket MSM for S when every segment is large (segment sizes >= msm_min)
  bool msm = rands && n > 0;
  for (size_t s = 0; msm && s < nseg; s++) msm = seg_off[s + 1] - seg_off[s] >= g.msm_min;
  MsmPlan mp{};
  if (msm) {
    mp = msm_plan((uint32_t)n, (uint32_t)nseg);
    if (!c.ensure(c.msm, mp.bytes)) return false;
  }
  // extra Miller pairs per segment after the n sets: (-g1, S), or the MSM's weighted
  // bucket / window sums
  const size_t X = msm ? mp.extra : 1;
  const size_t np = n + nseg * X;
  // ---- host tables, one staged upload:
  //   [pair list][groups][g2 chunks][seg_chunk][reduction levels][seg_off]
  // Level 0 of the Miller product: per segment, its pairs (sets, then the extra pairs)
  // in groups of <= G, strided so that a wave's lanes read adjacent pairs (k_ml_group).
  // Line buffer: all 68 events of every pair when that fits kLineBudget, else event
  // slices of EC events (the running points T in HBM between slices), so that memory stays
  // bounded at C5 scale.  The first slice is generated before the join like the unsliced
  // lines (sets on the main stream, extra pairs on side 2), later ones after it.
  const size_t event_bytes = (size_t)np * 72 * 4;
  int EC = ML_EVENTS;
  if (event_bytes * ML_EVENTS > g.line_budget)
    EC = (int)std::max<size_t>(1, g.line_budget / event_bytes);
  const bool sliced = EC < ML_EVENTS;
  // Miller segments: the verification segments, or (grouped single checks, grp > 1) runs of
  // grp checks whose pairs (i, n + i) share one Miller product and one final exponentiation
  const bool grouped = grp > 1 && single && !sliced && grp_r;
  const size_t nms = grouped ? (n + grp - 1) / grp : nseg;
  if (nms_out) *nms_out = nms;
  std::vector<uint32_t> &tab = c.host_tab;
  tab.clear();
  MlTables mt;
  if (grouped)
    mt = ml_tables(
        tab, nms, np, EC, d.nsimd, g.ml_rounds, g.ml_g,
        [&](size_t s) { return 2 * (uint32_t)(std::min(n, (s + 1) * grp) - s * grp); },
        [&](size_t s, std::vector<uint32_t> &t) {
          const uint32_t b = (uint32_t)(s * grp), e = (uint32_t)std::min(n, (s + 1) * grp);
          for (uint32_t i = b; i < e; i++) t.push_back(i);
          for (uint32_t i = b; i < e; i++) t.push_back((uint32_t)n + i);
        });
  else
    mt = ml_tables(
        tab, nseg, np, EC, d.nsimd, g.ml_rounds, g.ml_g,
        [&](size_t s) { return seg_off[s + 1] - seg_off[s] + (uint32_t)X; },
        [&](size_t s, std::vector<uint32_t> &t) {
          for (uint32_t i = seg_off[s]; i < seg_off[s + 1]; i++) t.push_back(i);
          for (size_t k = 0; k < X; k++) t.push_back((uint32_t)(n + s * X + k));
        });
  const size_t line_words = (size_t)mt.ncol * EC * 72;
  const size_t chunk_off = tab.size();
  const uint32_t CH = g.g2sum_ch;  // sets per level-1 G2-sum workgroup (WGR unless GBLS_G2SUM_CH)
  std::vector<uint32_t> seg_chunk(nseg + 1, 0);
  for (size_t s = 0; s < nseg; s++) {
    seg_chunk[s] = (uint32_t)((tab.size() - chunk_off) / 4);
    for (uint32_t h = 0; h < 2; h++) {
      uint32_t b = seg_off[s], e = seg_off[s + 1];
      do {
        uint32_t ce = std::min<uint32_t>(e, b + CH);
        tab.push_back((uint32_t)s);
        tab.push_back(h);
        tab.push_back(b);
        tab.push_back(ce);
        b = ce;
      } while (b < e);
    }
  }
  const size_t nchunks = (tab.size() - chunk_off) / 4;
  seg_chunk[nseg] = (uint32_t)nchunks;
  const size_t segchunk_off = tab.size();
  tab.insert(tab.end(), seg_chunk.begin(), seg_chunk.end());
  const size_t segoff_at = tab.size();
  tab.insert(tab.end(), seg_off, seg_off + nseg + 1);
  // ---- workspaces
  if (sliced && !c.ensure(c.Ts, np * sizeof(g2h))) return false;
  if (sig_groupcheck && !c.ensure(c.pre2, n * sizeof(int32_t) + 16)) return false;
  if (grouped && !c.ensure(c.ng1, n * sizeof(g1a) + 16)) return false;
  if (!c.ensure(c.U, 2 * n * sizeof(fp2) + 16) || !c.ensure(c.Q, 2 * n * sizeof(g2j) + 16) ||
      !c.ensure(c.H, np * sizeof(g2a)) || !c.ensure(c.P, np * sizeof(g1s)) ||
      !c.ensure(c.R, 2 * n * sizeof(g2j) + 16) ||
      !c.ensure(c.gpart, nchunks * (sizeof(g2j) + 4)) || !c.ensure(c.lines, line_words * 4) ||
      !c.ensure(c.V0, ML_EVENTS * mt.v0_n * sizeof(fp12)) ||
      !c.ensure(c.V1, ML_EVENTS * mt.v1_n * sizeof(fp12)) ||
      (g_ml_r28 && !c.ensure(c.V28, (size_t)ML_EVENTS * 168 * 4 * mt.ngroup)) ||
      (g_ml_r28 && mt.ngp && !c.ensure(c.Pc, (size_t)36 * 4 * mt.ncol)) ||
      !c.ensure(c.hparts, 4 * 64 * sizeof(fp12)))  // the split Horner's parts (<= 64 segments)
    return false;
  if (!c.upload_staged(c.tab, tab.data(), tab.size() * 4, st)) return false;
  const uint32_t N = (uint32_t)n, NP = (uint32_t)np, NS = (uint32_t)nseg;
  // latency regime: each segment's S = sum r_i sig_i stays Jacobian (no inversion), its lines
  // taken projectively (k_lines_w4j)
  g2j *sj = nullptr;
  if (!msm && !single && !sliced && X == 1 && nseg <= kW4Max) {
    if (!c.ensure(c.Sj, nseg * sizeof(g2j) + 16)) return false;
    sj = c.Sj.as<g2j>();
  }
  const uint32_t *T = c.tab.as<uint32_t>();
  const LineCols lc{mt.ngp ? T + mt.col_off : nullptr, mt.ncol};
  c.line_col = lc.col;  // for a grouped re-check of the same lines (grouped_verdicts)
  c.line_ncol = lc.ncol;
  g2j *gpart = c.gpart.as<g2j>();
  int32_t *gpart_err = reinterpret_cast<int32_t *>(gpart + nchunks);
  // ---- fork
  HIPCHK(hipEventRecord(c.ev_fork, st));
  HIPCHK(hipStreamWaitEvent(side1, c.ev_fork, 0));
  HIPCHK(hipStreamWaitEvent(side2, c.ev_fork, 0));
  // main stream first: its first kernels reach the GPU before the side streams' floods
  {
    StageTimer t(S_H2C_FIELD, st);
    launch_h2c_field(st, msgs, msg_off, N, nullptr, 0, c.U.as<fp2>());
  }
  {
    StageTimer t(S_H2C_MAP, st);
    launch_h2c_map(st, c.U.as<fp2>(), 2 * N, c.Q.as<g2j>());
  }
  const g1a *pks = nullptr;
  const int32_t *pre = nullptr;
  if (!resolve_pks(c, d, src, n, side1, &pks, &pre)) return false;
  HIPCHK(hipEventRecord(c.ev_pks, side1));
  {
    StageTimer t(S_G1MUL, side1);
    launch_mv_g1mul(side1, pks, grouped ? grp_r : rands, N, c.P.as<g1s>());
  }
  const int32_t *pre2 = nullptr;
  if (c.sig_c) {  // MultiVerifier::finish's decompression, inside this submission
    // sigs is then the lease's own output buffer (c.sigd, enqueue_host_batch)
    launch_g2_decompress(side2, c.sig_c, N, const_cast<g2a *>(sigs), c.sig_st);
    pre2 = c.sig_st;
    if (sig_groupcheck) {  // single checks (SingleVerifier::extend): decoding AND subgroup
      HIPCHK(hipMemcpyAsync(c.pre2.p, c.sig_st, (size_t)N * 4, hipMemcpyDeviceToDevice, side2));
      launch_g2_check(side2, sigs, N, c.pre2.as<int32_t>(), 1);
      pre2 = c.pre2.as<int32_t>();
    }
    c.sig_c = nullptr;
    c.sig_st = nullptr;
  } else if (sig_groupcheck) {
    launch_g2_check(side2, sigs, N, c.pre2.as<int32_t>(), 0);
    pre2 = c.pre2.as<int32_t>();
  }
  if (msm) {  // the keys' flags are read by the first MSM kernel
    HIPCHK(hipStreamWaitEvent(side2, c.ev_pks, 0));
    StageTimer t(S_MSM, side2);
    launch_msm(side2, mp, c.msm.as<uint8_t>(), sigs, rands, pks, pre, pre2, N, T + segoff_at,
               empty_is_error, c.H.as<g2a>(), c.P.as<g1s>(), seg_err);
  } else if (!single) {
    StageTimer t(S_G2MUL, side2);
    launch_mv_g2mul(side2, sigs, rands, N, c.R.as<g2j>());
  }
  if (!msm) {
    StageTimer t(S_G2SUM, side2);
    if (single) {
      HIPCHK(hipStreamWaitEvent(side2, c.ev_pks, 0));
      launch_single_S(side2, sigs, pks, pre, pre2, N, c.P.as<g1s>(), c.H.as<g2a>(), seg_err,
                      grouped ? c.ng1.as<g1a>() : nullptr);
      if (grouped)  // the (-g1, sig_i) pairs weighted by the same r_i: (-r_i g1, sig_i)
        launch_mv_g1mul(side2, c.ng1.as<g1a>(), grp_r, N, c.P.as<g1s>() + N);
    } else {  // the signature sums start at once; only their key flags wait for side 1
      launch_g2sum(side2, c.R.as<g2j>(), T + chunk_off, (uint32_t)nchunks, T + segchunk_off,
                   T + segoff_at, NS, N, pks, rands, pre, pre2, empty_is_error, gpart, gpart_err,
                   c.P.as<g1s>(), c.H.as<g2a>(), seg_err, sj, c.ev_pks);
    }
  }
  // experiment (GBLS_LINES_S_MAIN): the MSM's extra pairs' lines on the main stream after the
  // join (high priority) instead of on the signature-side stream
  const bool lines_s_main = msm && !sliced && g.lines_s_main;
  if (!lines_s_main) {  // the extra pairs' lines of the first event slice (all events when not sliced)
    StageTimer t(S_LINES_S, side2);
    if (!sj || !launch_lines_jac(side2, sj, 1, N, NS, lc, c.lines.as<uint32_t>()))
      launch_lines(side2, c.H.as<g2a>(), N, (uint32_t)(nseg * X), lc, 0, EC, c.Ts.as<g2h>(),
                   c.lines.as<uint32_t>(), g.lines_s_lane);
  }
  // latency regime: H(m) stays Jacobian (over Q[2 i]) and its lines take it projectively,
  // no inversion on the main chain
  const bool jac_h = !sliced && N <= kW4Max;
  {
    StageTimer t(S_H2C_CLEAR, st);
    if (!jac_h || !launch_h2c_clear_jac(st, c.Q.as<g2j>(), N))
      launch_h2c_clear(st, c.Q.as<g2j>(), N, c.H.as<g2a>());
  }
  {  // the sets' lines of the first event slice, before the join
    StageTimer t(S_LINES, st);
    if (!jac_h || !launch_lines_jac(st, c.Q.as<g2j>(), 2, 0, N, lc, c.lines.as<uint32_t>()))
      launch_lines(st, c.H.as<g2a>(), 0, N, lc, 0, EC, c.Ts.as<g2h>(), c.lines.as<uint32_t>());
  }
  HIPCHK(hipEventRecord(c.ev_side1, side1));
  HIPCHK(hipEventRecord(c.ev_side2, side2));
  HIPCHK(hipStreamWaitEvent(st, c.ev_side1, 0));
  HIPCHK(hipStreamWaitEvent(st, c.ev_side2, 0));
  if (lines_s_main) {
    StageTimer t(S_LINES_S, st);
    launch_lines(st, c.H.as<g2a>(), N, (uint32_t)(nseg * X), lc, 0, EC, c.Ts.as<g2h>(), c.lines.as<uint32_t>(),
                 g.lines_s_lane);
  }
  const uint32_t *Pc = nullptr;  // the points by line column (radix-2^28 Miller kernel)
  bool pcn = false;              // ... normalized
  // Points by line column for the radix-2^28 Miller kernel: normalized (x 2^8 / c, y 2^8 / c, one
  // inversion per pair, 4-product line evaluations) in the throughput regime; below it (blocks,
  // gossip, single batches, C3's grouped checks) the inversion's latency sits on the critical
  // path between the join and the Miller product, so the points keep their (x, y, c) form there
  if (g_ml_r28 && mt.ngp) {
    const bool normalize = g.ml_pcn && NP >= kPcnMinPairs;
    launch_ml_pcols(st, c.P.as<g1s>(), lc.col, NP, lc.ncol, c.Pc.as<uint32_t>(), normalize);
    Pc = c.Pc.as<uint32_t>();
    pcn = normalize;
  }
  for (int e0 = 0; e0 < ML_EVENTS; e0 += EC) {
    const int e1 = std::min(ML_EVENTS, e0 + EC);
    if (e0 > 0) {  // later slices: every pair, after the join
      StageTimer t(S_LINES, st);
      launch_lines(st, c.H.as<g2a>(), 0, NP, lc, e0, e1, c.Ts.as<g2h>(), c.lines.as<uint32_t>());
    }
    StageTimer t(S_ML_LEAF, st);
    launch_ml_group(st, c.lines.as<uint32_t>(), lc, mt.ngp, c.P.as<g1s>(), Pc, T + mt.plist_off,
                    T + mt.grp_off, (uint32_t)mt.ngroup, e0, e1, c.V0.as<fp12>(), c.V28.as<uint32_t>(), pcn);
  }
  ml_tail(c, st, mt, T, (uint32_t)nms, partials, n <= kSplitHornerMaxSets);
  if (st != caller) {
    HIPCHK(hipEventRecord(c.ev_out, st));
    HIPCHK(hipStreamWaitEvent(caller, c.ev_out, 0));
  }
  HIPCHK(hipGetLastError());
  return true;
}

// product of nparts partials per segment, final exponentiation, verdict per segment
bool pipeline_final(const fp12 *partials, const int32_t *err, size_t nparts, size_t nseg,
                    int32_t *verdicts, hipStream_t st) {
  StageTimer t(S_FINAL, st);
  launch_final_verdict(st, partials, err, (uint32_t)nparts, (uint32_t)nseg, verdicts);
  HIPCHK(hipGetLastError());
  return true;
}

// Grouped single checks (large batches of independent checks, the C3 shape): round 1 weights
// check i's two pairs by a secret random r_i on the G1 side, (r_i pk_i, H_i) and
// (-r_i g1, sig_i), and multiplies the pairs of kGroupChecks consecutive checks into one
// Miller product with one final exponentiation: prod_i (e(pk_i, H_i) e(-g1, sig_i))^r_i == 1.
// A group passes only if every member's check holds, except with probability ~2^-64 over
// r (the random-linear-combination soundness of Signature::multi_verify,
// bls/src/signature.rs:95-129).  Round 2 re-checks every member of a failed (or flagged) group on
// its own: its own Miller product of the SAME pairs, whose r_i-th power is 1 iff
// e(pk_i, H_i) == e(g1, sig_i) (r_i != 0 < q) -- the verdict of the reference's single check
// (SingleVerifier::verify_aggregate, helper_functions/src/verifier.rs).  The lines of round 1
// stay in HBM for round 2; only the Miller products, Horner steps and final exponentiations
// are redone, for ~8 % of the checks at 1 % invalid.
constexpr size_t kGroupChecks = 8;
constexpr size_t kGroupMinChecks = 2048;
constexpr size_t kGroupMaxChecks = 65536;  // lines of every pair resident (unsliced)

bool fill_random(uint64_t *r, size_t n) {
  uint8_t *p = reinterpret_cast<uint8_t *>(r);
  size_t want = n * sizeof(uint64_t), got = 0;
  while (got < want) {
    ssize_t k = getrandom(p + got, want - got, 0);
    if (k < 0) {
      if (errno == EINTR) continue;
      return fail(GBLS_ERR_HIP);
    }
    got += (size_t)k;
  }
  for (size_t i = 0; i < n; i++)
    if (!r[i]) r[i] = 1;
  return true;
}

// Round 2 runs entirely on the device (k_groups.hip): k_group_expand writes every check's
// verdict from its group's and compacts the members to re-check into a list whose length stays
// on the device; the re-checks then run in fixed passes of R slots (tables, Miller product,
// Horner step, final exponentiation writing through the list), slots past the count exiting at
// once.  No host synchronisation: the device entry points stay asynchronous on their stream.
bool grouped_verdicts(Ctx &c, Device &d, const uint8_t *msgs, const uint32_t *msg_off,
                      const g2a *sigs, const PkSource &src, bool sig_groupcheck, size_t n,
                      const uint32_t *seg_off, int32_t *verdicts, hipStream_t st, bool *done) {
  *done = false;
  const size_t gs = kGroupChecks, ng_max = (n + gs - 1) / gs;
  // re-check slots per pass: a quarter of the batch (>= 2048); a typical 1 %-invalid batch
  // re-checks ~8 % of its checks, so one pass does the work and the others exit at once
  const size_t R = std::min(n, std::max<size_t>(2048, (n + 3) / 4)), passes = (n + R - 1) / R;
  std::vector<uint64_t> r(n);
  // every buffer sized before round 1, so no growth (and no host wait) happens in between
  if (!fill_random(r.data(), n) || !c.upload_staged(c.rnd, r.data(), n * 8, st) ||
      !c.ensure(c.part, n * sizeof(fp12)) || !c.ensure(c.err, n * sizeof(int32_t) + 16) ||
      !c.ensure(c.gerr, n * sizeof(int32_t) + 16) || !c.ensure(c.gv, n * sizeof(int32_t) + 16) ||
      !c.ensure(c.redo, (n + 16) * sizeof(uint32_t)) || !c.ensure(c.rtab, 5 * R * sizeof(uint32_t)) ||
      !c.ensure(c.V0, ML_EVENTS * R * sizeof(fp12)) ||
      (g_ml_r28 && !c.ensure(c.V28, (size_t)ML_EVENTS * 168 * 4 * R)))
    return false;
  size_t nms = 0;
  if (!pipeline_partials(c, d, msgs, msg_off, sigs, src, nullptr, sig_groupcheck, n, seg_off, n, 1,
                         c.part.as<fp12>(), c.err.as<int32_t>(), st, (uint32_t)gs,
                         c.rnd.as<uint64_t>(), &nms))
    return false;
  if (nms != ng_max) return true;  // not grouped (line slices): per-check partials, caller goes on
  *done = true;
  launch_group_err(st, c.err.as<int32_t>(), (uint32_t)n, (uint32_t)gs, (uint32_t)nms,
                   c.gerr.as<int32_t>());
  if (!pipeline_final(c.part.as<fp12>(), c.gerr.as<int32_t>(), 1, nms, c.gv.as<int32_t>(), st))
    return false;
  uint32_t *redo = c.redo.as<uint32_t>(), *cnt = redo + n;
  HIPCHK(hipMemsetAsync(cnt, 0, sizeof(uint32_t), st));
  launch_group_expand(st, c.gv.as<int32_t>(), c.err.as<int32_t>(), (uint32_t)n, (uint32_t)gs, verdicts,
                      redo, cnt);
  // round 2: slot j of pass k re-checks redo[k R + j] -- its own Miller product of the SAME
  // pairs (lines resident since round 1), Horner step and final exponentiation
  HIPCHK(hipMemsetAsync(c.gerr.p, 0, R * sizeof(int32_t), st));
  uint32_t *plist = c.rtab.as<uint32_t>(), *grp = plist + 2 * R;
  for (size_t k = 0; k < passes; k++) {
    const uint32_t base = (uint32_t)(k * R);
    launch_redo_tables(st, redo, cnt, base, (uint32_t)R, (uint32_t)n, plist, grp);
    {
      StageTimer t(S_ML_LEAF, st);
      launch_ml_group(st, c.lines.as<uint32_t>(), LineCols{c.line_col, c.line_ncol}, 0, c.P.as<g1s>(), nullptr,
                      plist, grp,
                      (uint32_t)R, 0,
                      ML_EVENTS, c.V0.as<fp12>(), c.V28.as<uint32_t>());
    }
    {
      StageTimer t(S_ML_HORNER, st);
      launch_ml_horner(st, c.V0.as<fp12>(), (uint32_t)R, c.part.as<fp12>(), cnt, base);
    }
    StageTimer t(S_FINAL, st);
    launch_final_verdict(st, c.part.as<fp12>(), c.gerr.as<int32_t>(), 1, (uint32_t)R, verdicts, cnt, base, redo);
  }
  HIPCHK(hipGetLastError());
  return true;
}

bool pipeline_verdicts(Ctx &c, Device &d, const uint8_t *msgs, const uint32_t *msg_off,
                       const g2a *sigs, const PkSource &src, const uint64_t *rands,
                       bool sig_groupcheck, size_t n, const uint32_t *seg_off, size_t nseg,
                       int32_t *verdicts, hipStream_t st) {
  bool ident = !g.per_check.load() && !rands && n == nseg && n >= kGroupMinChecks &&
               n <= kGroupMaxChecks;
  for (size_t s = 0; ident && s <= nseg; s++) ident = seg_off[s] == s;
  if (ident) {
    bool done = false;
    if (!grouped_verdicts(c, d, msgs, msg_off, sigs, src, sig_groupcheck, n, seg_off, verdicts,
                          st, &done))
      return false;
    if (done) return true;
    return pipeline_final(c.part.as<fp12>(), c.err.as<int32_t>(), 1, nseg, verdicts, st);
  }
  if (!c.ensure(c.part, nseg * sizeof(fp12)) || !c.ensure(c.err, nseg * sizeof(int32_t) + 16))
    return false;
  return pipeline_partials(c, d, msgs, msg_off, sigs, src, rands, sig_groupcheck, n, seg_off, nseg,
                           1, c.part.as<fp12>(), c.err.as<int32_t>(), st) &&
         pipeline_final(c.part.as<fp12>(), c.err.as<int32_t>(), 1, nseg, verdicts, st);
}

// Upload a HOST key source for sets [b, e) as a device key source.
bool upload_pks(Ctx &c, const PkSource &host, size_t b, size_t e, hipStream_t st, PkSource *dev) {
  size_t n = e - b;
  *dev = PkSource();
  if (host.off) {
    uint32_t base = host.off[b], cnt = host.off[e] - base;
    std::vector<uint32_t> off(n + 1);
    for (size_t i = 0; i <= n; i++) off[i] = host.off[b + i] - base;
    if (!c.upload_staged(c.in5, off.data(), (n + 1) * 4, st)) return false;
    dev->off = c.in5.as<uint32_t>();
    if (host.pts) {
      if (!c.upload_staged(c.in2, host.pts + base, (size_t)cnt * sizeof(g1a), st)) return false;
      dev->pts = c.in2.as<g1a>();
    } else {
      if (!c.upload_staged(c.in2, host.idx + base, (size_t)cnt * 4, st)) return false;
      dev->idx = c.in2.as<uint32_t>();
    }
  } else if (host.pts) {
    if (!c.upload_staged(c.in2, host.pts + b, n * sizeof(g1a), st)) return false;
    dev->pts = c.in2.as<g1a>();
  } else if (host.idx) {
    if (!c.upload_staged(c.in2, host.idx + b, n * 4, st)) return false;
    dev->idx = c.in2.as<uint32_t>();
  } else {
    return fail(GBLS_ERR_ARG);
  }
  return true;
}

// One device: host batch [sets b..e) in segments seg (rebased, host) -> per-segment
// verdicts (host) when `verdicts`, or else the Miller partial + error flag of the single
// segment, copied device-to-device (hipMemcpyPeerAsync, xGMI) to part_dst / err_dst on
// device dst_dev.  rands == nullptr: independent single checks (r_i = 1, signature subgroup
// check, one segment per set).  Enqueues only; the caller synchronises `c.own` (or waits on it).
bool enqueue_host_batch(Ctx &c, Device &d, const uint8_t *msgs, const g2a *sigs,
                        const uint8_t *sigs_c, int32_t *sig_status, const PkSource &src,
                        const uint64_t *rands, size_t b, size_t e, const uint32_t *seg,
                        size_t nseg, int32_t *verdicts, fp12 *part_dst, int32_t *err_dst,
                        int dst_dev) {
  hipStream_t st = c.own;
  size_t n = e - b;
  if (!c.begin(st)) return false;
  const bool single = rands == nullptr;
  if (!c.upload_staged(c.in0, msgs + 32 * b, 32 * n, st) ||
      (!single && !c.upload_staged(c.in3, rands + b, n * 8, st)))
    return false;
  const g2a *dsigs;
  if (sigs_c) {  // compressed: decompressed on the device by the pipeline (side stream 2)
    if (!c.upload_staged(c.in1, sigs_c + 96 * b, 96 * n, st) ||
        !c.ensure(c.sigd, n * sizeof(g2a) + 16) || !c.ensure(c.sigst, n * 4 + 16))
      return false;
    c.sig_c = c.in1.as<uint8_t>();
    c.sig_st = c.sigst.as<int32_t>();
    dsigs = c.sigd.as<g2a>();
  } else {
    if (!c.upload_staged(c.in1, sigs + b, n * sizeof(g2a), st)) return false;
    dsigs = c.in1.as<g2a>();
  }
  PkSource dsrc;
  if (!upload_pks(c, src, b, e, st, &dsrc)) {
    c.sig_c = nullptr;
    c.sig_st = nullptr;
    return false;
  }
  bool ok;
  const uint64_t *drands = single ? nullptr : c.in3.as<uint64_t>();
  if (verdicts)
    ok = c.ensure(c.out1, nseg * sizeof(int32_t)) &&
         pipeline_verdicts(c, d, c.in0.as<uint8_t>(), nullptr, dsigs, dsrc, drands, single, n, seg,
                           nseg, c.out1.as<int32_t>(), st);
  else
    ok = c.ensure(c.part, sizeof(fp12)) && c.ensure(c.err, 16) &&
         pipeline_partials(c, d, c.in0.as<uint8_t>(), nullptr, dsigs, dsrc, drands, single, n, seg,
                           1, 0, c.part.as<fp12>(), c.err.as<int32_t>(), st);
  c.sig_c = nullptr;  // the option is for this call only, consumed or not
  c.sig_st = nullptr;
  if (!ok) return false;
  if (verdicts) {
    HIPCHK(hipMemcpyAsync(verdicts, c.out1.p, nseg * 4, hipMemcpyDeviceToHost, st));
  } else {
    HIPCHK(hipMemcpyPeerAsync(part_dst, dst_dev, c.part.p, d.hipdev, sizeof(fp12), st));
    HIPCHK(hipMemcpyPeerAsync(err_dst, dst_dev, c.err.p, d.hipdev, 4, st));
  }
  if (sigs_c) HIPCHK(hipMemcpyAsync(sig_status + b, c.sigst.p, n * 4, hipMemcpyDeviceToHost, st));
  return true;
}

// Host-pointer batch verification over every engine device.  Signatures are points
// (sigs) or, for MultiVerifier::finish, compressed bytes (sigs_c, 96 B each) decompressed on
// the device with their statuses written to sig_status.
bool verify_host(const uint8_t *msgs, const g2a *sigs, const uint8_t *sigs_c, int32_t *sig_status,
                 const PkSource &src, const uint64_t *rands, size_t n, const uint32_t *seg_off,
                 size_t nseg, int32_t *verdicts, int cls = 0) {
  std::shared_lock<std::shared_mutex> rl(g.reg_mu);
  const size_t ndev = g.devs.size();
  // ---- one large batch: per-device Miller partials, gathered device-to-device onto device 0
  // (hipMemcpyPeerAsync over xGMI, ordered by events, no host round trip), one final
  // exponentiation there
  if (nseg == 1 && ndev > 1 && n >= 2 * kShardMinSets && rands) {
    size_t k = std::min(ndev, n / kShardMinSets);
    Device &d0 = *g.devs[0];
    Lease L0(d0, cls);
    // L0's part / err become peer-copy destinations of the shard streams, which are not
    // ordered behind L0's previous call: if the pool handed out a context still busy on the
    // GPU, wait for that call on the host first (its final step may still read them)
    if (!L0.ok() || !L0->begin(L0->own) || !L0->drain()) return false;
    hipStream_t st0 = L0->own;
    if (!L0->ensure(L0->part, k * sizeof(fp12)) || !L0->ensure(L0->err, k * 4 + 16) ||
        !L0->ensure(L0->out1, 16))
      return false;
    std::vector<std::unique_ptr<Lease>> leases;
    std::vector<hipEvent_t> evs;
    bool ok = true;
    for (size_t j = 0; j < k && ok; j++) {
      size_t b = n * j / k, e = n * (j + 1) / k;
      Device &d = *g.devs[j];
      leases.emplace_back(new Lease(d, cls));
      Lease &L = *leases.back();
      uint32_t seg[2] = {0, (uint32_t)(e - b)};
      ok = L.ok() && enqueue_host_batch(*L, d, msgs, sigs, sigs_c, sig_status, src, rands, b, e,
                                        seg, 1, nullptr, L0->part.as<fp12>() + j,
                                        L0->err.as<int32_t>() + j, d0.hipdev);
      if (!ok) break;
      hipEvent_t ev;
      if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
        ok = fail(GBLS_ERR_HIP);
        break;
      }
      evs.push_back(ev);
      if (hipEventRecord(ev, L->own) != hipSuccess) ok = fail(GBLS_ERR_HIP);
    }
    if (ok && hipSetDevice(d0.hipdev) != hipSuccess) ok = fail(GBLS_ERR_HIP);
    for (size_t j = 0; ok && j < evs.size(); j++)
      if (hipStreamWaitEvent(st0, evs[j], 0) != hipSuccess) ok = fail(GBLS_ERR_HIP);
    ok = ok && pipeline_final(L0->part.as<fp12>(), L0->err.as<int32_t>(), k, 1,
                              L0->out1.as<int32_t>(), st0);
    if (ok && hipMemcpyAsync(verdicts, L0->out1.p, 4, hipMemcpyDeviceToHost, st0) != hipSuccess)
      ok = fail(GBLS_ERR_HIP);
    rl.unlock();  // enqueued: the host wait does not hold up registry updates
    // the final's stream waited on every shard, so its completion covers theirs (including the
    // shards' signature-status copies to the host); on a failure every shard is drained
    if (ok && hipStreamSynchronize(st0) != hipSuccess) ok = fail(GBLS_ERR_HIP);
    if (!ok)
      for (auto &L : leases) (void)hipStreamSynchronize((*L)->own);
    for (hipEvent_t ev : evs) (void)hipEventDestroy(ev);
    return ok;
  }
  // ---- whole segments per device, contiguous groups balanced by set count
  size_t k = 1;
  if (ndev > 1 && nseg > 1) k = std::min({ndev, nseg, std::max<size_t>(1, n / kShardMinSets)});
  std::vector<size_t> cut(k + 1, 0);  // segment boundaries of the groups
  cut[k] = nseg;
  for (size_t j = 1; j < k; j++) {
    size_t target = n * j / k, s = cut[j - 1];
    while (s < nseg && seg_off[s] < target) s++;
    cut[j] = std::max(s, cut[j - 1]);
  }
  std::vector<std::unique_ptr<Lease>> leases;
  std::vector<std::vector<uint32_t>> segs(k);
  bool ok = true;
  for (size_t j = 0; j < k && ok; j++) {
    size_t s0 = cut[j], s1 = cut[j + 1];
    if (s1 == s0) continue;
    size_t b = seg_off[s0], e = seg_off[s1];
    segs[j].resize(s1 - s0 + 1);
    for (size_t s = s0; s <= s1; s++) segs[j][s - s0] = seg_off[s] - (uint32_t)b;
    Device &d = k == 1 ? pick_device() : *g.devs[j];
    leases.emplace_back(new Lease(d, cls));
    Lease &L = *leases.back();
    ok = L.ok() && enqueue_host_batch(*L, d, msgs, sigs, sigs_c, sig_status, src, rands, b, e,
                                      segs[j].data(), s1 - s0, verdicts + s0, nullptr, nullptr, 0);
  }
  rl.unlock();  // enqueued: the host waits do not hold up registry updates
  for (auto &L : leases)
    if (hipStreamSynchronize((*L)->own) != hipSuccess) ok = fail(GBLS_ERR_HIP);
  return ok;
}

// ----- f3: cross-caller coalescing.  Concurrent host-pointer multi_verify calls (the
// node's gossip batches of <= 64 sets, p2p/src/attestation_verifier.rs:37,142-163, and
// the block verification pool's per-block batches, p2p/src/block_verification_pool.rs:
// 103-128) queue here; a caller that finds fewer than g.leaders x devices
// submissions in flight becomes a leader and verifies every queued request with the same
// key source kind as ONE segmented submission (each request keeps its own segments and
// verdicts).  Batches therefore grow with the load, while an idle engine runs a lone
// call immediately (no waiting window).
// (gbls_sched.h: queues, leaders, the collection window and the merge itself)
using CoReq = sched::Request<g1a, g2a>;
sched::Coalescer<CoReq> co;

bool coalesced_verify(CoReq &r) {
  sched::Config cfg;
  cfg.coalesce = g.coalesce.load();
  cfg.devices = (int)g.devs.size();
  cfg.leaders = g.leaders;
  cfg.merge_target = g.merge_target;
  cfg.merge_window_us = g.merge_window_us;
  if (g.block_hold) cfg.hold = &g.block_active;
  bool ok = co.submit(r, cfg, [](CoReq &m) {
    m.ok = verify_host(m.msgs, m.sigs, m.sigs_c, m.sig_status, m.src, m.rands, m.n, m.seg_off,
                       m.nseg, m.verdicts, m.prio);
    m.err = t_last_error;  // the leader's thread-local code, handed to every merged caller
  });
  t_last_error = r.err;
  return ok;
}

void fill(int32_t *v, size_t n, int32_t x) {
  for (size_t i = 0; i < n; i++) v[i] = x;
}

// Per-set verdicts of a batch by GPU bisection (f2): verify the batch; split every
// failing range into up to kFan pieces and verify all pieces of a round as segments of
// ONE submission, until the failing pieces are single sets.
constexpr size_t kFan = 16;
bool bisect_host(const uint8_t *msgs, const g2a *sigs, const PkSource &src,
                 const uint64_t *rands, size_t n, int32_t *set_verdicts) {
  struct Range {
    size_t b, e;
  };
  std::vector<Range> frontier{{0, n}};
  std::vector<uint8_t> gm;
  std::vector<g2a> gs;
  std::vector<g1a> gp;
  std::vector<uint32_t> gi, go;
  std::vector<uint64_t> gr;
  bool first = true;
  while (!frontier.empty()) {
    std::vector<Range> pieces;
    for (const Range &r : frontier) {
      size_t len = r.e - r.b;
      size_t parts = first ? 1 : std::min(kFan, len);
      for (size_t j = 0; j < parts; j++)
        pieces.push_back({r.b + len * j / parts, r.b + len * (j + 1) / parts});
    }
    first = false;
    // gather the pieces into one contiguous batch
    gm.clear(); gs.clear(); gp.clear(); gi.clear(); go.clear(); gr.clear();
    std::vector<uint32_t> seg{0};
    if (src.off) go.push_back(0);
    for (const Range &p : pieces) {
      for (size_t i = p.b; i < p.e; i++) {
        gm.insert(gm.end(), msgs + 32 * i, msgs + 32 * i + 32);
        gs.push_back(sigs[i]);
        gr.push_back(rands[i]);
        if (src.pts) gp.push_back(src.pts[i]);
        else if (src.off) {
          gi.insert(gi.end(), src.idx + src.off[i], src.idx + src.off[i + 1]);
          go.push_back((uint32_t)gi.size());
        } else gi.push_back(src.idx[i]);
      }
      seg.push_back((uint32_t)gs.size());
    }
    PkSource s2;
    if (src.pts) s2.pts = gp.data();
    else {
      s2.idx = gi.data();
      if (src.off) s2.off = go.data();
    }
    std::vector<int32_t> v(pieces.size(), FAILED);
    if (!verify_host(gm.data(), gs.data(), nullptr, nullptr, s2, gr.data(), gs.size(), seg.data(),
                     pieces.size(), v.data(), 0))
      return false;
    frontier.clear();
    for (size_t j = 0; j < pieces.size(); j++) {
      const Range &p = pieces[j];
      if (v[j] == GBLS_SUCCESS)
        fill(set_verdicts + p.b, p.e - p.b, GBLS_SUCCESS);
      else if (p.e - p.b == 1)
        set_verdicts[p.b] = GBLS_VERIFY_FAIL;
      else
        frontier.push_back(p);
    }
  }
  return true;
}

// the registry's streams and events on device d (created on first use, under reg_mu)
bool registry_streams(Device &d) {
  if (d.reg_st) return true;
  HIPCHK(hipSetDevice(d.hipdev));
  int least = 0, greatest = 0;  // registry updates are small: they jump the queued normal work
  HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  HIPCHK(hipStreamCreateWithPriority(&d.reg_st, hipStreamNonBlocking, greatest));
  HIPCHK(hipEventCreateWithFlags(&d.reg_ev, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&d.reg_tmp, hipEventDisableTiming));
  return true;
}
// Grow d's table to hold `need` bytes, stream-ordered on d.reg_st: a new table (zeroed past the
// loaded entries, the loaded ones copied), and the old one freed on d.retire_st once the copy
// and every kernel that read it have run (each context's last registry read, and the replica
// copies of earlier updates).  No host wait, no device synchronisation.
bool registry_grow(Device &d, size_t need, size_t loaded) {
  const size_t want = need + need / 4;
  void *nb = nullptr;
  bool pooled = true;
  if (hipMallocAsync(&nb, want, d.reg_st) != hipSuccess) {  // no stream-ordered allocator
    (void)hipGetLastError();
    pooled = false;
    HIPCHK(hipMalloc(&nb, want));
  }
  if (loaded) HIPCHK(hipMemcpyAsync(nb, d.reg.p, loaded, hipMemcpyDeviceToDevice, d.reg_st));
  HIPCHK(hipMemsetAsync(static_cast<uint8_t *>(nb) + loaded, 0, want - loaded, d.reg_st));
  // kept tables of earlier growths (no stream-ordered allocator) whose readers have finished
  for (size_t i = 0; i < d.reg_kept.size();) {
    if (hipEventQuery(d.reg_kept[i].ev) == hipSuccess) {
      (void)hipFree(d.reg_kept[i].p);
      (void)hipEventDestroy(d.reg_kept[i].ev);
      d.reg_kept.erase(d.reg_kept.begin() + (std::ptrdiff_t)i);
    } else {
      i++;
    }
  }
  (void)hipGetLastError();
  if (d.reg.p) {
    // the retire stream is created by the first growth that retires a table (a stream holds a
    // hardware queue from its creation; the engine's queue set is tuned, see kPrewarmCtx)
    if (!d.retire_st) HIPCHK(hipStreamCreateWithFlags(&d.retire_st, hipStreamNonBlocking));
    HIPCHK(hipEventRecord(d.reg_tmp, d.reg_st));
    HIPCHK(hipStreamWaitEvent(d.retire_st, d.reg_tmp, 0));
    bool ok = true;
    d.pool.for_each([&](Ctx &c) {
      if (c.reg_read && hipStreamWaitEvent(d.retire_st, c.ev_reg, 0) != hipSuccess) ok = false;
    });
    for (auto &o : g.devs)  // replica copies of earlier updates read device 0's table
      if (o->reg_ev_set && hipStreamWaitEvent(d.retire_st, o->reg_ev, 0) != hipSuccess) ok = false;
    if (!ok) return fail(GBLS_ERR_HIP);
    if (d.reg_pooled) {
      HIPCHK(hipFreeAsync(d.reg.p, d.retire_st));
    } else {  // readers may still be running: kept behind an event, never host-waited
      Device::Kept k{d.reg.p, nullptr};
      HIPCHK(hipEventCreateWithFlags(&k.ev, hipEventDisableTiming));
      HIPCHK(hipEventRecord(k.ev, d.retire_st));
      d.reg_kept.push_back(k);
    }
  }
  d.reg.p = nb;
  d.reg.cap = want;
  d.reg_pooled = pooled;
  return true;
}
}  // namespace

#define API_BEGIN                   \
  t_last_error = GBLS_ERR_NONE;     \
  if (!ensure_ready()) return FAILED;

extern "C" {

int gbls_init(uint32_t device_mask, uint32_t flags) {
  t_last_error = GBLS_ERR_NONE;
  return engine_init(device_mask, flags) ? GBLS_SUCCESS : FAILED;
}

uint32_t gbls_set_policy(uint32_t flags) {
  uint32_t prev = (g.coalesce.load() ? 0u : GBLS_INIT_NO_COALESCE) |
                  (g.per_check.load() ? GBLS_INIT_PER_CHECK : 0u);
  g.coalesce.store((flags & GBLS_INIT_NO_COALESCE) == 0);
  g.per_check.store((flags & GBLS_INIT_PER_CHECK) != 0);
  return prev;
}

int gbls_last_error(void) { return t_last_error; }
const char *gbls_version(void) { return "grandine-bls-mi355x 0.3 (gfx950)"; }
int gbls_device_count(void) { return g.ready.load() ? (int)g.devs.size() : 0; }

int gbls_g1_decompress(const uint8_t (*in)[48], size_t n, int validate, gbls_p1_affine *out,
                       int32_t *status) {
  fill(status, n, GBLS_BAD_ENCODING);
  API_BEGIN
  if (n == 0) return GBLS_SUCCESS;
  Lease L(pick_device());
  Ctx &c = *L;
  hipStream_t st = c.own;
  if (!L.ok() || !c.begin(st) || !c.upload_staged(c.in0, &in[0][0], 48 * n, st) ||
      !c.ensure(c.out0, n * sizeof(g1a)) || !c.ensure(c.out1, n * sizeof(int32_t)))
    return FAILED;
  launch_g1_decompress(st, c.in0.as<uint8_t>(), (uint32_t)n, validate, c.out0.as<g1a>(),
                       c.out1.as<int32_t>());
  if (hipMemcpyAsync(out, c.out0.p, n * sizeof(g1a), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(status, c.out1.p, n * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess) {
    fill(status, n, GBLS_BAD_ENCODING);
    return fail(GBLS_ERR_HIP), FAILED;
  }
  return GBLS_SUCCESS;
}

int gbls_g2_decompress(const uint8_t (*in)[96], size_t n, gbls_p2_affine *out, int32_t *status) {
  fill(status, n, GBLS_BAD_ENCODING);
  API_BEGIN
  if (n == 0) return GBLS_SUCCESS;
  Lease L(pick_device());
  Ctx &c = *L;
  hipStream_t st = c.own;
  if (!L.ok() || !c.begin(st) || !c.upload_staged(c.in0, &in[0][0], 96 * n, st) ||
      !c.ensure(c.out0, n * sizeof(g2a)) || !c.ensure(c.out1, n * sizeof(int32_t)))
    return FAILED;
  launch_g2_decompress(st, c.in0.as<uint8_t>(), (uint32_t)n, c.out0.as<g2a>(),
                       c.out1.as<int32_t>());
  if (hipMemcpyAsync(out, c.out0.p, n * sizeof(g2a), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(status, c.out1.p, n * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess) {
    fill(status, n, GBLS_BAD_ENCODING);
    return fail(GBLS_ERR_HIP), FAILED;
  }
  return GBLS_SUCCESS;
}

int gbls_g2_validate(const gbls_p2_affine *in, size_t n, int32_t *status) {
  fill(status, n, GBLS_POINT_NOT_IN_GROUP);
  API_BEGIN
  if (n == 0) return GBLS_SUCCESS;
  Lease L(pick_device());
  Ctx &c = *L;
  hipStream_t st = c.own;
  if (!L.ok() || !c.begin(st) || !c.upload_staged(c.in0, in, n * sizeof(g2a), st) ||
      !c.ensure(c.out1, n * sizeof(int32_t)))
    return FAILED;
  launch_g2_check(st, c.in0.as<g2a>(), (uint32_t)n, c.out1.as<int32_t>(), 0);
  if (hipMemcpyAsync(status, c.out1.p, n * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess) {
    fill(status, n, GBLS_POINT_NOT_IN_GROUP);
    return fail(GBLS_ERR_HIP), FAILED;
  }
  return GBLS_SUCCESS;
}

static int compress_impl(const void *in, size_t n, size_t in_sz, size_t out_sz, uint8_t *out,
                         int which) {
  API_BEGIN
  if (n == 0) return GBLS_SUCCESS;
  Lease L(pick_device());
  Ctx &c = *L;
  hipStream_t st = c.own;
  if (!L.ok() || !c.begin(st) || !c.upload_staged(c.in0, in, n * in_sz, st) ||
      !c.ensure(c.out0, n * out_sz))
    return FAILED;
  if (which == 1)
    launch_g1_compress(st, c.in0.as<g1a>(), (uint32_t)n, c.out0.as<uint8_t>());
  else
    launch_g2_compress(st, c.in0.as<g2a>(), (uint32_t)n, c.out0.as<uint8_t>());
  if (hipMemcpyAsync(out, c.out0.p, n * out_sz, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return fail(GBLS_ERR_HIP), FAILED;
  return GBLS_SUCCESS;
}
int gbls_g1_compress(const gbls_p1_affine *in, size_t n, uint8_t (*out)[48]) {
  return compress_impl(in, n, sizeof(g1a), 48, &out[0][0], 1);
}
int gbls_g2_compress(const gbls_p2_affine *in, size_t n, uint8_t (*out)[96]) {
  return compress_impl(in, n, sizeof(g2a), 96, &out[0][0], 2);
}

// segmented aggregation of points (which = 1: G1, 2: G2) or of registry keys (which = 3)
static int aggregate_impl(const void *pts, const uint32_t *idx, const uint32_t *seg_offsets,
                          size_t nseg, void *out, int32_t *status, int which) {
  fill(status, nseg, GBLS_AGGR_TYPE_MISMATCH);
  API_BEGIN
  if (nseg == 0) return GBLS_SUCCESS;
  if (!seg_offsets || seg_offsets[0] != 0) return fail(GBLS_ERR_ARG), FAILED;
  for (size_t s = 0; s < nseg; s++)
    if (seg_offsets[s + 1] < seg_offsets[s]) return fail(GBLS_ERR_ARG), FAILED;
  size_t n = seg_offsets[nseg];
  size_t psz = which == 2 ? sizeof(g2a) : sizeof(g1a);
  std::shared_lock<std::shared_mutex> rl(g.reg_mu);
  Device &d = pick_device();
  Lease L(d);
  Ctx &c = *L;
  hipStream_t st = c.own;
  if (!L.ok() || !c.begin(st) ||
      !c.upload_staged(c.in0, which == 3 ? (const void *)idx : pts, n * (which == 3 ? 4 : psz), st) ||
      !c.upload_staged(c.in1, seg_offsets, (nseg + 1) * 4, st) || !c.ensure(c.out0, nseg * psz) ||
      !c.ensure(c.out1, nseg * sizeof(int32_t)))
    return FAILED;
  if (which == 1)
    launch_g1_aggregate_seg(st, c.in0.as<g1a>(), c.in1.as<uint32_t>(), (uint32_t)nseg,
                            c.out0.as<g1a>(), c.out1.as<int32_t>());
  else if (which == 2)
    launch_g2_aggregate_seg(st, c.in0.as<g2a>(), c.in1.as<uint32_t>(), (uint32_t)nseg,
                            c.out0.as<g2a>(), c.out1.as<int32_t>());
  else if (!registry_read_begin(c, d, st))
    return FAILED;
  else
    launch_g1_aggregate_idx(st, d.reg.as<g1a>(), (uint32_t)g.reg_n, c.in0.as<uint32_t>(),
                            c.in1.as<uint32_t>(), (uint32_t)nseg, c.out0.as<g1a>(),
                            c.out1.as<int32_t>());
  if (which == 3 && !registry_read_end(c, st)) return FAILED;
  if (hipMemcpyAsync(out, c.out0.p, nseg * psz, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipMemcpyAsync(status, c.out1.p, nseg * 4, hipMemcpyDeviceToHost, st) != hipSuccess)
    return fail(GBLS_ERR_HIP), FAILED;
  rl.unlock();  // enqueued: the host wait below does not hold up registry updates
  if (hipStreamSynchronize(st) != hipSuccess) {
    fill(status, nseg, GBLS_AGGR_TYPE_MISMATCH);
    return fail(GBLS_ERR_HIP), FAILED;
  }
  return GBLS_SUCCESS;
}

int gbls_g1_aggregate_segments(const gbls_p1_affine *pks, const uint32_t *seg_offsets, size_t nseg,
                               gbls_p1_affine *out, int32_t *status) {
  return aggregate_impl(pks, nullptr, seg_offsets, nseg, out, status, 1);
}
int gbls_g2_aggregate_segments(const gbls_p2_affine *sigs, const uint32_t *seg_offsets,
                               size_t nseg, gbls_p2_affine *out, int32_t *status) {
  return aggregate_impl(sigs, nullptr, seg_offsets, nseg, out, status, 2);
}
int gbls_g1_aggregate_indexed(const uint32_t *idx, const uint32_t *seg_offsets, size_t nseg,
                              gbls_p1_affine *out, int32_t *status) {
  return aggregate_impl(nullptr, idx, seg_offsets, nseg, out, status, 3);
}

int gbls_g1_aggregate(const gbls_p1_affine *pks, size_t n, gbls_p1_affine *out) {
  t_last_error = GBLS_ERR_NONE;
  uint32_t off[2] = {0, (uint32_t)n};
  int32_t st = GBLS_AGGR_TYPE_MISMATCH;
  if (n == 0) {
    std::memset(out, 0, sizeof(*out));
    return GBLS_AGGR_TYPE_MISMATCH;
  }
  int rc = gbls_g1_aggregate_segments(pks, off, 1, out, &st);
  return rc != GBLS_SUCCESS ? rc : st;
}

int gbls_g2_aggregate(const gbls_p2_affine *sigs, size_t n, gbls_p2_affine *out) {
  t_last_error = GBLS_ERR_NONE;
  uint32_t off[2] = {0, (uint32_t)n};
  int32_t st = GBLS_AGGR_TYPE_MISMATCH;
  if (n == 0) {
    std::memset(out, 0, sizeof(*out));
    return GBLS_AGGR_TYPE_MISMATCH;
  }
  int rc = gbls_g2_aggregate_segments(sigs, off, 1, out, &st);
  return rc != GBLS_SUCCESS ? rc : st;
}

// m independent checks e(pk_i, H(m_i)) == e(g1, sig_i), each its own segment (r_i = 1),
// with the signature subgroup check.  mode 0: one key per check (pts); 1: aggregate pts
// per check (seg_off); 2: aggregate registry keys idx per check (seg_off).
static int single_checks(const g2a *sigs, const uint8_t *msg_data, const uint32_t *msg_off,
                         const void *keys, const uint32_t *seg_off, size_t m, int mode,
                         int32_t *verdicts) {
  fill(verdicts, m, GBLS_VERIFY_FAIL);
  API_BEGIN
  if (m == 0) return GBLS_SUCCESS;
  if (mode && !valid_offsets(seg_off, m, seg_off ? seg_off[m] : 0))
    return fail(GBLS_ERR_ARG), FAILED;
  size_t nkeys = mode ? seg_off[m] : m;
  std::shared_lock<std::shared_mutex> rl(g.reg_mu);
  Device &d = pick_device();
  Lease L(d);
  Ctx &c = *L;
  hipStream_t st = c.own;
  std::vector<uint32_t> ident(m + 1);
  for (size_t i = 0; i <= m; i++) ident[i] = (uint32_t)i;
  if (!L.ok() || !c.begin(st) || !c.upload_staged(c.in0, sigs, m * sizeof(g2a), st) ||
      !c.upload_staged(c.in1, msg_data, msg_off[m] ? msg_off[m] : 1, st) ||
      !c.upload_staged(c.in2, msg_off, (m + 1) * 4, st) ||
      !c.upload_staged(c.in4, keys, (nkeys ? nkeys : 1) * (mode == 2 ? 4 : sizeof(g1a)), st) ||
      !c.ensure(c.out1, m * sizeof(int32_t)))
    return FAILED;
  PkSource src;
  if (mode == 2)
    src.idx = c.in4.as<uint32_t>();
  else
    src.pts = c.in4.as<g1a>();
  if (mode) {
    if (!c.upload_staged(c.in5, seg_off, (m + 1) * 4, st)) return FAILED;
    src.off = c.in5.as<uint32_t>();
  }
  if (!pipeline_verdicts(c, d, c.in1.as<uint8_t>(), c.in2.as<uint32_t>(), c.in0.as<g2a>(), src,
                         nullptr, true, m, ident.data(), m, c.out1.as<int32_t>(), st))
    return FAILED;
  if (hipMemcpyAsync(verdicts, c.out1.p, m * 4, hipMemcpyDeviceToHost, st) != hipSuccess)
    return fail(GBLS_ERR_HIP), FAILED;
  rl.unlock();  // enqueued: the host wait does not hold up registry updates
  if (hipStreamSynchronize(st) != hipSuccess) {
    fill(verdicts, m, GBLS_VERIFY_FAIL);
    return fail(GBLS_ERR_HIP), FAILED;
  }
  return GBLS_SUCCESS;
}

// Single checks with 32-byte messages (every consensus caller: signing roots) go through the
// coalescer (f3): concurrent Signature::verify / fast_aggregate_verify calls -- sync-committee
// messages and contributions (operation_pools/src/sync_committee_agg_pool/tasks.rs:397-430),
// SingleVerifier::extend (helper_functions/src/verifier.rs:215-236) on many rayon workers --
// become segments of ONE submission instead of one pipeline each.  Signatures are points
// (sigs) or 96-byte encodings (sigs_c, decompressed in the same submission, statuses in
// sig_status: SingleVerifier::extend's try_from and verify cost one submission, not two).
// Keys: one point per check, or the sum of pks[pk_off[i] .. pk_off[i+1]) (fast_aggregate_verify).
static int single_checks_co(const uint8_t *msgs, const g2a *sigs, const uint8_t *sigs_c,
                            int32_t *sig_status, const g1a *pks, const uint32_t *pk_off, size_t m,
                            int32_t *verdicts) {
  fill(verdicts, m, GBLS_VERIFY_FAIL);
  if (sig_status) fill(sig_status, m, GBLS_BAD_ENCODING);
  API_BEGIN
  if (m == 0) return GBLS_SUCCESS;
  if (!msgs || !pks || (!sigs == !sigs_c) || (sigs_c && !sig_status)) return fail(GBLS_ERR_ARG), FAILED;
  if (pk_off && !valid_offsets(pk_off, m, pk_off[m])) return fail(GBLS_ERR_ARG), FAILED;
  std::vector<uint32_t> ident(m + 1);
  for (size_t i = 0; i <= m; i++) ident[i] = (uint32_t)i;
  CoReq r{msgs, sigs, PkSource(), nullptr, m, ident.data(), m, verdicts};
  r.src.pts = pks;
  r.src.off = pk_off;
  r.sigs_c = sigs_c;
  r.sig_status = sig_status;
  if (!coalesced_verify(r)) {
    fill(verdicts, m, GBLS_VERIFY_FAIL);
    if (sig_status) fill(sig_status, m, GBLS_BAD_ENCODING);
    return FAILED;
  }
  return GBLS_SUCCESS;
}
static bool msgs_are_roots(const uint32_t *msg_off, size_t m) {
  for (size_t i = 0; i <= m; i++)
    if (msg_off[i] != 32 * i) return false;
  return true;
}

int gbls_aggregate_verify_batch(const gbls_p2_affine *sigs, const uint8_t *msg_data,
                                const uint32_t *msg_off, const gbls_p1_affine *pks, size_t m,
                                int32_t *verdicts) {
  if (m && msg_off && msgs_are_roots(msg_off, m))
    return single_checks_co(msg_data, reinterpret_cast<const g2a *>(sigs), nullptr, nullptr,
                            reinterpret_cast<const g1a *>(pks), nullptr, m, verdicts);
  return single_checks(reinterpret_cast<const g2a *>(sigs), msg_data, msg_off, pks, nullptr, m, 0,
                       verdicts);
}

int gbls_verify(const gbls_p2_affine *sig, const uint8_t *msg, size_t msg_len,
                const gbls_p1_affine *pk) {
  uint32_t off[2] = {0, (uint32_t)msg_len};
  int32_t v = GBLS_VERIFY_FAIL;
  uint8_t dummy = 0;
  if (gbls_aggregate_verify_batch(sig, msg_len ? msg : &dummy, off, pk, 1, &v) != GBLS_SUCCESS)
    return GBLS_VERIFY_FAIL;
  return v;
}

int gbls_fast_aggregate_verify_batch(const gbls_p2_affine *sigs, const uint8_t *msg_data,
                                     const uint32_t *msg_off, const gbls_p1_affine *pks,
                                     const uint32_t *seg_off, size_t m, int32_t *verdicts) {
  if (m && msg_off && msgs_are_roots(msg_off, m))
    return single_checks_co(msg_data, reinterpret_cast<const g2a *>(sigs), nullptr, nullptr,
                            reinterpret_cast<const g1a *>(pks), seg_off, m, verdicts);
  return single_checks(reinterpret_cast<const g2a *>(sigs), msg_data, msg_off, pks, seg_off, m, 1,
                       verdicts);
}

int gbls_verify_batch_compressed(const uint8_t (*msgs)[32], const uint8_t (*sigs)[96],
                                 const gbls_p1_affine *pks, const uint32_t *pk_off, size_t m,
                                 int32_t *sig_status, int32_t *verdicts) {
  return single_checks_co(msgs ? &msgs[0][0] : nullptr, nullptr, sigs ? &sigs[0][0] : nullptr,
                          sig_status, reinterpret_cast<const g1a *>(pks), pk_off, m, verdicts);
}

int gbls_fast_aggregate_verify_indexed(const gbls_p2_affine *sigs, const uint8_t *msg_data,
                                       const uint32_t *msg_off, const uint32_t *pk_idx,
                                       const uint32_t *seg_off, size_t m, int32_t *verdicts) {
  return single_checks(reinterpret_cast<const g2a *>(sigs), msg_data, msg_off, pk_idx, seg_off,
                       m, 2, verdicts);
}

int gbls_fast_aggregate_verify(const gbls_p2_affine *sig, const uint8_t *msg, size_t msg_len,
                               const gbls_p1_affine *pks, size_t n) {
  t_last_error = GBLS_ERR_NONE;
  if (n == 0) return GBLS_VERIFY_FAIL;  // blst: AGGR_TYPE_MISMATCH -> not SUCCESS
  uint32_t moff[2] = {0, (uint32_t)msg_len};
  uint32_t soff[2] = {0, (uint32_t)n};
  int32_t v = GBLS_VERIFY_FAIL;
  uint8_t dummy = 0;
  if (gbls_fast_aggregate_verify_batch(sig, msg_len ? msg : &dummy, moff, pks, soff, 1, &v) !=
      GBLS_SUCCESS)
    return GBLS_VERIFY_FAIL;
  return v;
}

int gbls_multi_verify_segments(const uint8_t (*msgs)[32], const gbls_p2_affine *sigs,
                               const gbls_p1_affine *pks, const uint64_t *rands, size_t n,
                               const uint32_t *seg_off, size_t nseg, int32_t *verdicts) {
  fill(verdicts, nseg, GBLS_VERIFY_FAIL);
  API_BEGIN
  if (nseg == 0) return GBLS_SUCCESS;
  if (!valid_offsets(seg_off, nseg, n)) return fail(GBLS_ERR_ARG), FAILED;
  CoReq r{&msgs[0][0], reinterpret_cast<const g2a *>(sigs), PkSource(), rands, n, seg_off,
          nseg, verdicts};
  r.src.pts = reinterpret_cast<const g1a *>(pks);
  if (!coalesced_verify(r)) {
    fill(verdicts, nseg, GBLS_VERIFY_FAIL);
    return FAILED;
  }
  return GBLS_SUCCESS;
}

int gbls_multi_verify(const uint8_t (*msgs)[32], const gbls_p2_affine *sigs,
                      const gbls_p1_affine *pks, const uint64_t *rands, size_t n) {
  t_last_error = GBLS_ERR_NONE;  // the early verdicts below are verdicts, not engine errors
  if (n == 0) return GBLS_VERIFY_FAIL;
  for (size_t i = 0; i < n; i++)
    if (rands[i] == 0) return GBLS_VERIFY_FAIL;  // NonZeroU64 contract
  uint32_t off[2] = {0, (uint32_t)n};
  int32_t v = GBLS_VERIFY_FAIL;
  if (gbls_multi_verify_segments(msgs, sigs, pks, rands, n, off, 1, &v) != GBLS_SUCCESS)
    return GBLS_VERIFY_FAIL;
  return v;
}

int gbls_multi_verify_indexed(const uint8_t (*msgs)[32], const gbls_p2_affine *sigs,
                              const uint32_t *pk_idx, const uint32_t *pk_off,
                              const uint64_t *rands, size_t n) {
  API_BEGIN
  if (n == 0) return GBLS_VERIFY_FAIL;
  if (pk_off && !valid_offsets(pk_off, n, pk_off[n])) return fail(GBLS_ERR_ARG), GBLS_VERIFY_FAIL;
  uint32_t off[2] = {0, (uint32_t)n};
  int32_t v = GBLS_VERIFY_FAIL;
  CoReq r{&msgs[0][0], reinterpret_cast<const g2a *>(sigs), PkSource(), rands, n, off, 1, &v};
  r.src.idx = pk_idx;
  r.src.off = pk_off;
  if (!coalesced_verify(r)) return GBLS_VERIFY_FAIL;
  return v;
}

int gbls_multi_verify_compressed_ex(const uint8_t (*msgs)[32], const uint8_t (*sigs)[96],
                                    const gbls_p1_affine *pks, const uint32_t *pk_idx,
                                    const uint32_t *pk_off, const uint64_t *rands, size_t n,
                                    int32_t *sig_status, uint32_t call_flags) {
  t_last_error = GBLS_ERR_NONE;
  if (!sig_status) return fail(GBLS_ERR_ARG), GBLS_VERIFY_FAIL;
  fill(sig_status, n, GBLS_BAD_ENCODING);
  API_BEGIN
  if (n == 0) return GBLS_VERIFY_FAIL;
  if (!pks == !pk_idx) return fail(GBLS_ERR_ARG), GBLS_VERIFY_FAIL;
  if (pk_off && !valid_offsets(pk_off, n, pk_off[n])) return fail(GBLS_ERR_ARG), GBLS_VERIFY_FAIL;
  uint32_t off[2] = {0, (uint32_t)n};
  int32_t v = GBLS_VERIFY_FAIL;
  CoReq r{&msgs[0][0], nullptr, PkSource(), rands, n, off, 1, &v};
  r.src.pts = reinterpret_cast<const g1a *>(pks);
  r.src.idx = pk_idx;
  r.src.off = pk_off;
  r.sigs_c = &sigs[0][0];
  r.sig_status = sig_status;
  r.prio = (call_flags & GBLS_CALL_BLOCK) ? 1 : 0;
  struct BlockActive {  // normal submissions keep off the reserved CUs meanwhile
    bool on;
    explicit BlockActive(bool b) : on(b) {
      if (on) g.block_active.fetch_add(1);
    }
    ~BlockActive() {
      if (on && g.block_active.fetch_sub(1) == 1) co.wake();  // held normal callers go on
    }
  } block_active(r.prio != 0);
  if (!coalesced_verify(r)) {
    fill(sig_status, n, GBLS_BAD_ENCODING);
    return GBLS_VERIFY_FAIL;
  }
  for (size_t i = 0; i < n; i++)  // MultiVerifier::finish: a decoding error comes first
    if (sig_status[i] != GBLS_SUCCESS) return sig_status[i];
  return v;
}

int gbls_multi_verify_compressed(const uint8_t (*msgs)[32], const uint8_t (*sigs)[96],
                                 const gbls_p1_affine *pks, const uint32_t *pk_idx,
                                 const uint32_t *pk_off, const uint64_t *rands, size_t n,
                                 int32_t *sig_status) {
  return gbls_multi_verify_compressed_ex(msgs, sigs, pks, pk_idx, pk_off, rands, n, sig_status, 0);
}

int gbls_multi_verify_bisect(const uint8_t (*msgs)[32], const gbls_p2_affine *sigs,
                             const gbls_p1_affine *pks, const uint32_t *pk_idx,
                             const uint32_t *pk_off, const uint64_t *rands, size_t n,
                             int32_t *set_verdicts) {
  fill(set_verdicts, n, GBLS_VERIFY_FAIL);
  API_BEGIN
  if (n == 0) return GBLS_SUCCESS;
  if (pk_off && !valid_offsets(pk_off, n, pk_off[n])) return fail(GBLS_ERR_ARG), FAILED;
  PkSource src;
  src.pts = reinterpret_cast<const g1a *>(pks);
  src.idx = pks ? nullptr : pk_idx;
  src.off = pks ? nullptr : pk_off;
  if (!src.pts && !src.idx) return fail(GBLS_ERR_ARG), FAILED;
  if (!bisect_host(&msgs[0][0], reinterpret_cast<const g2a *>(sigs), src, rands, n,
                   set_verdicts)) {
    fill(set_verdicts, n, GBLS_VERIFY_FAIL);
    return FAILED;
  }
  return GBLS_SUCCESS;
}

// ---- device-pointer variants (inputs resident in HBM, asynchronous on the caller's stream)
static int device_verify(const uint8_t *msgs, const g2a *sigs, const PkSource &src,
                         const uint64_t *rands, size_t n, const uint32_t *seg_off, size_t nseg,
                         int32_t *verdicts, fp12 *partials, int32_t *seg_err, void *stream) {
  API_BEGIN
  if (nseg == 0) return GBLS_SUCCESS;
  if (!valid_offsets(seg_off, nseg, n)) return fail(GBLS_ERR_ARG), FAILED;
  Device *d = current_device();
  if (!d) return fail(GBLS_ERR_ARG), FAILED;
  std::shared_lock<std::shared_mutex> rl(g.reg_mu);
  Lease L(*d, true, (hipStream_t)stream);
  Ctx &c = *L;
  hipStream_t st = (hipStream_t)stream;
  if (!L.ok() || !c.begin(st)) return FAILED;
  bool ok = verdicts ? pipeline_verdicts(c, *d, msgs, nullptr, sigs, src, rands, false, n, seg_off,
                                         nseg, verdicts, st)
                     : pipeline_partials(c, *d, msgs, nullptr, sigs, src, rands, false, n,
                                         seg_off, nseg, 0, partials, seg_err, st);
  return ok ? GBLS_SUCCESS : FAILED;
}

int gbls_multi_verify_segments_device(const uint8_t *msgs, const gbls_p2_affine *sigs,
                                      const gbls_p1_affine *pks, const uint64_t *rands, size_t n,
                                      const uint32_t *seg_off, size_t nseg, int32_t *verdicts,
                                      void *stream) {
  PkSource src;
  src.pts = reinterpret_cast<const g1a *>(pks);
  return device_verify(msgs, reinterpret_cast<const g2a *>(sigs), src, rands, n, seg_off, nseg,
                       verdicts, nullptr, nullptr, stream);
}

int gbls_multi_verify_indexed_segments_device(const uint8_t *msgs, const gbls_p2_affine *sigs,
                                              const uint32_t *pk_idx, const uint32_t *pk_off,
                                              const uint64_t *rands, size_t n,
                                              const uint32_t *seg_off, size_t nseg,
                                              int32_t *verdicts, void *stream) {
  PkSource src;
  src.idx = pk_idx;
  src.off = pk_off;
  return device_verify(msgs, reinterpret_cast<const g2a *>(sigs), src, rands, n, seg_off, nseg,
                       verdicts, nullptr, nullptr, stream);
}

int gbls_multi_verify_partials_device(const uint8_t *msgs, const gbls_p2_affine *sigs,
                                      const gbls_p1_affine *pks, const uint64_t *rands, size_t n,
                                      const uint32_t *seg_off, size_t nseg, gbls_fp12 *partials,
                                      int32_t *seg_err, void *stream) {
  PkSource src;
  src.pts = reinterpret_cast<const g1a *>(pks);
  return device_verify(msgs, reinterpret_cast<const g2a *>(sigs), src, rands, n, seg_off, nseg,
                       nullptr, reinterpret_cast<fp12 *>(partials), seg_err, stream);
}

int gbls_multi_verify_indexed_partials_device(const uint8_t *msgs, const gbls_p2_affine *sigs,
                                              const uint32_t *pk_idx, const uint32_t *pk_off,
                                              const uint64_t *rands, size_t n,
                                              const uint32_t *seg_off, size_t nseg,
                                              gbls_fp12 *partials, int32_t *seg_err,
                                              void *stream) {
  PkSource src;
  src.idx = pk_idx;
  src.off = pk_off;
  return device_verify(msgs, reinterpret_cast<const g2a *>(sigs), src, rands, n, seg_off, nseg,
                       nullptr, reinterpret_cast<fp12 *>(partials), seg_err, stream);
}

int gbls_final_verify_partials_device(const gbls_fp12 *partials, const int32_t *seg_err,
                                      size_t nparts, size_t nseg, int32_t *verdicts, void *stream) {
  API_BEGIN
  if (nseg == 0) return GBLS_SUCCESS;
  if (nparts == 0) return fail(GBLS_ERR_ARG), FAILED;
  Device *d = current_device();
  if (!d) return fail(GBLS_ERR_ARG), FAILED;
  Lease L(*d, true, (hipStream_t)stream);
  hipStream_t st = (hipStream_t)stream;
  if (!L.ok() || !L->begin(st)) return FAILED;
  return pipeline_final(reinterpret_cast<const fp12 *>(partials), seg_err, nparts, nseg, verdicts,
                        st)
             ? GBLS_SUCCESS
             : FAILED;
}

// C3 on device-resident inputs: m sync-committee checks, 32-byte messages, keys from the
// registry (pk_idx / pk_off device arrays, pk_off[0] == 0 and non-decreasing)
int gbls_fast_aggregate_verify_indexed_device(const gbls_p2_affine *sigs, const uint8_t *msgs,
                                              const uint32_t *pk_idx, const uint32_t *pk_off,
                                              size_t m, int32_t *verdicts, void *stream) {
  API_BEGIN
  if (m == 0) return GBLS_SUCCESS;
  Device *d = current_device();
  if (!d) return fail(GBLS_ERR_ARG), FAILED;
  std::shared_lock<std::shared_mutex> rl(g.reg_mu);
  Lease L(*d, true, (hipStream_t)stream);
  Ctx &c = *L;
  hipStream_t st = (hipStream_t)stream;
  std::vector<uint32_t> ident(m + 1);
  for (size_t i = 0; i <= m; i++) ident[i] = (uint32_t)i;
  if (!L.ok() || !c.begin(st)) return FAILED;
  PkSource src;
  src.idx = pk_idx;
  src.off = pk_off;
  return pipeline_verdicts(c, *d, msgs, nullptr, reinterpret_cast<const g2a *>(sigs), src, nullptr,
                           true, m, ident.data(), m, verdicts, st)
             ? GBLS_SUCCESS
             : FAILED;
}

// ---- validator registry (f1): bulk decompress + validate on the device, replicated.
// The keys are decompressed ONCE (on the first engine device) and the 96-B affine table
// slice is copied device-to-device to every other replica (hipMemcpyPeerAsync over xGMI
// between GPUs), so 8 GPUs cost one decompression of the registry, not eight.  The new
// size is committed only when every replica holds the slice; a failure part-way truncates
// the registry to `first`, so no index can resolve to replicas that disagree (indices past
// the size are BAD_ENCODING everywhere).

// ---- validator registry (f1): bulk decompress + validate on the device, replicated.
// The keys are decompressed ONCE (on the first engine device) and the 96-B affine table
// slice is copied device-to-device to every other replica (hipMemcpyPeerAsync over xGMI
// between GPUs), so 8 GPUs cost one decompression of the registry, not eight.  Every write is
// enqueued under the exclusive registry lock on the devices' registry streams; verifications
// already in flight keep running (a growth frees the old table behind them, on the GPU), later
// ones wait for the update on the GPU, and the host wait for the statuses happens after the
// lock is released.  A failure truncates the registry to `first`, so no index can resolve to
// replicas that disagree (indices past the size are BAD_ENCODING everywhere).
int gbls_registry_set(size_t first, const uint8_t (*pks)[48], size_t n, int32_t *status) {
  fill(status, n, GBLS_BAD_ENCODING);
  API_BEGIN
  std::vector<int32_t> st0(n);
  std::vector<hipEvent_t> done;
  struct EvGuard {
    std::vector<hipEvent_t> &v;
    ~EvGuard() {
      for (hipEvent_t e : v) (void)hipEventDestroy(e);
    }
  } guard{done};
  size_t new_n = 0;  // the size this call commits
  // a failure truncates the registry to `first`; after the lock was released (the host waits)
  // only while no later registry_set has moved the size on from this call's
  auto broken = [&](std::unique_lock<std::shared_mutex> &wl) {
    const bool relock = !wl.owns_lock();
    if (relock) wl.lock();
    if (!relock || g.reg_n == new_n) g.reg_n = std::min(g.reg_n, first);
    fill(status, n, GBLS_BAD_ENCODING);
    return FAILED;
  };
  std::unique_lock<std::shared_mutex> wl(g.reg_mu);
  {
    new_n = std::max(g.reg_n, first + n);
    if (new_n > 0xffffffffull) return fail(GBLS_ERR_ARG), FAILED;
    Device &d0 = *g.devs[0];
    for (auto &dp : g.devs) {
      Device &d = *dp;
      if (!registry_streams(d) || hipSetDevice(d.hipdev) != hipSuccess) return fail(GBLS_ERR_HIP), broken(wl);
      if (&d == &d0)  // earlier replica copies read device 0's table: overwrite it after them
        for (auto &o : g.devs)
          if (o.get() != &d0 && o->reg_ev_set && hipStreamWaitEvent(d0.reg_st, o->reg_ev, 0) != hipSuccess)
            return fail(GBLS_ERR_HIP), broken(wl);
      if (first < g.reg_n && new_n * sizeof(g1a) <= d.reg.cap) {
        // loaded slots are rewritten in place: after every kernel still reading them (each
        // context's last registry read), so no reader sees a half-written key
        bool ok = true;
        d.pool.for_each([&](Ctx &c) {
          if (c.reg_read && hipStreamWaitEvent(d.reg_st, c.ev_reg, 0) != hipSuccess) ok = false;
        });
        if (!ok) return fail(GBLS_ERR_HIP), broken(wl);
      }
      if (new_n * sizeof(g1a) > d.reg.cap) {
        if (!registry_grow(d, new_n * sizeof(g1a), g.reg_n * sizeof(g1a))) return broken(wl);
      } else if (first > g.reg_n &&  // a gap past the loaded keys: never-loaded slots are zero
                 hipMemsetAsync(d.reg.as<g1a>() + g.reg_n, 0, (first - g.reg_n) * sizeof(g1a),
                                d.reg_st) != hipSuccess) {
        return fail(GBLS_ERR_HIP), broken(wl);
      }
    }
    if (n) {
      if (hipSetDevice(d0.hipdev) != hipSuccess) return fail(GBLS_ERR_HIP), broken(wl);
      Lease L(d0);  // workspaces and staging; the work itself runs on the registry stream
      Ctx &c = *L;
      hipStream_t st = d0.reg_st;
      if (!L.ok() || !c.begin(st) || !c.upload_staged(c.in0, &pks[0][0], 48 * n, st) ||
          !c.ensure(c.out1, n * sizeof(int32_t)))
        return broken(wl);
      g1a *slice0 = d0.reg.as<g1a>() + first;
      launch_g1_decompress(st, c.in0.as<uint8_t>(), (uint32_t)n, 1, slice0, c.out1.as<int32_t>());
      if (hipMemcpyAsync(st0.data(), c.out1.p, n * 4, hipMemcpyDeviceToHost, st) != hipSuccess ||
          hipEventRecord(d0.reg_tmp, st) != hipSuccess)
        return fail(GBLS_ERR_HIP), broken(wl);
      // replicas: each copies the decoded slice on its own registry stream, behind its growth
      for (size_t j = 1; j < g.devs.size(); j++) {
        Device &d = *g.devs[j];
        g1a *dst = d.reg.as<g1a>() + first;
        if (hipSetDevice(d.hipdev) != hipSuccess || hipStreamWaitEvent(d.reg_st, d0.reg_tmp, 0) != hipSuccess)
          return fail(GBLS_ERR_HIP), broken(wl);
        hipError_t e = d.hipdev == d0.hipdev
                           ? hipMemcpyAsync(dst, slice0, n * sizeof(g1a), hipMemcpyDeviceToDevice, d.reg_st)
                           : hipMemcpyPeerAsync(dst, d.hipdev, slice0, d0.hipdev, n * sizeof(g1a), d.reg_st);
        if (e != hipSuccess) return fail(GBLS_ERR_HIP), broken(wl);
      }
    }
    // later readers wait (on the GPU) for this update; this call waits on its own events
    for (auto &dp : g.devs) {
      Device &d = *dp;
      hipEvent_t e = nullptr;
      if (hipSetDevice(d.hipdev) != hipSuccess || hipEventRecord(d.reg_ev, d.reg_st) != hipSuccess ||
          hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess)
        return fail(GBLS_ERR_HIP), broken(wl);
      done.push_back(e);
      if (hipEventRecord(e, d.reg_st) != hipSuccess) return fail(GBLS_ERR_HIP), broken(wl);
      d.reg_ev_set = true;
    }
    g.reg_n = new_n;
  }
  wl.unlock();
  for (hipEvent_t e : done)
    if (hipEventSynchronize(e) != hipSuccess) return fail(GBLS_ERR_HIP), broken(wl);
  if (n) std::memcpy(status, st0.data(), n * 4);
  return GBLS_SUCCESS;
}

size_t gbls_registry_size(void) {
  std::shared_lock<std::shared_mutex> rl(g.reg_mu);
  return g.reg_n;
}

int gbls_sk_to_pk(const uint8_t (*sks)[32], size_t n, gbls_p1_affine *out) {
  API_BEGIN
  if (n == 0) return GBLS_SUCCESS;
  Lease L(pick_device());
  Ctx &c = *L;
  hipStream_t st = c.own;
  if (!L.ok() || !c.begin(st) || !c.upload_staged(c.in0, &sks[0][0], 32 * n, st) ||
      !c.ensure(c.out0, n * sizeof(g1a)))
    return FAILED;
  launch_sk_to_pk(st, c.in0.as<uint8_t>(), (uint32_t)n, c.out0.as<g1a>());
  if (hipMemcpyAsync(out, c.out0.p, n * sizeof(g1a), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return fail(GBLS_ERR_HIP), FAILED;
  return GBLS_SUCCESS;
}

// hash_to_G2 of n messages into c.out1 (affine), optional custom DST (device pointer)
static bool h2c_affine(Ctx &c, const uint8_t *msg_data, const uint32_t *msg_off, size_t n,
                       const uint8_t *dst_dev, uint32_t dst_len, hipStream_t st) {
  if (!c.upload_staged(c.in1, msg_data, msg_off[n] ? msg_off[n] : 1, st) ||
      !c.upload_staged(c.in2, msg_off, (n + 1) * 4, st) || !c.ensure(c.U, 2 * n * sizeof(fp2)) ||
      !c.ensure(c.Q, 2 * n * sizeof(g2j)) || !c.ensure(c.out1, n * sizeof(g2a)))
    return false;
  launch_h2c_field(st, c.in1.as<uint8_t>(), c.in2.as<uint32_t>(), (uint32_t)n, dst_dev, dst_len,
                   c.U.as<fp2>());
  launch_h2c_map(st, c.U.as<fp2>(), (uint32_t)(2 * n), c.Q.as<g2j>());
  launch_h2c_clear(st, c.Q.as<g2j>(), (uint32_t)n, c.out1.as<g2a>());
  return hipGetLastError() == hipSuccess || fail(GBLS_ERR_HIP);
}

int gbls_sign(const uint8_t (*sks)[32], const uint8_t *msg_data, const uint32_t *msg_off, size_t n,
              gbls_p2_affine *out) {
  API_BEGIN
  if (n == 0) return GBLS_SUCCESS;
  Lease L(pick_device());
  Ctx &c = *L;
  hipStream_t st = c.own;
  if (!L.ok() || !c.begin(st) || !c.upload_staged(c.in0, &sks[0][0], 32 * n, st) ||
      !c.ensure(c.out0, n * sizeof(g2a)))
    return FAILED;
  if (!h2c_affine(c, msg_data, msg_off, n, nullptr, 0, st)) return FAILED;
  launch_sign(st, c.in0.as<uint8_t>(), c.out1.as<g2a>(), (uint32_t)n, c.out0.as<g2a>());
  if (hipMemcpyAsync(out, c.out0.p, n * sizeof(g2a), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return fail(GBLS_ERR_HIP), FAILED;
  return GBLS_SUCCESS;
}

int gbls_hash_to_g2(const uint8_t *msg_data, const uint32_t *msg_off, size_t n, const uint8_t *dst,
                    size_t dst_len, gbls_p2_affine *out) {
  API_BEGIN
  if (n == 0) return GBLS_SUCCESS;
  // dst == NULL (with dst_len 0): the signature scheme's own DST (BLS_SIG_..._POP_)
  if (dst_len > 255 || !msg_data || !msg_off || !out || (!dst && dst_len)) return fail(GBLS_ERR_ARG), FAILED;
  Lease L(pick_device());
  Ctx &c = *L;
  hipStream_t st = c.own;
  if (!L.ok() || !c.begin(st) || (dst && !c.upload_staged(c.in3, dst, dst_len ? dst_len : 1, st)))
    return FAILED;
  if (!h2c_affine(c, msg_data, msg_off, n, dst ? c.in3.as<uint8_t>() : nullptr, (uint32_t)dst_len, st))
    return FAILED;
  if (hipMemcpyAsync(out, c.out1.p, n * sizeof(g2a), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return fail(GBLS_ERR_HIP), FAILED;
  return GBLS_SUCCESS;
}

double gbls_measure_mad64_peak(void) {
  if (!ensure_ready()) return 0.0;
  Lease L(pick_device());
  if (!L.ok()) return 0.0;
  hipStream_t st = L->own;
  L->begin(st);
  Buf sink;
  if (!sink.ensure(64)) return 0.0;
  const unsigned blocks = 256 * 8, threads = 256;
  const uint32_t iters = 4096;
  launch_mad_peak(st, blocks, sink.as<uint64_t>(), 16, 1);  // warm
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a, st);
  launch_mad_peak(st, blocks, sink.as<uint64_t>(), iters, 7);
  (void)hipEventRecord(b, st);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  (void)hipFree(sink.p);
  double mads = (double)blocks * threads * iters * 16.0;
  return ms > 0 ? mads / (ms * 1e-3) : 0.0;
}

int gbls_profile(int enable) {
  if (enable) {  // a stock of timing events, created before the profiled calls
    std::lock_guard<std::mutex> lk(prof.mu);
    while (prof.free_ev.size() < 2048) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) break;
      prof.free_ev.push_back(e);
    }
  }
  bool prev = prof.on.exchange(enable != 0);
  return prev ? 1 : 0;
}

int gbls_profile_read(double *ms, uint32_t *calls, int max_stages) {
  std::lock_guard<std::mutex> lk(prof.mu);
  for (auto &r : prof.pending) {
    float t = 0;
    if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&t, r.a, r.b) == hipSuccess) {
      prof.ms[r.stage] += t;
      prof.calls[r.stage] += 1;
    }
    prof.free_ev.push_back(r.a);
    prof.free_ev.push_back(r.b);
  }
  prof.pending.clear();
  int n = max_stages < S_COUNT ? max_stages : S_COUNT;
  for (int i = 0; i < n; i++) {
    if (ms) ms[i] = prof.ms[i];
    if (calls) calls[i] = prof.calls[i];
  }
  return S_COUNT;
}

void gbls_profile_reset(void) {
  std::lock_guard<std::mutex> lk(prof.mu);
  for (int i = 0; i < S_COUNT; i++) {
    prof.ms[i] = 0;
    prof.calls[i] = 0;
  }
}

const char *gbls_stage_name(int stage) {
  return (stage >= 0 && stage < S_COUNT) ? kStageNames[stage] : "";
}

}  // extern "C"
