// C ABI of the MI355X BLS12-381 engine: host-side orchestration of the gfx950 kernels
// (k_*.hip).  Entry points, their reference counterparts and semantics are documented
// in include/grandine_bls_gpu.h.
//
// Concurrency model: a process-wide engine (one HIP device, one stream, grow-only
// device workspaces) guarded by a mutex; callers from many threads are serialised
// onto the stream.  Every failure is fail-closed (VERIFY_FAIL + gbls_last_error).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/grandine_bls_gpu.h"
#include "gbls_common.h"

using namespace gbls;

static_assert(sizeof(g1a) == sizeof(gbls_p1_affine), "p1 layout");
static_assert(sizeof(g2a) == sizeof(gbls_p2_affine), "p2 layout");
static_assert(sizeof(fp12) == sizeof(gbls_fp12), "fp12 layout");

namespace {

thread_local int t_last_error = GBLS_ERR_NONE;

struct Buf {
  void *p = nullptr;
  size_t cap = 0;
  bool ensure(size_t bytes) {
    if (bytes <= cap) return true;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = bytes < 4096 ? 4096 : bytes + bytes / 4;
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
  S_ML_REDUCE, S_ML_HORNER, S_FINAL, S_COUNT
};
const char *kStageNames[S_COUNT] = {"k_h2c_field", "k_h2c_map",   "k_h2c_clear", "k_mv_g1mul",
                                    "k_mv_g2mul",  "k_g2sum",      "k_lines",     "k_lines_S",
                                    "k_ml_leaf",   "k_ml_reduce",  "k_ml_horner", "k_final_verdict"};

struct Engine {
  std::mutex mu;
  bool ready = false;
  int device = -1;
  hipStream_t stream = nullptr;
  hipStream_t side1 = nullptr, side2 = nullptr;  // fork/join streams of the pipeline
  hipEvent_t ev_fork = nullptr, ev_side1 = nullptr, ev_side2 = nullptr;
  // workspaces
  Buf in0, in1, in2, in3, in4, in5, in6, U, Q, H, P, R, gpart, lines, V0, V1, tab, segoff, part,
      err, out0, out1;
  // profiling
  bool prof = false;
  struct Rec {
    int stage;
    hipEvent_t a, b;
  };
  std::vector<Rec> pending;
  double ms[S_COUNT] = {0};
  uint32_t calls[S_COUNT] = {0};
} g;

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

struct StageTimer {  // RAII: events around one stage's launches when profiling
  hipEvent_t a = nullptr, b = nullptr;
  hipStream_t st;
  int stage;
  StageTimer(int s, hipStream_t stream) : st(stream), stage(s) {
    if (!g.prof) return;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) return;
    (void)hipEventRecord(a, st);
  }
  ~StageTimer() {
    if (!g.prof || !a || !b) return;
    (void)hipEventRecord(b, st);
    g.pending.push_back({stage, a, b});
  }
};

bool engine_init_locked(uint32_t device_mask) {
  if (g.ready) return true;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return fail(GBLS_ERR_NO_DEVICE);
  int dev = 0;
  if (device_mask) {
    while (dev < 32 && !((device_mask >> dev) & 1)) dev++;
  } else {
    (void)hipGetDevice(&dev);
  }
  if (dev >= ndev) return fail(GBLS_ERR_NO_DEVICE);
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return fail(GBLS_ERR_NO_DEVICE);
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return fail(GBLS_ERR_NO_DEVICE);
  HIPCHK(hipSetDevice(dev));
  HIPCHK(hipStreamCreateWithFlags(&g.stream, hipStreamNonBlocking));
  HIPCHK(hipStreamCreateWithFlags(&g.side1, hipStreamNonBlocking));
  HIPCHK(hipStreamCreateWithFlags(&g.side2, hipStreamNonBlocking));
  HIPCHK(hipEventCreateWithFlags(&g.ev_fork, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&g.ev_side1, hipEventDisableTiming));
  HIPCHK(hipEventCreateWithFlags(&g.ev_side2, hipEventDisableTiming));
  g.device = dev;
  g.ready = true;
  return true;
}

bool ensure_ready() {
  if (g.ready) {
    (void)hipSetDevice(g.device);
    return true;
  }
  return engine_init_locked(0);
}

template <class T>
bool upload(Buf &b, const T *host, size_t count, hipStream_t st) {
  if (!b.ensure(count * sizeof(T) + 16)) return fail(GBLS_ERR_HIP);
  if (count) HIPCHK(hipMemcpyAsync(b.p, host, count * sizeof(T), hipMemcpyHostToDevice, st));
  return true;
}
template <class T>
bool upload(Buf &b, const T *host, size_t count) {
  return upload(b, host, count, g.stream);
}
template <class T>
bool download(T *host, const Buf &b, size_t count) {
  if (count) HIPCHK(hipMemcpyAsync(host, b.p, count * sizeof(T), hipMemcpyDeviceToHost, g.stream));
  return true;
}
bool sync() {
  HIPCHK(hipStreamSynchronize(g.stream));
  HIPCHK(hipGetLastError());
  return true;
}

// ----- the verification pipeline on device pointers.
// Sets [0, n) grouped in segments by seg_off (HOST array, nseg + 1 entries); per segment
// a Miller partial (no final exponentiation) and an error flag.  rands == nullptr
// means r_i = 1 (single checks); pre[i] != 0 marks a set that failed a pre-check.
bool pipeline_partials(const uint8_t *msgs, const uint32_t *msg_off, const g2a *sigs,
                       const g1a *pks, const uint64_t *rands, const int32_t *pre, size_t n,
                       const uint32_t *seg_off, size_t nseg, fp12 *partials, int32_t *seg_err,
                       hipStream_t st) {
  const size_t np = n + nseg;
  // ---- host tables, one upload: [couples][g2 chunks][seg_chunk][reduction levels]
  std::vector<uint32_t> tab;
  std::vector<uint32_t> cnt(nseg);
  for (size_t s = 0; s < nseg; s++) {  // level-0 couples of each segment's pair list
    std::vector<uint32_t> list;
    for (uint32_t i = seg_off[s]; i < seg_off[s + 1]; i++) list.push_back(i);
    list.push_back((uint32_t)(n + s));
    for (size_t j = 0; j < list.size(); j += 2) {
      tab.push_back(list[j]);
      tab.push_back(j + 1 < list.size() ? list[j + 1] : NONE);
      cnt[s]++;
    }
  }
  const size_t ncouple = tab.size() / 2;
  const size_t chunk_off = tab.size();
  const uint32_t CH = 4 * WGR;  // sets per level-1 G2-sum workgroup
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
  struct Level {
    size_t tab_off, nin, nout;
  };
  std::vector<Level> levels;
  size_t cur_n = ncouple;
  while (*std::max_element(cnt.begin(), cnt.end()) > 1) {
    Level L{tab.size(), cur_n, 0};
    size_t in_base = 0;
    std::vector<uint32_t> next(nseg);
    for (size_t s = 0; s < nseg; s++) {
      uint32_t c = cnt[s];
      for (uint32_t q = 0; q < c; q += 4) {
        tab.push_back((uint32_t)(in_base + q));
        tab.push_back(std::min<uint32_t>(4, c - q));
        next[s]++;
      }
      in_base += c;
    }
    L.nout = (tab.size() - L.tab_off) / 2;
    levels.push_back(L);
    cnt = next;
    cur_n = L.nout;
  }
  // ---- workspaces
  const size_t line_words = (size_t)np * ML_EVENTS * 72;
  size_t v1_n = 1, v0_n = ncouple;
  for (size_t l = 0; l < levels.size(); l++)
    (l & 1 ? v0_n : v1_n) = std::max(l & 1 ? v0_n : v1_n, levels[l].nout);
  if (!g.U.ensure(2 * n * sizeof(fp2)) || !g.Q.ensure(2 * n * sizeof(g2j)) ||
      !g.H.ensure(np * sizeof(g2a)) || !g.P.ensure(np * sizeof(g1a)) ||
      !g.R.ensure(2 * n * sizeof(g2j) + 16) || !g.gpart.ensure(nchunks * (sizeof(g2j) + 4)) ||
      !g.lines.ensure(line_words * 4) || !g.V0.ensure(ML_EVENTS * v0_n * sizeof(fp12)) ||
      !g.V1.ensure(ML_EVENTS * v1_n * sizeof(fp12)) || !g.segoff.ensure((nseg + 1) * 4))
    return fail(GBLS_ERR_HIP);
  if (!upload(g.tab, tab.data(), tab.size(), st)) return false;
  HIPCHK(hipMemcpyAsync(g.segoff.p, seg_off, (nseg + 1) * 4, hipMemcpyHostToDevice, st));
  const uint32_t N = (uint32_t)n, NP = (uint32_t)np, NS = (uint32_t)nseg;
  const uint32_t *T = g.tab.as<uint32_t>();
  g2j *gpart = g.gpart.as<g2j>();
  int32_t *gpart_err = reinterpret_cast<int32_t *>(gpart + nchunks);
  // ---- fork: side stream 1 = G1 scalar products, side stream 2 = G2 sum + its lines,
  // main stream = hash_to_G2 + the sets' lines; join before the Miller tree.
  HIPCHK(hipEventRecord(g.ev_fork, st));
  HIPCHK(hipStreamWaitEvent(g.side1, g.ev_fork, 0));
  HIPCHK(hipStreamWaitEvent(g.side2, g.ev_fork, 0));
  {
    StageTimer t(S_G1MUL, g.side1);
    launch_mv_g1mul(g.side1, pks, rands, N, g.P.as<g1a>());
  }
  {
    StageTimer t(S_G2MUL, g.side2);
    launch_mv_g2mul(g.side2, sigs, rands, N, g.R.as<g2j>());
  }
  {
    StageTimer t(S_G2SUM, g.side2);
    launch_g2sum(g.side2, g.R.as<g2j>(), T + chunk_off, (uint32_t)nchunks, T + segchunk_off,
                 g.segoff.as<uint32_t>(), NS, N, pks, pre, gpart, gpart_err, g.P.as<g1a>(),
                 g.H.as<g2a>(), seg_err);
  }
  {
    StageTimer t(S_LINES_S, g.side2);
    launch_lines(g.side2, g.H.as<g2a>(), N, NS, NP, g.lines.as<uint32_t>());
  }
  {
    StageTimer t(S_H2C_FIELD, st);
    launch_h2c_field(st, msgs, msg_off, N, nullptr, 0, g.U.as<fp2>());
  }
  {
    StageTimer t(S_H2C_MAP, st);
    launch_h2c_map(st, g.U.as<fp2>(), 2 * N, g.Q.as<g2j>());
  }
  {
    StageTimer t(S_H2C_CLEAR, st);
    launch_h2c_clear(st, g.Q.as<g2j>(), N, g.H.as<g2a>());
  }
  {
    StageTimer t(S_LINES, st);
    launch_lines(st, g.H.as<g2a>(), 0, N, NP, g.lines.as<uint32_t>());
  }
  HIPCHK(hipEventRecord(g.ev_side1, g.side1));
  HIPCHK(hipEventRecord(g.ev_side2, g.side2));
  HIPCHK(hipStreamWaitEvent(st, g.ev_side1, 0));
  HIPCHK(hipStreamWaitEvent(st, g.ev_side2, 0));
  {
    StageTimer t(S_ML_LEAF, st);
    launch_ml_leaf(st, g.lines.as<uint32_t>(), NP, g.P.as<g1a>(), T, (uint32_t)ncouple,
                   g.V0.as<fp12>());
  }
  fp12 *cur = g.V0.as<fp12>(), *other = g.V1.as<fp12>();
  {
    StageTimer t(S_ML_REDUCE, st);
    for (const Level &L : levels) {
      launch_ml_reduce(st, cur, (uint32_t)L.nin, T + L.tab_off, (uint32_t)L.nout, other);
      std::swap(cur, other);
    }
  }
  {
    StageTimer t(S_ML_HORNER, st);
    launch_ml_horner(st, cur, NS, partials);
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

bool pipeline_verdicts(const uint8_t *msgs, const uint32_t *msg_off, const g2a *sigs,
                       const g1a *pks, const uint64_t *rands, const int32_t *pre, size_t n,
                       const uint32_t *seg_off, size_t nseg, int32_t *verdicts, hipStream_t st) {
  if (!g.part.ensure(nseg * sizeof(fp12)) || !g.err.ensure(nseg * sizeof(int32_t)))
    return fail(GBLS_ERR_HIP);
  return pipeline_partials(msgs, msg_off, sigs, pks, rands, pre, n, seg_off, nseg,
                           g.part.as<fp12>(), g.err.as<int32_t>(), st) &&
         pipeline_final(g.part.as<fp12>(), g.err.as<int32_t>(), 1, nseg, verdicts, st);
}

std::vector<uint32_t> identity_offsets(size_t m) {
  std::vector<uint32_t> v(m + 1);
  for (size_t i = 0; i <= m; i++) v[i] = (uint32_t)i;
  return v;
}

}  // namespace

#define API_LOCK                             \
  std::lock_guard<std::mutex> lock__(g.mu);  \
  t_last_error = GBLS_ERR_NONE;              \
  if (!ensure_ready()) return -1;

extern "C" {

int gbls_init(uint32_t device_mask, uint32_t flags) {
  (void)flags;
  std::lock_guard<std::mutex> lock(g.mu);
  t_last_error = GBLS_ERR_NONE;
  return engine_init_locked(device_mask) ? GBLS_SUCCESS : -1;
}

int gbls_last_error(void) { return t_last_error; }
const char *gbls_version(void) { return "grandine-bls-mi355x 0.2 (gfx950)"; }

int gbls_g1_decompress(const uint8_t (*in)[48], size_t n, int validate, gbls_p1_affine *out,
                       int32_t *status) {
  API_LOCK
  if (n == 0) return GBLS_SUCCESS;
  if (!upload(g.in0, &in[0][0], 48 * n) || !g.out0.ensure(n * sizeof(g1a)) ||
      !g.out1.ensure(n * sizeof(int32_t)))
    return -1;
  launch_g1_decompress(g.stream, g.in0.as<uint8_t>(), (uint32_t)n, validate, g.out0.as<g1a>(),
                       g.out1.as<int32_t>());
  if (!download(reinterpret_cast<g1a *>(out), g.out0, n) || !download(status, g.out1, n) || !sync())
    return -1;
  return GBLS_SUCCESS;
}

int gbls_g2_decompress(const uint8_t (*in)[96], size_t n, gbls_p2_affine *out, int32_t *status) {
  API_LOCK
  if (n == 0) return GBLS_SUCCESS;
  if (!upload(g.in0, &in[0][0], 96 * n) || !g.out0.ensure(n * sizeof(g2a)) ||
      !g.out1.ensure(n * sizeof(int32_t)))
    return -1;
  launch_g2_decompress(g.stream, g.in0.as<uint8_t>(), (uint32_t)n, g.out0.as<g2a>(),
                       g.out1.as<int32_t>());
  if (!download(reinterpret_cast<g2a *>(out), g.out0, n) || !download(status, g.out1, n) || !sync())
    return -1;
  return GBLS_SUCCESS;
}

int gbls_g2_validate(const gbls_p2_affine *in, size_t n, int32_t *status) {
  API_LOCK
  if (n == 0) return GBLS_SUCCESS;
  if (!upload(g.in0, reinterpret_cast<const g2a *>(in), n) || !g.out1.ensure(n * sizeof(int32_t)))
    return -1;
  launch_g2_check(g.stream, g.in0.as<g2a>(), (uint32_t)n, g.out1.as<int32_t>(), 0);
  if (!download(status, g.out1, n) || !sync()) return -1;
  return GBLS_SUCCESS;
}

int gbls_g1_compress(const gbls_p1_affine *in, size_t n, uint8_t (*out)[48]) {
  API_LOCK
  if (n == 0) return GBLS_SUCCESS;
  if (!upload(g.in0, reinterpret_cast<const g1a *>(in), n) || !g.out0.ensure(48 * n)) return -1;
  launch_g1_compress(g.stream, g.in0.as<g1a>(), (uint32_t)n, g.out0.as<uint8_t>());
  if (!download(&out[0][0], g.out0, 48 * n) || !sync()) return -1;
  return GBLS_SUCCESS;
}

int gbls_g2_compress(const gbls_p2_affine *in, size_t n, uint8_t (*out)[96]) {
  API_LOCK
  if (n == 0) return GBLS_SUCCESS;
  if (!upload(g.in0, reinterpret_cast<const g2a *>(in), n) || !g.out0.ensure(96 * n)) return -1;
  launch_g2_compress(g.stream, g.in0.as<g2a>(), (uint32_t)n, g.out0.as<uint8_t>());
  if (!download(&out[0][0], g.out0, 96 * n) || !sync()) return -1;
  return GBLS_SUCCESS;
}

int gbls_g1_aggregate_segments(const gbls_p1_affine *pks, const uint32_t *seg_offsets, size_t nseg,
                               gbls_p1_affine *out, int32_t *status) {
  API_LOCK
  if (nseg == 0) return GBLS_SUCCESS;
  size_t n = seg_offsets[nseg];
  if (!upload(g.in0, reinterpret_cast<const g1a *>(pks), n) ||
      !upload(g.in1, seg_offsets, nseg + 1) || !g.out0.ensure(nseg * sizeof(g1a)) ||
      !g.out1.ensure(nseg * sizeof(int32_t)))
    return -1;
  launch_g1_aggregate_seg(g.stream, g.in0.as<g1a>(), g.in1.as<uint32_t>(), (uint32_t)nseg,
                          g.out0.as<g1a>(), g.out1.as<int32_t>());
  if (!download(reinterpret_cast<g1a *>(out), g.out0, nseg) || !download(status, g.out1, nseg) ||
      !sync())
    return -1;
  return GBLS_SUCCESS;
}

int gbls_g1_aggregate(const gbls_p1_affine *pks, size_t n, gbls_p1_affine *out) {
  uint32_t off[2] = {0, (uint32_t)n};
  int32_t st = GBLS_SUCCESS;
  if (n == 0) {
    std::memset(out, 0, sizeof(*out));
    return GBLS_AGGR_TYPE_MISMATCH;
  }
  int rc = gbls_g1_aggregate_segments(pks, off, 1, out, &st);
  return rc != GBLS_SUCCESS ? rc : st;
}

int gbls_g2_aggregate(const gbls_p2_affine *sigs, size_t n, gbls_p2_affine *out) {
  API_LOCK
  uint32_t off[2] = {0, (uint32_t)n};
  if (!upload(g.in0, reinterpret_cast<const g2a *>(sigs), n) || !upload(g.in1, off, 2) ||
      !g.out0.ensure(sizeof(g2a)))
    return -1;
  launch_g2_aggregate_seg(g.stream, g.in0.as<g2a>(), g.in1.as<uint32_t>(), 1, g.out0.as<g2a>());
  if (!download(reinterpret_cast<g2a *>(out), g.out0, 1) || !sync()) return -1;
  return GBLS_SUCCESS;
}

// m independent checks e(pk_i, H(m_i)) == e(g1, sig_i), each its own segment
// (r_i = 1), with the signature subgroup check folded into the pre-flags.
int gbls_aggregate_verify_batch(const gbls_p2_affine *sigs, const uint8_t *msg_data,
                                const uint32_t *msg_off, const gbls_p1_affine *pks, size_t m,
                                int32_t *verdicts) {
  API_LOCK
  if (m == 0) return GBLS_SUCCESS;
  for (size_t i = 0; i < m; i++) verdicts[i] = GBLS_VERIFY_FAIL;
  std::vector<uint32_t> ident = identity_offsets(m);
  if (!upload(g.in0, reinterpret_cast<const g2a *>(sigs), m) ||
      !upload(g.in1, msg_data, msg_off[m] ? msg_off[m] : 1) || !upload(g.in2, msg_off, m + 1) ||
      !upload(g.in3, reinterpret_cast<const g1a *>(pks), m) || !g.in5.ensure(m * sizeof(int32_t)) ||
      !g.out1.ensure(m * sizeof(int32_t)))
    return -1;
  if (hipMemsetAsync(g.in5.p, 0, m * sizeof(int32_t), g.stream) != hipSuccess)
    return (t_last_error = GBLS_ERR_HIP), -1;
  launch_g2_check(g.stream, g.in0.as<g2a>(), (uint32_t)m, g.in5.as<int32_t>(), 1);
  if (!pipeline_verdicts(g.in1.as<uint8_t>(), g.in2.as<uint32_t>(), g.in0.as<g2a>(), g.in3.as<g1a>(),
                         nullptr, g.in5.as<int32_t>(), m, ident.data(), m, g.out1.as<int32_t>(),
                         g.stream))
    return -1;
  if (!download(verdicts, g.out1, m) || !sync()) {
    for (size_t i = 0; i < m; i++) verdicts[i] = GBLS_VERIFY_FAIL;
    return -1;
  }
  return GBLS_SUCCESS;
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
  API_LOCK
  if (m == 0) return GBLS_SUCCESS;
  for (size_t i = 0; i < m; i++) verdicts[i] = GBLS_VERIFY_FAIL;
  size_t npk = seg_off[m];
  std::vector<uint32_t> ident = identity_offsets(m);
  if (!upload(g.in0, reinterpret_cast<const g2a *>(sigs), m) ||
      !upload(g.in1, msg_data, msg_off[m] ? msg_off[m] : 1) || !upload(g.in2, msg_off, m + 1) ||
      !upload(g.in4, reinterpret_cast<const g1a *>(pks), npk ? npk : 1) ||
      !upload(g.in5, seg_off, m + 1) || !g.in3.ensure(m * sizeof(g1a)) ||
      !g.out0.ensure(m * sizeof(int32_t)) || !g.out1.ensure(m * sizeof(int32_t)))
    return -1;
  // aggregate pks per message (status AGGR_TYPE_MISMATCH for empty -> pre-flag)
  launch_g1_aggregate_seg(g.stream, g.in4.as<g1a>(), g.in5.as<uint32_t>(), (uint32_t)m,
                          g.in3.as<g1a>(), g.out0.as<int32_t>());
  launch_g2_check(g.stream, g.in0.as<g2a>(), (uint32_t)m, g.out0.as<int32_t>(), 1);
  if (!pipeline_verdicts(g.in1.as<uint8_t>(), g.in2.as<uint32_t>(), g.in0.as<g2a>(), g.in3.as<g1a>(),
                         nullptr, g.out0.as<int32_t>(), m, ident.data(), m, g.out1.as<int32_t>(),
                         g.stream))
    return -1;
  if (!download(verdicts, g.out1, m) || !sync()) {
    for (size_t i = 0; i < m; i++) verdicts[i] = GBLS_VERIFY_FAIL;
    return -1;
  }
  return GBLS_SUCCESS;
}

int gbls_fast_aggregate_verify(const gbls_p2_affine *sig, const uint8_t *msg, size_t msg_len,
                               const gbls_p1_affine *pks, size_t n) {
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
  API_LOCK
  for (size_t s = 0; s < nseg; s++) verdicts[s] = GBLS_VERIFY_FAIL;
  if (nseg == 0) return GBLS_SUCCESS;
  if (seg_off[nseg] != n) return (t_last_error = GBLS_ERR_ARG), -1;
  if (!upload(g.in0, &msgs[0][0], 32 * n) || !upload(g.in1, reinterpret_cast<const g2a *>(sigs), n) ||
      !upload(g.in2, reinterpret_cast<const g1a *>(pks), n) || !upload(g.in3, rands, n) ||
      !g.out1.ensure(nseg * sizeof(int32_t)))
    return -1;
  if (!pipeline_verdicts(g.in0.as<uint8_t>(), nullptr, g.in1.as<g2a>(), g.in2.as<g1a>(),
                         g.in3.as<uint64_t>(), nullptr, n, seg_off, nseg, g.out1.as<int32_t>(),
                         g.stream))
    return -1;
  if (!download(verdicts, g.out1, nseg) || !sync()) {
    for (size_t s = 0; s < nseg; s++) verdicts[s] = GBLS_VERIFY_FAIL;
    return -1;
  }
  return GBLS_SUCCESS;
}

int gbls_multi_verify(const uint8_t (*msgs)[32], const gbls_p2_affine *sigs,
                      const gbls_p1_affine *pks, const uint64_t *rands, size_t n) {
  if (n == 0) return GBLS_VERIFY_FAIL;
  for (size_t i = 0; i < n; i++)
    if (rands[i] == 0) return GBLS_VERIFY_FAIL;  // NonZeroU64 contract
  uint32_t off[2] = {0, (uint32_t)n};
  int32_t v = GBLS_VERIFY_FAIL;
  if (gbls_multi_verify_segments(msgs, sigs, pks, rands, n, off, 1, &v) != GBLS_SUCCESS)
    return GBLS_VERIFY_FAIL;
  return v;
}

int gbls_multi_verify_segments_device(const uint8_t *msgs, const gbls_p2_affine *sigs,
                                      const gbls_p1_affine *pks, const uint64_t *rands, size_t n,
                                      const uint32_t *seg_off, size_t nseg, int32_t *verdicts,
                                      void *stream) {
  API_LOCK
  if (nseg == 0) return GBLS_SUCCESS;
  if (seg_off[nseg] != n) return (t_last_error = GBLS_ERR_ARG), -1;
  hipStream_t st = stream ? (hipStream_t)stream : g.stream;
  return pipeline_verdicts(msgs, nullptr, reinterpret_cast<const g2a *>(sigs),
                           reinterpret_cast<const g1a *>(pks), rands, nullptr, n, seg_off, nseg,
                           verdicts, st)
             ? GBLS_SUCCESS
             : -1;
}

int gbls_multi_verify_partials_device(const uint8_t *msgs, const gbls_p2_affine *sigs,
                                      const gbls_p1_affine *pks, const uint64_t *rands, size_t n,
                                      const uint32_t *seg_off, size_t nseg, gbls_fp12 *partials,
                                      int32_t *seg_err, void *stream) {
  API_LOCK
  if (nseg == 0) return GBLS_SUCCESS;
  if (seg_off[nseg] != n) return (t_last_error = GBLS_ERR_ARG), -1;
  hipStream_t st = stream ? (hipStream_t)stream : g.stream;
  return pipeline_partials(msgs, nullptr, reinterpret_cast<const g2a *>(sigs),
                           reinterpret_cast<const g1a *>(pks), rands, nullptr, n, seg_off, nseg,
                           reinterpret_cast<fp12 *>(partials), seg_err, st)
             ? GBLS_SUCCESS
             : -1;
}

int gbls_final_verify_partials_device(const gbls_fp12 *partials, const int32_t *seg_err,
                                      size_t nparts, size_t nseg, int32_t *verdicts, void *stream) {
  API_LOCK
  if (nseg == 0) return GBLS_SUCCESS;
  hipStream_t st = stream ? (hipStream_t)stream : g.stream;
  return pipeline_final(reinterpret_cast<const fp12 *>(partials), seg_err, nparts, nseg, verdicts,
                        st)
             ? GBLS_SUCCESS
             : -1;
}

int gbls_sk_to_pk(const uint8_t (*sks)[32], size_t n, gbls_p1_affine *out) {
  API_LOCK
  if (n == 0) return GBLS_SUCCESS;
  if (!upload(g.in0, &sks[0][0], 32 * n) || !g.out0.ensure(n * sizeof(g1a))) return -1;
  launch_sk_to_pk(g.stream, g.in0.as<uint8_t>(), (uint32_t)n, g.out0.as<g1a>());
  if (!download(reinterpret_cast<g1a *>(out), g.out0, n) || !sync()) return -1;
  return GBLS_SUCCESS;
}

// hash_to_G2 of n messages into g.out1 (affine), optional custom DST (device pointer)
static bool h2c_affine_locked(const uint8_t *msg_data, const uint32_t *msg_off, size_t n,
                              const uint8_t *dst_dev, uint32_t dst_len) {
  if (!upload(g.in1, msg_data, msg_off[n] ? msg_off[n] : 1) || !upload(g.in2, msg_off, n + 1) ||
      !g.U.ensure(2 * n * sizeof(fp2)) || !g.Q.ensure(2 * n * sizeof(g2j)) ||
      !g.out1.ensure(n * sizeof(g2a)))
    return false;
  launch_h2c_field(g.stream, g.in1.as<uint8_t>(), g.in2.as<uint32_t>(), (uint32_t)n, dst_dev, dst_len,
                   g.U.as<fp2>());
  launch_h2c_map(g.stream, g.U.as<fp2>(), (uint32_t)(2 * n), g.Q.as<g2j>());
  launch_h2c_clear(g.stream, g.Q.as<g2j>(), (uint32_t)n, g.out1.as<g2a>());
  return hipGetLastError() == hipSuccess || fail(GBLS_ERR_HIP);
}

int gbls_sign(const uint8_t (*sks)[32], const uint8_t *msg_data, const uint32_t *msg_off, size_t n,
              gbls_p2_affine *out) {
  API_LOCK
  if (n == 0) return GBLS_SUCCESS;
  if (!upload(g.in0, &sks[0][0], 32 * n) || !g.out0.ensure(n * sizeof(g2a))) return -1;
  if (!h2c_affine_locked(msg_data, msg_off, n, nullptr, 0)) return -1;
  launch_sign(g.stream, g.in0.as<uint8_t>(), g.out1.as<g2a>(), (uint32_t)n, g.out0.as<g2a>());
  if (!download(reinterpret_cast<g2a *>(out), g.out0, n) || !sync()) return -1;
  return GBLS_SUCCESS;
}

int gbls_hash_to_g2(const uint8_t *msg_data, const uint32_t *msg_off, size_t n, const uint8_t *dst,
                    size_t dst_len, gbls_p2_affine *out) {
  API_LOCK
  if (n == 0) return GBLS_SUCCESS;
  if (dst_len > 255) return (t_last_error = GBLS_ERR_ARG), -1;
  if (!upload(g.in3, dst, dst_len ? dst_len : 1)) return -1;
  if (!h2c_affine_locked(msg_data, msg_off, n, g.in3.as<uint8_t>(), (uint32_t)dst_len)) return -1;
  if (!download(reinterpret_cast<g2a *>(out), g.out1, n) || !sync()) return -1;
  return GBLS_SUCCESS;
}

double gbls_measure_mad64_peak(void) {
  std::lock_guard<std::mutex> lock(g.mu);
  if (!ensure_ready()) return 0.0;
  Buf sink;
  if (!sink.ensure(64)) return 0.0;
  const unsigned blocks = 256 * 8, threads = 256;
  const uint32_t iters = 4096;
  launch_mad_peak(g.stream, blocks, sink.as<uint64_t>(), 16, 1);  // warm
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a, g.stream);
  launch_mad_peak(g.stream, blocks, sink.as<uint64_t>(), iters, 7);
  (void)hipEventRecord(b, g.stream);
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
  std::lock_guard<std::mutex> lock(g.mu);
  int prev = g.prof ? 1 : 0;
  g.prof = enable != 0;
  return prev;
}

int gbls_profile_read(double *ms, uint32_t *calls, int max_stages) {
  std::lock_guard<std::mutex> lock(g.mu);
  for (auto &r : g.pending) {
    float t = 0;
    if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&t, r.a, r.b) == hipSuccess) {
      g.ms[r.stage] += t;
      g.calls[r.stage] += 1;
    }
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  g.pending.clear();
  int n = max_stages < S_COUNT ? max_stages : S_COUNT;
  for (int i = 0; i < n; i++) {
    if (ms) ms[i] = g.ms[i];
    if (calls) calls[i] = g.calls[i];
  }
  return S_COUNT;
}

void gbls_profile_reset(void) {
  std::lock_guard<std::mutex> lock(g.mu);
  for (int i = 0; i < S_COUNT; i++) {
    g.ms[i] = 0;
    g.calls[i] = 0;
  }
}

const char *gbls_stage_name(int stage) {
  return (stage >= 0 && stage < S_COUNT) ? kStageNames[stage] : "";
}

}  // extern "C"
