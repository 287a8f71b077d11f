// C ABI of the MI355X BLS12-381 engine: host-side orchestration of the gfx950
// kernels in gbls_kernels.h.  Entry points, their reference counterparts and
// semantics are documented in include/grandine_bls_gpu.h.
//
// Concurrency model: a process-wide engine (one HIP device, one stream, grow-only
// device workspaces) guarded by a mutex; callers from many threads are serialised
// onto the stream.  Every failure is fail-closed (VERIFY_FAIL + gbls_last_error).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/grandine_bls_gpu.h"
#include "gbls_kernels.h"

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

struct Engine {
  std::mutex mu;
  bool ready = false;
  int device = -1;
  hipStream_t stream = nullptr;
  // workspaces
  Buf in0, in1, in2, in3, in4, in5, H, P, R, S, f, F, part, bad, err, out0, out1;
} g;

bool fail(int code) {
  t_last_error = code;
  return false;
}

#define HIPCHK(x)                     \
  do {                                \
    if ((x) != hipSuccess) {          \
      t_last_error = GBLS_ERR_HIP;    \
      return false;                   \
    }                                 \
  } while (0)

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

inline unsigned nblk(size_t n) { return (unsigned)((n + WG - 1) / WG); }

template <class T>
bool upload(Buf &b, const T *host, size_t count) {
  if (!b.ensure(count * sizeof(T) + 16)) return fail(GBLS_ERR_HIP);
  if (count) HIPCHK(hipMemcpyAsync(b.p, host, count * sizeof(T), hipMemcpyHostToDevice, g.stream));
  return true;
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

// ----- multi_verify pipeline on device pointers (sets n, segments nseg)
bool mv_partials(const uint8_t *msgs, const g2a *sigs, const g1a *pks, const uint64_t *rands,
                 size_t n, const uint32_t *seg_off, size_t nseg, fp12 *partials, int32_t *seg_err,
                 hipStream_t st) {
  if (!g.H.ensure(n * sizeof(g2a)) || !g.P.ensure(n * sizeof(g1a)) ||
      !g.R.ensure(n * sizeof(g2j)) || !g.f.ensure(n * sizeof(fp12)) ||
      !g.bad.ensure(n * sizeof(int32_t)) || !g.S.ensure(nseg * sizeof(g2j)) ||
      !g.F.ensure(nseg * sizeof(fp12)))
    return fail(GBLS_ERR_HIP);
  unsigned b = nblk(n);
  k_hash_to_g2<<<b, WG, 0, st>>>(msgs, nullptr, (uint32_t)n, nullptr, 0, g.H.as<g2a>());
  k_mv_g1mul<<<b, WG, 0, st>>>(pks, rands, (uint32_t)n, g.P.as<g1a>(), g.bad.as<int32_t>());
  k_mv_g2mul<<<b, WG, 0, st>>>(sigs, rands, (uint32_t)n, g.R.as<g2j>());
  k_seg_g2_sum<<<(unsigned)nseg, WG, 0, st>>>(g.R.as<g2j>(), seg_off, (uint32_t)nseg, g.S.as<g2j>());
  k_miller<<<b, WG, 0, st>>>(g.P.as<g1a>(), g.H.as<g2a>(), (uint32_t)n, g.f.as<fp12>());
  k_seg_fp12_prod<<<(unsigned)nseg, WG, 0, st>>>(g.f.as<fp12>(), g.bad.as<int32_t>(), seg_off,
                                                 (uint32_t)nseg, g.F.as<fp12>(), seg_err);
  k_seg_partial<<<nblk(nseg), WG, 0, st>>>(g.F.as<fp12>(), g.S.as<g2j>(), (uint32_t)nseg, partials);
  HIPCHK(hipGetLastError());
  return true;
}

bool mv_segments_device(const uint8_t *msgs, const g2a *sigs, const g1a *pks,
                        const uint64_t *rands, size_t n, const uint32_t *seg_off, size_t nseg,
                        int32_t *verdicts, hipStream_t st) {
  if (!g.part.ensure(nseg * sizeof(fp12)) || !g.err.ensure(nseg * sizeof(int32_t)))
    return fail(GBLS_ERR_HIP);
  if (!mv_partials(msgs, sigs, pks, rands, n, seg_off, nseg, g.part.as<fp12>(),
                   g.err.as<int32_t>(), st))
    return false;
  k_final_verify<<<nblk(nseg), WG, 0, st>>>(g.part.as<fp12>(), g.err.as<int32_t>(), 1,
                                            (uint32_t)nseg, verdicts);
  HIPCHK(hipGetLastError());
  return true;
}

// ----- m independent pairing checks (sigs/pks/msgs already on device in in0..in3)
bool av_batch_device(const g2a *sigs, const uint8_t *msg, const uint32_t *off, const g1a *pks,
                     const int32_t *pre, size_t m, int32_t *verdicts_dev) {
  if (!g.H.ensure(m * sizeof(g2a)) || !g.f.ensure(m * sizeof(fp12)) ||
      !g.bad.ensure(m * sizeof(int32_t)))
    return fail(GBLS_ERR_HIP);
  unsigned b = nblk(m);
  k_hash_to_g2<<<b, WG, 0, g.stream>>>(msg, off, (uint32_t)m, nullptr, 0, g.H.as<g2a>());
  k_av_miller<<<b, WG, 0, g.stream>>>(sigs, pks, g.H.as<g2a>(), pre, (uint32_t)m, g.f.as<fp12>(),
                                      g.bad.as<int32_t>());
  k_final_verify<<<b, WG, 0, g.stream>>>(g.f.as<fp12>(), g.bad.as<int32_t>(), 1, (uint32_t)m,
                                         verdicts_dev);
  HIPCHK(hipGetLastError());
  return true;
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
const char *gbls_version(void) { return "grandine-bls-mi355x 0.1 (gfx950)"; }

int gbls_g1_decompress(const uint8_t (*in)[48], size_t n, int validate, gbls_p1_affine *out,
                       int32_t *status) {
  API_LOCK
  if (n == 0) return GBLS_SUCCESS;
  if (!upload(g.in0, &in[0][0], 48 * n) || !g.out0.ensure(n * sizeof(g1a)) ||
      !g.out1.ensure(n * sizeof(int32_t)))
    return -1;
  k_g1_decompress<<<nblk(n), WG, 0, g.stream>>>(g.in0.as<uint8_t>(), (uint32_t)n, validate,
                                                g.out0.as<g1a>(), g.out1.as<int32_t>());
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
  k_g2_decompress<<<nblk(n), WG, 0, g.stream>>>(g.in0.as<uint8_t>(), (uint32_t)n,
                                                g.out0.as<g2a>(), g.out1.as<int32_t>());
  if (!download(reinterpret_cast<g2a *>(out), g.out0, n) || !download(status, g.out1, n) || !sync())
    return -1;
  return GBLS_SUCCESS;
}

int gbls_g2_validate(const gbls_p2_affine *in, size_t n, int32_t *status) {
  API_LOCK
  if (n == 0) return GBLS_SUCCESS;
  if (!upload(g.in0, reinterpret_cast<const g2a *>(in), n) || !g.out1.ensure(n * sizeof(int32_t)))
    return -1;
  k_g2_validate<<<nblk(n), WG, 0, g.stream>>>(g.in0.as<g2a>(), (uint32_t)n, g.out1.as<int32_t>());
  if (!download(status, g.out1, n) || !sync()) return -1;
  return GBLS_SUCCESS;
}

int gbls_g1_compress(const gbls_p1_affine *in, size_t n, uint8_t (*out)[48]) {
  API_LOCK
  if (n == 0) return GBLS_SUCCESS;
  if (!upload(g.in0, reinterpret_cast<const g1a *>(in), n) || !g.out0.ensure(48 * n)) return -1;
  k_g1_compress<<<nblk(n), WG, 0, g.stream>>>(g.in0.as<g1a>(), (uint32_t)n, g.out0.as<uint8_t>());
  if (!download(&out[0][0], g.out0, 48 * n) || !sync()) return -1;
  return GBLS_SUCCESS;
}

int gbls_g2_compress(const gbls_p2_affine *in, size_t n, uint8_t (*out)[96]) {
  API_LOCK
  if (n == 0) return GBLS_SUCCESS;
  if (!upload(g.in0, reinterpret_cast<const g2a *>(in), n) || !g.out0.ensure(96 * n)) return -1;
  k_g2_compress<<<nblk(n), WG, 0, g.stream>>>(g.in0.as<g2a>(), (uint32_t)n, g.out0.as<uint8_t>());
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
  k_g1_aggregate_seg<<<(unsigned)nseg, WG, 0, g.stream>>>(
      g.in0.as<g1a>(), g.in1.as<uint32_t>(), (uint32_t)nseg, g.out0.as<g1a>(), g.out1.as<int32_t>());
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
  k_g2_aggregate_seg<<<1, WG, 0, g.stream>>>(g.in0.as<g2a>(), g.in1.as<uint32_t>(), 1,
                                             g.out0.as<g2a>());
  if (!download(reinterpret_cast<g2a *>(out), g.out0, 1) || !sync()) return -1;
  return GBLS_SUCCESS;
}

int gbls_aggregate_verify_batch(const gbls_p2_affine *sigs, const uint8_t *msg_data,
                                const uint32_t *msg_off, const gbls_p1_affine *pks, size_t m,
                                int32_t *verdicts) {
  API_LOCK
  if (m == 0) return GBLS_SUCCESS;
  for (size_t i = 0; i < m; i++) verdicts[i] = GBLS_VERIFY_FAIL;
  if (!upload(g.in0, reinterpret_cast<const g2a *>(sigs), m) ||
      !upload(g.in1, msg_data, msg_off[m]) || !upload(g.in2, msg_off, m + 1) ||
      !upload(g.in3, reinterpret_cast<const g1a *>(pks), m) ||
      !g.out1.ensure(m * sizeof(int32_t)))
    return -1;
  if (!av_batch_device(g.in0.as<g2a>(), g.in1.as<uint8_t>(), g.in2.as<uint32_t>(), g.in3.as<g1a>(),
                       nullptr, m, g.out1.as<int32_t>()))
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
  if (!upload(g.in0, reinterpret_cast<const g2a *>(sigs), m) ||
      !upload(g.in1, msg_data, msg_off[m]) || !upload(g.in2, msg_off, m + 1) ||
      !upload(g.in4, reinterpret_cast<const g1a *>(pks), npk) || !upload(g.in5, seg_off, m + 1) ||
      !g.in3.ensure(m * sizeof(g1a)) || !g.out0.ensure(m * sizeof(int32_t)) ||
      !g.out1.ensure(m * sizeof(int32_t)))
    return -1;
  k_g1_aggregate_seg<<<(unsigned)m, WG, 0, g.stream>>>(g.in4.as<g1a>(), g.in5.as<uint32_t>(),
                                                       (uint32_t)m, g.in3.as<g1a>(),
                                                       g.out0.as<int32_t>());
  if (!av_batch_device(g.in0.as<g2a>(), g.in1.as<uint8_t>(), g.in2.as<uint32_t>(), g.in3.as<g1a>(),
                       g.out0.as<int32_t>(), m, g.out1.as<int32_t>()))
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
      !upload(g.in4, seg_off, nseg + 1) || !g.out1.ensure(nseg * sizeof(int32_t)))
    return -1;
  if (!mv_segments_device(g.in0.as<uint8_t>(), g.in1.as<g2a>(), g.in2.as<g1a>(),
                          g.in3.as<uint64_t>(), n, g.in4.as<uint32_t>(), nseg,
                          g.out1.as<int32_t>(), g.stream))
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
  hipStream_t st = stream ? (hipStream_t)stream : g.stream;
  return mv_segments_device(msgs, reinterpret_cast<const g2a *>(sigs),
                            reinterpret_cast<const g1a *>(pks), rands, n, seg_off, nseg, verdicts,
                            st)
             ? GBLS_SUCCESS
             : -1;
}

int gbls_multi_verify_partials_device(const uint8_t *msgs, const gbls_p2_affine *sigs,
                                      const gbls_p1_affine *pks, const uint64_t *rands, size_t n,
                                      const uint32_t *seg_off, size_t nseg, gbls_fp12 *partials,
                                      int32_t *seg_err, void *stream) {
  API_LOCK
  if (nseg == 0) return GBLS_SUCCESS;
  hipStream_t st = stream ? (hipStream_t)stream : g.stream;
  return mv_partials(msgs, reinterpret_cast<const g2a *>(sigs), reinterpret_cast<const g1a *>(pks),
                     rands, n, seg_off, nseg, reinterpret_cast<fp12 *>(partials), seg_err, st)
             ? GBLS_SUCCESS
             : -1;
}

int gbls_final_verify_partials_device(const gbls_fp12 *partials, const int32_t *seg_err,
                                      size_t nparts, size_t nseg, int32_t *verdicts, void *stream) {
  API_LOCK
  if (nseg == 0) return GBLS_SUCCESS;
  hipStream_t st = stream ? (hipStream_t)stream : g.stream;
  k_final_verify<<<nblk(nseg), WG, 0, st>>>(reinterpret_cast<const fp12 *>(partials), seg_err,
                                            (uint32_t)nparts, (uint32_t)nseg, verdicts);
  return hipGetLastError() == hipSuccess ? GBLS_SUCCESS : ((t_last_error = GBLS_ERR_HIP), -1);
}

int gbls_sk_to_pk(const uint8_t (*sks)[32], size_t n, gbls_p1_affine *out) {
  API_LOCK
  if (n == 0) return GBLS_SUCCESS;
  if (!upload(g.in0, &sks[0][0], 32 * n) || !g.out0.ensure(n * sizeof(g1a))) return -1;
  k_sk_to_pk<<<nblk(n), WG, 0, g.stream>>>(g.in0.as<uint8_t>(), (uint32_t)n, g.out0.as<g1a>());
  if (!download(reinterpret_cast<g1a *>(out), g.out0, n) || !sync()) return -1;
  return GBLS_SUCCESS;
}

int gbls_sign(const uint8_t (*sks)[32], const uint8_t *msg_data, const uint32_t *msg_off, size_t n,
              gbls_p2_affine *out) {
  API_LOCK
  if (n == 0) return GBLS_SUCCESS;
  if (!upload(g.in0, &sks[0][0], 32 * n) || !upload(g.in1, msg_data, msg_off[n] ? msg_off[n] : 1) ||
      !upload(g.in2, msg_off, n + 1) || !g.H.ensure(n * sizeof(g2a)) ||
      !g.out0.ensure(n * sizeof(g2a)))
    return -1;
  k_hash_to_g2<<<nblk(n), WG, 0, g.stream>>>(g.in1.as<uint8_t>(), g.in2.as<uint32_t>(), (uint32_t)n,
                                             nullptr, 0, g.H.as<g2a>());
  k_sign<<<nblk(n), WG, 0, g.stream>>>(g.in0.as<uint8_t>(), g.H.as<g2a>(), (uint32_t)n,
                                       g.out0.as<g2a>());
  if (!download(reinterpret_cast<g2a *>(out), g.out0, n) || !sync()) return -1;
  return GBLS_SUCCESS;
}

int gbls_hash_to_g2(const uint8_t *msg_data, const uint32_t *msg_off, size_t n, const uint8_t *dst,
                    size_t dst_len, gbls_p2_affine *out) {
  API_LOCK
  if (n == 0) return GBLS_SUCCESS;
  if (dst_len > 255) return (t_last_error = GBLS_ERR_ARG), -1;
  if (!upload(g.in1, msg_data, msg_off[n] ? msg_off[n] : 1) || !upload(g.in2, msg_off, n + 1) ||
      !upload(g.in3, dst, dst_len ? dst_len : 1) || !g.out0.ensure(n * sizeof(g2a)))
    return -1;
  k_hash_to_g2<<<nblk(n), WG, 0, g.stream>>>(g.in1.as<uint8_t>(), g.in2.as<uint32_t>(), (uint32_t)n,
                                             g.in3.as<uint8_t>(), (uint32_t)dst_len,
                                             g.out0.as<g2a>());
  if (!download(reinterpret_cast<g2a *>(out), g.out0, n) || !sync()) return -1;
  return GBLS_SUCCESS;
}

double gbls_measure_mad64_peak(void) {
  std::lock_guard<std::mutex> lock(g.mu);
  if (!ensure_ready()) return 0.0;
  Buf sink;
  if (!sink.ensure(64)) return 0.0;
  const unsigned blocks = 256 * 8, threads = 256;
  const uint32_t iters = 4096;
  k_mad_peak<<<blocks, threads, 0, g.stream>>>(sink.as<uint64_t>(), 16, 1);  // warm
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventRecord(a, g.stream);
  k_mad_peak<<<blocks, threads, 0, g.stream>>>(sink.as<uint64_t>(), iters, 7);
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

}  // extern "C"
