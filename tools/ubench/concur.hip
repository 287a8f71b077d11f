// Concurrency probe: does a small kernel on a second stream run beside a heavy
// one-wave-per-SIMD kernel (k_h2c_clear: 256 VGPR + 248 AGPR + 12 B scratch;
// k_h2c_map: 256 + 35, no scratch; k_lines: 256 + 132) or wait for it to drain?
// Prints, per heavy kernel and wave count: the heavy kernel's time alone, the small
// kernel's time alone, and when the small kernel finished relative to the heavy one.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I grandine_amd/csrc \
//   tools/ubench/concur.hip -o /tmp/concur
#include "../../grandine_amd/csrc/k_lines.hip"  // first: it enables the gang line steps
#include "../../grandine_amd/csrc/k_h2c_clear.hip"
#include "../../grandine_amd/csrc/k_h2c_map.hip"

#include <cstdio>

using namespace gbls;

__global__ void k_small(const uint32_t *in, uint32_t n, uint32_t *out) {
  uint32_t i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = in[i] * 3u + 1u;
}

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e_ = (x);                                              \
    if (e_ != hipSuccess) {                                           \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); \
      return 1;                                                       \
    }                                                                 \
  } while (0)

int main() {
  const uint32_t NMAX = 16384;
  g2j *Q;
  g2a *H;
  fp2 *U;
  uint32_t *a, *b, *lines;
  CK(hipMalloc(&Q, 2 * NMAX * sizeof(g2j)));
  CK(hipMalloc(&H, 2 * NMAX * sizeof(g2a)));
  CK(hipMalloc(&U, 2 * NMAX * sizeof(fp2)));
  CK(hipMalloc(&a, 1 << 20));
  CK(hipMalloc(&b, 1 << 20));
  CK(hipMalloc(&lines, (size_t)NMAX * ML_EVENTS * 72 * 4));
  CK(hipMemset(Q, 0, 2 * NMAX * sizeof(g2j)));
  CK(hipMemset(H, 0, 2 * NMAX * sizeof(g2a)));
  CK(hipMemset(U, 0, 2 * NMAX * sizeof(fp2)));
  CK(hipMemset(a, 0, 1 << 20));
  hipStream_t sa, sb;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  hipEvent_t e0, e1, e2, f0, f1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&e2));
  CK(hipEventCreate(&f0));
  CK(hipEventCreate(&f1));
  const char *names[3] = {"clear", "map", "lines"};
  for (int kind = 0; kind < 3; kind++) {
    for (uint32_t n : {1024u, 4096u, 16384u}) {
      auto heavy = [&](hipStream_t s) {
        if (kind == 0) launch_h2c_clear(s, Q, n, H);
        if (kind == 1) launch_h2c_map(s, U, n / 2, Q);
        if (kind == 2) launch_lines(s, H, 0, n, n, lines);
      };
      float t_heavy = 0, t_small = 0, t_fin_small = 0, t_fin_heavy = 0;
      for (int rep = 0; rep < 3; rep++) {
        CK(hipEventRecord(e0, sa));
        heavy(sa);
        CK(hipEventRecord(e2, sa));
        CK(hipStreamSynchronize(sa));
        CK(hipEventElapsedTime(&t_heavy, e0, e2));
        CK(hipEventRecord(f0, sb));
        k_small<<<64, 256, 0, sb>>>(a, 16384, b);
        CK(hipEventRecord(f1, sb));
        CK(hipStreamSynchronize(sb));
        CK(hipEventElapsedTime(&t_small, f0, f1));
        // concurrent: heavy on sa, then (after it has started) small on sb
        CK(hipEventRecord(e0, sa));
        heavy(sa);
        CK(hipEventRecord(e2, sa));
        CK(hipStreamWaitEvent(sb, e0, 0));
        k_small<<<64, 256, 0, sb>>>(a, 16384, b);
        CK(hipEventRecord(e1, sb));
        CK(hipDeviceSynchronize());
        CK(hipEventElapsedTime(&t_fin_small, e0, e1));
        CK(hipEventElapsedTime(&t_fin_heavy, e0, e2));
      }
      std::printf("%-6s n=%-6u heavy %.3f ms  small alone %.3f ms  concurrent: small done at %.3f, heavy at %.3f ms\n",
                  names[kind], n, t_heavy, t_small, t_fin_small, t_fin_heavy);
    }
  }
  return 0;
}
