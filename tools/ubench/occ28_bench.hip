// Does a second wave per SIMD speed up the radix-2^28 lane chains?  The cofactor chain
// ([|x|] P: 63 lazy doublings + 5 mixed additions of an affine base parked in LDS) compiled for
// two waves per SIMD (amdgpu_waves_per_eu: 256 VGPRs, no scratch), launched with and without a
// dynamic LDS pad that leaves room for only four one-wave blocks per CU (one wave per SIMD),
// timed over 65 536 and 131 072 lanes.
// usage: occ28_bench  (prints one line per (occupancy, lanes): ms per launch, chains/s)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "gbls_common.h"
#include "bls_curve28.h"

namespace gbls {
struct g2a28_lds {
  r28::g2a28 v;
  uint32_t pad;
};
template <int OCC>
__global__ void __launch_bounds__(WG) __attribute__((amdgpu_waves_per_eu(OCC, OCC)))
k_chain(g2j *Q, uint32_t n) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  __shared__ g2a28_lds pl[WG];
  r28::g2a28 *pp = &pl[threadIdx.x].v;
  r28::g2j28 h;
  r28::g2j_load12(h, Q[i]);
  pp->x = h.x;
  pp->y = h.y;
  for (int b = 62; b >= 0; b--) {
    jac_dbl(h, h);
    if ((k::X_ABS >> b) & 1) r28::jac_add_aff28<false>(h, h, *pp);
  }
  r28::g2j_store12(Q[i], h);
}
}  // namespace gbls
using namespace gbls;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main() {
  const uint32_t nmax = 131072;
  std::vector<g2j> h(nmax);
  uint32_t s = 12345;
  for (auto &p : h) {  // small random limbs (< 2^380 each word pattern): values < p
    uint32_t *w = reinterpret_cast<uint32_t *>(&p);
    for (size_t k = 0; k < sizeof(g2j) / 4; k++) {
      s = s * 1664525u + 1013904223u;
      w[k] = (k % 12 == 11) ? (s & 0x0fffffffu) : s;
    }
  }
  g2j *d;
  CK(hipMalloc(&d, nmax * sizeof(g2j)));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (uint32_t n : {65536u, 131072u}) {
    for (int occ = 1; occ <= 2; occ++) {
      CK(hipMemcpy(d, h.data(), n * sizeof(g2j), hipMemcpyHostToDevice));
      // occ 1: 40 KB of LDS per one-wave block (160 KB per CU / 4); occ 2: the 14.6 KB static
      const size_t pad = occ == 1 ? 40960 - sizeof(g2a28_lds) * WG : 0;
      auto run = [&]() { k_chain<2><<<nblk(n), WG, pad>>>(d, n); };
      run();
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(a));
      const int reps = 5;
      for (int r = 0; r < reps; r++) run();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      ms /= reps;
      printf("occupancy %d lanes %u: %.3f ms per launch, %.3e chains/s\n", occ, n, ms, n / (ms * 1e-3));
    }
  }
  return 0;
}
