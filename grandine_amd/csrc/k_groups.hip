// gfx950 kernels of the grouped single checks' second round (gbls_capi.hip grouped_verdicts),
// entirely on the device so that the device entry points stay asynchronous: the verdict of
// every check from its group's verdict, the compacted list of members to re-check, and the
// re-check's Miller tables.
#include "gbls_common.h"

namespace gbls {

// check i passes with its group (gv = the group verdicts of round 1, which already include
// every member's error flag); a member of a failed group without an error flag of its own is
// appended to redo (order irrelevant: each re-check is its own segment and writes its own
// verdict through the redo index)
__global__ void __launch_bounds__(WG) k_group_expand(const int32_t *gv, const int32_t *err, uint32_t n,
                                                     uint32_t gs, int32_t *verdicts, uint32_t *redo,
                                                     uint32_t *cnt) {
  const uint32_t i = blockIdx.x * WG + threadIdx.x;
  if (i >= n) return;
  const bool pass = gv[i / gs] == ST_SUCCESS;
  verdicts[i] = pass ? ST_SUCCESS : ST_VERIFY_FAIL;
  if (!pass && err[i] == 0) redo[atomicAdd(cnt, 1u)] = i;
}

// Miller tables of re-check slots [base, base + R): slot j = check redo[base + j] alone, its
// two pairs (i, n + i) one group; a slot past the count evaluates one line of pair 0 (cheap,
// and its Horner step and final exponentiation are skipped)
__global__ void __launch_bounds__(WG) k_redo_tables(const uint32_t *redo, const uint32_t *cnt, uint32_t base,
                                                    uint32_t R, uint32_t n, uint32_t *plist, uint32_t *grp) {
  const uint32_t j = blockIdx.x * WG + threadIdx.x;
  if (j >= R) return;
  const bool on = base + j < *cnt;
  const uint32_t i = on ? redo[base + j] : 0;
  plist[2 * j] = i;
  plist[2 * j + 1] = n + i;
  grp[3 * j] = 2 * j;
  grp[3 * j + 1] = 1;
  grp[3 * j + 2] = on ? 2 : 1;
}

void launch_group_expand(hipStream_t st, const int32_t *gv, const int32_t *err, uint32_t n, uint32_t gs,
                         int32_t *verdicts, uint32_t *redo, uint32_t *cnt) {
  if (n) k_group_expand<<<nblk(n), WG, 0, st>>>(gv, err, n, gs, verdicts, redo, cnt);
}
void launch_redo_tables(hipStream_t st, const uint32_t *redo, const uint32_t *cnt, uint32_t base, uint32_t R,
                        uint32_t n, uint32_t *plist, uint32_t *grp) {
  if (R) k_redo_tables<<<nblk(R), WG, 0, st>>>(redo, cnt, base, R, n, plist, grp);
}

}  // namespace gbls
