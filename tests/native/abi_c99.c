/* C99 consumer of include/grandine_bls_gpu.h: includes the header in a -std=c99 -Wall -Wextra
 * -Werror -pedantic translation unit, calls EVERY entry point once with one-element arguments and
 * links against grandine_amd/lib/libgrandine_bls.so.  Without a GPU (the CPU suite) every call
 * must fail closed: verification entry points return GBLS_VERIFY_FAIL, verdict and status
 * arrays are filled with a failure code, and gbls_last_error() is GBLS_ERR_NO_DEVICE.
 * Prints "name rc" per call; tests/test_rust_binding.py checks the output. */
#include <stdio.h>
#include <string.h>

#include "grandine_bls_gpu.h"

#define CALL(name, expr)                                         \
  do {                                                           \
    int rc_ = (int)(expr);                                       \
    printf("%s %d %d\n", name, rc_, gbls_last_error());          \
  } while (0)

int main(void) {
  static uint8_t m32[1][32], s96[1][96], k48[1][48], sk[1][32], msg[32], dst[8];
  static gbls_p1_affine p1[2];
  static gbls_p2_affine p2[2];
  static gbls_fp12 f12[1];
  static uint64_t rands[1] = {1};
  static uint32_t off2[2] = {0, 1}, moff[2] = {0, 32}, idx[1] = {0}, calls[32];
  static int32_t st[2], v[2];
  static double ms[32];
  const char *ver;

  CALL("gbls_init", gbls_init(0, 0));
  CALL("gbls_set_policy", gbls_set_policy(0));
  CALL("gbls_device_count", gbls_device_count());
  ver = gbls_version();
  printf("gbls_version %s\n", ver ? ver : "(null)");
  CALL("gbls_g1_decompress", gbls_g1_decompress((const uint8_t(*)[48])k48, 1, 1, p1, st));
  printf("status %d\n", st[0]);
  CALL("gbls_g2_decompress", gbls_g2_decompress((const uint8_t(*)[96])s96, 1, p2, st));
  CALL("gbls_g2_validate", gbls_g2_validate(p2, 1, st));
  CALL("gbls_g1_compress", gbls_g1_compress(p1, 1, k48));
  CALL("gbls_g2_compress", gbls_g2_compress(p2, 1, s96));
  CALL("gbls_g1_aggregate", gbls_g1_aggregate(p1, 1, p1 + 1));
  CALL("gbls_g1_aggregate_segments", gbls_g1_aggregate_segments(p1, off2, 1, p1 + 1, st));
  CALL("gbls_g2_aggregate", gbls_g2_aggregate(p2, 1, p2 + 1));
  CALL("gbls_g2_aggregate_segments", gbls_g2_aggregate_segments(p2, off2, 1, p2 + 1, st));
  CALL("gbls_registry_set", gbls_registry_set(0, (const uint8_t(*)[48])k48, 1, st));
  CALL("gbls_registry_size", gbls_registry_size());
  CALL("gbls_g1_aggregate_indexed", gbls_g1_aggregate_indexed(idx, off2, 1, p1, st));
  CALL("gbls_verify", gbls_verify(p2, msg, 32, p1));
  CALL("gbls_fast_aggregate_verify", gbls_fast_aggregate_verify(p2, msg, 32, p1, 1));
  CALL("gbls_aggregate_verify_batch", gbls_aggregate_verify_batch(p2, msg, moff, p1, 1, v));
  printf("verdict %d\n", v[0]);
  CALL("gbls_verify_batch_compressed",
       gbls_verify_batch_compressed((const uint8_t(*)[32])m32, (const uint8_t(*)[96])s96, p1, NULL, 1,
                                    st, v));
  CALL("gbls_fast_aggregate_verify_batch",
       gbls_fast_aggregate_verify_batch(p2, msg, moff, p1, off2, 1, v));
  CALL("gbls_fast_aggregate_verify_indexed",
       gbls_fast_aggregate_verify_indexed(p2, msg, moff, idx, off2, 1, v));
  CALL("gbls_multi_verify", gbls_multi_verify((const uint8_t(*)[32])m32, p2, p1, rands, 1));
  CALL("gbls_multi_verify_segments",
       gbls_multi_verify_segments((const uint8_t(*)[32])m32, p2, p1, rands, 1, off2, 1, v));
  CALL("gbls_multi_verify_indexed",
       gbls_multi_verify_indexed((const uint8_t(*)[32])m32, p2, idx, NULL, rands, 1));
  CALL("gbls_multi_verify_compressed",
       gbls_multi_verify_compressed((const uint8_t(*)[32])m32, (const uint8_t(*)[96])s96, p1, NULL,
                                    NULL, rands, 1, st));
  CALL("gbls_multi_verify_compressed_ex",
       gbls_multi_verify_compressed_ex((const uint8_t(*)[32])m32, (const uint8_t(*)[96])s96, p1,
                                       NULL, NULL, rands, 1, st, GBLS_CALL_BLOCK));
  CALL("gbls_multi_verify_bisect",
       gbls_multi_verify_bisect((const uint8_t(*)[32])m32, p2, p1, NULL, NULL, rands, 1, v));
  /* device-pointer entry points: host memory is never dereferenced without a device */
  CALL("gbls_multi_verify_segments_device",
       gbls_multi_verify_segments_device(&m32[0][0], p2, p1, rands, 1, off2, 1, v, NULL));
  CALL("gbls_multi_verify_indexed_segments_device",
       gbls_multi_verify_indexed_segments_device(&m32[0][0], p2, idx, NULL, rands, 1, off2, 1, v,
                                                 NULL));
  CALL("gbls_fast_aggregate_verify_indexed_device",
       gbls_fast_aggregate_verify_indexed_device(p2, &m32[0][0], idx, off2, 1, v, NULL));
  CALL("gbls_multi_verify_partials_device",
       gbls_multi_verify_partials_device(&m32[0][0], p2, p1, rands, 1, off2, 1, f12, st, NULL));
  CALL("gbls_multi_verify_indexed_partials_device",
       gbls_multi_verify_indexed_partials_device(&m32[0][0], p2, idx, NULL, rands, 1, off2, 1, f12,
                                                 st, NULL));
  CALL("gbls_final_verify_partials_device",
       gbls_final_verify_partials_device(f12, st, 1, 1, v, NULL));
  CALL("gbls_sk_to_pk", gbls_sk_to_pk((const uint8_t(*)[32])sk, 1, p1));
  CALL("gbls_sign", gbls_sign((const uint8_t(*)[32])sk, msg, moff, 1, p2));
  CALL("gbls_hash_to_g2", gbls_hash_to_g2(msg, moff, 1, dst, sizeof dst, p2));
  printf("gbls_measure_mad64_peak %g\n", gbls_measure_mad64_peak());
  CALL("gbls_profile", gbls_profile(0));
  CALL("gbls_profile_read", gbls_profile_read(ms, calls, 32));
  gbls_profile_reset();
  printf("gbls_stage_name %s\n", gbls_stage_name(0));
  (void)memset(st, 0, sizeof st);
  return 0;
}
