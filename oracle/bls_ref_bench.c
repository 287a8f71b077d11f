/* oracle/bls_ref_bench.c -- CPU baseline driver for bench.py (TEST INFRASTRUCTURE).
 *
 * Generates n synthetic sets shaped like bench.py's C2 workload (interop-style keys,
 * distinct 32-byte messages, sig = sk * H(m), nonzero 64-bit scalars), then times one
 * ref_multi_verify over them with T worker threads, and prints one JSON line:
 *   {"n": n, "threads": T, "seconds": s, "sets_per_s": n / s, "ok": 1}
 * usage: bls_ref_bench N THREADS
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

int ref_multi_verify(const uint8_t *, const uint8_t *, const uint8_t *, const uint64_t *, size_t, int);
void ref_sk_to_pk(const uint8_t *, uint8_t *);
void ref_sign(const uint8_t *, const uint8_t *, size_t, uint8_t *);

static void sha256_bytes(const uint8_t *m, size_t len, uint8_t out[32]);

typedef struct {
  size_t b, e;
  uint8_t *sks, *msgs, *pks, *sigs;
} gen_t;
static void *gen_worker(void *arg) {
  gen_t *g = (gen_t *)arg;
  for (size_t i = g->b; i < g->e; i++) {
    ref_sk_to_pk(g->sks + 32 * i, g->pks + 96 * i);
    ref_sign(g->sks + 32 * i, g->msgs + 32 * i, 32, g->sigs + 192 * i);
  }
  return NULL;
}
static double now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}
int main(int argc, char **argv) {
  size_t n = argc > 1 ? strtoul(argv[1], 0, 10) : 256;
  int T = argc > 2 ? atoi(argv[2]) : 1;
  uint8_t *sks = malloc(32 * n), *msgs = malloc(32 * n), *pks = malloc(96 * n), *sigs = malloc(192 * n);
  uint64_t *rands = malloc(8 * n);
  for (size_t i = 0; i < n; i++) {
    uint8_t buf[40];
    memcpy(buf, "cpu-sk", 6);
    memcpy(buf + 6, &i, 8);
    sha256_bytes(buf, 14, sks + 32 * i);
    sks[32 * i] &= 0x3f; /* < 2^254 < r: a valid nonzero scalar (probability ~1) */
    memcpy(buf, "cpu-m/", 6);
    sha256_bytes(buf, 14, msgs + 32 * i);
    uint64_t x = 0x9E3779B97F4A7C15ull * (i + 1);
    x ^= x >> 29;
    rands[i] = x ? x : 1;
  }
  pthread_t *th = calloc(T, sizeof(pthread_t));
  gen_t *g = calloc(T, sizeof(gen_t));
  for (int t = 0; t < T; t++) {
    g[t] = (gen_t){n * t / T, n * (t + 1) / T, sks, msgs, pks, sigs};
    pthread_create(&th[t], 0, gen_worker, &g[t]);
  }
  for (int t = 0; t < T; t++) pthread_join(th[t], 0);
  double t0 = now();
  int ok = ref_multi_verify(msgs, sigs, pks, rands, n, T);
  double dt = now() - t0;
  printf("{\"n\": %zu, \"threads\": %d, \"seconds\": %.4f, \"sets_per_s\": %.1f, \"ok\": %d}\n", n, T, dt,
         n / dt, ok);
  return ok ? 0 : 1;
}

/* minimal SHA-256 for input generation */
static const uint32_t K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
#define RR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))
static void sha256_bytes(const uint8_t *m, size_t len, uint8_t out[32]) {
  uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint8_t blk[64] = {0};
  memcpy(blk, m, len); /* len < 56 */
  blk[len] = 0x80;
  uint64_t bits = (uint64_t)len * 8;
  for (int i = 0; i < 8; i++) blk[63 - i] = (uint8_t)(bits >> (8 * i));
  uint32_t w[64];
  for (int i = 0; i < 16; i++) w[i] = ((uint32_t)blk[4 * i] << 24) | (blk[4 * i + 1] << 16) | (blk[4 * i + 2] << 8) | blk[4 * i + 3];
  for (int i = 16; i < 64; i++)
    w[i] = w[i - 16] + (RR(w[i - 15], 7) ^ RR(w[i - 15], 18) ^ (w[i - 15] >> 3)) + w[i - 7] +
           (RR(w[i - 2], 17) ^ RR(w[i - 2], 19) ^ (w[i - 2] >> 10));
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int i = 0; i < 64; i++) {
    uint32_t t1 = hh + (RR(e, 6) ^ RR(e, 11) ^ RR(e, 25)) + ((e & f) ^ (~e & g)) + K[i] + w[i];
    uint32_t t2 = (RR(a, 2) ^ RR(a, 13) ^ RR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  for (int i = 0; i < 8; i++)
    for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(h[i] >> (24 - 8 * k));
}
