// Shared declarations of the engine's translation units.  Each k_*.hip file holds a
// group of gfx950 kernels plus host launchers (declared here); gbls_capi.hip is the
// host orchestration behind the C ABI.  Splitting the kernels over translation units
// keeps every hipcc invocation small and lets the build run them in parallel.
#pragma once
#include <hip/hip_runtime.h>

#include "bls_hash.h"
#include "bls_pairing.h"

namespace gbls {

constexpr int WG = 64;    // per-lane kernels: one wave per workgroup
constexpr int WGR = 256;  // segment reductions: 4 waves, LDS tree
constexpr uint32_t NONE = 0xffffffffu;
// Stages with a quad-gang (latency) and a lane-per-item (throughput) variant pick the
// latter from these launch sizes on (measured on MI355X, 12 x 4096-set C2 step: Miller lines
// 3.32 ms quad vs 2.44 ms lane at 49152 pairs; cofactor clearing 4.99 vs 4.40 ms at 32768
// sets, the other streams filling the SIMDs a lane launch leaves free).  r06: with the
// radix-2^28 lane kernels and their lazy combinations the lane form also wins from 8192 points
// when two submissions are in flight (C3, 10 000 messages per launch: 835-855k -> 879k
// messages/s in one box, profiles/r06/y_ab_lane_min.txt; C2's launches are 4096 or >= 65536).
// One threshold for all three stages: g_lane_min (GBLS_LANE_MIN overrides it).
constexpr uint32_t kLaneRegimeSets = 8192;
// ... and Miller lines of up to this many pairs run on 16-lane DPP rows (bls_gang.h),
// 16 x 4096 lanes being one wave per SIMD
constexpr uint32_t kRowRegimeMax = 6144;
// ... and the smallest launches run one wave per point (bls_w4.h): cofactor clearing and
// Miller lines of up to this many points
#ifndef GBLS_W4_MAX
#define GBLS_W4_MAX 1024
#endif
constexpr uint32_t kW4Max = GBLS_W4_MAX;
// cofactor clearing on rows up to this many points (4096 -> 2048 in r04: a single 4096-set batch
// runs 802k sets/s with quad gangs vs 772k with rows, a C4 epoch of 2048-set launches 540k with
// rows vs 480k with quad gangs; profiles/r04/q_*)
constexpr uint32_t kRowClearMax = 2048;
extern uint32_t g_row_clear_max;         // kRowClearMax unless GBLS_ROW_CLEAR_MAX is set
extern uint32_t g_ml_r28;                // k_ml_group in radix-2^28 arithmetic (GBLS_ML_R28)
// k_msm_chunk: points summed per lane (mixed additions).  r05 (partials folded by k_msm_fold):
// C2 4.25 / 4.27M at K = 16 (884 waves), 4.18 / 4.24M at K = 8 (1716), 4.22 / 4.18M at K = 6
// (2271) -- within noise; the side-stream MSM overlaps the main chain, so its fill is not the
// step's bound.  GBLS_MSM_K selects another K.
constexpr uint32_t kMsmChunk = 16;
// segments below 4096 sets (C4's 2048-set segments): K = 4, more and shorter chunk chains on the
// signature side, which sets their join (C4 565-580k vs 529-566k with K = 16, one box,
// profiles/r06/zz_ab_c4_msm_k.txt)
constexpr uint32_t kMsmChunkSmall = 4;
constexpr int kMsmFoldLevels = 3;        // k_msm_fold: pairwise levels over each bucket's partials
constexpr uint32_t kMsmFold = 1u << kMsmFoldLevels;  // chunk partials per fold group
extern uint32_t g_msm_k;                 // GBLS_MSM_K, else 0: kMsmChunkSmall / kMsmChunk (msm_plan)
extern uint32_t g_msm_r28;               // k_msm_chunk28 / k_msm_fold28 (GBLS_MSM_R28=0: the engine-form kernels)
extern uint32_t g_ml_kara;               // k_ml_group28: Karatsuba Fp2 sparse products (GBLS_ML_KARA)
extern uint32_t g_ml_prefetch;           // k_ml_group28: next pair's line loaded during the product (GBLS_ML_PREFETCH)
extern uint32_t g_ml_dma;                // k_ml_group28: line staged in LDS by DMA loads (GBLS_ML_DMA)
extern uint32_t g_ml_xcd;                // k_ml_group: XCD-grouped block order (GBLS_ML_XCD)
extern uint32_t g_lane_r28;              // lane-regime clearing / lines in radix 2^28 (GBLS_LANE_R28)
extern uint32_t g_clear_staged;          // lane clearing in five stages, chains at two waves per SIMD (GBLS_CLEAR_STAGED=1; off)
extern uint32_t g_map_rows_max;          // hash_to_G2 maps of up to this many field elements on 16-lane rows (GBLS_MAP_ROWS_MAX)
extern uint32_t g_lane_min;              // launches of at least this many points take the lane regime (GBLS_LANE_MIN)
// line-coefficient buffer bound per submission (19.6 KB per pair: 4 GB = 214k pairs,
// a C5 shard of 131 072 sets unsliced; tiny next to 288 GB of HBM): above it the Miller
// lines are made in event slices (GBLS_LINE_BUDGET_MB overrides it)
constexpr size_t kLineBudget = (size_t)4 << 30;

inline unsigned nblk(size_t n, unsigned per = WG) { return (unsigned)((n + per - 1) / per); }

// k_decode.hip -- encodings, aggregation, key material, roofline probe
void launch_g1_decompress(hipStream_t st, const uint8_t *in, uint32_t n, int validate, g1a *out,
                          int32_t *status);
void launch_g2_decompress(hipStream_t st, const uint8_t *in, uint32_t n, g2a *out, int32_t *status);
void launch_g2_check(hipStream_t st, const g2a *in, uint32_t n, int32_t *status, int accumulate);
void launch_g1_compress(hipStream_t st, const g1a *in, uint32_t n, uint8_t *out);
void launch_g2_compress(hipStream_t st, const g2a *in, uint32_t n, uint8_t *out);
void launch_g1_aggregate_seg(hipStream_t st, const g1a *pks, const uint32_t *off, uint32_t nseg,
                             g1a *out, int32_t *status);
void launch_g2_aggregate_seg(hipStream_t st, const g2a *pts, const uint32_t *off, uint32_t nseg,
                             g2a *out, int32_t *status);
// validator registry (f1): keys by index
void launch_g1_aggregate_idx(hipStream_t st, const g1a *reg, uint32_t nreg, const uint32_t *idx,
                             const uint32_t *off, uint32_t nseg, g1a *out, int32_t *status);
void launch_g1_gather_idx(hipStream_t st, const g1a *reg, uint32_t nreg, const uint32_t *idx,
                          uint32_t n, g1a *out, int32_t *status);
void launch_sk_to_pk(hipStream_t st, const uint8_t *sks, uint32_t n, g1a *out);
void launch_sign(hipStream_t st, const uint8_t *sks, const g2a *H, uint32_t n, g2a *out);
void launch_mad_peak(hipStream_t st, unsigned blocks, uint64_t *sink, uint32_t iters, uint32_t seed);

// k_h2c.hip -- hash_to_G2 stages
void launch_h2c_field(hipStream_t st, const uint8_t *msg, const uint32_t *off, uint32_t n,
                      const uint8_t *dst, uint32_t dlen, fp2 *U);
void launch_h2c_map(hipStream_t st, const fp2 *U, uint32_t nu, g2j *Q);
void launch_h2c_clear(hipStream_t st, const g2j *Q, uint32_t n, g2a *H);
// the latency regime's pipeline form (n <= kW4Max, else false): the cleared points stay
// Jacobian, written over Q[2 i]
bool launch_h2c_clear_jac(hipStream_t st, g2j *Q, uint32_t n);

// k_scalar.hip -- random-scalar products and the per-segment signature sum
// P_i = r_i pk_i as line-evaluation points (bls_pairing.h g1s), quad per set
void launch_mv_g1mul(hipStream_t st, const g1a *pks, const uint64_t *rands, uint32_t n, g1s *P);
void launch_mv_g2mul(hipStream_t st, const g2a *sigs, const uint64_t *rands, uint32_t n, g2j *R);
// chunks: 4 words per level-1 workgroup {segment, half, begin, end}; seg_chunk[nseg+1].
// seg_err[s] = a set of s failed (infinite pk, zero scalar, pre[i] != 0) or, when
// empty_is_error, s has no sets; an empty segment's partial is the identity otherwise.
void launch_g2sum(hipStream_t st, const g2j *R, const uint32_t *chunks, uint32_t nchunks,
                  const uint32_t *seg_chunk, const uint32_t *seg_off, uint32_t nseg, uint32_t n,
                  const g1a *pks, const uint64_t *rands, const int32_t *pre, const int32_t *pre2,
                  int empty_is_error, g2j *part, int32_t *part_err, g1s *P, g2a *H,
                  int32_t *seg_err, g2j *Sj = nullptr, hipEvent_t keys_ready = nullptr);
// single checks (r = 1, one set per segment): the extra pair of segment s is (-g1, sig_s)
// ng1_out: grouped single checks -- -g1 (affine) per check into ng1_out instead of the
// pair's G1 point P[n + i], which the caller then scales by r_i (launch_mv_g1mul)
void launch_single_S(hipStream_t st, const g2a *sigs, const g1a *pks, const int32_t *pre,
                     const int32_t *pre2, uint32_t n, g1s *P, g2a *H, int32_t *seg_err,
                     g1a *ng1_out = nullptr);
// gerr[g] = OR of err[i] over the checks [g gs, (g + 1) gs) of group g
void launch_group_err(hipStream_t st, const int32_t *err, uint32_t n, uint32_t gs, uint32_t ngrp,
                      int32_t *gerr);

// k_msm.hip -- S_s = sum r_i sig_i of every segment by a signed-digit bucket MSM
struct MsmPlan {
  uint32_t nseg;
  int c, W;             // window bits, windows
  uint32_t nb;          // buckets (nseg * W * 2^(c-1))
  uint32_t max_chunks;  // bound on the chunk count (grid of the chunk kernel)
  uint32_t K;           // points per chunk
  uint32_t max_folds;   // bound on the level-0 fold-pair count (grid of the fold kernels)
  bool tree;            // per-window bucket trees (c = 13) or per-bucket pairs (c = 5)
  uint32_t extra;       // extra Miller pairs per segment: W (tree) or W * 2^(c-1)
  bool r28;             // chunk sums and folds in radix 2^28 (g_msm_r28)
  size_t o_cnt, o_start, o_cur, o_cstart, o_fstart[kMsmFoldLevels], o_list, o_chunk, o_t0, o_a0, o_t1, o_a1,
      o_sig28, bytes;
};
// default: segments at least this large use the bucket MSM.  2048 -> 4096 in r04 (a C4 epoch of
// 2048-set segments ran 542-572k sets/s with per-set products vs 375-390k with that round's MSM,
// profiles/r04/k_*); back to 2048 in r06, after the radix-2^28 MSM and the lazy additions: C4
// 546-575k with the MSM vs 511-557k with per-set products in two boxes, seven runs each way
// (profiles/r06/zz_ab_msm_min.txt), C2 / C1 unchanged (their segments are >= 4096 / < 2048)
constexpr uint32_t kMsmMinPerSeg = 2048;
MsmPlan msm_plan(uint32_t n, uint32_t nseg);
// writes each segment's p.extra Miller pairs (P[n + s * extra + k] = a constant G1 weight,
// H[...] = affine bucket or window sum), zeroes seg_err and flags empty segments when
// empty_is_error
// (pks, pre, pre2: the segment error flags of k_msm_count, as k_g2sum_final sets them)
void launch_msm(hipStream_t st, const MsmPlan &p, uint8_t *ws, const g2a *sigs,
                const uint64_t *rands, const g1a *pks, const int32_t *pre, const int32_t *pre2,
                uint32_t n, const uint32_t *seg_off, int empty_is_error, g2a *H, g1s *P,
                int32_t *seg_err);

// k_lines.hip -- Miller-loop line functions of every pair
// Where a pair's lines live: column col[pair] of ncol (col null: column = pair); word w of
// event e at (e * 72 + w) * ncol + column (bls_pairing.h line_word)
struct LineCols {
  const uint32_t *col;
  uint32_t ncol;
};
// lines of events [e0, e1) of pairs [first, first + count) (H indexed by pair), stored at
// event e - e0; Ts: the running point between event slices (null: full range)
void launch_lines(hipStream_t st, const g2a *H, uint32_t first, uint32_t count, LineCols lc,
                  int e0, int e1, g2h *Ts, uint32_t *lines, bool lane = false);
// all events of pairs [first, first + count) from Jacobian points Qj[stride i] (count <=
// kW4Max, else false)
bool launch_lines_jac(hipStream_t st, const g2j *Qj, uint32_t stride, uint32_t first, uint32_t count,
                      LineCols lc, uint32_t *lines);

// k_miller.hip -- Miller product tree + Horner
// groups: (first index into plist, stride, count) per group, segment by segment
// events [e0, e1): lines at event e - e0, products to V0[e * ngroup + g]; the lines of pair j
// of group g at column j ngp + g when ngp != 0 (the tables' layout), else at lc's column
// Pc (nullable): the points by line column (launch_ml_pcols), read by the radix-2^28 kernel
void launch_ml_group(hipStream_t st, const uint32_t *lines, LineCols lc, uint32_t ngp, const g1s *P,
                     const uint32_t *Pc, const uint32_t *plist, const uint32_t *groups, uint32_t ngroup,
                     int e0, int e1, fp12 *V0, uint32_t *V28, bool pcn = false);
// Pc[w * ncol + col[pair]] = word w of P[pair] (36 words per point), pairs [0, np)
void launch_ml_pcols(hipStream_t st, const g1s *P, const uint32_t *col, uint32_t np, uint32_t ncol,
                     uint32_t *Pc, bool normalize);
void launch_ml_reduce(hipStream_t st, const fp12 *Vin, uint32_t nin, const uint32_t *red,
                      uint32_t nout, fp12 *Vout);
// lim (device count, optional): only segments s with base + s < *lim run (the others exit)
// tmp (optional, >= 4 nseg values): up to 64 segments run the chain in 4 parallel parts
void launch_ml_horner(hipStream_t st, const fp12 *V, uint32_t nseg, fp12 *partial,
                      const uint32_t *lim = nullptr, uint32_t base = 0, fp12 *tmp = nullptr);

// k_fexp.hip -- product of partials, final exponentiation, verdict
// lim / base as in launch_ml_horner; scatter (optional): segment s's verdict goes to
// verdict[scatter[base + s]] instead of verdict[s]
void launch_final_verdict(hipStream_t st, const fp12 *partials, const int32_t *err,
                          uint32_t nparts, uint32_t nseg, int32_t *verdict,
                          const uint32_t *lim = nullptr, uint32_t base = 0,
                          const uint32_t *scatter = nullptr);

// k_groups.hip -- second round of the grouped single checks, on the device
void launch_group_expand(hipStream_t st, const int32_t *gv, const int32_t *err, uint32_t n, uint32_t gs,
                         int32_t *verdicts, uint32_t *redo, uint32_t *cnt);
void launch_redo_tables(hipStream_t st, const uint32_t *redo, const uint32_t *cnt, uint32_t base, uint32_t R,
                        uint32_t n, uint32_t *plist, uint32_t *grp);

}  // namespace gbls
