// Host-side Miller product tables of a submission (one staged upload with the rest of its host
// tables).  Host-only C++ (no HIP): gbls_capi.hip builds them for every pipeline;
// tests/native/tables_check.cpp checks their invariants on the CPU.
//
// Level 0: per Miller segment, its pairs in groups of <= G, strided so that a wave's lanes read
// adjacent pairs (k_ml_group); then 4-ary reduction levels down to one product per segment
// (k_ml_reduce), whose Horner step (k_ml_horner) gives the segment's partial.  This is the
// batch form of blst's miller_loop_n over every pair of a multi_verify
// (reference bls/src/signature.rs:117-126).
#pragma once

#include <algorithm>
#include <cstddef>
#include <cstdint>
#include <vector>

namespace gbls {

constexpr uint32_t kTableWave = 64;  // lanes per k_ml_group wave (gbls_common.h WG)

// Line columns (pair j of group g at j ngp + g) cost ncol = gmax x ngp columns of line buffer;
// with uneven groups (one big segment beside many 1-2 pair segments) that can be many times the
// pair count, so the column layout is used only while ncol <= kColSlack4 / 4 x npairs or
// ncol <= npairs + kColPad (small launches: the wave padding), else the lines stay pair-indexed;
// the line buffer stays within 1.25x the budget the event slices were sized for (+ the pad).
constexpr uint64_t kColSlack4 = 5;
constexpr uint64_t kColPad = 4096;

struct MlTables {
  struct Level {
    size_t tab_off, nin, nout;
  };
  size_t plist_off = 0, grp_off = 0, ngroup = 0, v0_n = 1, v1_n = 1;
  std::vector<Level> levels;
  uint32_t G = 1;  // pairs per k_ml_group lane (at most)
  // the lines' column table (col_off: npairs entries, col[pair] = j ngp + g for pair j of group
  // g), ngp = groups rounded up to a wave, ncol = ngp x the largest group; ngp = 0: the lines
  // stay pair-indexed (col_off unset, ncol = npairs)
  size_t col_off = 0;
  uint32_t ngp = 0, ncol = 0;
};

// count(s): pairs of Miller segment s (>= 1); emit(s, tab): appends their pair indices.
// npairs: pairs listed; EC: events per launch (line slices); nsimd: SIMDs of the device;
// ml_rounds: k_ml_group waves per SIMD for large launches; ml_g: forced G (0: chosen).
template <class Count, class Emit>
MlTables ml_tables(std::vector<uint32_t> &tab, size_t nms, size_t npairs, int EC, uint32_t nsimd,
                   uint32_t ml_rounds, uint32_t ml_g, Count count, Emit emit) {
  MlTables mt;
  // G, the pairs per k_ml_group lane.  Small launches: the largest power of two <= 64 that
  // still gives >= 65536 lanes per launch (EC events).  Large launches: the smallest G
  // whose launch is at most ml_rounds waves per SIMD, EC x ceil(groups / 64) waves, so that
  // the waves fill whole rounds of the chip's SIMDs (a launch just past a multiple of them
  // idles most of the chip for one more wave-duration, at one wave per SIMD).
  uint32_t G = 1;
  while (G < 64 && (uint64_t)EC * npairs / (2 * G) >= 65536) G *= 2;
  {
    auto waves = [&](uint32_t gs) {
      uint64_t ng = 0;
      for (size_t s = 0; s < nms; s++) ng += (count(s) + gs - 1) / gs;
      return (uint64_t)EC * ((ng + kTableWave - 1) / kTableWave);
    };
    const uint64_t cap = (uint64_t)ml_rounds * nsimd;
    uint32_t lo = 1, hi = (uint32_t)std::max<size_t>(npairs, 1);  // smallest G with waves(G) <= cap
    while (lo < hi) {
      uint32_t mid = lo + (hi - lo) / 2;
      if (waves(mid) <= cap)
        hi = mid;
      else
        lo = mid + 1;
    }
    // (when even one group per segment exceeds the cap, e.g. thousands of tiny segments beside
    // a large one, the search ends at G = npairs: keep the lane-count rule's G instead of
    // serialising the large segment in one lane)
    if (lo >= 8 && waves(lo) <= cap) G = lo;
  }
  if (ml_g) G = ml_g;
  mt.G = G;
  mt.plist_off = tab.size();
  for (size_t s = 0; s < nms; s++) emit(s, tab);
  mt.grp_off = tab.size();
  std::vector<uint32_t> cnt(nms);
  uint32_t at = 0;
  for (size_t s = 0; s < nms; s++) {
    const uint32_t m = count(s), ng = (m + G - 1) / G;
    for (uint32_t k = 0; k < ng; k++) {
      tab.push_back(at + k);
      tab.push_back(ng);
      tab.push_back((m - k + ng - 1) / ng);
    }
    cnt[s] = ng;
    at += m;
  }
  mt.ngroup = (tab.size() - mt.grp_off) / 3;
  size_t cur_n = mt.ngroup;
  while (nms && *std::max_element(cnt.begin(), cnt.end()) > 1) {
    MlTables::Level L{tab.size(), cur_n, 0};
    size_t in_base = 0;
    std::vector<uint32_t> next(nms);
    for (size_t s = 0; s < nms; s++) {
      const uint32_t k = cnt[s];
      for (uint32_t q = 0; q < k; q += 4) {
        tab.push_back((uint32_t)(in_base + q));
        tab.push_back(std::min<uint32_t>(4, k - q));
        next[s]++;
      }
      in_base += k;
    }
    L.nout = (tab.size() - L.tab_off) / 2;
    mt.levels.push_back(L);
    cnt = next;
    cur_n = L.nout;
  }
  mt.v0_n = mt.ngroup;
  for (size_t l = 0; l < mt.levels.size(); l++)
    (l & 1 ? mt.v0_n : mt.v1_n) = std::max(l & 1 ? mt.v0_n : mt.v1_n, mt.levels[l].nout);
  // line columns: pair j of group g at j ngp + g, so that a wave of k_ml_group (64 consecutive
  // groups from a multiple of 64) reads 64 consecutive, 256-byte-aligned words per load
  uint32_t gmax = 0;
  for (size_t q = 0; q < mt.ngroup; q++) gmax = std::max(gmax, tab[mt.grp_off + 3 * q + 2]);
  const uint32_t ngp = (uint32_t)((mt.ngroup + kTableWave - 1) / kTableWave * kTableWave);
  mt.ncol = (uint32_t)npairs;
  const uint64_t cols = (uint64_t)gmax * ngp;
  if (mt.ngroup && cols < (1ull << 32) && (4 * cols <= kColSlack4 * (uint64_t)npairs || cols <= npairs + kColPad)) {
    const size_t off = tab.size();
    tab.resize(off + npairs, 0xffffffffu);
    bool ok = true;
    for (size_t q = 0; q < mt.ngroup && ok; q++) {
      const uint32_t a = tab[mt.grp_off + 3 * q], st = tab[mt.grp_off + 3 * q + 1],
                     c = tab[mt.grp_off + 3 * q + 2];
      for (uint32_t j = 0; j < c; j++) {
        const uint32_t pair = tab[mt.plist_off + a + (size_t)j * st];
        if (pair >= npairs || tab[off + pair] != 0xffffffffu) {
          ok = false;
          break;
        }
        tab[off + pair] = j * ngp + (uint32_t)q;
      }
    }
    for (size_t p = 0; ok && p < npairs; p++) ok = tab[off + p] != 0xffffffffu;
    if (ok) {  // every pair listed exactly once
      mt.col_off = off;
      mt.ngp = ngp;
      mt.ncol = (uint32_t)cols;
    } else {
      tab.resize(off);
    }
  }
  return mt;
}

}  // namespace gbls
