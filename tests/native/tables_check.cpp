// CPU check of the Miller product tables (grandine_amd/csrc/gbls_tables.h), run by
// tests/test_host_sanitizers.py under ASan/UBSan.  The invariants the kernels rely on:
//   * every pair of every segment appears exactly once in the pair list and in one group;
//   * groups of a segment hold <= G pairs and the reduction levels end in one value per segment;
//   * with the line-column layout, the column of pair j of group g is j ngp + g and is < ncol;
//   * the line buffer, ncol x EC x 72 words, stays within 1.25x the budget EC was sized for,
//     also when one large segment sits beside many tiny ones (the column layout
//     with ncol = gmax x ngp could exceed the budget several times over).
#include <cassert>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "gbls_tables.h"

using namespace gbls;

static int fails = 0;
#define CHECK(c)                                                     \
  do {                                                               \
    if (!(c)) {                                                      \
      std::fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); \
      fails++;                                                       \
    }                                                                \
  } while (0)

// segments of the given set counts, X extra pairs each (pipeline_partials' layout: the sets'
// pairs [0, n), then the extra pairs n + s X + k)
static void run(const char *name, const std::vector<uint32_t> &sizes, uint32_t X, uint64_t budget) {
  const size_t nseg = sizes.size();
  std::vector<uint32_t> off(nseg + 1, 0);
  for (size_t s = 0; s < nseg; s++) off[s + 1] = off[s] + sizes[s];
  const size_t n = off[nseg], np = n + nseg * X;
  const uint64_t event_bytes = (uint64_t)np * 72 * 4;
  int EC = 68;
  if (event_bytes * 68 > budget) EC = (int)std::max<uint64_t>(1, budget / event_bytes);
  std::vector<uint32_t> tab;
  MlTables mt = ml_tables(
      tab, nseg, np, EC, 1024, 2, 0, [&](size_t s) { return sizes[s] + X; },
      [&](size_t s, std::vector<uint32_t> &t) {
        for (uint32_t i = off[s]; i < off[s + 1]; i++) t.push_back(i);
        for (uint32_t k = 0; k < X; k++) t.push_back((uint32_t)(n + s * X + k));
      });
  // groups: every pair once, <= G per group
  std::vector<int> seen(np, 0);
  for (size_t q = 0; q < mt.ngroup; q++) {
    const uint32_t a = tab[mt.grp_off + 3 * q], st = tab[mt.grp_off + 3 * q + 1], c = tab[mt.grp_off + 3 * q + 2];
    CHECK(c >= 1 && c <= mt.G);
    for (uint32_t j = 0; j < c; j++) {
      const uint32_t pair = tab[mt.plist_off + a + (size_t)j * st];
      CHECK(pair < np);
      if (pair < np) seen[pair]++;
      if (mt.ngp) {
        const uint32_t col = tab[mt.col_off + pair];
        CHECK(col == j * mt.ngp + (uint32_t)q);
        CHECK(col < mt.ncol);
      }
    }
  }
  for (size_t p = 0; p < np; p++) CHECK(seen[p] == 1);
  // reduction levels: the last one has one output per segment
  if (!mt.levels.empty()) CHECK(mt.levels.back().nout == nseg);
  else CHECK(mt.ngroup == nseg);
  // the line buffer bound
  const uint64_t line_bytes = (uint64_t)mt.ncol * EC * 72 * 4;
  const uint64_t bound = std::max<uint64_t>(budget, event_bytes) * 5 / 4 + (uint64_t)4096 * EC * 72 * 4;
  // no lane multiplies more than 4096 pairs (a segment is split into groups)
  CHECK(mt.G <= 4096);
  CHECK(line_bytes <= bound);
  CHECK(mt.ncol >= np);
  std::printf("%-10s nseg %6zu pairs %8zu EC %2d G %3u ngroup %6zu ncol %8u (%s) lines %.1f MB (bound %.1f MB)\n",
              name, nseg, np, EC, mt.G, mt.ngroup, mt.ncol, mt.ngp ? "columns" : "pair-indexed",
              line_bytes / 1e6, bound / 1e6);
}

int main() {
  const uint64_t GB4 = 4ull << 30;
  // C2: 16 batches of 4096 sets, 208 MSM pairs each
  run("c2", std::vector<uint32_t>(16, 4096), 208, GB4);
  // a single batch, a block (131 sets, one extra pair)
  run("c2-one", {4096}, 208, GB4);
  run("block", {131}, 1, GB4);
  // C5 sliced: 2^20 sets in 16 segments under a 4 GB budget
  run("c5", std::vector<uint32_t>(16, 65536), 5, GB4);
  // mixed: one 65536-set segment beside 4000 one- and two-set segments (coalesced gossip),
  // under a small budget -- the uneven groups that made gmax x ngp blow past the budget
  {
    std::vector<uint32_t> sz{65536};
    for (int i = 0; i < 4000; i++) sz.push_back(1 + (i & 1));
    run("mixed", sz, 1, 256ull << 20);
    run("mixed-4G", sz, 1, GB4);
  }
  {
    std::vector<uint32_t> sz;
    for (int i = 0; i < 64; i++) sz.push_back(i % 8 == 0 ? 8192 : 3);
    run("mixed-2", sz, 1, 64ull << 20);
  }
  if (fails) {
    std::printf("tables_check: %d failures\n", fails);
    return 1;
  }
  std::printf("tables_check: OK\n");
  return 0;
}
