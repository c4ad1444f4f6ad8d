// Row-group index of a loader panel whose rows are grouped by stock code (ascending) with
// strictly ascending trade dates inside a stock -- the stored panel's order.
//
// The index is what every date-sharded rank needs before it can pick its rows
// (csrc_host/shard_rows.cpp): the first row of every stock segment (segment k = global stock id
// k) and the set of trade dates (a byte mask over YYYYMMDD, from which every rank derives the
// same global date axis without a collective), plus the check that the order holds.  The CSV
// reader builds it while it parses (csv_panel.cpp, mfa_csv_parse_ix: the row's code and date
// are still in cache), so the per-rank selection never scans the 16-byte code column again;
// mfa_row_index builds it in one threaded pass over columns from any other source.
#pragma once
#include <cstdint>
#include <cstring>
#include <vector>

namespace mfa_ix {

constexpr int32_t kDateLo = 19000101, kDateHi = 21000101;  // mask span of YYYYMMDD ints

inline int cmp16(const uint8_t* a, const uint8_t* b) { return std::memcmp(a, b, 16); }
// equality of two 16-byte codes as two 8-byte words
inline bool eq16(const uint8_t* a, const uint8_t* b) {
  uint64_t a0, a1, b0, b1;
  std::memcpy(&a0, a, 8);
  std::memcpy(&a1, a + 8, 8);
  std::memcpy(&b0, b, 8);
  std::memcpy(&b1, b + 8, 8);
  return ((a0 ^ b0) | (a1 ^ b1)) == 0;
}

// One thread's contiguous share [r0, r1) of the rows, fed row by row in order.
struct Chunk {
  std::vector<int64_t> first;  // segment starts seen in the chunk (r0 always, settled at merge)
  int64_t r0 = 0;
  int err = 0;  // -1 order violated, -2 trade date outside the mask span
  void row(const uint8_t* codes, const int32_t* dates, int64_t r, uint8_t* mask) {
    const int32_t d = dates[r];
    if (d < kDateLo || d >= kDateHi) {
      err = err ? err : -2;
      return;
    }
    // test before storing: after a date's first sighting its line stays shared between the
    // threads' caches instead of bouncing on every row
    if (!mask[d - kDateLo]) mask[d - kDateLo] = 1;
    if (r == r0) {
      first.push_back(r);
      return;
    }
    const uint8_t* c = codes + 16 * r;
    if (eq16(c, c - 16)) {
      if (d <= dates[r - 1]) err = err ? err : -1;
    } else {
      if (cmp16(c, c - 16) < 0) err = err ? err : -1;
      first.push_back(r);
    }
  }
};

// Owned by the caller through an opaque handle (the segment count is not known in advance).
struct Index {
  std::vector<int64_t> seg_first;
  int err = 0;
};

// Concatenate the chunks (ascending r0), settling each chunk's first row against the row
// before it.
inline Index* merge(std::vector<Chunk>& ch, const uint8_t* codes, const int32_t* dates) {
  auto* ix = new Index;
  size_t n = 0;
  for (auto& c : ch) n += c.first.size();
  ix->seg_first.reserve(n);
  for (size_t t = 0; t < ch.size(); ++t) {
    Chunk& c = ch[t];
    if (c.err && !ix->err) ix->err = c.err;
    if (c.first.empty()) continue;
    size_t k0 = 0;
    const int64_t r = c.first[0];
    if (r > 0) {
      const uint8_t* a = codes + 16 * r;
      if (eq16(a, a - 16)) {
        if (dates[r] <= dates[r - 1] && !ix->err) ix->err = -1;
        k0 = 1;  // continues the previous chunk's segment
      } else if (cmp16(a, a - 16) < 0 && !ix->err) {
        ix->err = -1;
      }
    }
    ix->seg_first.insert(ix->seg_first.end(), c.first.begin() + k0, c.first.end());
  }
  return ix;
}

}  // namespace mfa_ix
