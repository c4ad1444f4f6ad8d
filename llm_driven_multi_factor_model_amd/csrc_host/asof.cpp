// Point-in-time as-of join (K12) for statement -> daily-price alignment.
//
// Reference: Barra_factor_cal/load_data.py:41-62 (robust_merge_asof): for every ts_code, a
// pandas merge_asof(direction='backward') of the daily rows (left_on trade_date) onto the
// statement rows (right_on f_ann_date / ann_date), looping over stocks in Python.
//
// Here both sides arrive as (group code, int64 key) arrays sorted by (group, key); each thread
// takes a contiguous range of groups and runs a two-pointer sweep: for left row i the result is
// the LAST right row of the same group with right_key <= left_key (-1 if none), i.e. the most
// recently announced statement as of that trading day.  Ties among right rows resolve to the
// last one, as pandas merge_asof does.
#include <algorithm>
#include <cstdint>
#include <thread>
#include <vector>

extern "C" __attribute__((visibility("default"))) int mfa_asof_join(
    const int32_t* lg, const int64_t* lk, int64_t nl, const int32_t* rg, const int64_t* rk,
    int64_t nr, int64_t* out, int nthreads) {
  if (nl <= 0) return 0;
  const int nt = nthreads > 0 ? nthreads : (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  // split the LEFT rows at group boundaries
  std::vector<int64_t> cut(nt + 1, nl);
  cut[0] = 0;
  for (int t = 1; t < nt; ++t) {
    int64_t c = nl * t / nt;
    while (c < nl && c > 0 && lg[c] == lg[c - 1]) ++c;
    cut[t] = std::max(c, cut[t - 1]);
  }
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      int64_t a = cut[t], b = cut[t + 1];
      if (a >= b) return;
      // first right row of the first group in range
      int64_t j = std::lower_bound(rg, rg + nr, lg[a]) - rg;
      for (int64_t i = a; i < b; ++i) {
        const int32_t g = lg[i];
        while (j < nr && rg[j] < g) ++j;
        // advance within the group while right key <= left key
        int64_t best = -1;
        int64_t k = j;
        while (k < nr && rg[k] == g && rk[k] <= lk[i]) { best = k; ++k; }
        out[i] = best;
        // keys are sorted within the group: the next left row starts from the last match
        if (best >= 0) j = best;
      }
    });
  for (auto& x : th) x.join();
  return 0;
}
