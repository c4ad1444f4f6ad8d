// Sanitizer harness for the native host runtime (csrc_host/*.cpp): built by
// tests/test_host_sanitizers.py with -fsanitize=address,undefined and, separately,
// -fsanitize=thread (the CSV reader and the as-of join are multi-threaded), then run on CPU.
//
// Exercises: CSV edge cases (CRLF, empty and "nan" fields, long strings truncated to the
// 16-byte slot, three date spellings, no trailing newline, chunk boundaries at every thread
// count) and the as-of join against a brute-force oracle on random sorted groups.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

extern "C" {
int64_t mfa_csv_shape(const char* path, int* ncol);
int64_t mfa_csv_parse(const char* path, int ncol, const int* types, void** outs, int nthreads);
int mfa_asof_join(const int32_t* lg, const int64_t* lk, int64_t nl, const int32_t* rg,
                  const int64_t* rk, int64_t nr, int64_t* out, int nthreads);
int mfa_write_matrix_csv(const char* path, const char* header, const char* const* labels,
                         long long rows, long long cols, const float* data, int nthreads);
}

static int fails = 0;
#define CHECK(c)                                                    \
  do {                                                              \
    if (!(c)) {                                                     \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++fails;                                                      \
    }                                                               \
  } while (0)

static void csv_case(const char* path, int rows, bool crlf, bool trailing_nl) {
  FILE* f = std::fopen(path, "wb");
  const char* eol = crlf ? "\r\n" : "\n";
  std::fprintf(f, "date,stocknames,capital,ret%s", eol);
  for (int i = 0; i < rows; ++i) {
    const int y = 2020 + i % 5, m = 1 + i % 12, d = 1 + i % 28;
    char date[32];
    if (i % 3 == 0) std::snprintf(date, sizeof date, "%04d/%02d/%02d", y, m, d);
    else if (i % 3 == 1) std::snprintf(date, sizeof date, "%04d-%02d-%02d", y, m, d);
    else std::snprintf(date, sizeof date, "%04d%02d%02d", y, m, d);
    std::string name = (i % 7 == 0) ? "a_very_long_stock_name_beyond_16_bytes" : "0000" + std::to_string(i) + ".SZ";
    const bool last = i == rows - 1;
    if (i % 11 == 0)
      std::fprintf(f, "%s,%s,,nan%s", date, name.c_str(), (last && !trailing_nl) ? "" : eol);
    else
      std::fprintf(f, "%s,%s,%.6f,%.6f%s", date, name.c_str(), 1000.0 + i, 0.001 * (i % 13),
                   (last && !trailing_nl) ? "" : eol);
  }
  std::fclose(f);
  int ncol = 0;
  const int64_t n = mfa_csv_shape(path, &ncol);
  CHECK(ncol == 4);
  CHECK(n == rows);
  for (int nt : {1, 2, 3, 7, 16}) {
    std::vector<int32_t> dates(rows);
    std::vector<char> names((size_t)rows * 16);
    std::vector<double> cap(rows), ret(rows);
    const int types[4] = {2, 1, 0, 0};
    void* outs[4] = {dates.data(), names.data(), cap.data(), ret.data()};
    const int64_t got = mfa_csv_parse(path, 4, types, outs, nt);
    CHECK(got == rows);
    for (int i = 0; i < rows; ++i) {
      const int y = 2020 + i % 5, m = 1 + i % 12, d = 1 + i % 28;
      CHECK(dates[i] == y * 10000 + m * 100 + d);
      if (i % 11 == 0) {
        CHECK(std::isnan(cap[i]) && std::isnan(ret[i]));
      } else {
        CHECK(std::fabs(cap[i] - (1000.0 + i)) < 1e-9);
        CHECK(std::fabs(ret[i] - 0.001 * (i % 13)) < 1e-9);
      }
      CHECK(strnlen(&names[(size_t)i * 16], 16) >= 1);  // fixed 16-byte slot, NUL-padded when shorter
    }
  }
}

static void asof_case(unsigned seed, int groups, int nl_per, int nr_per, int nt) {
  std::mt19937 rng(seed);
  std::vector<int32_t> lg, rg;
  std::vector<int64_t> lk, rk;
  for (int g = 0; g < groups; ++g) {
    const int nl = rng() % (nl_per + 1), nr = rng() % (nr_per + 1);
    int64_t k = rng() % 10;
    for (int i = 0; i < nl; ++i) { k += rng() % 3; lg.push_back(g); lk.push_back(k); }
    k = rng() % 10;
    for (int i = 0; i < nr; ++i) { k += rng() % 4; rg.push_back(g); rk.push_back(k); }
  }
  const int64_t nl = (int64_t)lg.size(), nr = (int64_t)rg.size();
  std::vector<int64_t> out(nl, -2);
  mfa_asof_join(lg.data(), lk.data(), nl, rg.data(), rk.data(), nr, out.data(), nt);
  for (int64_t i = 0; i < nl; ++i) {
    int64_t best = -1;
    for (int64_t j = 0; j < nr; ++j)
      if (rg[j] == lg[i] && rk[j] <= lk[i]) best = j;  // last match (ties -> last)
    CHECK(out[i] == best);
  }
}

// Matrix writer: multi-threaded row blocks (64 rows) written in order; special values; the
// result re-read through the native parser must round-trip every finite value exactly.
static void write_case(const char* path, int rows, int cols, int nt) {
  std::mt19937 rng(rows * 31 + cols);
  std::vector<float> v((size_t)rows * cols);
  for (auto& x : v) x = std::ldexp((float)(rng() % 2000001) - 1000000.0f, (int)(rng() % 60) - 50);
  if (!v.empty()) v[0] = std::nanf("");
  if (v.size() > 1) v[1] = -0.0f;
  std::vector<std::string> lab(rows);
  std::vector<const char*> lp(rows);
  for (int r = 0; r < rows; ++r) { lab[r] = std::to_string(20200000 + r); lp[r] = lab[r].c_str(); }
  std::string header = "date";
  for (int c = 0; c < cols; ++c) header += ",c" + std::to_string(c);
  CHECK(mfa_write_matrix_csv(path, header.c_str(), lp.data(), rows, cols, v.data(), nt) == 0);
  int ncol = 0;
  const int64_t n = mfa_csv_shape(path, &ncol);
  CHECK(n == rows && ncol == cols + 1);
  if (n != rows || ncol != cols + 1) return;
  std::vector<int> types(ncol, 0);
  std::vector<std::vector<double>> buf(ncol, std::vector<double>(rows));
  std::vector<void*> outs(ncol);
  for (int c = 0; c < ncol; ++c) outs[c] = buf[c].data();
  CHECK(mfa_csv_parse(path, ncol, types.data(), outs.data(), nt) == rows);
  for (int r = 0; r < rows; ++r)
    for (int c = 0; c < cols; ++c) {
      const float x = v[(size_t)r * cols + c], y = (float)buf[c + 1][r];
      CHECK(std::isnan(x) ? std::isnan(y) : x == y);
    }
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  const std::string p = dir + "/mfa_san.csv";
  csv_case(p.c_str(), 1, false, false);
  csv_case(p.c_str(), 97, false, true);
  csv_case(p.c_str(), 1000, true, true);
  csv_case(p.c_str(), 1001, true, false);
  for (unsigned s = 0; s < 6; ++s)
    for (int nt : {1, 2, 5, 16}) asof_case(s, 1 + s * 7, 40, 12, nt);
  asof_case(99, 0, 1, 1, 4);
  for (int nt : {1, 3, 8}) write_case(p.c_str(), 130, 17, nt);
  write_case(p.c_str(), 1, 1, 2);
  std::remove(p.c_str());
  std::printf("host runtime sanitizer check: %s (%d failures)\n", fails ? "FAIL" : "ok", fails);
  return fails ? 1 : 0;
}
