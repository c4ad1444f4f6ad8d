// Multi-threaded writer of a labelled float32 matrix as CSV, in pandas ``DataFrame.to_csv``'s
// text format.  Used for the demo.py outputs whose size scales with stocks x dates
// (specific_returns.csv: 2520 x 5000 = 156 MB; pandas takes 6-30 s, mostly float formatting).
//
// Value text = numpy's float32 repr, which pandas writes: shortest round-trip digits,
// positional for 1e-4 <= |x| < 1e16 (with a trailing ".0" on integral values) and scientific
// ("1.2e-05") otherwise.  NaN = empty field (pandas na_rep="").  Labels are written verbatim:
// the caller falls back to pandas when one would need CSV quoting.
//
// Rows are formatted into per-thread buffers in parallel, then written in order.
#include <charconv>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

void put_float(std::string& out, float v) {
  if (std::isnan(v)) return;
  if (std::isinf(v)) {
    out.append(v > 0 ? "inf" : "-inf");
    return;
  }
  char buf[64];
  // shortest round-trip digits, as d.ddde[+-]XX
  const std::to_chars_result r = std::to_chars(buf, buf + sizeof(buf) - 1, v, std::chars_format::scientific);
  *r.ptr = '\0';  // to_chars does not terminate; atoi below reads the exponent
  const double a = std::fabs((double)v);  // numpy compares the float's exact value
  if (!(a == 0.0 || (a >= 1e-4 && a < 1e16))) {
    out.append(buf, r.ptr);
    return;
  }
  // positional: the same shortest digits, zero padded (numpy format_float_positional)
  const char* p = buf;
  if (*p == '-') out.push_back(*p++);
  char dig[32];
  int nd = 0;
  while (p < r.ptr && *p != 'e') {
    if (*p != '.') dig[nd++] = *p;
    ++p;
  }
  const int ex = (p < r.ptr) ? std::atoi(p + 1) : 0;
  if (ex >= 0) {
    for (int i = 0; i <= ex; ++i) out.push_back(i < nd ? dig[i] : '0');
    out.push_back('.');
    if (nd > ex + 1) out.append(dig + ex + 1, nd - ex - 1);
    else out.push_back('0');
  } else {
    out.append("0.");
    out.append((size_t)(-ex - 1), '0');
    out.append(dig, nd);
  }
}

}  // namespace

extern "C" {

// header: the first line without its newline.  labels: `rows` NUL-terminated row labels.
// data: row-major [rows][cols] float32.  Returns 0, or -1 if the file cannot be written.
__attribute__((visibility("default"))) int mfa_write_matrix_csv(const char* path,
                                                                const char* header,
                                                                const char* const* labels,
                                                                long long rows, long long cols,
                                                                const float* data, int nthreads) {
  FILE* fh = std::fopen(path, "wb");
  if (!fh) return -1;
  std::fputs(header, fh);
  std::fputc('\n', fh);
  int nt = nthreads > 0 ? nthreads : (int)std::thread::hardware_concurrency();
  if (nt < 1) nt = 1;
  if (nt > 64) nt = 64;
  // blocks of rows: each block formatted by one thread, blocks written in order
  const long long blk = 64;
  const long long nblk = (rows + blk - 1) / blk;
  std::vector<std::string> bufs(nblk);
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t) {
    th.emplace_back([&, t]() {
      for (long long b = t; b < nblk; b += nt) {
        std::string& s = bufs[b];
        const long long r1 = (b + 1) * blk < rows ? (b + 1) * blk : rows;
        s.reserve((size_t)(r1 - b * blk) * (size_t)cols * 13);
        for (long long r = b * blk; r < r1; ++r) {
          s.append(labels[r]);
          const float* row = data + r * cols;
          for (long long c = 0; c < cols; ++c) {
            s.push_back(',');
            put_float(s, row[c]);
          }
          s.push_back('\n');
        }
      }
    });
  }
  for (auto& x : th) x.join();
  int rc = 0;
  for (auto& s : bufs)
    if (std::fwrite(s.data(), 1, s.size(), fh) != s.size()) rc = -1;
  if (std::fclose(fh) != 0) rc = -1;
  return rc;
}

}  // extern "C"
