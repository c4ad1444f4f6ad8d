// Native multi-threaded CSV reader for Barra-format panels (barra_data_csi.csv, factor dumps).
//
// The reference reads its 401,749 x 15 panel with pandas (Barra-master/demo.py:22) and loads
// Mongo collections into DataFrames (Barra_factor_cal/load_data.py:27-39).  This host-side
// runtime component memory-maps the file, splits it into line-aligned chunks, and parses every
// chunk on its own std::thread straight into caller-allocated columnar buffers:
//   type 0 = float64 (empty / "nan" -> NaN), 1 = fixed-width string (16 bytes, NUL padded),
//   type 2 = date -> int32 YYYYMMDD (accepts YYYY/MM/DD, YYYY-MM-DD, YYYYMMDD),
//   type 3 = float32: parsed as float64, then rounded to float32 -- the reference's load-time
//            downcast (Barra_factor_cal/load_data.py:13-25, quirk Q27), done while parsing so the
//            device upload moves half the bytes (and, into pinned buffers, by DMA).
// C ABI for ctypes; no Python objects are touched.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#include "row_index.h"

namespace {

struct Map {
  const char* p = nullptr;
  size_t n = 0;
  int fd = -1;
  bool open(const char* path) {
    fd = ::open(path, O_RDONLY);
    if (fd < 0) return false;
    struct stat st;
    if (fstat(fd, &st) != 0) return false;
    n = (size_t)st.st_size;
    if (n == 0) return true;
    void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) return false;
    p = (const char*)m;
    madvise(m, n, MADV_SEQUENTIAL);
    return true;
  }
  ~Map() {
    if (p) munmap((void*)p, n);
    if (fd >= 0) ::close(fd);
  }
};

inline const char* next_line(const char* s, const char* e) {
  const void* nl = memchr(s, '\n', (size_t)(e - s));
  return nl ? (const char*)nl + 1 : e;
}

double parse_double(const char* s, const char* e) {
  while (s < e && (*s == ' ' || *s == '"')) ++s;
  while (e > s && (e[-1] == ' ' || e[-1] == '"' || e[-1] == '\r')) --e;
  if (s == e) return NAN;
  char buf[64];
  size_t len = (size_t)(e - s);
  if (len >= sizeof(buf)) len = sizeof(buf) - 1;
  memcpy(buf, s, len);
  buf[len] = 0;
  char* end = nullptr;
  const double v = strtod(buf, &end);
  return end == buf ? NAN : v;
}

int32_t parse_date(const char* s, const char* e) {
  int32_t v = 0, nd = 0;
  for (; s < e; ++s) {
    if (*s >= '0' && *s <= '9') { v = v * 10 + (*s - '0'); ++nd; }
    else if (*s == ' ' || *s == '\r' || *s == '"') continue;
    else if (nd >= 8) break;  // time part after the date
  }
  // handle Y/M/D without zero padding is not supported: Barra dates are zero padded
  return nd >= 8 ? v / (int32_t)std::pow(10, nd - 8) : -1;
}

// ix (optional): the row-group index chunk of this range, fed each row right after it is parsed
// (its code and date are still in cache); kc / dc = the code and date columns.
void parse_range(const char* s, const char* e, int64_t row0, int ncol, const int* types,
                 void** outs, mfa_ix::Chunk* ix = nullptr, int kc = -1, int dc = -1,
                 uint8_t* mask = nullptr) {
  int64_t r = row0;
  while (s < e) {
    const char* le = next_line(s, e);
    const char* line_end = le;
    while (line_end > s && (line_end[-1] == '\n' || line_end[-1] == '\r')) --line_end;
    if (line_end == s) { s = le; continue; }
    const char* f = s;
    for (int c = 0; c < ncol; ++c) {
      const char* fe = f;
      while (fe < line_end && *fe != ',') ++fe;
      switch (types[c]) {
        case 0: ((double*)outs[c])[r] = parse_double(f, fe); break;
        case 1: {
          char* dst = (char*)outs[c] + r * 16;
          memset(dst, 0, 16);
          const char* a = f;
          const char* b = fe;
          while (a < b && (*a == '"' || *a == ' ')) ++a;
          while (b > a && (b[-1] == '"' || b[-1] == ' ' || b[-1] == '\r')) --b;
          memcpy(dst, a, (size_t)((b - a) < 16 ? (b - a) : 16));
          break;
        }
        case 2: ((int32_t*)outs[c])[r] = parse_date(f, fe); break;
        case 3: ((float*)outs[c])[r] = (float)parse_double(f, fe); break;
        default: break;
      }
      f = fe < line_end ? fe + 1 : line_end;
    }
    if (ix) ix->row((const uint8_t*)outs[kc], (const int32_t*)outs[dc], r, mask);
    ++r;
    s = le;
  }
}

}  // namespace

extern "C" {

// Number of data rows (excluding the header) and columns of the header line; -1 on error.
__attribute__((visibility("default"))) int64_t mfa_csv_shape(const char* path, int* ncol) {
  Map m;
  if (!m.open(path)) return -1;
  if (m.n == 0) { *ncol = 0; return 0; }
  const char* e = m.p + m.n;
  const char* h = next_line(m.p, e);
  int c = 1;
  for (const char* q = m.p; q < h; ++q) c += (*q == ',');
  *ncol = c;
  // parallel newline count
  const int nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<int64_t> cnt(nt, 0);
  std::vector<std::thread> th;
  const size_t body = (size_t)(e - h);
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      const char* a = h + body * t / nt;
      const char* b = h + body * (t + 1) / nt;
      int64_t k = 0;
      for (const char* q = a; q < b; ++q) k += (*q == '\n');
      cnt[t] = k;
    });
  for (auto& x : th) x.join();
  int64_t rows = 0;
  for (auto k : cnt) rows += k;
  if (m.n > 0 && e[-1] != '\n') rows += 1;  // last line without newline
  return rows;
}

}  // extern "C"

namespace {

int64_t parse_file(const char* path, int ncol, const int* types, void** outs, int nthreads,
                   int kc, int dc, uint8_t* mask, void** index) {
  Map m;
  if (!m.open(path)) return -1;
  if (m.n == 0) return 0;
  const char* e = m.p + m.n;
  const char* h = next_line(m.p, e);
  const int nt = nthreads > 0 ? nthreads
                              : (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  // line-aligned chunk boundaries
  std::vector<const char*> b(nt + 1);
  b[0] = h;
  b[nt] = e;
  const size_t body = (size_t)(e - h);
  for (int t = 1; t < nt; ++t) {
    const char* q = h + body * t / nt;
    if (q < b[t - 1]) q = b[t - 1];
    b[t] = q > h ? next_line(q - 1, e) : h;
  }
  // rows before each chunk
  std::vector<int64_t> start(nt + 1, 0);
  {
    std::vector<std::thread> th;
    std::vector<int64_t> cnt(nt, 0);
    for (int t = 0; t < nt; ++t)
      th.emplace_back([&, t] {
        int64_t k = 0;
        for (const char* q = b[t]; q < b[t + 1];) {
          const char* le = next_line(q, b[t + 1]);
          const char* x = le;
          while (x > q && (x[-1] == '\n' || x[-1] == '\r')) --x;
          if (x > q) ++k;
          q = le;
        }
        cnt[t] = k;
      });
    for (auto& x : th) x.join();
    for (int t = 0; t < nt; ++t) start[t + 1] = start[t] + cnt[t];
  }
  const bool want_ix = index && kc >= 0 && dc >= 0 && mask;
  std::vector<mfa_ix::Chunk> ch(want_ix ? nt : 0);
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      mfa_ix::Chunk* c = want_ix ? &ch[t] : nullptr;
      if (c) c->r0 = start[t];
      parse_range(b[t], b[t + 1], start[t], ncol, types, outs, c, kc, dc, mask);
    });
  for (auto& x : th) x.join();
  if (want_ix) *index = mfa_ix::merge(ch, (const uint8_t*)outs[kc], (const int32_t*)outs[dc]);
  return start[nt];
}

}  // namespace

extern "C" {

// Parse all data rows into caller buffers outs[c] (typed by types[c]); returns rows parsed.
__attribute__((visibility("default"))) int64_t mfa_csv_parse(const char* path, int ncol,
                                                              const int* types, void** outs,
                                                              int nthreads) {
  return parse_file(path, ncol, types, outs, nthreads, -1, -1, nullptr, nullptr);
}

// mfa_csv_parse + the row-group index of the parsed rows (row_index.h), built while parsing:
// kc = the code column (type 1), dc = the trade-date column (type 2), mask = caller's
// mfa_date_span() zeroed bytes; *index = a handle for mfa_row_index_* (csrc_host/shard_rows.cpp).
__attribute__((visibility("default"))) int64_t mfa_csv_parse_ix(const char* path, int ncol,
                                                                 const int* types, void** outs,
                                                                 int nthreads, int kc, int dc,
                                                                 uint8_t* mask, void** index) {
  *index = nullptr;
  if (kc < 0 || dc < 0 || kc >= ncol || dc >= ncol || types[kc] != 1 || types[dc] != 2)
    return parse_file(path, ncol, types, outs, nthreads, -1, -1, nullptr, nullptr);
  return parse_file(path, ncol, types, outs, nthreads, kc, dc, mask, index);
}

}  // extern "C"
