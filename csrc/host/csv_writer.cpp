// Native CSV formatter for the per-epoch synthetic table (reference: `DataFrame.to_csv` after
// `Transform.inverse`, Server/dtds/distributed.py:584-590 and Server/dtds/data/utils/transform.py).
//
// Output matches pandas' default writer on the decoded frame byte for byte:
//   * floats: Python repr() (shortest round-trip digits; fixed notation when the decimal point
//     position is in (-4, 16], otherwise d.ddde[+-]XX with >= 2 exponent digits; "-0.0" kept);
//     NaN -> empty field (pandas na_rep)
//   * categoricals: vocabulary string of the integer code (QUOTE_MINIMAL quoting)
//   * non-negative columns: the caller maps v = exp(x) - 1 (ceil when v < 0) with numpy's exp --
//     libm's exp differs from numpy's in the last ulp for some inputs -- and v == -1 is written " "
// Rows are formatted in parallel by worker threads, in row chunks handed out in order, and the
// calling thread writes each chunk as soon as it is formatted (the file write overlaps the
// formatting of the later chunks instead of following all of it).
#include "csv_writer.h"

#include <algorithm>
#include <atomic>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <exception>
#include <future>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace fedtgan {
namespace {

// Python repr() of a double written at p (at most 26 bytes); returns the end.  NaN writes nothing
// (pandas na_rep).  Shortest round-trip digits from std::to_chars, laid out as repr does.
char* put_py_float(char* p, double x) {
  if (std::isnan(x)) return p;
  if (std::isinf(x)) {
    if (x < 0) *p++ = '-';
    std::memcpy(p, "inf", 3);
    return p + 3;
  }
  char buf[40];
  const auto res = std::to_chars(buf, buf + sizeof(buf), x, std::chars_format::scientific);
  // buf: [-]d[.ddd]e[+-]XX
  const char* q = buf;
  if (*q == '-') {
    *p++ = '-';
    ++q;
  }
  char digits[24];
  int nd = 0;
  for (; q < res.ptr && *q != 'e'; ++q)
    if (*q != '.') digits[nd++] = *q;
  int e10 = 0;
  if (q < res.ptr) {   // 'e', sign, digits
    ++q;
    const bool eneg = *q == '-';
    ++q;
    for (; q < res.ptr; ++q) e10 = e10 * 10 + (*q - '0');
    if (eneg) e10 = -e10;
  }
  while (nd > 1 && digits[nd - 1] == '0') --nd;   // (to_chars shortest never emits them; robustness)
  const int decpt = e10 + 1;                      // value = 0.d1d2... x 10^decpt
  if (decpt > -4 && decpt <= 16) {
    if (decpt <= 0) {
      *p++ = '0';
      *p++ = '.';
      for (int i = 0; i < -decpt; ++i) *p++ = '0';
      std::memcpy(p, digits, (size_t)nd);
      p += nd;
    } else if (decpt < nd) {
      std::memcpy(p, digits, (size_t)decpt);
      p += decpt;
      *p++ = '.';
      std::memcpy(p, digits + decpt, (size_t)(nd - decpt));
      p += nd - decpt;
    } else {
      std::memcpy(p, digits, (size_t)nd);
      p += nd;
      for (int i = 0; i < decpt - nd; ++i) *p++ = '0';
      *p++ = '.';
      *p++ = '0';
    }
  } else {
    *p++ = digits[0];
    if (nd > 1) {
      *p++ = '.';
      std::memcpy(p, digits + 1, (size_t)(nd - 1));
      p += nd - 1;
    }
    const int ex = decpt - 1;
    *p++ = 'e';
    *p++ = ex < 0 ? '-' : '+';
    const int ax = ex < 0 ? -ex : ex;
    if (ax >= 100) *p++ = (char)('0' + ax / 100);
    *p++ = (char)('0' + (ax / 10) % 10);
    *p++ = (char)('0' + ax % 10);
  }
  return p;
}

void append_py_float(std::string& out, double x) {
  char b[40];
  out.append(b, (size_t)(put_py_float(b, x) - b));
}

std::string quote_field(const std::string& s) {
  if (s.find_first_of(",\"\n\r") == std::string::npos) return s;
  std::string q = "\"";
  for (char ch : s) {
    if (ch == '"') q.push_back('"');
    q.push_back(ch);
  }
  q.push_back('"');
  return q;
}

void append_field(std::string& out, const std::string& s) { out += quote_field(s); }

}  // namespace

// Rows [r0, r1) into one string.  Every vocabulary entry is quoted once up front and each row is
// written through a raw pointer into a buffer sized for its worst case (26 bytes per number), so the
// hot loop does no allocation, no searching and no growing appends.
std::string format_csv_rows(const double* values, int64_t rows, int64_t cols, int64_t r0, int64_t r1,
                            const std::vector<int>& kinds, const std::vector<std::vector<std::string>>& vocabs) {
  (void)rows;
  std::vector<std::vector<std::string>> qv(vocabs.size());
  size_t row_max = 1;
  for (int64_t j = 0; j < cols; ++j) {
    size_t w = 26;
    if (kinds[(size_t)j] == 1) {
      w = 0;
      for (const auto& e : vocabs[(size_t)j]) {
        qv[(size_t)j].push_back(quote_field(e));
        w = std::max(w, qv[(size_t)j].back().size());
      }
    }
    row_max += w + 1;
  }
  std::string out;
  out.resize((size_t)(r1 - r0) * row_max);
  char* p = &out[0];
  for (int64_t r = r0; r < r1; ++r) {
    const double* row = values + r * cols;
    for (int64_t j = 0; j < cols; ++j) {
      if (j) *p++ = ',';
      const double x = row[j];
      switch (kinds[(size_t)j]) {
        case 1: {  // vocabulary
          const auto& voc = qv[(size_t)j];
          const int64_t k = (int64_t)x;
          if (k < 0 || k >= (int64_t)voc.size()) throw std::runtime_error("csv: category code out of range");
          const std::string& f = voc[(size_t)k];
          std::memcpy(p, f.data(), f.size());
          p += f.size();
          break;
        }
        case 2:    // non-negative column, already mapped by exp(x)-1 (+ceil) on the host with numpy's exp
          if (x == -1.0) *p++ = ' ';
          else p = put_py_float(p, x);
          break;
        default:
          p = put_py_float(p, x);
      }
    }
    *p++ = '\n';
  }
  out.resize((size_t)(p - out.data()));
  return out;
}

std::string format_py_float(double x) {
  std::string s;
  append_py_float(s, x);
  return s;
}

void write_csv_file(const std::string& path, const double* values, int64_t rows, int64_t cols,
                    const std::vector<std::string>& names, const std::vector<int>& kinds,
                    const std::vector<std::vector<std::string>>& vocabs, int threads) {
  if ((int64_t)kinds.size() != cols || (int64_t)names.size() != cols || (int64_t)vocabs.size() != cols)
    throw std::runtime_error("csv: column descriptor size mismatch");
  if (threads <= 0) {
    unsigned hc = std::thread::hardware_concurrency();
    threads = (int)std::min<unsigned>(hc ? hc : 4, 16);
  }
  const int64_t min_rows = 2048;
  threads = (int)std::max<int64_t>(1, std::min<int64_t>(threads, (rows + min_rows - 1) / min_rows));
  // ~4 chunks per thread (at least 512 rows each): the first chunk is ready after ~1/(4*threads) of
  // the formatting time, and the write of chunk c overlaps the formatting of chunks > c
  const int64_t chunk = std::max<int64_t>(512, (rows + 4 * threads - 1) / (4 * threads));
  const int nchunks = (int)std::max<int64_t>(1, (rows + chunk - 1) / chunk);
  std::vector<std::string> parts((size_t)nchunks);
  std::vector<std::promise<void>> ready((size_t)nchunks);
  std::vector<std::future<void>> done;
  done.reserve((size_t)nchunks);
  for (auto& r : ready) done.push_back(r.get_future());
  std::atomic<int> next{0};
  std::vector<std::thread> pool;
  for (int t = 0; t < threads; ++t) {
    pool.emplace_back([&]() {
      for (int c = next.fetch_add(1); c < nchunks; c = next.fetch_add(1)) {
        try {
          const int64_t r0 = (int64_t)c * chunk, r1 = std::min(rows, r0 + chunk);
          parts[(size_t)c] = format_csv_rows(values, rows, cols, r0, r1, kinds, vocabs);
          ready[(size_t)c].set_value();
        } catch (...) {
          ready[(size_t)c].set_exception(std::current_exception());
        }
      }
    });
  }
  std::string header;
  for (int64_t j = 0; j < cols; ++j) {
    if (j) header.push_back(',');
    append_field(header, names[(size_t)j]);
  }
  header.push_back('\n');
  FILE* f = std::fopen(path.c_str(), "wb");
  std::exception_ptr err;
  if (!f) err = std::make_exception_ptr(std::runtime_error("csv: cannot open " + path));
  else std::fwrite(header.data(), 1, header.size(), f);
  for (int c = 0; c < nchunks; ++c) {
    try {
      done[(size_t)c].get();
    } catch (...) {
      if (!err) err = std::current_exception();
    }
    if (f && !err) std::fwrite(parts[(size_t)c].data(), 1, parts[(size_t)c].size(), f);
    std::string().swap(parts[(size_t)c]);
  }
  for (auto& th : pool) th.join();
  if (f) std::fclose(f);
  if (err) std::rethrow_exception(err);
}

}  // namespace fedtgan
