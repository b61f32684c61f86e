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
//   * date columns (`Server/dtds/data/utils/transform.py:51-52`, `date.py:113-200`): re-joined from their
//     categorical part columns (year / month / day / hour / minute / second codes -> values through
//     per-part tables), impossible days repaired as the reference does, and printed the way pandas
//     prints the re-joined column (date only, full timestamp, or the yymmdd integer; see
//     resolve_date_styles)
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
#include <mutex>
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

namespace {

// Python's strptime %y: 69..99 -> 1969..1999, 0..68 -> 2000..2068
int year_of_y2(int y2) { return y2 < 69 ? 2000 + y2 : 1900 + y2; }

// one date column's fields for a row; false when any part is "empty" (the whole field is then " ")
struct DateFields {
  int y2 = -1, year = 1900, month = 1, day = 1, hour = 0, minute = 0, second = 0;
};

bool date_fields(const double* row, const CsvColumn& c, DateFields& f) {
  int v[6] = {-1, -1, -1, -1, -1, -1};
  for (const auto& p : c.parts) {
    const int64_t code = (int64_t)row[p.src];
    if (code < 0 || code >= (int64_t)p.lut.size()) throw std::runtime_error("csv: date part code out of range");
    const int x = p.lut[(size_t)code];
    if (x < 0) return false;
    v[p.elem] = x;
  }
  if (v[0] >= 0) {
    f.y2 = v[0];
    f.year = year_of_y2(v[0]);
  }
  if (v[1] >= 0) f.month = v[1];
  if (v[2] >= 0) f.day = v[2];
  if (v[3] >= 0) f.hour = v[3];
  if (v[4] >= 0) f.minute = v[4];
  if (v[5] >= 0) f.second = v[5];
  // impossible days (`Server/dtds/data/utils/date.py:113-200`, the reference's leap rule on the two-digit
  // year: only "00" keeps February 29); applied when the first three parts are year, month, day
  if (c.parts.size() >= 3 && v[0] >= 0 && v[1] >= 0 && v[2] >= 0) {
    static const int dim[13] = {0, 31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
    if (f.month < 1 || f.month > 12) throw std::runtime_error("csv: date month out of range");
    if (f.day > dim[f.month]) {
      if (f.month == 2) f.day = (f.y2 % 4 == 0 && f.y2 % 100 == 0 && f.y2 % 400 == 0) ? 29 : 28;
      else f.day = 30;
    }
  }
  return true;
}

char* put_2(char* p, int x) {
  *p++ = (char)('0' + (x / 10) % 10);
  *p++ = (char)('0' + x % 10);
  return p;
}

char* put_date(char* p, const DateFields& f, int style) {
  if (style == DATE_STYLE_YYMMDD) {   // int(ts.strftime("%y%m%d"))
    const auto r = std::to_chars(p, p + 12, (f.year % 100) * 10000 + f.month * 100 + f.day);
    return r.ptr;
  }
  const auto r = std::to_chars(p, p + 6, f.year);
  p = r.ptr;
  *p++ = '-';
  p = put_2(p, f.month);
  *p++ = '-';
  p = put_2(p, f.day);
  if (style == DATE_STYLE_FULL) {
    *p++ = ' ';
    p = put_2(p, f.hour);
    *p++ = ':';
    p = put_2(p, f.minute);
    *p++ = ':';
    p = put_2(p, f.second);
  }
  return p;
}

}  // namespace

// Rows [r0, r1) into one string.  Every vocabulary entry is quoted once up front and each row is
// written through a raw pointer into a buffer sized for its worst case (26 bytes per number), so the
// hot loop does no allocation, no searching and no growing appends.
// rows [r0, r1) formatted into buf (grown as needed, never shrunk or zero-filled again); returns the length
static size_t format_csv_into(std::vector<char>& buf, const double* values, int64_t cols, int64_t r0, int64_t r1,
                              const std::vector<CsvColumn>& out, const std::vector<int>& date_style,
                              const double* aux, int64_t aux_cols) {
  std::vector<std::vector<std::string>> qv(out.size());
  size_t row_max = 1;
  for (size_t j = 0; j < out.size(); ++j) {
    const CsvColumn& c = out[j];
    if (c.kind != CSV_DATE && (c.src < 0 || c.src >= cols + (aux ? aux_cols : 0)))
      throw std::runtime_error("csv: source column out of range");
    size_t w = 26;
    if (c.kind == CSV_VOCAB) {
      w = 0;
      for (const auto& e : c.vocab) {
        qv[j].push_back(quote_field(e));
        w = std::max(w, qv[j].back().size());
      }
    } else if (c.kind == CSV_DATE) {
      for (const auto& p : c.parts)
        if (p.src < 0 || p.src >= cols || p.elem < 0 || p.elem > 5) throw std::runtime_error("csv: date part");
      w = 32;
    }
    row_max += w + 1;
  }
  const size_t need = (size_t)(r1 - r0) * row_max;
  if (buf.size() < need) buf.resize(need);
  char* const b0 = buf.data();
  char* p = b0;
  for (int64_t r = r0; r < r1; ++r) {
    const double* row = values + r * cols;
    const double* arow = aux ? aux + r * aux_cols : nullptr;   // column src >= cols is arow[src - cols]
    auto val = [&](int s) { return s < cols ? row[s] : arow[s - cols]; };
    for (size_t j = 0; j < out.size(); ++j) {
      if (j) *p++ = ',';
      const CsvColumn& c = out[j];
      switch (c.kind) {
        case CSV_VOCAB: {
          const auto& voc = qv[j];
          const int64_t k = (int64_t)val(c.src);
          if (k < 0 || k >= (int64_t)voc.size()) throw std::runtime_error("csv: category code out of range");
          const std::string& f = voc[(size_t)k];
          std::memcpy(p, f.data(), f.size());
          p += f.size();
          break;
        }
        case CSV_NONNEG: {   // already mapped by exp(x)-1 (+ceil) on the host with numpy's exp
          const double x = val(c.src);
          if (x == -1.0) *p++ = ' ';
          else p = put_py_float(p, x);
          break;
        }
        case CSV_DATE: {
          DateFields f;
          if (date_fields(row, c, f)) p = put_date(p, f, date_style[j]);
          else *p++ = ' ';
          break;
        }
        default:
          p = put_py_float(p, val(c.src));
      }
    }
    *p++ = '\n';
  }
  return (size_t)(p - b0);
}

std::string format_csv_columns(const double* values, int64_t cols, int64_t r0, int64_t r1,
                               const std::vector<CsvColumn>& out, const std::vector<int>& date_style,
                               const double* aux, int64_t aux_cols) {
  std::vector<char> buf;
  const size_t n = format_csv_into(buf, values, cols, r0, r1, out, date_style, aux, aux_cols);
  return std::string(buf.data(), n);
}

// Chunk buffers kept across tables (write_csv_columns runs once per epoch, on the runtime's writer thread): a
// fresh zero-filled string per chunk cost a page fault per 4 KB of text on every table -- ~45 MB of first
// touches per 40k-row Intrusion table, most of the formatter's time, and page-table contention with the
// training thread.  One table at a time (the mutex); the buffers are reused as they are.
std::mutex g_csv_mu;
std::vector<std::vector<char>> g_csv_bufs;

std::vector<int> resolve_date_styles(const double* values, int64_t rows, int64_t cols, const std::vector<CsvColumn>& out) {
  // pandas writes the re-joined column by its dtype, which depends on the whole column: with any "empty"
  // row it is an object column of Timestamps (str(): "YYYY-MM-DD HH:MM:SS"); otherwise datetime64, printed
  // date-only when every time of day is midnight.  The yymmdd form is an integer either way.
  std::vector<int> style(out.size(), DATE_STYLE_DAY);
  for (size_t j = 0; j < out.size(); ++j) {
    const CsvColumn& c = out[j];
    if (c.kind != CSV_DATE) continue;
    if (c.date_mode == 1) {
      style[j] = DATE_STYLE_YYMMDD;
      continue;
    }
    bool any_empty = false, any_time = false;
    for (int64_t r = 0; r < rows && !any_empty; ++r) {
      DateFields f;
      if (!date_fields(values + r * cols, c, f)) any_empty = true;
      else if (f.hour || f.minute || f.second) any_time = true;
    }
    style[j] = (any_empty || any_time) ? DATE_STYLE_FULL : DATE_STYLE_DAY;
  }
  return style;
}

std::vector<CsvColumn> simple_columns(int64_t cols, const std::vector<int>& kinds,
                                      const std::vector<std::vector<std::string>>& vocabs) {
  std::vector<CsvColumn> out((size_t)cols);
  for (int64_t j = 0; j < cols; ++j) {
    out[(size_t)j].kind = kinds[(size_t)j];
    out[(size_t)j].src = (int)j;
    out[(size_t)j].vocab = vocabs[(size_t)j];
  }
  return out;
}

std::string format_csv_rows(const double* values, int64_t rows, int64_t cols, int64_t r0, int64_t r1,
                            const std::vector<int>& kinds, const std::vector<std::vector<std::string>>& vocabs) {
  const auto out = simple_columns(cols, kinds, vocabs);
  return format_csv_columns(values, cols, r0, r1, out, resolve_date_styles(values, rows, cols, out), nullptr, 0);
}

std::string format_py_float(double x) {
  std::string s;
  append_py_float(s, x);
  return s;
}

void write_csv_columns(const std::string& path, const double* values, int64_t rows, int64_t cols,
                       const std::vector<std::string>& names, const std::vector<CsvColumn>& out, int threads,
                       const double* aux, int64_t aux_cols) {
  if (names.size() != out.size()) throw std::runtime_error("csv: column descriptor size mismatch");
  const std::vector<int> style = resolve_date_styles(values, rows, cols, out);
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
  std::lock_guard<std::mutex> lock(g_csv_mu);
  if (g_csv_bufs.size() < (size_t)nchunks) g_csv_bufs.resize((size_t)nchunks);
  std::vector<size_t> lens((size_t)nchunks, 0);
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
          lens[(size_t)c] = format_csv_into(g_csv_bufs[(size_t)c], values, cols, r0, r1, out, style, aux, aux_cols);
          ready[(size_t)c].set_value();
        } catch (...) {
          ready[(size_t)c].set_exception(std::current_exception());
        }
      }
    });
  }
  std::string header;
  for (size_t j = 0; j < names.size(); ++j) {
    if (j) header.push_back(',');
    append_field(header, names[j]);
  }
  header.push_back('\n');
  FILE* f = std::fopen(path.c_str(), "wb");
  std::exception_ptr err;
  // a short write (full disk, I/O error) or a failed close is an error like a formatting failure: the
  // caller must not record a truncated table as written
  auto put = [&](const char* b, size_t n) {
    if (f && !err && std::fwrite(b, 1, n, f) != n)
      err = std::make_exception_ptr(std::runtime_error("csv: short write to " + path));
  };
  if (!f) err = std::make_exception_ptr(std::runtime_error("csv: cannot open " + path));
  else put(header.data(), header.size());
  for (int c = 0; c < nchunks; ++c) {
    try {
      done[(size_t)c].get();
    } catch (...) {
      if (!err) err = std::current_exception();
    }
    put(g_csv_bufs[(size_t)c].data(), lens[(size_t)c]);
  }
  for (auto& th : pool) th.join();
  if (f && std::fclose(f) != 0 && !err) err = std::make_exception_ptr(std::runtime_error("csv: close failed for " + path));
  if (err) std::rethrow_exception(err);
}

void write_csv_file(const std::string& path, const double* values, int64_t rows, int64_t cols,
                    const std::vector<std::string>& names, const std::vector<int>& kinds,
                    const std::vector<std::vector<std::string>>& vocabs, int threads) {
  if ((int64_t)kinds.size() != cols || (int64_t)names.size() != cols || (int64_t)vocabs.size() != cols)
    throw std::runtime_error("csv: column descriptor size mismatch");
  write_csv_columns(path, values, rows, cols, names, simple_columns(cols, kinds, vocabs), threads);
}

}  // namespace fedtgan
