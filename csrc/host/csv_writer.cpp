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
// Rows are formatted in parallel blocks by worker threads and written with one fwrite each.
#include "csv_writer.h"

#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace fedtgan {
namespace {

void append_py_float(std::string& out, double x) {
  if (std::isnan(x)) return;  // pandas writes NaN as an empty field
  if (std::isinf(x)) {
    out += (x > 0) ? "inf" : "-inf";
    return;
  }
  char buf[64];
  auto res = std::to_chars(buf, buf + sizeof(buf), x, std::chars_format::scientific);
  *res.ptr = '\0';
  // buf: [-]d[.ddd]e[+-]XX
  const char* p = buf;
  bool neg = false;
  if (*p == '-') {
    neg = true;
    ++p;
  }
  char digits[32];
  int nd = 0;
  while (*p && *p != 'e') {
    if (*p != '.') digits[nd++] = *p;
    ++p;
  }
  int e10 = 0;
  if (*p == 'e') e10 = std::atoi(p + 1);
  // strip trailing zeros of the mantissa (to_chars shortest never emits them, but keep it robust)
  while (nd > 1 && digits[nd - 1] == '0') --nd;
  const int decpt = e10 + 1;  // value = 0.d1d2... x 10^decpt
  if (neg) out.push_back('-');
  if (decpt > -4 && decpt <= 16) {
    if (decpt <= 0) {
      out += "0.";
      out.append((size_t)(-decpt), '0');
      out.append(digits, (size_t)nd);
    } else if (decpt < nd) {
      out.append(digits, (size_t)decpt);
      out.push_back('.');
      out.append(digits + decpt, (size_t)(nd - decpt));
    } else {
      out.append(digits, (size_t)nd);
      out.append((size_t)(decpt - nd), '0');
      out += ".0";
    }
  } else {
    out.push_back(digits[0]);
    if (nd > 1) {
      out.push_back('.');
      out.append(digits + 1, (size_t)(nd - 1));
    }
    const int ex = decpt - 1;
    out.push_back('e');
    out.push_back(ex < 0 ? '-' : '+');
    const int ax = ex < 0 ? -ex : ex;
    if (ax < 10) out.push_back('0');
    out += std::to_string(ax);
  }
}

void append_field(std::string& out, const std::string& s) {
  bool q = s.find_first_of(",\"\n\r") != std::string::npos;
  if (!q) {
    out += s;
    return;
  }
  out.push_back('"');
  for (char ch : s) {
    if (ch == '"') out.push_back('"');
    out.push_back(ch);
  }
  out.push_back('"');
}

}  // namespace

std::string format_csv_rows(const double* values, int64_t rows, int64_t cols, int64_t r0, int64_t r1,
                            const std::vector<int>& kinds, const std::vector<std::vector<std::string>>& vocabs) {
  std::string out;
  out.reserve((size_t)(r1 - r0) * (size_t)cols * 12);
  for (int64_t r = r0; r < r1; ++r) {
    const double* row = values + r * cols;
    for (int64_t j = 0; j < cols; ++j) {
      if (j) out.push_back(',');
      const double x = row[j];
      switch (kinds[(size_t)j]) {
        case 1: {  // vocabulary
          const auto& voc = vocabs[(size_t)j];
          int64_t k = (int64_t)x;
          if (k < 0 || k >= (int64_t)voc.size()) throw std::runtime_error("csv: category code out of range");
          append_field(out, voc[(size_t)k]);
          break;
        }
        case 2: {  // non-negative column, already mapped by exp(x)-1 (+ceil) on the host with numpy's exp
          if (x == -1.0) out.push_back(' ');
          else append_py_float(out, x);
          break;
        }
        default:
          append_py_float(out, x);
      }
    }
    out.push_back('\n');
  }
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
  std::vector<std::string> parts((size_t)threads);
  std::vector<std::thread> pool;
  const int64_t per = (rows + threads - 1) / threads;
  for (int t = 0; t < threads; ++t) {
    const int64_t r0 = t * per, r1 = std::min(rows, r0 + per);
    if (r0 >= r1) continue;
    pool.emplace_back([&, t, r0, r1]() { parts[(size_t)t] = format_csv_rows(values, rows, cols, r0, r1, kinds, vocabs); });
  }
  std::string header;
  for (int64_t j = 0; j < cols; ++j) {
    if (j) header.push_back(',');
    append_field(header, names[(size_t)j]);
  }
  header.push_back('\n');
  for (auto& th : pool) th.join();
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) throw std::runtime_error("csv: cannot open " + path);
  std::fwrite(header.data(), 1, header.size(), f);
  for (auto& p : parts) std::fwrite(p.data(), 1, p.size(), f);
  std::fclose(f);
}

}  // namespace fedtgan
