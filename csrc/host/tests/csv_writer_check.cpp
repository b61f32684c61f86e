// Host-only check of the native CSV writer, built with sanitizers by tests/test_host_sanitizers.py
// (AddressSanitizer + UndefinedBehaviorSanitizer, and ThreadSanitizer for the worker pool).
// Writes a table with every column kind through the multi-threaded path and compares it with the
// single-threaded formatting of the same rows.
#include <cmath>
#include <cstdio>
#include <fstream>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "../csv_writer.h"

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "/tmp/csv_writer_check.csv";
  const int64_t rows = 20000, cols = 6;
  std::vector<double> v((size_t)(rows * cols));
  std::mt19937_64 g(7);
  std::normal_distribution<double> nd;
  for (int64_t r = 0; r < rows; ++r) {
    v[r * cols + 0] = nd(g) * std::pow(10.0, (double)(r % 30) - 15);   // floats across magnitudes
    v[r * cols + 1] = (double)(r % 3);                                  // vocabulary codes
    v[r * cols + 2] = (r % 5 == 0) ? -1.0 : std::fabs(nd(g)) * 100;     // non-negative (-1 -> blank)
    v[r * cols + 3] = (r % 11 == 0) ? NAN : nd(g);                      // NaN -> empty field
    v[r * cols + 4] = (r % 2) ? -0.0 : 1e16;
    v[r * cols + 5] = (double)(r % 2);
  }
  std::vector<std::string> names = {"x", "cat", "nonneg", "nan", "edge", "q,uoted"};
  std::vector<int> kinds = {0, 1, 2, 0, 0, 1};
  std::vector<std::vector<std::string>> vocabs(cols);
  vocabs[1] = {"a", "b,c", "say \"hi\""};
  vocabs[5] = {"0", "1"};
  fedtgan::write_csv_file(path, v.data(), rows, cols, names, kinds, vocabs, 8);
  std::ifstream f(path);
  std::stringstream ss;
  ss << f.rdbuf();
  const std::string multi = ss.str();
  const std::string single = fedtgan::format_csv_rows(v.data(), rows, cols, 0, rows, kinds, vocabs);
  const size_t hdr = multi.find('\n') + 1;
  if (multi.substr(hdr) != single) {
    std::fprintf(stderr, "multi-threaded output differs from the single-threaded one\n");
    return 1;
  }
  std::printf("ok %zu bytes\n", multi.size());
  return 0;
}
