#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace fedtgan {

// output column kinds of the native CSV formatter (fed_tgan_amd/data/decode.py KIND_*)
enum { CSV_FLOAT = 0, CSV_VOCAB = 1, CSV_NONNEG = 2, CSV_DATE = 3 };
enum { DATE_STYLE_DAY = 0, DATE_STYLE_FULL = 1, DATE_STYLE_YYMMDD = 2 };

// one categorical part of a date column: its source column of codes, the date element it carries
// (0 year (two digits), 1 month, 2 day, 3 hour, 4 minute, 5 second) and code -> value (-1: "empty")
struct CsvDatePart {
  int src = 0;
  int elem = 0;
  std::vector<int> lut;
};

struct CsvColumn {
  int kind = CSV_FLOAT;
  int src = 0;                       // source column in the value matrix (not used by CSV_DATE)
  std::vector<std::string> vocab;    // CSV_VOCAB: code -> string
  int date_mode = 0;                 // CSV_DATE: 0 timestamp, 1 the yymmdd integer
  std::vector<CsvDatePart> parts;    // CSV_DATE: in the format's order
};

std::string format_py_float(double x);

std::vector<int> resolve_date_styles(const double* values, int64_t rows, int64_t cols, const std::vector<CsvColumn>& out);

// aux (nullable): a second [rows, aux_cols] matrix; a column's src >= cols reads aux[r, src - cols] (e.g.
// the non-negative columns mapped on the host, so the main matrix is read in place, never copied)
std::string format_csv_columns(const double* values, int64_t cols, int64_t r0, int64_t r1,
                               const std::vector<CsvColumn>& out, const std::vector<int>& date_style,
                               const double* aux = nullptr, int64_t aux_cols = 0);

void write_csv_columns(const std::string& path, const double* values, int64_t rows, int64_t cols,
                       const std::vector<std::string>& names, const std::vector<CsvColumn>& out, int threads,
                       const double* aux = nullptr, int64_t aux_cols = 0);

// one output column per value column (kinds 0..2)
std::string format_csv_rows(const double* values, int64_t rows, int64_t cols, int64_t r0, int64_t r1,
                            const std::vector<int>& kinds, const std::vector<std::vector<std::string>>& vocabs);

void write_csv_file(const std::string& path, const double* values, int64_t rows, int64_t cols,
                    const std::vector<std::string>& names, const std::vector<int>& kinds,
                    const std::vector<std::vector<std::string>>& vocabs, int threads);

}  // namespace fedtgan
