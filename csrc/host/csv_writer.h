#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace fedtgan {

std::string format_py_float(double x);

std::string format_csv_rows(const double* values, int64_t rows, int64_t cols, int64_t r0, int64_t r1,
                            const std::vector<int>& kinds, const std::vector<std::vector<std::string>>& vocabs);

void write_csv_file(const std::string& path, const double* values, int64_t rows, int64_t cols,
                    const std::vector<std::string>& names, const std::vector<int>& kinds,
                    const std::vector<std::vector<std::string>>& vocabs, int threads);

}  // namespace fedtgan
