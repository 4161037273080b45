// ob_host.hpp -- host-side inference helpers shared by the builder and the C ABI.
#pragma once
#include <cstdint>
#include <vector>

namespace ob {
// inference.rs:4-34: out = {std_err, p_value, ci_lower, ci_upper}
void bootstrap_stats(const double* v, int64_t n, double out[4]);
// math/rif.rs:14-88
void rif(const double* y, int64_t n, double tau, double* out);
// bootstrap_stats per group of row columns (values of a group's columns pooled in replicate order,
// builder.rs:963-971) over rows with ok != 0; out: groups.size() x 4. Multithreaded.
void aggregate(const double* rows, const uint8_t* ok, uint64_t n_reps, int row_len,
               const std::vector<std::vector<int>>& groups, double* out);
}  // namespace ob
