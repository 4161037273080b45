// ob_host.hpp -- host-side inference helpers shared by the builder and the C ABI.
#pragma once
#include <cstdint>

namespace ob {
// inference.rs:4-34: out = {std_err, p_value, ci_lower, ci_upper}
void bootstrap_stats(const double* v, int64_t n, double out[4]);
// math/rif.rs:14-88
void rif(const double* y, int64_t n, double tau, double* out);
}  // namespace ob
