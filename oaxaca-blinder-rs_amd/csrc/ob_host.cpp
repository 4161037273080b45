// ob_host.cpp -- host-side inference: bootstrap_stats (inference.rs:4-34) and the RIF
// transform (math/rif.rs:14-88), plus the error/version entry points of the C ABI.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "ob_common.hpp"
#include "ob_host.hpp"

namespace ob {

std::string& last_error() {
  static thread_local std::string msg;
  return msg;
}

// NaN-last total order so std::nth_element is well defined; for NaN-free input the selected
// order statistics are the ones `sort_unstable_by(partial_cmp)` puts at those indices.
static inline bool total_less(double a, double b) {
  if (std::isnan(a)) return false;
  if (std::isnan(b)) return true;
  return a < b;
}

void bootstrap_stats(const double* v, int64_t n, double out[4]) {
  if (n == 0) {  // inference.rs:5-7
    out[0] = out[1] = out[2] = out[3] = NAN;
    return;
  }
  const double nf = (double)n;
  double mean = 0.0;
  for (int64_t i = 0; i < n; ++i) mean += v[i];
  mean /= nf;
  double ss = 0.0;
  for (int64_t i = 0; i < n; ++i) ss += (v[i] - mean) * (v[i] - mean);
  out[0] = std::sqrt(ss / (nf - 1.0));  // inference.rs:9-15 (n - 1 denominator)
  int64_t pos = 0, neg = 0;
  for (int64_t i = 0; i < n; ++i) {
    pos += v[i] >= 0.0;
    neg += v[i] <= 0.0;
  }
  const double pp = (double)pos / nf, pn = (double)neg / nf;
  out[1] = std::min(2.0 * std::min(pp, pn), 1.0);  // inference.rs:20-22
  // percentile CI, floor indices (inference.rs:25-31)
  const int64_t lo = (int64_t)std::floor(0.025 * nf);
  const int64_t hi = std::min<int64_t>((int64_t)std::floor(0.975 * nf), n - 1);
  std::vector<double> s(v, v + n);
  std::nth_element(s.begin(), s.begin() + hi, s.end(), total_less);
  out[3] = s[hi];
  if (lo < n) {
    std::nth_element(s.begin(), s.begin() + lo, s.begin() + hi + 1, total_less);
    out[2] = s[lo];
  } else {
    out[2] = NAN;
  }
}

void rif(const double* y, int64_t n, double tau, double* out) {
  if (n < 2) {  // rif.rs:18-20
    if (n > 0) std::memcpy(out, y, sizeof(double) * n);
    return;
  }
  const double nf = (double)n;
  std::vector<double> s(y, y + n);
  std::sort(s.begin(), s.end(), total_less);
  const double h = (nf - 1.0) * tau, hf = std::floor(h), hc = std::ceil(h), frac = h - hf;
  const double q = (hf == hc) ? s[(int64_t)hf] : s[(int64_t)hf] + frac * (s[(int64_t)hc] - s[(int64_t)hf]);
  double mean = 0.0;
  for (int64_t i = 0; i < n; ++i) mean += y[i];
  mean /= nf;
  double var = 0.0;
  for (int64_t i = 0; i < n; ++i) var += (y[i] - mean) * (y[i] - mean);
  var /= (nf - 1.0);
  const double sd = std::sqrt(var);
  int64_t i75 = (int64_t)std::ceil(0.75 * nf);
  i75 = i75 == 0 ? 0 : i75 - 1;
  int64_t i25 = (int64_t)std::ceil(0.25 * nf);
  i25 = i25 == 0 ? 0 : i25 - 1;
  const double iqr = s[std::min(i75, n - 1)] - s[std::min(i25, n - 1)];
  double spread = (iqr > 1e-8) ? std::fmin(sd, iqr / 1.34) : sd;
  if (spread < 1e-8) spread = 1.0;
  const double bw = 0.9 * spread * std::pow(nf, -0.2);  // Silverman (rif.rs:59)
  const double c = 1.0 / std::sqrt(2.0 * M_PI);
  double dens = 0.0;
  for (int64_t i = 0; i < n; ++i) {
    const double u = (q - y[i]) / bw;
    dens += c * std::exp(-0.5 * (u * u));
  }
  dens /= (nf * bw);
  if (dens < 1e-8) dens = 1e-8;
  for (int64_t i = 0; i < n; ++i) out[i] = q + (tau - (y[i] <= q ? 1.0 : 0.0)) / dens;
}

void aggregate(const double* rows, const uint8_t* ok, uint64_t n_reps, int row_len,
               const std::vector<std::vector<int>>& groups, double* out) {
  std::vector<uint64_t> good;
  good.reserve(n_reps);
  for (uint64_t r = 0; r < n_reps; ++r)
    if (ok[r]) good.push_back(r);
  auto work = [&](size_t lo, size_t hi) {
    std::vector<double> v;
    for (size_t g = lo; g < hi; ++g) {
      v.clear();
      v.reserve(good.size() * groups[g].size());
      for (uint64_t r : good)
        for (int c : groups[g]) v.push_back(rows[r * (uint64_t)row_len + c]);
      bootstrap_stats(v.data(), (int64_t)v.size(), out + 4 * g);
    }
  };
  const size_t ng = groups.size();
  const size_t nth = std::min<size_t>({ng, 16, std::max(1u, std::thread::hardware_concurrency())});
  if (nth <= 1 || good.size() < 4096) {
    work(0, ng);
    return;
  }
  std::vector<std::thread> th;
  for (size_t t = 0; t < nth; ++t) {  // strided split keeps the per-thread work even
    th.emplace_back([&, t]() {
      for (size_t g = t; g < ng; g += nth) work(g, g + 1);
    });
  }
  for (auto& t : th) t.join();
}

}  // namespace ob

extern "C" {

int ob_aggregate(const double* rows, const uint8_t* ok, uint64_t n_reps, int32_t row_len, const int32_t* cols,
                 int32_t n_cols, double* out) {
  if (n_cols < 0 || row_len <= 0 || (n_cols > 0 && (!cols || !out)) || (n_reps > 0 && (!rows || !ok)))
    return ob::fail(OB_E_INVALID, "bad arguments");
  std::vector<std::vector<int>> groups((size_t)n_cols);
  for (int32_t c = 0; c < n_cols; ++c) {
    if (cols[c] < 0 || cols[c] >= row_len) return ob::fail(OB_E_INVALID, "column %d out of range", cols[c]);
    groups[c] = {cols[c]};
  }
  ob::aggregate(rows, ok, n_reps, row_len, groups, out);
  return OB_OK;
}


const char* ob_last_error(void) { return ob::last_error().c_str(); }

const char* ob_version(void) { return "oaxaca-boot-mi355x 0.2.0 (gfx950, OBRS-3)"; }

int ob_bootstrap_stats(const double* estimates, int64_t n, double point_estimate, double out[4]) {
  (void)point_estimate;  // unused by the reference too (inference.rs:4)
  if (!out || (n > 0 && !estimates) || n < 0) return ob::fail(OB_E_INVALID, "bad arguments");
  ob::bootstrap_stats(estimates, n, out);
  return OB_OK;
}

int ob_rif(const double* y, int64_t n, double tau, double* out) {
  if (n < 0 || (n > 0 && (!y || !out))) return ob::fail(OB_E_INVALID, "bad arguments");
  ob::rif(y, n, tau, out);
  return OB_OK;
}

}  // extern "C"
