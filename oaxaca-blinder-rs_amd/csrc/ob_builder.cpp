// ob_builder.cpp -- native host runtime mirroring `OaxacaBuilder` (oaxaca_blinder/src/builder.rs)
// over a column frame, with the bootstrap driver delegated to the MI355X engine.
//
//   clean_dataframe        builder.rs:760-784
//   create_dummies_manual  builder.rs:380-418
//   split_groups           builder.rs:61-102
//   prepare_data           builder.rs:294-378
//   run                    builder.rs:787-951 (point estimate, bootstrap, aggregation)
//   process_component      builder.rs:849-865, process_detailed_components builder.rs:953-983
//   decompose_quantile     builder.rs:711-757
//   get_data_matrices      builder.rs:252-291
// Polars semantics that matter here are kept: rows with a null in any used column are dropped,
// categorical levels are the sorted unique strings (byte order), group A is the first sorted
// level that is not the reference, a third level is ignored, outcome/weights must be Float64.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "ob_common.hpp"
#include "ob_engine.hpp"
#include "ob_host.hpp"
#include "ob_mm.hpp"
#include "ob_spec.h"

namespace ob {

struct Col {
  std::string name;
  int kind = OB_COL_F64;
  std::vector<double> f;       // OB_COL_F64 values (OB_COL_I64 values cast on use)
  std::vector<int64_t> i;      // OB_COL_I64
  std::vector<std::string> s;  // OB_COL_STR
  std::vector<uint8_t> valid;  // 1 = non-null
};

struct Frame {
  int64_t nrows = 0;
  std::vector<Col> cols;
  int find(const std::string& n) const {
    for (size_t c = 0; c < cols.size(); ++c)
      if (cols[c].name == n) return (int)c;
    return -1;
  }
};

struct Config {
  std::string outcome, group, reference_group;
  std::vector<std::string> outcomes;  // RIF multi-tau: y columns of one panel (empty: {outcome})
  std::vector<std::string> predictors, categorical, normalize;
  bool has_weights = false;
  std::string weights;
  bool has_selection = false;
  std::string selection;
  std::vector<std::string> selection_predictors;
  uint64_t reps = 20;
  int ref = OB_REF_GROUP_A;
  bool has_seed = false;
  uint64_t seed = 0;
};

static const char* dtype_name(int kind) {
  switch (kind) {
    case OB_COL_F64: return "f64";
    case OB_COL_I64: return "i64";
    default: return "str";
  }
}

static int load_frame(const ob_column* cols, int n_cols, int64_t n_rows, Frame& out) {
  if (n_cols < 0 || n_rows < 0 || (n_cols > 0 && !cols)) return fail(OB_E_INVALID, "bad frame arguments");
  out.nrows = n_rows;
  out.cols.clear();
  for (int c = 0; c < n_cols; ++c) {
    const ob_column& src = cols[c];
    if (!src.name) return fail(OB_E_INVALID, "column %d has no name", c);
    if (out.find(src.name) >= 0)
      return fail(OB_E_POLARS, "%sduplicate: column with name '%s' has more than one occurrence",
                  error_prefix(OB_E_POLARS), src.name);
    Col col;
    col.name = src.name;
    col.kind = src.kind;
    col.valid.assign(n_rows, 1);
    if (src.kind == OB_COL_F64) {
      if (n_rows && !src.f64) return fail(OB_E_INVALID, "column '%s' has no f64 data", src.name);
      col.f.assign(src.f64, src.f64 + n_rows);
      if (src.valid) col.valid.assign(src.valid, src.valid + n_rows);
    } else if (src.kind == OB_COL_I64) {
      if (n_rows && !src.i64) return fail(OB_E_INVALID, "column '%s' has no i64 data", src.name);
      col.i.assign(src.i64, src.i64 + n_rows);
      if (src.valid) col.valid.assign(src.valid, src.valid + n_rows);
    } else if (src.kind == OB_COL_STR) {
      if (n_rows && !src.str) return fail(OB_E_INVALID, "column '%s' has no string data", src.name);
      col.s.resize(n_rows);
      for (int64_t r = 0; r < n_rows; ++r) {
        if (src.str[r]) {
          col.s[r] = src.str[r];
        } else {
          col.valid[r] = 0;
        }
      }
    } else {
      return fail(OB_E_INVALID, "column '%s' has unknown kind %d", src.name, src.kind);
    }
    for (auto& v : col.valid) v = v ? 1 : 0;
    out.cols.push_back(std::move(col));
  }
  return OB_OK;
}

static Col take_col(const Col& c, const std::vector<int64_t>& rows) {
  Col o;
  o.name = c.name;
  o.kind = c.kind;
  o.valid.resize(rows.size());
  if (c.kind == OB_COL_F64) o.f.resize(rows.size());
  if (c.kind == OB_COL_I64) o.i.resize(rows.size());
  if (c.kind == OB_COL_STR) o.s.resize(rows.size());
  for (size_t r = 0; r < rows.size(); ++r) {
    const int64_t src = rows[r];
    o.valid[r] = c.valid[src];
    if (c.kind == OB_COL_F64) o.f[r] = c.f[src];
    if (c.kind == OB_COL_I64) o.i[r] = c.i[src];
    if (c.kind == OB_COL_STR) o.s[r] = c.s[src];
  }
  return o;
}

static Frame take(const Frame& f, const std::vector<int64_t>& rows) {
  Frame o;
  o.nrows = (int64_t)rows.size();
  for (const Col& c : f.cols) o.cols.push_back(take_col(c, rows));
  return o;
}

static int config_from(const ob_builder_config* c, Config& out) {
  if (!c || !c->outcome || !c->group || !c->reference_group) return fail(OB_E_INVALID, "incomplete builder config");
  out.outcome = c->outcome;
  out.group = c->group;
  out.reference_group = c->reference_group;
  auto names = [](const char* const* v, int n, std::vector<std::string>& o) -> int {
    o.clear();
    if (n < 0 || (n > 0 && !v)) return fail(OB_E_INVALID, "bad name list");
    for (int i = 0; i < n; ++i) {
      if (!v[i]) return fail(OB_E_INVALID, "null name");
      o.emplace_back(v[i]);
    }
    return OB_OK;
  };
  OB_TRY(names(c->predictors, c->n_predictors, out.predictors));
  OB_TRY(names(c->categorical, c->n_categorical, out.categorical));
  OB_TRY(names(c->normalize, c->n_normalize, out.normalize));
  out.has_weights = c->weights != nullptr;
  if (c->weights) out.weights = c->weights;
  out.has_selection = c->selection_outcome != nullptr;
  if (c->selection_outcome) out.selection = c->selection_outcome;
  OB_TRY(names(c->selection_predictors, c->n_selection_predictors, out.selection_predictors));
  out.reps = c->bootstrap_reps;
  out.ref = c->reference_coeffs;
  if (out.ref < OB_REF_GROUP_A || out.ref > OB_REF_NEUMARK)
    return fail(OB_E_INVALID, "unknown reference coefficients %d", out.ref);
  out.has_seed = c->has_seed != 0;
  out.seed = c->seed;
  return OB_OK;
}

// builder.rs:760-784
static int clean_dataframe(const Frame& f, const Config& c, Frame& out) {
  std::vector<std::string> cols = {c.outcome, c.group};
  cols.insert(cols.end(), c.predictors.begin(), c.predictors.end());
  cols.insert(cols.end(), c.categorical.begin(), c.categorical.end());
  if (c.has_weights) cols.push_back(c.weights);
  if (c.has_selection) cols.push_back(c.selection);
  cols.insert(cols.end(), c.selection_predictors.begin(), c.selection_predictors.end());
  std::vector<int> idx;
  for (const auto& name : cols) {
    const int i = f.find(name);
    if (i < 0) return fail(OB_E_COLUMN, "%s%s", error_prefix(OB_E_COLUMN), name.c_str());
    idx.push_back(i);
  }
  std::vector<int64_t> keep;
  keep.reserve(f.nrows);
  for (int64_t r = 0; r < f.nrows; ++r) {
    bool ok = true;
    for (int i : idx) ok = ok && f.cols[i].valid[r];
    if (ok) keep.push_back(r);
  }
  out = take(f, keep);
  return OB_OK;
}

static int expect_str(const Col& c) {
  if (c.kind != OB_COL_STR)
    return fail(OB_E_POLARS, "%sinvalid series dtype: expected `String`, got `%s` for `%s`", error_prefix(OB_E_POLARS),
                dtype_name(c.kind), c.name.c_str());
  return OB_OK;
}

static std::vector<std::string> sorted_levels(const Col& c) {
  std::vector<std::string> lv;
  for (size_t r = 0; r < c.s.size(); ++r)
    if (c.valid[r]) lv.push_back(c.s[r]);
  std::sort(lv.begin(), lv.end());
  lv.erase(std::unique(lv.begin(), lv.end()), lv.end());
  return lv;
}

struct Dummies {
  std::vector<Col> cols;
  size_t m = 0;
  std::string base_name;
};

// builder.rs:380-418: base = first sorted level, one f64 0/1 column "{col}_{level}" per other level
static int create_dummies(const Col& series, Dummies& out) {
  OB_TRY(expect_str(series));
  const auto levels = sorted_levels(series);
  out.m = levels.size();
  if (levels.empty())
    return fail(OB_E_GROUP, "%sCould not get reference category for %s", error_prefix(OB_E_GROUP), series.name.c_str());
  out.base_name = series.name + "_" + levels[0];
  for (size_t l = 1; l < levels.size(); ++l) {
    Col d;
    d.name = series.name + "_" + levels[l];
    d.kind = OB_COL_F64;
    d.f.resize(series.s.size());
    d.valid.assign(series.s.size(), 1);
    for (size_t r = 0; r < series.s.size(); ++r) d.f[r] = (series.valid[r] && series.s[r] == levels[l]) ? 1.0 : 0.0;
    out.cols.push_back(std::move(d));
  }
  return OB_OK;
}

struct Split {
  std::vector<int64_t> a, b;
  std::string name_a;
};

// builder.rs:61-102
static int split_groups(const Frame& f, const Config& c, Split& out) {
  const int gi = f.find(c.group);
  if (gi < 0) return fail(OB_E_COLUMN, "%s%s", error_prefix(OB_E_COLUMN), c.group.c_str());
  const Col& g = f.cols[gi];
  OB_TRY(expect_str(g));
  const auto levels = sorted_levels(g);
  if (levels.size() < 2) return fail(OB_E_GROUP, "%sNot enough groups for comparison", error_prefix(OB_E_GROUP));
  const std::string& b = c.reference_group;
  out.name_a = levels[0] == b ? levels[1] : levels[0];
  out.a.clear();
  out.b.clear();
  for (int64_t r = 0; r < f.nrows; ++r) {
    if (!g.valid[r]) continue;
    if (g.s[r] == out.name_a) out.a.push_back(r);
    if (g.s[r] == b) out.b.push_back(r);
  }
  return OB_OK;
}

struct Design {
  int64_t n = 0;
  std::vector<double> x;  // column-major n x p (no intercept)
  std::vector<double> y, w;
};

static int numeric_value(const Col& c, int64_t r, double& v) {
  if (c.kind == OB_COL_F64) {
    v = c.f[r];
  } else if (c.kind == OB_COL_I64) {
    v = (double)c.i[r];
  } else {
    return fail(OB_E_POLARS, "%scannot cast column `%s` of dtype `str` to `f64`", error_prefix(OB_E_POLARS),
                c.name.c_str());
  }
  return OB_OK;
}

// builder.rs:294-378 for the rows of one group. X columns = predictors then dummies.
static int prepare_data(const Frame& f, const std::vector<int64_t>& rows, const Config& c,
                        const std::vector<std::string>& dummy_names, bool want_w, Design& d) {
  const int yi = f.find(c.outcome);
  if (yi < 0) return fail(OB_E_COLUMN, "%s%s", error_prefix(OB_E_COLUMN), c.outcome.c_str());
  if (f.cols[yi].kind != OB_COL_F64)  // `.f64()?` (builder.rs:308)
    return fail(OB_E_POLARS, "%sinvalid series dtype: expected `Float64`, got `%s` for `%s`", error_prefix(OB_E_POLARS),
                dtype_name(f.cols[yi].kind), c.outcome.c_str());
  const int64_t n = (int64_t)rows.size();
  const size_t p = c.predictors.size() + dummy_names.size();
  d.n = n;
  d.x.assign((size_t)n * p, 0.0);
  const size_t ny = c.outcomes.empty() ? 1 : c.outcomes.size();
  d.y.resize((size_t)n * ny);  // column-major n x ny
  for (size_t t = 0; t < ny; ++t) {
    const int ti = c.outcomes.empty() ? yi : f.find(c.outcomes[t]);
    if (ti < 0 || f.cols[ti].kind != OB_COL_F64) return fail(OB_E_INVALID, "outcome column %zu missing", t);
    for (int64_t r = 0; r < n; ++r) d.y[t * n + r] = f.cols[ti].f[rows[r]];
  }
  size_t col = 0;
  for (const auto& name : c.predictors) {
    const int ci = f.find(name);
    if (ci < 0) return fail(OB_E_COLUMN, "%s%s", error_prefix(OB_E_COLUMN), name.c_str());
    for (int64_t r = 0; r < n; ++r) OB_TRY(numeric_value(f.cols[ci], rows[r], d.x[col * n + r]));
    ++col;
  }
  for (const auto& name : dummy_names) {  // missing dummy -> zero column (builder.rs:340-343)
    const int ci = f.find(name);
    if (ci >= 0)
      for (int64_t r = 0; r < n; ++r) OB_TRY(numeric_value(f.cols[ci], rows[r], d.x[col * n + r]));
    ++col;
  }
  d.w.clear();
  if (want_w && c.has_weights) {
    const int wi = f.find(c.weights);
    if (wi < 0) return fail(OB_E_COLUMN, "%s%s", error_prefix(OB_E_COLUMN), c.weights.c_str());
    if (f.cols[wi].kind != OB_COL_F64)
      return fail(OB_E_POLARS, "%sinvalid series dtype: expected `Float64`, got `%s` for `%s`",
                  error_prefix(OB_E_POLARS), dtype_name(f.cols[wi].kind), c.weights.c_str());
    d.w.resize(n);
    for (int64_t r = 0; r < n; ++r) d.w[r] = f.cols[wi].f[rows[r]];
  }
  return OB_OK;
}

// clean -> dummies -> split (builder.rs:787-808), shared by run/get_data_matrices.
struct Staged {
  Frame df;
  std::vector<std::string> dummy_names;
  std::unordered_map<std::string, size_t> category_counts;
  std::unordered_map<std::string, std::string> base_categories;
  Split split;
};

static int stage(const Frame& input, const Config& c, Staged& st) {
  OB_TRY(clean_dataframe(input, c, st.df));
  for (const auto& cat : c.categorical) {
    const int ci = st.df.find(cat);
    Dummies dm;
    OB_TRY(create_dummies(st.df.cols[ci], dm));
    st.category_counts[cat] = dm.m;
    st.base_categories[cat] = dm.base_name;
    for (auto& col : dm.cols) {
      if (st.df.find(col.name) >= 0)
        return fail(OB_E_POLARS, "%sduplicate: column with name '%s' has more than one occurrence",
                    error_prefix(OB_E_POLARS), col.name.c_str());
      st.dummy_names.push_back(col.name);
      st.df.cols.push_back(std::move(col));
    }
  }
  OB_TRY(split_groups(st.df, c, st.split));
  return OB_OK;
}

static bool starts_with(const std::string& s, const std::string& pre) {
  return s.size() >= pre.size() && std::equal(pre.begin(), pre.end(), s.begin());
}

}  // namespace ob

// ---------------------------------------------------------------------------------------------
// prepared run: panel in HBM + point estimate; boot ranges; aggregation
// ---------------------------------------------------------------------------------------------
struct ob_results {
  double total_gap = 0.0;
  int64_t n_a = 0, n_b = 0, n_failed = 0;
  struct Comp {
    std::string name;
    double estimate, std_err, t_stat, p_value, ci_lower, ci_upper;
  };
  std::vector<Comp> tables[5];
  std::vector<double> residuals, xa_mean, xb_mean, beta_star;
};

struct ob_prepared {
  ob_ctx* ctx = nullptr;
  ob_panel* panel = nullptr;
  ob::Config cfg;
  int ref = OB_REF_GROUP_A;
  uint64_t seed = 0;
  int k = 0, n_base = 0, row_len = 0;
  std::vector<std::string> names;         // K final predictor names
  std::vector<std::string> detail_names;  // K + n_base (base categories appended)
  std::vector<double> point_row, resid_b;  // n_y x row_len, n_y x n_b
  int64_t n_a = 0, n_b = 0;
  int n_y = 1;
  int64_t n_resid = 0;                     // residuals per outcome: n_b, or B's selected rows (Heckman)
  std::vector<std::string> selection_names;  // Heckman: intercept + selection predictors
};

struct ob_matrices {
  int64_t n_a = 0, n_b = 0;
  int32_t k = 0;
  std::vector<double> xa, ya, xb, yb;
  std::vector<std::string> names;
};

namespace ob {

static uint64_t fresh_seed() {
  std::random_device rd;
  return ((uint64_t)rd() << 32) ^ (uint64_t)rd();
}

static int prepare(ob_ctx* ctx, const Frame& input, const Config& c, ob_prepared** out) {
  const bool heck = c.has_selection;
  if (heck && (c.ref == OB_REF_POOLED || c.ref == OB_REF_NEUMARK))
    return fail(OB_E_UNSUPPORTED,
                "Heckman selection with pooled reference coefficients: the reference's pooled beta* has no IMR "
                "entry and its decomposition panics on the dimension mismatch (builder.rs:547-589)");
  if (heck && !c.normalize.empty())
    return fail(OB_E_UNSUPPORTED, "Heckman selection with normalized categoricals is outside the engine's scope");
  if (heck && !c.outcomes.empty())
    return fail(OB_E_UNSUPPORTED, "Heckman selection takes one outcome");
  Staged st;
  OB_TRY(stage(input, c, st));
  if (st.split.a.empty() || st.split.b.empty())  // builder.rs:431-435
    return fail(OB_E_GROUP, "%sOne group has no data", error_prefix(OB_E_GROUP));
  Design da, db;
  OB_TRY(prepare_data(st.df, st.split.a, c, st.dummy_names, true, da));
  OB_TRY(prepare_data(st.df, st.split.b, c, st.dummy_names, true, db));
  const int p = (int)(c.predictors.size() + st.dummy_names.size());
  const int k = p + 1;
  // ols() check order for A then B (ols.rs:60-66 negative weights, ols.rs:98-105 n <= k)
  for (const Design* d : {&da, &db}) {
    if (heck) break;  // the Heckman OLS is unweighted and its row count varies: checked on the GPU
    if (c.has_weights)
      for (double w : d->w)
        if (w < 0.0) return fail(OB_E_GROUP, "%sWeights cannot be negative", error_prefix(OB_E_GROUP));
    if ((double)d->n <= (double)k)
      return fail(OB_E_INSUFFICIENT,
                  "%sInsufficient data for OLS calculation: n_obs (%lld) must be strictly greater than k (%d)",
                  error_prefix(OB_E_INSUFFICIENT), (long long)d->n, k);
  }
  // names: [intercept, predictors, dummies] and the pooled list with the indicator
  std::vector<std::string> names = {"__ob_intercept__"};
  names.insert(names.end(), c.predictors.begin(), c.predictors.end());
  names.insert(names.end(), st.dummy_names.begin(), st.dummy_names.end());
  std::vector<std::string> pooled = {"__ob_intercept__"};
  pooled.insert(pooled.end(), c.predictors.begin(), c.predictors.end());
  pooled.push_back("__ob_group_indicator__");
  pooled.insert(pooled.end(), st.dummy_names.begin(), st.dummy_names.end());
  std::vector<int32_t> nstart = {0}, nidx, nm, pstart = {0}, pidx, has;
  std::vector<std::string> base_names;
  for (const auto& var : c.normalize) {
    const std::string pre = var + "_";
    for (int i = 0; i < (int)names.size(); ++i)
      if (starts_with(names[i], pre)) nidx.push_back(i);
    for (int i = 0; i < (int)pooled.size(); ++i)
      if (starts_with(pooled[i], pre)) pidx.push_back(i);
    nstart.push_back((int32_t)nidx.size());
    pstart.push_back((int32_t)pidx.size());
    auto cc = st.category_counts.find(var);
    nm.push_back(cc == st.category_counts.end() ? -1 : (int32_t)cc->second);
    auto bc = st.base_categories.find(var);
    has.push_back(bc != st.base_categories.end() ? 1 : 0);
    if (bc != st.base_categories.end()) base_names.push_back(bc->second);
  }
  ob_panel_desc pd{};
  pd.p = p;
  pd.n_num = (int32_t)c.predictors.size();
  pd.weighted = c.has_weights ? 1 : 0;
  pd.a = {da.n, da.x.data(), da.n, da.y.data(), c.has_weights ? da.w.data() : nullptr};
  pd.b = {db.n, db.x.data(), db.n, db.y.data(), c.has_weights ? db.w.data() : nullptr};
  pd.n_norm = (int32_t)c.normalize.size();
  pd.norm_start = nstart.data();
  pd.norm_idx = nidx.data();
  pd.norm_m = nm.data();
  pd.pooled_start = pstart.data();
  pd.pooled_idx = pidx.data();
  pd.has_base = has.data();
  pd.n_y = c.outcomes.empty() ? 1 : (int32_t)c.outcomes.size();
  // Heckman: selection outcome s (f64, prepare_selection_data's `.f64()?`) and z per group
  std::vector<double> hs[2], hz[2];
  int64_t n_b_sel = 0;
  if (heck) {
    const int si = st.df.find(c.selection);
    if (si < 0) return fail(OB_E_COLUMN, "%s%s", error_prefix(OB_E_COLUMN), c.selection.c_str());
    if (st.df.cols[si].kind != OB_COL_F64)
      return fail(OB_E_POLARS, "%sinvalid series dtype: expected `Float64`, got `%s` for `%s`", error_prefix(OB_E_POLARS),
                  dtype_name(st.df.cols[si].kind), c.selection.c_str());
    const std::vector<int64_t>* grows[2] = {&st.split.a, &st.split.b};
    const size_t nz = c.selection_predictors.size();
    for (int g = 0; g < 2; ++g) {
      const auto& rows = *grows[g];
      const size_t n = rows.size();
      hs[g].resize(n);
      for (size_t r = 0; r < n; ++r) hs[g][r] = st.df.cols[si].f[rows[r]];
      hz[g].assign(n * nz, 0.0);
      for (size_t j = 0; j < nz; ++j) {
        const int ci = st.df.find(c.selection_predictors[j]);
        if (ci < 0) return fail(OB_E_COLUMN, "%s%s", error_prefix(OB_E_COLUMN), c.selection_predictors[j].c_str());
        for (size_t r = 0; r < n; ++r) OB_TRY(numeric_value(st.df.cols[ci], rows[r], hz[g][j * n + r]));
      }
    }
    for (double v : hs[1]) n_b_sel += v == 1.0 ? 1 : 0;
    pd.heckman = 1;
    pd.n_zsel = (int32_t)nz;
    pd.sa = hs[0].data();
    pd.sb = hs[1].data();
    pd.za = hz[0].data();
    pd.zb = hz[1].data();
    names.push_back("IMR");  // estimation.rs:148-149
  }
  ob_prepared* pr = new ob_prepared();
  pr->ctx = ctx;
  pr->cfg = c;
  pr->ref = c.ref;
  pr->seed = c.has_seed ? c.seed : fresh_seed();
  int rc = ob_panel_create(ctx, &pd, &pr->panel);
  if (rc != OB_OK) {
    delete pr;
    return rc;
  }
  pr->k = heck ? k + 1 : k;
  pr->n_base = ob_panel_n_base(pr->panel);
  pr->row_len = ob_panel_row_len(pr->panel);
  pr->names = names;
  pr->detail_names = names;
  pr->detail_names.insert(pr->detail_names.end(), base_names.begin(), base_names.end());
  pr->n_a = da.n;
  pr->n_b = db.n;
  pr->n_y = pd.n_y;
  pr->n_resid = heck ? n_b_sel : db.n;
  if (heck) {
    pr->selection_names = {"__ob_intercept__"};
    pr->selection_names.insert(pr->selection_names.end(), c.selection_predictors.begin(),
                               c.selection_predictors.end());
  }
  pr->point_row.assign((size_t)pr->row_len * pr->n_y, 0.0);
  pr->resid_b.assign((size_t)pr->n_resid * pr->n_y, 0.0);  // Heckman: zeros (estimation.rs:152-153)
  rc = ob_point_estimate(pr->panel, pr->ref, pr->point_row.data(), heck ? nullptr : pr->resid_b.data());
  if (rc != OB_OK) {
    ob_panel_destroy(pr->panel);
    delete pr;
    return rc;
  }
  *out = pr;
  return OB_OK;
}

// builder.rs:841-950 over successful rows in replicate order, for outcome t (rows/ok: its block).
static int finish(const ob_prepared* pr, int t_out, const double* rows, const uint8_t* ok, uint64_t n_reps,
                  ob_results** out) {
  const int k = pr->k, kd = k + pr->n_base, rl = pr->row_len;
  const double* point_row = pr->point_row.data() + (size_t)t_out * rl;
  uint64_t ng = 0;
  for (uint64_t r = 0; r < n_reps; ++r) ng += ok[r] ? 1 : 0;
  if (ng < n_reps)
    fprintf(stderr,
            "Warning: %llu out of %llu bootstrap replications failed and were discarded. The analysis is based on "
            "%llu successful replications.\n",
            (unsigned long long)(n_reps - ng), (unsigned long long)n_reps, (unsigned long long)ng);
  ob_results* res = new ob_results();
  res->total_gap = point_row[OB_ROW_TOTAL_GAP];
  res->n_a = pr->n_a;
  res->n_b = pr->n_b;
  res->n_failed = (int64_t)(n_reps - ng);
  res->residuals.assign(pr->resid_b.begin() + (size_t)t_out * pr->n_resid,
                        pr->resid_b.begin() + (size_t)(t_out + 1) * pr->n_resid);
  const double* tail = point_row + 6 + 2 * kd;
  res->xa_mean.assign(tail + 2 * k, tail + 3 * k);
  res->xb_mean.assign(tail + 3 * k, tail + 4 * k);
  res->beta_star.assign(tail + 4 * k, tail + 5 * k);

  struct Job {
    int table;
    std::string name;
    double point;
    std::vector<int> cols;  // row offsets whose values feed this component, in order
  };
  std::vector<Job> jobs;
  const char* two[2] = {"explained", "unexplained"};
  const char* three[3] = {"endowments", "coefficients", "interaction"};
  for (int i = 0; i < 2; ++i) jobs.push_back({OB_TABLE_TWO_FOLD, two[i], point_row[i], {i}});
  for (int i = 0; i < 3; ++i) jobs.push_back({OB_TABLE_THREE_FOLD, three[i], point_row[2 + i], {2 + i}});
  // process_detailed_components: estimates merged by variable name (builder.rs:963-971)
  for (int t = 0; t < 2; ++t) {
    const int base = 6 + t * kd;
    for (int i = 0; i < kd; ++i) {
      Job j{t == 0 ? OB_TABLE_DETAILED_EXPLAINED : OB_TABLE_DETAILED_UNEXPLAINED, pr->detail_names[i],
            point_row[base + i], {}};
      for (int q = 0; q < kd; ++q)
        if (pr->detail_names[q] == pr->detail_names[i]) j.cols.push_back(base + q);
      jobs.push_back(std::move(j));
    }
  }
  // Heckman: detailed_selection (builder.rs:510-530), after the 5K' coefficient/mean tail
  const int sel0 = 6 + 2 * kd + 5 * k;
  for (size_t i = 0; i < pr->selection_names.size(); ++i)
    jobs.push_back({OB_TABLE_DETAILED_SELECTION, pr->selection_names[i], point_row[sel0 + i], {sel0 + (int)i}});
  std::vector<std::vector<int>> groups;
  for (const Job& j : jobs) groups.push_back(j.cols);
  std::vector<double> st(4 * jobs.size());
  aggregate(rows, ok, n_reps, rl, groups, st.data());
  std::vector<ob_results::Comp> comps(jobs.size());
  for (size_t ji = 0; ji < jobs.size(); ++ji) {
    const double* s4 = st.data() + 4 * ji;
    const double t = std::fabs(s4[0]) > 1e-9 ? jobs[ji].point / s4[0] : 0.0;  // builder.rs:851-855
    comps[ji] = {jobs[ji].name, jobs[ji].point, s4[0], t, s4[1], s4[2], s4[3]};
  }
  for (size_t ji = 0; ji < jobs.size(); ++ji) res->tables[jobs[ji].table].push_back(comps[ji]);
  *out = res;
  return OB_OK;
}

// prepare + every replicate + finish for each outcome: out[t] for t < n_y (OaxacaBuilder::run).
static int run_all(ob_ctx* ctx, const Frame& f, const Config& c, ob_results** out) {
  ob_prepared* pr = nullptr;
  OB_TRY(prepare(ctx, f, c, &pr));
  const size_t ny = (size_t)pr->n_y;
  std::vector<double> rows((size_t)c.reps * pr->row_len * ny);
  std::vector<uint8_t> ok(c.reps * ny, 0);
  int rc = OB_OK;
  if (c.reps > 0) rc = ob_boot_run(pr->panel, pr->seed, 0, c.reps, pr->ref, rows.data(), ok.data());
  for (size_t t = 0; t < ny && rc == OB_OK; ++t) {
    rc = finish(pr, (int)t, rows.data() + t * c.reps * pr->row_len, ok.data() + t * c.reps, c.reps, &out[t]);
    if (rc != OB_OK)
      for (size_t u = 0; u < t; ++u) {
        delete out[u];
        out[u] = nullptr;
      }
  }
  ob_panel_destroy(pr->panel);
  delete pr;
  return rc;
}

}  // namespace ob

// ---------------------------------------------------------------------------------------------
// Machado-Mata: QuantileDecompositionBuilder::run (quantile_decomposition.rs:21-445)
// ---------------------------------------------------------------------------------------------
struct ob_qd_results {
  int64_t n_a = 0, n_b = 0, n_failed = 0;
  std::vector<std::string> keys;
  std::vector<std::vector<ob_results::Comp>> comps;  // per key: Total Gap, Characteristics, Coefficients
};

namespace ob {

struct QdConfig {
  std::string outcome, group, reference_group;
  std::vector<std::string> predictors, categorical;
  std::vector<double> quantiles;
  int sims = 200;
  uint64_t reps = 20;
  bool has_seed = false;
  uint64_t seed = 0;
};

// prepare_data (quantile_decomposition.rs:96-141): y must be Float64 without nulls; X columns =
// predictors then dummies (intercept implicit); a null predictor value reads as NaN (to_ndarray).
static int qd_design(const Frame& f, const std::vector<int64_t>& rows, const QdConfig& c,
                     const std::vector<std::string>& dummy_names, Design& d) {
  const int yi = f.find(c.outcome);
  if (f.cols[yi].kind != OB_COL_F64)
    return fail(OB_E_POLARS, "%sinvalid series dtype: expected `Float64`, got `%s` for `%s`", error_prefix(OB_E_POLARS),
                dtype_name(f.cols[yi].kind), c.outcome.c_str());
  const int64_t n = (int64_t)rows.size();
  d.n = n;
  d.y.resize(n);
  for (int64_t r = 0; r < n; ++r) {
    if (!f.cols[yi].valid[rows[r]])
      return fail(OB_E_GROUP, "%sNull outcome encountered", error_prefix(OB_E_GROUP));
    d.y[r] = f.cols[yi].f[rows[r]];
  }
  std::vector<std::string> xs = c.predictors;
  xs.insert(xs.end(), dummy_names.begin(), dummy_names.end());
  d.x.assign((size_t)n * xs.size(), 0.0);
  for (size_t j = 0; j < xs.size(); ++j) {
    const int ci = f.find(xs[j]);
    for (int64_t r = 0; r < n; ++r) {
      if (!f.cols[ci].valid[rows[r]]) {
        d.x[j * n + r] = NAN;
        continue;
      }
      OB_TRY(numeric_value(f.cols[ci], rows[r], d.x[j * n + r]));
    }
  }
  return OB_OK;
}

static int qd_run(ob_ctx* ctx, const Frame& f, const QdConfig& c, ob_qd_results** out) {
  std::vector<std::string> need = {c.outcome, c.group};  // df.select (:284-287): no null cleaning
  need.insert(need.end(), c.predictors.begin(), c.predictors.end());
  need.insert(need.end(), c.categorical.begin(), c.categorical.end());
  for (const auto& nm : need)
    if (f.find(nm) < 0) return fail(OB_E_COLUMN, "%s%s", error_prefix(OB_E_COLUMN), nm.c_str());
  if (c.quantiles.empty()) return fail(OB_E_INVALID, "no target quantiles");
  Frame df = f;
  std::vector<std::string> dummy_names;
  for (const auto& cat : c.categorical) {  // create_dummies_manual (:143-161); a null level reads NaN
    const int ci = df.find(cat);
    Dummies dm;
    OB_TRY(create_dummies(df.cols[ci], dm));
    for (auto& col : dm.cols) {
      if (df.find(col.name) >= 0)
        return fail(OB_E_POLARS, "%sduplicate: column with name '%s' has more than one occurrence",
                    error_prefix(OB_E_POLARS), col.name.c_str());
      for (int64_t r = 0; r < df.nrows; ++r)
        if (!df.cols[ci].valid[r]) col.f[r] = NAN;
      dummy_names.push_back(col.name);
      df.cols.push_back(std::move(col));
    }
  }
  const Col& g = df.cols[df.find(c.group)];  // run_single_pass (:178-206)
  OB_TRY(expect_str(g));
  const auto levels = sorted_levels(g);
  if (levels.size() < 2) return fail(OB_E_GROUP, "%sNot enough groups", error_prefix(OB_E_GROUP));
  const std::string& name_b = c.reference_group;
  const std::string name_a = levels[0] != name_b ? levels[0] : levels[1];
  std::vector<int64_t> ra, rb;
  for (int64_t r = 0; r < df.nrows; ++r) {
    if (!g.valid[r]) continue;
    if (g.s[r] == name_a) ra.push_back(r);
    if (g.s[r] == name_b) rb.push_back(r);
  }
  if (ra.size() < 2 || rb.size() < 2)
    return fail(OB_E_GROUP, "%sOne group has insufficient data", error_prefix(OB_E_GROUP));
  Design da, db;
  OB_TRY(qd_design(df, ra, c, dummy_names, da));
  OB_TRY(qd_design(df, rb, c, dummy_names, db));
  const int p = (int)(c.predictors.size() + dummy_names.size());
  if (p + 1 > kMmMaxK)
    return fail(OB_E_UNSUPPORTED, "Machado-Mata takes at most %d predictor columns (dummies included), got %d",
                kMmMaxK - 1, p);
  ob_panel_desc pd{};
  pd.p = p;
  pd.n_num = (int32_t)c.predictors.size();
  pd.a = {da.n, da.x.data(), da.n, da.y.data(), nullptr};
  pd.b = {db.n, db.x.data(), db.n, db.y.data(), nullptr};
  pd.n_y = 1;
  ob_panel* panel = nullptr;
  OB_TRY(ob_panel_create(ctx, &pd, &panel));
  const int nq = (int)c.quantiles.size();
  std::vector<double> rows((size_t)(1 + c.reps) * 3 * nq);
  std::vector<uint8_t> ok(1 + c.reps, 0);
  const uint64_t seed = c.has_seed ? c.seed : fresh_seed();
  int rc = mm_run(panel, seed, c.sims, c.quantiles.data(), nq, 0, c.reps, true, rows.data(), ok.data(), nullptr);
  ob_panel_destroy(panel);
  if (rc != OB_OK) return rc;
  if (!ok[0])  // the point pass failed (:231-236)
    return fail(OB_E_LINALG, "%sFailed to estimate a sufficient number of quantile regressions.",
                error_prefix(OB_E_LINALG));
  ob_qd_results* res = new ob_qd_results();
  for (int64_t r = 0; r < f.nrows; ++r) {  // n_a / n_b over the whole frame (:423-441)
    if (!g.valid[r]) continue;
    res->n_a += g.s[r] == name_a;
    res->n_b += g.s[r] == name_b;
  }
  uint64_t ng = 0;
  for (uint64_t r = 0; r < c.reps; ++r) ng += ok[1 + r] ? 1 : 0;
  res->n_failed = (int64_t)(c.reps - ng);
  // keys "q{floor(100 tau)}" (:270); a repeated key keeps the later quantile (HashMap::insert)
  std::vector<int> slot_of_key;
  for (int j = 0; j < nq; ++j) {
    const std::string key = "q" + std::to_string((uint32_t)(c.quantiles[j] * 100.0));
    auto it = std::find(res->keys.begin(), res->keys.end(), key);
    if (it == res->keys.end()) {
      res->keys.push_back(key);
      slot_of_key.push_back(j);
    } else {
      slot_of_key[it - res->keys.begin()] = j;
    }
  }
  static const char* names[3] = {"Total Gap", "Characteristics", "Coefficients"};
  std::vector<double> v;
  for (size_t e = 0; e < res->keys.size(); ++e) {
    const int j = slot_of_key[e];
    std::vector<ob_results::Comp> cs;
    for (int k = 0; k < 3; ++k) {
      v.clear();
      for (uint64_t r = 0; r < c.reps; ++r)
        if (ok[1 + r]) v.push_back(rows[(1 + r) * 3 * nq + 3 * j + k]);
      double s4[4];
      bootstrap_stats(v.data(), (int64_t)v.size(), s4);
      const double pt = rows[3 * j + k];
      cs.push_back({names[k], pt, s4[0], std::fabs(s4[0]) > 1e-9 ? pt / s4[0] : 0.0, s4[1], s4[2], s4[3]});
    }
    res->comps.push_back(std::move(cs));
  }
  *out = res;
  return OB_OK;
}

}  // namespace ob

extern "C" {

int ob_quantile_decomposition_run(ob_ctx* ctx, const ob_column* cols, int32_t n_cols, int64_t n_rows,
                                  const ob_qd_config* cfg, ob_qd_results** out) {
  if (!ctx || !cfg || !out) return ob::fail(OB_E_INVALID, "null pointer");
  *out = nullptr;
  if (!cfg->outcome || !cfg->group || !cfg->reference_group) return ob::fail(OB_E_INVALID, "incomplete config");
  ob::QdConfig c;
  c.outcome = cfg->outcome;
  c.group = cfg->group;
  c.reference_group = cfg->reference_group;
  for (int i = 0; i < cfg->n_predictors; ++i) c.predictors.emplace_back(cfg->predictors[i]);
  for (int i = 0; i < cfg->n_categorical; ++i) c.categorical.emplace_back(cfg->categorical[i]);
  if (cfg->quantiles && cfg->n_quantiles > 0)
    c.quantiles.assign(cfg->quantiles, cfg->quantiles + cfg->n_quantiles);
  else
    c.quantiles = {0.1, 0.25, 0.5, 0.75, 0.9};  // :56
  c.sims = cfg->simulations;
  c.reps = cfg->bootstrap_reps;
  c.has_seed = cfg->has_seed != 0;
  c.seed = cfg->seed;
  ob::Frame f;
  OB_TRY(ob::load_frame(cols, n_cols, n_rows, f));
  return ob::qd_run(ctx, f, c, out);
}

int ob_qd_results_dims(const ob_qd_results* r, int32_t* n_entries, int64_t* n_a, int64_t* n_b) {
  if (!r) return ob::fail(OB_E_INVALID, "null pointer");
  if (n_entries) *n_entries = (int32_t)r->keys.size();
  if (n_a) *n_a = r->n_a;
  if (n_b) *n_b = r->n_b;
  return OB_OK;
}

int ob_qd_results_get(const ob_qd_results* r, int32_t i, const char** key, ob_component* comps) {
  if (!r || i < 0 || i >= (int32_t)r->keys.size()) return ob::fail(OB_E_INVALID, "entry index out of range");
  if (key) *key = r->keys[i].c_str();
  if (comps)
    for (int k = 0; k < 3; ++k) {
      const auto& c = r->comps[i][k];
      comps[k] = {c.name.c_str(), c.estimate, c.std_err, c.t_stat, c.p_value, c.ci_lower, c.ci_upper};
    }
  return OB_OK;
}

int64_t ob_qd_results_n_failed(const ob_qd_results* r) { return r ? r->n_failed : 0; }

void ob_qd_results_free(ob_qd_results* r) { delete r; }

}  // extern "C"

extern "C" {

int ob_builder_prepare(ob_ctx* ctx, const ob_column* cols, int32_t n_cols, int64_t n_rows,
                       const ob_builder_config* cfg, ob_prepared** out) {
  if (!ctx || !out) return ob::fail(OB_E_INVALID, "null pointer");
  *out = nullptr;
  ob::Frame f;
  ob::Config c;
  OB_TRY(ob::config_from(cfg, c));
  OB_TRY(ob::load_frame(cols, n_cols, n_rows, f));
  return ob::prepare(ctx, f, c, out);
}

int ob_prepared_row_len(const ob_prepared* p) { return p ? p->row_len : 0; }
int ob_prepared_n_y(const ob_prepared* p) { return p ? p->n_y : 0; }
uint64_t ob_prepared_seed(const ob_prepared* p) { return p ? p->seed : 0; }
ob_panel* ob_prepared_panel(ob_prepared* p) { return p ? p->panel : nullptr; }

int ob_prepared_boot(ob_prepared* p, uint64_t first_rep, uint64_t n_reps, double* rows, uint8_t* ok) {
  if (!p) return ob::fail(OB_E_INVALID, "null pointer");
  return ob_boot_run(p->panel, p->seed, first_rep, n_reps, p->ref, rows, ok);
}

int ob_prepared_boot_sharded(ob_prepared* p, uint64_t first_rep, uint64_t n_reps, double* rows, uint8_t* ok) {
  if (!p) return ob::fail(OB_E_INVALID, "null pointer");
  // the RCCL all-gather moves only the columns finish() aggregates: two-fold, three-fold, total
  // gap, detailed [0, 6 + 2 Kd) and a Heckman row's selection terms after its 5K' tail
  const int kd = p->k + p->n_base, sel0 = 6 + 2 * kd + 5 * p->k;
  std::vector<int32_t> cols;
  for (int c = 0; c < 6 + 2 * kd; ++c) cols.push_back(c);
  for (size_t i = 0; i < p->selection_names.size(); ++i) cols.push_back(sel0 + (int)i);
  // the narrowing holds for this call only: the panel's own column set is restored afterwards, so a
  // later ob_boot_run_sharded on ob_prepared_panel(p) gathers what its caller asked for
  const std::vector<int32_t> saved = p->panel->gather_cols;
  OB_TRY(ob_panel_set_gather_columns(p->panel, cols.data(), (int32_t)cols.size()));
  const int rc = ob_boot_run_sharded(p->panel, p->seed, first_rep, n_reps, p->ref, rows, ok);
  const int rc2 = ob_panel_set_gather_columns(p->panel, saved.data(), (int32_t)saved.size());
  return rc != OB_OK ? rc : rc2;
}

int ob_prepared_boot_device(ob_prepared* p, uint64_t first_rep, uint64_t n_reps, double* d_rows, uint8_t* d_ok,
                            void* hip_stream) {
  if (!p) return ob::fail(OB_E_INVALID, "null pointer");
  return ob_boot_run_device(p->panel, p->seed, first_rep, n_reps, p->ref, d_rows, d_ok, hip_stream);
}

int ob_prepared_finish(ob_prepared* p, const double* rows, const uint8_t* ok, uint64_t n_reps, ob_results** out) {
  if (!p || !out || (n_reps && (!rows || !ok))) return ob::fail(OB_E_INVALID, "null pointer");
  *out = nullptr;
  return ob::finish(p, 0, rows, ok, n_reps, out);
}

void ob_prepared_destroy(ob_prepared* p) {
  if (!p) return;
  ob_panel_destroy(p->panel);
  delete p;
}

int ob_builder_run(ob_ctx* ctx, const ob_column* cols, int32_t n_cols, int64_t n_rows, const ob_builder_config* cfg,
                   ob_results** out) {
  if (!ctx || !out) return ob::fail(OB_E_INVALID, "null pointer");
  *out = nullptr;
  ob::Frame f;
  ob::Config c;
  OB_TRY(ob::config_from(cfg, c));
  OB_TRY(ob::load_frame(cols, n_cols, n_rows, f));
  return ob::run_all(ctx, f, c, out);
}

// builder.rs:711-757: RIF of each group's outcome on the cleaned data, then run() on vstack(A, B).
// Several quantiles share one panel: the RIF columns are the panel's outcomes (n_y = n_taus), so
// one Gram pass serves every tau; out[t] is bitwise the single-tau run.
static int decompose_quantiles(ob_ctx* ctx, const ob_column* cols, int32_t n_cols, int64_t n_rows,
                               const ob_builder_config* cfg, const double* taus, int32_t n_taus, ob_results** out) {
  if (!ctx || !out || !taus || n_taus < 1) return ob::fail(OB_E_INVALID, "null pointer or no quantiles");
  for (int32_t t = 0; t < n_taus; ++t) out[t] = nullptr;
  ob::Frame f, df;
  ob::Config c;
  OB_TRY(ob::config_from(cfg, c));
  OB_TRY(ob::load_frame(cols, n_cols, n_rows, f));
  OB_TRY(ob::clean_dataframe(f, c, df));
  ob::Split sp;
  OB_TRY(ob::split_groups(df, c, sp));
  const int yi = df.find(c.outcome);
  if (df.cols[yi].kind != OB_COL_F64)
    return ob::fail(OB_E_POLARS, "%sinvalid series dtype: expected `Float64`, got `%s`", ob::error_prefix(OB_E_POLARS),
                    ob::dtype_name(df.cols[yi].kind));
  std::vector<int64_t> order = sp.a;
  order.insert(order.end(), sp.b.begin(), sp.b.end());
  ob::Frame mod = ob::take(df, order);
  const int mi = mod.find(c.outcome);
  const size_t na = sp.a.size(), nb = sp.b.size();
  std::vector<double> ya(na), yb(nb), ra(na), rb(nb);
  for (size_t i = 0; i < na; ++i) ya[i] = mod.cols[mi].f[i];
  for (size_t i = 0; i < nb; ++i) yb[i] = mod.cols[mi].f[na + i];
  for (int32_t t = 0; t < n_taus; ++t) {
    ob::rif(ya.data(), (int64_t)na, taus[t], ra.data());
    ob::rif(yb.data(), (int64_t)nb, taus[t], rb.data());
    ob::Col rc = mod.cols[mi];
    rc.name = "__ob_rif_" + std::to_string(t) + "__";
    for (size_t i = 0; i < na; ++i) rc.f[i] = ra[i];
    for (size_t i = 0; i < nb; ++i) rc.f[na + i] = rb[i];
    if (n_taus == 1) {
      mod.cols[mi] = std::move(rc);  // the reference's own layout: the outcome column replaced
      mod.cols[mi].name = c.outcome;
    } else {
      c.outcomes.push_back(rc.name);
      mod.cols.push_back(std::move(rc));
    }
  }
  c.has_selection = false;  // the new builder carries no Heckman settings (builder.rs:743-754)
  c.selection_predictors.clear();
  return ob::run_all(ctx, mod, c, out);
}

int ob_builder_decompose_quantile(ob_ctx* ctx, const ob_column* cols, int32_t n_cols, int64_t n_rows,
                                  const ob_builder_config* cfg, double quantile, ob_results** out) {
  return decompose_quantiles(ctx, cols, n_cols, n_rows, cfg, &quantile, 1, out);
}

int ob_builder_decompose_quantiles(ob_ctx* ctx, const ob_column* cols, int32_t n_cols, int64_t n_rows,
                                   const ob_builder_config* cfg, const double* taus, int32_t n_taus,
                                   ob_results** out) {
  return decompose_quantiles(ctx, cols, n_cols, n_rows, cfg, taus, n_taus, out);
}

int ob_builder_data_matrices(const ob_column* cols, int32_t n_cols, int64_t n_rows, const ob_builder_config* cfg,
                             ob_matrices** out) {
  if (!out) return ob::fail(OB_E_INVALID, "null pointer");
  *out = nullptr;
  ob::Frame f;
  ob::Config c;
  OB_TRY(ob::config_from(cfg, c));
  OB_TRY(ob::load_frame(cols, n_cols, n_rows, f));
  ob::Staged st;
  OB_TRY(ob::stage(f, c, st));
  ob::Design da, db;
  OB_TRY(ob::prepare_data(st.df, st.split.a, c, st.dummy_names, false, da));
  OB_TRY(ob::prepare_data(st.df, st.split.b, c, st.dummy_names, false, db));
  ob_matrices* m = new ob_matrices();
  m->k = (int32_t)(c.predictors.size() + st.dummy_names.size() + 1);
  m->n_a = da.n;
  m->n_b = db.n;
  auto with_intercept = [&](const ob::Design& d, std::vector<double>& x) {
    x.assign((size_t)d.n * m->k, 1.0);
    std::copy(d.x.begin(), d.x.end(), x.begin() + d.n);
  };
  with_intercept(da, m->xa);
  with_intercept(db, m->xb);
  m->ya = da.y;
  m->yb = db.y;
  m->names = {"__ob_intercept__"};
  m->names.insert(m->names.end(), c.predictors.begin(), c.predictors.end());
  m->names.insert(m->names.end(), st.dummy_names.begin(), st.dummy_names.end());
  *out = m;
  return OB_OK;
}

double ob_results_total_gap(const ob_results* r) { return r ? r->total_gap : NAN; }
int64_t ob_results_n_a(const ob_results* r) { return r ? r->n_a : 0; }
int64_t ob_results_n_b(const ob_results* r) { return r ? r->n_b : 0; }
int64_t ob_results_n_failed(const ob_results* r) { return r ? r->n_failed : 0; }

int ob_results_count(const ob_results* r, int32_t table) {
  if (!r || table < 0 || table > 4) return -1;
  return (int)r->tables[table].size();
}

int ob_results_component(const ob_results* r, int32_t table, int32_t i, ob_component* out) {
  if (!r || !out || table < 0 || table > 4 || i < 0 || i >= (int)r->tables[table].size())
    return ob::fail(OB_E_INVALID, "component index out of range");
  const auto& c = r->tables[table][i];
  *out = {c.name.c_str(), c.estimate, c.std_err, c.t_stat, c.p_value, c.ci_lower, c.ci_upper};
  return OB_OK;
}

int ob_results_vector(const ob_results* r, int32_t which, const double** data, int64_t* len) {
  if (!r || !data || !len) return ob::fail(OB_E_INVALID, "null pointer");
  const std::vector<double>* v = nullptr;
  switch (which) {
    case OB_VEC_RESIDUALS: v = &r->residuals; break;
    case OB_VEC_XA_MEAN: v = &r->xa_mean; break;
    case OB_VEC_XB_MEAN: v = &r->xb_mean; break;
    case OB_VEC_BETA_STAR: v = &r->beta_star; break;
    default: return ob::fail(OB_E_INVALID, "unknown vector %d", which);
  }
  *data = v->data();
  *len = (int64_t)v->size();
  return OB_OK;
}

void ob_results_free(ob_results* r) { delete r; }

int ob_matrices_dims(const ob_matrices* m, int64_t* n_a, int64_t* n_b, int32_t* k) {
  if (!m || !n_a || !n_b || !k) return ob::fail(OB_E_INVALID, "null pointer");
  *n_a = m->n_a;
  *n_b = m->n_b;
  *k = m->k;
  return OB_OK;
}

int ob_matrices_get(const ob_matrices* m, const double** x_a, const double** y_a, const double** x_b,
                    const double** y_b) {
  if (!m || !x_a || !y_a || !x_b || !y_b) return ob::fail(OB_E_INVALID, "null pointer");
  *x_a = m->xa.data();
  *y_a = m->ya.data();
  *x_b = m->xb.data();
  *y_b = m->yb.data();
  return OB_OK;
}

const char* ob_matrices_name(const ob_matrices* m, int32_t i) {
  if (!m || i < 0 || i >= (int32_t)m->names.size()) return nullptr;
  return m->names[i].c_str();
}

void ob_matrices_free(ob_matrices* m) { delete m; }

}  // extern "C"
