// ob_csv.cpp -- the CSV front end of the reference CLI (main.rs:161-165, polars LazyCsvReader with
// has_header = true), as the ingestion step before the builder: a header row, one column per
// field, dtypes inferred from the first 100 data rows like polars' default infer_schema_length
// (i64 if every non-empty field parses as an integer, else f64 if every one parses as a float,
// else str), an empty field is a null, RFC 4180 double quotes. A later field that does not
// parse as its column's inferred dtype is an error (polars: "could not parse ... as dtype").
// Large unquoted files are parsed by several threads, one line range each.
#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "ob_common.hpp"

struct ob_csv {
  int64_t nrows = 0;
  std::vector<std::string> names;
  std::vector<int32_t> kinds;
  std::vector<std::vector<double>> f;
  std::vector<std::vector<int64_t>> i;
  std::vector<std::vector<std::string>> s;
  std::vector<std::vector<const char*>> sp;  // ob_column.str views (NULL = null)
  std::vector<std::vector<uint8_t>> valid;
};

namespace {

constexpr int kInferRows = 100;

struct Field {
  const char* p;
  size_t n;
  bool quoted;
};

// Splits one line [b, e) into fields; quoted fields keep their quotes for unquote().
void split_line(const char* b, const char* e, std::vector<Field>& out) {
  out.clear();
  const char* p = b;
  while (true) {
    const char* start = p;
    bool quoted = false;
    if (p < e && *p == '"') {
      quoted = true;
      ++p;
      while (p < e) {
        if (*p == '"') {
          if (p + 1 < e && p[1] == '"') {
            p += 2;
            continue;
          }
          ++p;
          break;
        }
        ++p;
      }
      while (p < e && *p != ',') ++p;
    } else {
      while (p < e && *p != ',') ++p;
    }
    out.push_back({start, (size_t)(p - start), quoted});
    if (p >= e) break;
    ++p;  // the comma
    if (p == e) {
      out.push_back({p, 0, false});
      break;
    }
  }
}

std::string unquote(const Field& f) {
  if (!f.quoted) return std::string(f.p, f.n);
  std::string r;
  const char* p = f.p + 1;
  const char* e = f.p + f.n;
  while (p < e) {
    if (*p == '"') {
      if (p + 1 < e && p[1] == '"') {
        r.push_back('"');
        p += 2;
        continue;
      }
      break;
    }
    r.push_back(*p++);
  }
  return r;
}

bool parse_i64(const std::string& t, int64_t& v) {
  if (t.empty()) return false;
  const char* b = t.c_str();
  char* end = nullptr;
  errno = 0;
  long long x = std::strtoll(b, &end, 10);
  if (errno != 0 || end != b + t.size()) return false;
  v = (int64_t)x;
  return true;
}

bool parse_f64(const std::string& t, double& v) {
  if (t.empty()) return false;
  const char* b = t.c_str();
  char* end = nullptr;
  v = std::strtod(b, &end);
  return end == b + t.size();
}

// Line starts/ends (a trailing '\r' is stripped). Quoted newlines are not split when the
// file contains quotes (then the scan runs sequentially with quote tracking).
void find_lines(const char* data, size_t size, std::vector<std::pair<size_t, size_t>>& lines) {
  const bool has_quote = size && std::memchr(data, '"', size) != nullptr;  // an empty file maps no data
  size_t b = 0;
  bool inq = false;
  for (size_t k = 0; k < size; ++k) {
    const char c = data[k];
    if (has_quote && c == '"') inq = !inq;
    if (c == '\n' && !inq) {
      size_t e = k;
      if (e > b && data[e - 1] == '\r') --e;
      lines.push_back({b, e});
      b = k + 1;
    }
  }
  if (b < size) {
    size_t e = size;
    if (e > b && data[e - 1] == '\r') --e;
    lines.push_back({b, e});
  }
}

}  // namespace

extern "C" {

int ob_csv_read(const char* path, ob_csv** out) {
  if (!path || !out) return ob::fail(OB_E_INVALID, "null pointer");
  *out = nullptr;
  FILE* fp = std::fopen(path, "rb");
  if (!fp) return ob::fail(OB_E_POLARS, "%sNo such file or directory (os error 2): %s", ob::error_prefix(OB_E_POLARS), path);
  std::fseek(fp, 0, SEEK_END);
  const long sz = std::ftell(fp);
  std::fseek(fp, 0, SEEK_SET);
  std::vector<char> buf((size_t)std::max(sz, 0L));
  const size_t got = sz > 0 ? std::fread(buf.data(), 1, (size_t)sz, fp) : 0;
  std::fclose(fp);
  if ((long)got != sz) return ob::fail(OB_E_POLARS, "%sshort read of %s", ob::error_prefix(OB_E_POLARS), path);
  const char* data = buf.data();
  std::vector<std::pair<size_t, size_t>> lines;
  find_lines(data, got, lines);
  // drop empty trailing lines
  while (!lines.empty() && lines.back().first == lines.back().second) lines.pop_back();
  if (lines.empty()) return ob::fail(OB_E_POLARS, "%sempty CSV", ob::error_prefix(OB_E_POLARS));

  ob_csv* c = new ob_csv();
  std::vector<Field> fl;
  split_line(data + lines[0].first, data + lines[0].second, fl);
  for (const Field& f : fl) c->names.push_back(unquote(f));
  const size_t ncol = c->names.size();
  const int64_t nrows = (int64_t)lines.size() - 1;
  c->nrows = nrows;

  // dtype inference over the first kInferRows rows
  std::vector<int> can_int(ncol, 1), can_float(ncol, 1), any(ncol, 0);
  for (int64_t r = 0; r < std::min<int64_t>(nrows, kInferRows); ++r) {
    split_line(data + lines[r + 1].first, data + lines[r + 1].second, fl);
    for (size_t j = 0; j < ncol && j < fl.size(); ++j) {
      const std::string t = unquote(fl[j]);
      if (t.empty()) continue;
      any[j] = 1;
      int64_t iv;
      double dv;
      if (fl[j].quoted || !parse_i64(t, iv)) can_int[j] = 0;
      if (fl[j].quoted || !parse_f64(t, dv)) can_float[j] = 0;
    }
  }
  c->kinds.resize(ncol);
  c->f.resize(ncol);
  c->i.resize(ncol);
  c->s.resize(ncol);
  c->sp.resize(ncol);
  c->valid.resize(ncol);
  for (size_t j = 0; j < ncol; ++j) {
    // an all-null inference window is a string column, as in polars
    c->kinds[j] = !any[j] ? OB_COL_STR : (can_int[j] ? OB_COL_I64 : (can_float[j] ? OB_COL_F64 : OB_COL_STR));
    if (c->kinds[j] == OB_COL_F64) c->f[j].assign(nrows, 0.0);
    if (c->kinds[j] == OB_COL_I64) c->i[j].assign(nrows, 0);
    if (c->kinds[j] == OB_COL_STR) c->s[j].assign(nrows, std::string());
    c->valid[j].assign(nrows, 1);
  }

  // parse all rows, in line ranges over threads
  const int nth = (int)std::min<int64_t>(16, std::max<int64_t>(1, nrows / 50000));
  std::vector<std::string> errs(nth);
  auto work = [&](int t) {
    std::vector<Field> f2;
    const int64_t r0 = nrows * t / nth, r1 = nrows * (t + 1) / nth;
    for (int64_t r = r0; r < r1 && errs[t].empty(); ++r) {
      split_line(data + lines[r + 1].first, data + lines[r + 1].second, f2);
      if (f2.size() != ncol) {
        errs[t] = "found " + std::to_string(f2.size()) + " fields in row " + std::to_string(r) + ", expected " +
                  std::to_string(ncol);
        return;
      }
      for (size_t j = 0; j < ncol; ++j) {
        std::string tv = unquote(f2[j]);
        if (tv.empty() && !f2[j].quoted) {
          c->valid[j][r] = 0;
          continue;
        }
        if (c->kinds[j] == OB_COL_STR) {
          c->s[j][r] = std::move(tv);
        } else if (c->kinds[j] == OB_COL_I64) {
          if (!parse_i64(tv, c->i[j][r])) {
            errs[t] = "could not parse `" + tv + "` as dtype `i64` at column '" + c->names[j] + "'";
            return;
          }
        } else if (!parse_f64(tv, c->f[j][r])) {
          errs[t] = "could not parse `" + tv + "` as dtype `f64` at column '" + c->names[j] + "'";
          return;
        }
      }
    }
  };
  if (nth == 1) {
    work(0);
  } else {
    std::vector<std::thread> ts;
    for (int t = 0; t < nth; ++t) ts.emplace_back(work, t);
    for (auto& th : ts) th.join();
  }
  for (const std::string& e : errs)
    if (!e.empty()) {
      delete c;
      return ob::fail(OB_E_POLARS, "%s%s", ob::error_prefix(OB_E_POLARS), e.c_str());
    }
  for (size_t j = 0; j < ncol; ++j)
    if (c->kinds[j] == OB_COL_STR) {
      c->sp[j].resize(nrows);
      for (int64_t r = 0; r < nrows; ++r) c->sp[j][r] = c->valid[j][r] ? c->s[j][r].c_str() : nullptr;
    }
  *out = c;
  return OB_OK;
}

int ob_csv_dims(const ob_csv* c, int64_t* nrows, int32_t* ncols) {
  if (!c) return ob::fail(OB_E_INVALID, "null pointer");
  if (nrows) *nrows = c->nrows;
  if (ncols) *ncols = (int32_t)c->names.size();
  return OB_OK;
}

int ob_csv_column(const ob_csv* c, int32_t j, ob_column* out) {
  if (!c || !out || j < 0 || j >= (int32_t)c->names.size()) return ob::fail(OB_E_INVALID, "bad column index");
  std::memset(out, 0, sizeof(*out));
  out->name = c->names[j].c_str();
  out->kind = c->kinds[j];
  if (out->kind == OB_COL_F64) out->f64 = c->f[j].data();
  if (out->kind == OB_COL_I64) out->i64 = c->i[j].data();
  if (out->kind == OB_COL_STR) out->str = c->sp[j].data();
  out->valid = c->valid[j].data();
  return OB_OK;
}

void ob_csv_free(ob_csv* c) { delete c; }

}  // extern "C"
