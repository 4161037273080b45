// Host-side sanitizer driver: the C-ABI host paths of liboaxaca_boot -- CSV front
// end (ob_csv.cpp), frame logic of the builder (ob_builder.cpp: clean_dataframe, dummies,
// split_groups, prepare_data via ob_builder_data_matrices), inference (ob_host.cpp) and the
// no-GPU failure of the device entry points -- built with -fsanitize=address,undefined on the
// host side (tests/asan/Makefile) and run by tests/test_asan.py. Exit code 0 = every check held;
// the sanitizers abort on the first finding.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/oaxaca_boot.h"
#include "../../oaxaca-blinder-rs_amd/csrc/ob_shard_layout.h"

static int failures = 0;
#define CHECK(c)                                                        \
  do {                                                                  \
    if (!(c)) {                                                         \
      std::fprintf(stderr, "CHECK failed at %d: %s\n", __LINE__, #c);  \
      ++failures;                                                       \
    }                                                                   \
  } while (0)

static std::string write_file(const char* dir, const char* name, const std::string& text) {
  std::string path = std::string(dir) + "/" + name;
  FILE* f = std::fopen(path.c_str(), "wb");
  std::fwrite(text.data(), 1, text.size(), f);
  std::fclose(f);
  return path;
}

static void csv_and_frames(const char* dir) {
  // quotes with embedded separators and doubled quotes, nulls, ints, floats, strings
  std::string text = "wage,education,experience,gender,sector,note\n";
  const char* sectors[] = {"a", "b", "c"};
  for (int i = 0; i < 400; ++i) {
    char line[256];
    const bool null_exp = i % 37 == 5;
    std::snprintf(line, sizeof line, "%.6f,%d,%s,%s,%s,\"n, \"\"%d\"\"\"\n", 10.0 + 0.05 * i + (i % 7), 8 + i % 13,
                  null_exp ? "" : std::to_string(i % 40).c_str(), i % 2 ? "F" : "M", sectors[i % 3], i);
    text += line;
  }
  ob_csv* csv = nullptr;
  CHECK(ob_csv_read(write_file(dir, "frame.csv", text).c_str(), &csv) == OB_OK);
  int64_t nrows = 0;
  int32_t ncols = 0;
  CHECK(ob_csv_dims(csv, &nrows, &ncols) == OB_OK && nrows == 400 && ncols == 6);
  std::vector<ob_column> cols(ncols);
  for (int32_t i = 0; i < ncols; ++i) CHECK(ob_csv_column(csv, i, &cols[i]) == OB_OK);
  CHECK(cols[0].kind == OB_COL_F64 && cols[1].kind == OB_COL_I64 && cols[3].kind == OB_COL_STR);
  CHECK(cols[2].valid && cols[2].valid[5] == 0);
  CHECK(std::strcmp(cols[5].str[3], "n, \"3\"") == 0);

  const char* preds[] = {"education", "experience"};
  const char* cats[] = {"sector"};
  ob_builder_config cfg{};
  cfg.outcome = "wage";
  cfg.group = "gender";
  cfg.reference_group = "F";
  cfg.predictors = preds;
  cfg.n_predictors = 2;
  cfg.categorical = cats;
  cfg.n_categorical = 1;
  cfg.normalize = cats;
  cfg.n_normalize = 1;
  cfg.bootstrap_reps = 20;
  ob_matrices* m = nullptr;
  CHECK(ob_builder_data_matrices(cols.data(), ncols, nrows, &cfg, &m) == OB_OK);
  int64_t na = 0, nb = 0;
  int32_t k = 0;
  CHECK(ob_matrices_dims(m, &na, &nb, &k) == OB_OK);
  CHECK(na + nb == 400 - 11 && k == 5);  // nulls dropped; intercept, 2 numeric, 2 sector dummies
  const double *xa = nullptr, *ya = nullptr, *xb = nullptr, *yb = nullptr;
  CHECK(ob_matrices_get(m, &xa, &ya, &xb, &yb) == OB_OK);
  double s = 0.0;
  for (int64_t i = 0; i < na * k; ++i) s += xa[i];
  for (int64_t i = 0; i < nb; ++i) s += yb[i];
  CHECK(std::isfinite(s));
  for (int32_t i = 0; i < k; ++i) CHECK(ob_matrices_name(m, i) != nullptr);
  ob_matrices_free(m);

  // weights column + a missing predictor
  cfg.weights = "experience";
  CHECK(ob_builder_data_matrices(cols.data(), ncols, nrows, &cfg, &m) == OB_OK);
  ob_matrices_free(m);
  const char* bad[] = {"nope"};
  cfg.predictors = bad;
  cfg.n_predictors = 1;
  CHECK(ob_builder_data_matrices(cols.data(), ncols, nrows, &cfg, &m) == OB_E_COLUMN);
  CHECK(ob_last_error() && std::strlen(ob_last_error()) > 0);
  ob_csv_free(csv);

  // CSV errors: missing file, ragged row, empty file; an unterminated quote must not crash
  ob_csv* e = nullptr;
  CHECK(ob_csv_read((std::string(dir) + "/missing.csv").c_str(), &e) != OB_OK);
  CHECK(ob_csv_read(write_file(dir, "ragged.csv", "a,b\n1,2\n3\n").c_str(), &e) != OB_OK);
  if (ob_csv_read(write_file(dir, "quote.csv", "a,b\n1,\"open\n").c_str(), &e) == OB_OK) ob_csv_free(e);  // no crash
  CHECK(ob_csv_read(write_file(dir, "empty.csv", "").c_str(), &e) != OB_OK);
}

static void inference() {
  std::vector<double> v(1001);
  for (size_t i = 0; i < v.size(); ++i) v[i] = std::sin(0.37 * (double)i) + 0.001 * (double)i;
  double out[4];
  CHECK(ob_bootstrap_stats(v.data(), (int64_t)v.size(), 0.25, out) == OB_OK && out[0] > 0.0);
  CHECK(ob_bootstrap_stats(v.data(), 0, 0.25, out) == OB_OK && std::isnan(out[0]));
  // rows of 7 columns, some replicates failed
  const int reps = 300, rl = 7;
  std::vector<double> rows(reps * rl);
  std::vector<uint8_t> ok(reps);
  for (int r = 0; r < reps; ++r) {
    ok[r] = r % 11 != 3;
    for (int c = 0; c < rl; ++c) rows[r * rl + c] = std::cos(0.1 * r + c);
  }
  const int32_t sel[] = {0, 2, 6};
  std::vector<double> agg(3 * 4);
  CHECK(ob_aggregate(rows.data(), ok.data(), reps, rl, sel, 3, agg.data()) == OB_OK);
  std::vector<double> rif(v.size());
  CHECK(ob_rif(v.data(), (int64_t)v.size(), 0.5, rif.data()) == OB_OK);
  CHECK(ob_rif(nullptr, 5, 0.5, rif.data()) == OB_E_INVALID);
}

static void no_gpu() {
  ob_ctx* ctx = nullptr;
  const int rc = ob_ctx_create(0, &ctx);
  if (rc == OB_OK) {  // a gfx950 is present: nothing more to check here (the GPU suite covers it)
    ob_ctx_destroy(ctx);
    return;
  }
  CHECK(rc == OB_E_HIP && ctx == nullptr);
}

// ob_shard_layout.h through a simulated all-gather: every rank computes its shard of fake rows
// (a pure function of (outcome, replicate, column), like the engine's), packs the gathered
// columns into an exactly-sized send block (ASan catches any offset past it), the blocks land
// where ncclAllGather puts them, and each rank's delivery must give every replicate's gathered
// columns, its own replicates' other columns, and NaN for the rest.
static double fake(int t, uint64_t rep, int c) { return t * 1e6 + (double)rep * 16.0 + c; }

static void shard_layout() {
  const int rl = 7, ny = 3;
  const std::vector<std::vector<int>> col_sets = {{0, 1, 2, 3, 4, 5, 6}, {0, 2, 5}};
  const int worlds[] = {1, 2, 3, 8};
  const uint64_t ns[] = {1, 2, 5, 37, 64, 1001};
  for (const auto& cols : col_sets)
    for (int world : worlds)
      for (uint64_t n : ns) {
        const uint64_t first = 11;
        const int nc = (int)cols.size();
        const ob_shard_range s0 = ob_shard_of(first, n, 0, world);
        std::vector<double> recv(ob_recv_block_off(s0, world, ny, 0, nc));
        std::vector<uint8_t> recv_ok(ob_recv_block_off(s0, world, ny, 0, 1));
        uint64_t covered = 0;
        for (int r = 0; r < world; ++r) {
          const ob_shard_range s = ob_shard_of(first, n, r, world);
          CHECK(s.per == s0.per && s.count <= s.per && s.lo == covered && s.first == first + s.lo);
          covered += s.count;
          std::vector<double> rows((size_t)ny * s.count * rl);
          std::vector<uint8_t> ok((size_t)ny * s.count);
          for (int t = 0; t < ny; ++t)
            for (uint64_t i = 0; i < s.count; ++i) {
              for (int c = 0; c < rl; ++c) rows.at(ob_shard_row_off(s, t, i, rl, c)) = fake(t, s.first + i, c);
              ok.at(ob_shard_ok_off(s, t, i)) = (uint8_t)(1 + ((s.first + i) & 1));
            }
          std::vector<double> send((size_t)ny * ob_send_elems(s, nc));
          std::vector<uint8_t> send_ok((size_t)ny * s.per);
          for (int t = 0; t < ny; ++t)
            for (uint64_t i = 0; i < s.per; ++i) {
              for (int q = 0; q < nc; ++q)
                send.at(ob_send_off(s, t, i, nc, q)) = i < s.count ? rows.at(ob_shard_row_off(s, t, i, rl, cols[q])) : 0.0;
              send_ok.at(ob_send_ok_off(s, t, i)) = i < s.count ? ok.at(ob_shard_ok_off(s, t, i)) : 0;
            }
          for (int t = 0; t < ny; ++t) {  // ncclAllGather per outcome: rank r's block of t
            std::memcpy(&recv.at(ob_recv_block_off(s, world, t, r, nc)), &send.at(ob_send_off(s, t, 0, nc, 0)),
                        sizeof(double) * ob_send_elems(s, nc));
            std::memcpy(&recv_ok.at(ob_recv_block_off(s, world, t, r, 1)), &send_ok.at(ob_send_ok_off(s, t, 0)), s.per);
          }
        }
        CHECK(covered == n);
        for (int me = 0; me < world; ++me) {
          const ob_shard_range s = ob_shard_of(first, n, me, world);
          for (int t = 0; t < ny; ++t)
            for (uint64_t j = 0; j < n; ++j) {
              CHECK(recv_ok.at(ob_recv_ok_off(s, world, t, j)) == (uint8_t)(1 + ((first + j) & 1)));
              for (int c = 0; c < rl; ++c) {
                int q = -1;
                for (int k = 0; k < nc; ++k)
                  if (cols[k] == c) q = k;
                const bool own = j >= s.lo && j < s.lo + s.count;
                const double want = fake(t, first + j, c);
                if (q >= 0) CHECK(recv.at(ob_recv_off(s, world, t, j, nc, q)) == want);
                else if (own) CHECK(ob_shard_row_off(s, t, j - s.lo, rl, c) < (size_t)ny * s.count * rl);
                CHECK(ob_deliver_off(n, t, j, rl, c) < (size_t)ny * n * rl);
              }
            }
        }
      }
}

int main(int argc, char** argv) {
  const char* dir = argc > 1 ? argv[1] : "/tmp";
  csv_and_frames(dir);
  inference();
  no_gpu();
  shard_layout();
  std::printf("host_asan: %s (%d failed checks)\n", failures ? "FAIL" : "ok", failures);
  return failures ? 1 : 0;
}
