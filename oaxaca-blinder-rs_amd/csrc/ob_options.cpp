// ob_options.cpp -- the option table behind ob_set_option (ob_options.hpp).
#include "ob_options.hpp"

#include <atomic>
#include <cstdlib>
#include <cstring>
#include <limits>

#include "../../include/oaxaca_boot.h"
#include "ob_common.hpp"

namespace {

struct Entry {
  const char* name;  // ob_set_option's name; OB_TUNING builds read "OB_" + upper-case name too
  ob::Opt opt;
};

constexpr Entry kNames[] = {
    {"gram_path", ob::Opt::GramPath},         {"gram_digits", ob::Opt::GramDigits},
    {"hk_erfc", ob::Opt::HkErfc},             {"mm_reduce", ob::Opt::MmReduce},
    {"mm_trace", ob::Opt::MmTrace},           {"mm_state_gb", ob::Opt::MmStateGb},
    {"mm_delta1", ob::Opt::MmDelta1},         {"mm_delta2", ob::Opt::MmDelta2},
    {"mm_tol1", ob::Opt::MmTol1},             {"mm_fit_stride", ob::Opt::MmFitStride},
    {"mm_kappa", ob::Opt::MmKappa},           {"mm_band0", ob::Opt::MmBand0},
    {"gram_diag", ob::Opt::GramDiag},         {"l1_diag", ob::Opt::L1Diag},
    {"gram_tile", ob::Opt::GramTile},         {"debug_count_overflow", ob::Opt::DebugCountOverflow},
    {"rs_double", ob::Opt::RsDouble},         {"rs_pieces", ob::Opt::RsPieces},
    {"tail_stream", ob::Opt::TailStream},
};
static_assert(sizeof(kNames) / sizeof(kNames[0]) == (size_t)ob::Opt::Count, "one name per option");

// Every option starts unset (NaN); a function-local static initializes the table once, thread-safely.
std::atomic<double>* table() {
  static std::atomic<double>* t = [] {
    auto* a = new std::atomic<double>[(size_t)ob::Opt::Count];
    for (size_t i = 0; i < (size_t)ob::Opt::Count; ++i) a[i].store(std::numeric_limits<double>::quiet_NaN());
    return a;
  }();
  return t;
}

#if OB_TUNING
// OB_<NAME> from the environment (tuning builds only); gram_path also takes "f64" / "i8".
double env_value(const char* name) {
  char key[64] = "OB_";
  size_t i = 3;
  for (const char* c = name; *c && i + 1 < sizeof(key); ++c) key[i++] = (char)(*c >= 'a' && *c <= 'z' ? *c - 32 : *c);
  key[i] = 0;
  const char* e = std::getenv(key);
  if (!e || !*e) return std::numeric_limits<double>::quiet_NaN();
  if (!std::strcmp(name, "gram_path")) return !std::strcmp(e, "f64") ? 1.0 : (!std::strcmp(e, "i8") ? 2.0 : 0.0);
  return std::atof(e);
}
#endif

}  // namespace

namespace ob {

double opt(Opt o) {
  const double v = table()[(size_t)o].load(std::memory_order_relaxed);
#if OB_TUNING
  if (std::isnan(v)) {
    for (const Entry& e : kNames)
      if (e.opt == o) return env_value(e.name);
  }
#else
  if (o == Opt::GramDiag || o == Opt::L1Diag) return std::numeric_limits<double>::quiet_NaN();
#endif
  return v;
}

}  // namespace ob

extern "C" {

int ob_set_option(const char* name, double value) {
  if (!name) return ob::fail(OB_E_INVALID, "null option name");
  for (const Entry& e : kNames)
    if (!std::strcmp(e.name, name)) {
#if !OB_TUNING
      if ((e.opt == ob::Opt::GramDiag || e.opt == ob::Opt::L1Diag) && !std::isnan(value))
        return ob::fail(OB_E_UNSUPPORTED, "option '%s' exists only in a tuning build (make tuning)", name);
#endif
      table()[(size_t)e.opt].store(value, std::memory_order_relaxed);
      return OB_OK;
    }
  return ob::fail(OB_E_INVALID, "unknown option '%s'", name);
}

int ob_get_option(const char* name, double* value) {
  if (!name || !value) return ob::fail(OB_E_INVALID, "null pointer");
  for (const Entry& e : kNames)
    if (!std::strcmp(e.name, name)) {
      *value = table()[(size_t)e.opt].load(std::memory_order_relaxed);  // what ob_set_option stored (NaN: unset)
      return OB_OK;
    }
  return ob::fail(OB_E_INVALID, "unknown option '%s'", name);
}

int ob_tuning_build(void) { return OB_TUNING; }

}  // extern "C"
