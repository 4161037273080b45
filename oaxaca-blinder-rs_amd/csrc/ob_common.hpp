// ob_common.hpp -- error plumbing shared by the engine, the builder and the C ABI.
#pragma once
#include <cstdarg>
#include <cstdio>
#include <string>

#include "../../include/oaxaca_boot.h"

namespace ob {

// Thread-local message behind ob_last_error(); the code travels as the return value.
std::string& last_error();

inline int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  last_error() = buf;
  return code;
}

// OaxacaError's Display prefixes (error.rs:21-33) so messages read like the reference's.
inline const char* error_prefix(int code) {
  switch (code) {
    case OB_E_POLARS: return "Polars error: ";
    case OB_E_COLUMN: return "Column not found: ";
    case OB_E_GROUP: return "Invalid group variable: ";
    case OB_E_LINALG: return "Nalgebra error: ";
    case OB_E_DIAG: return "Diagnostic error: ";
    case OB_E_INSUFFICIENT: return "Insufficient data: ";
    default: return "";
  }
}

struct Error {
  int code;
  std::string msg;
};

}  // namespace ob

#define OB_TRY(expr)            \
  do {                          \
    int rc_ = (expr);           \
    if (rc_ != OB_OK) return rc_; \
  } while (0)
