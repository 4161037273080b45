// ob_options.hpp -- process-wide engine options for tests and A/B tooling.
//
// The shipped library reads no environment variable: every switch below is set through the C ABI
// (ob_set_option, include/oaxaca_boot.h) by a caller that asks for it -- the parity tests (the f64
// Gram against the i8 Gram, the unreduced Machado-Mata solve against the reduced one, the library
// erfc against npdf_ncdf). A build with -DOB_TUNING=1 (`make tuning`, liboaxaca_boot_tuning.so)
// also reads OB_<NAME> from the environment for an option nobody set, and compiles the timing
// ablation kernels (gram_diag, l1_diag) that the A/B scripts under tools/ drive.
#pragma once

#include <cmath>

#ifndef OB_TUNING
#define OB_TUNING 0
#endif

namespace ob {

enum class Opt : int {
  GramPath,     // 1: f64 MFMA Gram, 2: i8 Gram (an error if its images do not fit); unset: i8 when it fits
  GramDigits,   // 7: seven digit slices on every column tile
  HkErfc,       // 0: the library erfc beside a second exp in the probit/IMR kernels
  MmReduce,     // 0: no Machado-Mata row reduction, 1: always; unset: when both groups have >= 2^16 rows
  MmTrace,      // nonzero: per-iteration Machado-Mata trace on stderr
  MmStateGb,    // Machado-Mata IPM state budget (GB of HBM)
  MmDelta1,     // Machado-Mata start offsets and band parameters (tuning: results do not depend on them)
  MmDelta2,
  MmTol1,
  MmFitStride,
  MmKappa,
  MmBand0,
  GramDiag,     // timing ablations (OB_TUNING builds only): wrong results by design
  L1Diag,
  GramTile,     // i8 Gram kernel: 1 = 8 waves, 32 pairs per block; 2 = 4 waves, 64 pairs (oz_gram_w_kernel);
                // 3 = that wide tile with each chunk's sub-tiles split over two blocks
  DebugCountOverflow,  // nonzero: engine_counts raises its overflow word after the count kernel (tests the
                       // error path that a real count above 255 would take, p < 1e-500 per row)
  RsDouble,     // 1: two count-image / m1 buffers, so a boot's resample runs under the previous Gram;
                // 0: one; unset: the engine's rule (engine_boot)
  RsPieces,     // level 1 and counts of a segment in this many replicate pieces, counts of piece k
                // beside level 1 of piece k + 1 (1: one launch each); unset: the engine's rule
  TailStream,   // 1: a boot's reduce / solve on a stream of their own, so the next segment's Gram
                // need not wait for them (two partial buffers); 0: on the caller's stream; unset: rule
  Count
};

// The option's value, or NaN when it is unset (the caller then uses its built-in default).
double opt(Opt o);

// Convenience: the option as an int / a double, or the default when unset.
inline int opt_int(Opt o, int dflt) {
  const double v = opt(o);
  return std::isnan(v) ? dflt : (int)v;
}
inline double opt_double(Opt o, double dflt) {
  const double v = opt(o);
  return std::isnan(v) ? dflt : v;
}

}  // namespace ob
