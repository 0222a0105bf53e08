// Host-only plumbing shared by the HIP translation units and the plain C++
// one (host_image.cpp, which the sanitizer builds compile on their own):
// image geometry constants, the error type and KRY_REQUIRE.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <string>

#include "../../include/krylov_hip.h"

namespace kry {

constexpr int kSlice = 64;           // SELL slice height = one wavefront
// diagonal-offset image (kry_csr::dia_*): slices of kDiaSlice rows, lane l
// of the wave owns rows 2l and 2l + 1 of its slice
constexpr int kDiaSlice = 128;
constexpr int kDiaPad = 32;  // slot-column descriptors past the last one (unconditional reads of a round)
// paired-row SELL-128 image (kry_csr::sp_*): lane l owns rows 2l, 2l + 1
constexpr int kPairSlice = 128;
constexpr int kCbRows = 256;         // rows per column-blocked segment (one per thread)
// rank-sorted SELL-128 image (kry_csr::rs_*): runs of stored entries sorted by column
constexpr int kRsChunk = 16;

// ---------------------------------------------------------------- errors
void set_error(const std::string &msg);

struct Error {
  int code;
  std::string msg;
};

#define KRY_REQUIRE(cond, code, msg)                                           \
  do {                                                                         \
    if (!(cond)) throw ::kry::Error{(code), (msg)};                            \
  } while (0)

}  // namespace kry
