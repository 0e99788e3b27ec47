// common.hpp — shared definitions for the gp2d HIP engine (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <string>

// The product library is compiled with -DGP2D_RELEASE=1 (__graft_entry__.build_lib).  A few
// tuning constants of the headers can be overridden by -DGP2D_<NAME> in measurement builds
// (tools/microbench compiles the headers into its own benches); in a release compile any such
// override is an error, so no measurement switch reaches a shipped libgp2d.so.
#if defined(GP2D_RELEASE) &&                                                                   \
    (defined(GP2D_STAMP) || defined(GP2D_OZ_P) || defined(GP2D_OZ_PW) || defined(GP2D_OZ_PB) || \
     defined(GP2D_KS_OCC) || defined(GP2D_KS_PPL) || defined(GP2D_CRT_RPL) || defined(GP2D_CRT_OCC))
#error "gp2d: measurement overrides (-DGP2D_<NAME>) are not allowed in a GP2D_RELEASE build"
#endif

namespace gp2d {

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));

// Tile of the whole engine: point counts are padded to 64, matrix orders to 128.
constexpr int PT_TILE = 64;
constexpr int NB = 128;

void set_error(const std::string& msg);

inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return -1;
  }
  return 0;
}

#define GP2D_REQUIRE(cond, msg)            \
  do {                                     \
    if (!(cond)) {                         \
      ::gp2d::set_error(msg);              \
      return -2;                           \
    }                                      \
  } while (0)

#define GP2D_CHECK(expr)                   \
  do {                                     \
    int _rc = (expr);                      \
    if (_rc != 0) return _rc;              \
  } while (0)

}  // namespace gp2d
