// dgraph_amd — host-side error checking.
//
// Replaces the reference's error macros (DGraph/distributed/include/macros.hpp:18-34),
// which called exit(EXIT_FAILURE); here every failure throws c10::Error so a failing
// rank surfaces a Python exception instead of killing the process mid-collective.
#pragma once
#include <hip/hip_runtime_api.h>
#include <c10/util/Exception.h>

#define DG_HIP_CHECK(expr)                                                       \
  do {                                                                           \
    hipError_t _e = (expr);                                                      \
    TORCH_CHECK(_e == hipSuccess, "HIP error ", hipGetErrorString(_e), " at ",   \
                __FILE__, ":", __LINE__, " in ", #expr);                         \
  } while (0)
