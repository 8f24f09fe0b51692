// Compile-time ABI check between the reference's types (restated: quantize.cuh:14-25 QParams, HIP's
// dim3, half) and the library's C declarations (include/mxmoe_gg.h): the casts in
// ref_harness_call.cpp's registry adapter are only sound if these hold.
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cstddef>

#include "mxmoe_gg.h"

namespace refside {
struct QParams {  // quantize.cuh:14-25
  int2 qbits{make_int2(16, 16)};
  int gsize{-1};
  bool sym{false};
};
}  // namespace refside

static_assert(sizeof(refside::QParams) == sizeof(mxmoe_qparams), "QParams size");
static_assert(alignof(refside::QParams) == alignof(mxmoe_qparams), "QParams alignment");
static_assert(offsetof(refside::QParams, qbits) == offsetof(mxmoe_qparams, a_bits), "qbits.x = a_bits");
static_assert(offsetof(refside::QParams, qbits) + sizeof(int) == offsetof(mxmoe_qparams, w_bits), "qbits.y = w_bits");
static_assert(offsetof(refside::QParams, gsize) == offsetof(mxmoe_qparams, gsize), "gsize");
static_assert(offsetof(refside::QParams, sym) == offsetof(mxmoe_qparams, sym), "sym");
static_assert(sizeof(bool) == sizeof(uint8_t), "bool sym is one byte");
static_assert(sizeof(dim3) == sizeof(mxmoe_dim3) && offsetof(dim3, x) == offsetof(mxmoe_dim3, x) &&
                  offsetof(dim3, y) == offsetof(mxmoe_dim3, y) && offsetof(dim3, z) == offsetof(mxmoe_dim3, z),
              "dim3");
static_assert(sizeof(half) == 2 && sizeof(half*) == sizeof(void*), "half**");

extern "C" int mxmoe_layout_check(void) { return 1; }
