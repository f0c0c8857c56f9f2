// Host-side constant folding (fixed-point multipliers), error state, version.
#include <cmath>
#include <cstring>
#include <limits>
#include <string>

#include "tk_common.h"

namespace tk {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace tk

extern "C" {

const char* tk_last_error(void) { return tk::g_last_error.c_str(); }
int tk_abi_version(void) { return TK_ABI_VERSION; }
const char* tk_build_arch(void) { return "gfx950"; }
#ifndef TK_SOURCE_HASH
#define TK_SOURCE_HASH "unknown"
#endif
const char* tk_build_info(void) { return TK_SOURCE_HASH; }

// GetFixedPointMultiplierShift (src/relay/qnn/utils.cc:33-57).
int tk_fixed_point_multiplier_shift(double multiplier, int32_t* significand, int32_t* shift) {
  if (!significand || !shift) {
    tk::set_error("tk_fixed_point_multiplier_shift: null output");
    return TK_ERR_INVALID_ARG;
  }
  if (multiplier == 0.0) {
    *significand = 0;
    *shift = 0;
    return TK_OK;
  }
  int exponent = 0;
  double sig = std::frexp(multiplier, &exponent);
  sig = std::round(sig * static_cast<double>(1ll << 31));
  int64_t q = static_cast<int64_t>(sig);
  if (q > (1ll << 31)) {
    tk::set_error("tk_fixed_point_multiplier_shift: significand overflow");
    return TK_ERR_INVALID_ARG;
  }
  if (q == (1ll << 31)) {
    q /= 2;
    ++exponent;
  }
  *significand = static_cast<int32_t>(q);
  *shift = exponent;
  return TK_OK;
}

// Mirrors the branch structure of RequantizeLowerInt (src/relay/qnn/op/requantize.cc:218-257):
// per-tensor when the scale is rank-0 (IsConstScalar), skip when the float32 scales are
// structurally equal, power-of-two fast path only on the per-tensor UPWARD branch.
int tk_requantize_prepare(const float* input_scales, int n_scales, float output_scale, int rounding,
                          int32_t* multipliers, int32_t* shifts, int* mode) {
  if (!input_scales || !multipliers || !shifts || !mode || n_scales < 0) {
    tk::set_error("tk_requantize_prepare: invalid argument");
    return TK_ERR_INVALID_ARG;
  }
  if (rounding != TK_ROUND_UPWARD && rounding != TK_ROUND_TONEAREST) {
    tk::set_error("tk_requantize_prepare: rounding must be UPWARD or TONEAREST");
    return TK_ERR_INVALID_ARG;
  }
  auto check_shift = [](int32_t s) {
    int rs = s > 0 ? 0 : -s;
    // 1 << (30 + rs) must stay inside int64 (the reference would shift out of range: UB)
    return rs + 31 <= 62 && s <= 31;
  };
  if (n_scales == 0) {
    float s_in = input_scales[0];
    if (std::memcmp(&s_in, &output_scale, sizeof(float)) == 0) {
      *mode = TK_RQ_IDENTITY;
      multipliers[0] = 0;
      shifts[0] = 0;
      return TK_OK;
    }
    double dm = static_cast<double>(s_in) / static_cast<double>(output_scale);
    int rc = tk_fixed_point_multiplier_shift(dm, &multipliers[0], &shifts[0]);
    if (rc) return rc;
    if (!check_shift(shifts[0])) {
      tk::set_error("tk_requantize_prepare: multiplier out of the representable shift range");
      return TK_ERR_UNSUPPORTED;
    }
    if (rounding == TK_ROUND_UPWARD) {
      if (multipliers[0] == (1 << 30)) {
        int e = shifts[0] - 1;
        if (e == 0 || -e > 31) {
          tk::set_error("tk_requantize_prepare: power-of-two shift outside the int32 path");
          return TK_ERR_UNSUPPORTED;
        }
        *mode = TK_RQ_TENSOR_POW2;
      } else {
        *mode = TK_RQ_TENSOR_UPWARD;
      }
    } else {
      *mode = TK_RQ_TENSOR_TONEAREST;
    }
    return TK_OK;
  }
  for (int i = 0; i < n_scales; ++i) {
    double dm = static_cast<double>(input_scales[i]) / static_cast<double>(output_scale);
    int rc = tk_fixed_point_multiplier_shift(dm, &multipliers[i], &shifts[i]);
    if (rc) return rc;
    if (!check_shift(shifts[i])) {
      tk::set_error("tk_requantize_prepare: per-axis multiplier out of range");
      return TK_ERR_UNSUPPORTED;
    }
  }
  *mode = rounding == TK_ROUND_UPWARD ? TK_RQ_AXIS_UPWARD : TK_RQ_AXIS_TONEAREST;
  return TK_OK;
}

}  // extern "C"
