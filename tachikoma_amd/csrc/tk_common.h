// Shared host/device helpers for the tachikoma gfx950 kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/tachikoma.h"

namespace tk {

// ---------------------------------------------------------------- errors
void set_error(const std::string& msg);

#define TK_CHECK_ARG(cond, msg)                         \
  do {                                                  \
    if (!(cond)) {                                      \
      ::tk::set_error(std::string(__func__) + ": " + (msg)); \
      return TK_ERR_INVALID_ARG;                        \
    }                                                   \
  } while (0)

#define TK_HIP(call)                                                                  \
  do {                                                                                \
    hipError_t e_ = (call);                                                           \
    if (e_ != hipSuccess) {                                                           \
      ::tk::set_error(std::string(#call) + " failed: " + hipGetErrorString(e_));      \
      return TK_ERR_HIP;                                                              \
    }                                                                                 \
  } while (0)

#define TK_LAUNCH_CHECK()                                                             \
  do {                                                                                \
    hipError_t e_ = hipGetLastError();                                                \
    if (e_ != hipSuccess) {                                                           \
      ::tk::set_error(std::string(__func__) + ": launch failed: " + hipGetErrorString(e_)); \
      return TK_ERR_HIP;                                                              \
    }                                                                                 \
  } while (0)

// ---------------------------------------------------------------- tensors
inline int64_t numel(const tk_tensor* t) {
  int64_t n = 1;
  for (int i = 0; i < t->ndim; ++i) n *= t->shape[i];
  return n;
}
inline int elem_bytes(const tk_tensor* t) { return (t->dtype.bits + 7) / 8; }
inline int64_t nbytes(const tk_tensor* t) { return numel(t) * elem_bytes(t); }
inline char* ptr(const tk_tensor* t) { return static_cast<char*>(t->data) + t->byte_offset; }
inline bool is_int(const tk_tensor* t, int bits) {
  return t->dtype.code == TK_DL_INT && t->dtype.bits == bits && t->dtype.lanes == 1;
}
inline bool is_uint(const tk_tensor* t, int bits) {
  return t->dtype.code == TK_DL_UINT && t->dtype.bits == bits && t->dtype.lanes == 1;
}
inline bool is_int8ish(const tk_tensor* t) { return is_int(t, 8) || is_uint(t, 8); }
inline bool is_integer(const tk_tensor* t) {
  return (t->dtype.code == TK_DL_INT || t->dtype.code == TK_DL_UINT) && t->dtype.lanes == 1 &&
         (t->dtype.bits == 8 || t->dtype.bits == 16 || t->dtype.bits == 32 || t->dtype.bits == 64);
}
inline bool is_f32(const tk_tensor* t) {
  return t->dtype.code == TK_DL_FLOAT && t->dtype.bits == 32 && t->dtype.lanes == 1;
}
inline bool compact(const tk_tensor* t) { return t->strides == nullptr; }

// dtype id used as a template switch in kernels
enum DT { DT_I8 = 0, DT_U8 = 1, DT_I16 = 2, DT_U16 = 3, DT_I32 = 4, DT_U32 = 5, DT_I64 = 6, DT_U64 = 7 };
inline int dt_of(const tk_tensor* t) {
  int b = t->dtype.bits, u = t->dtype.code == TK_DL_UINT;
  switch (b) {
    case 8: return u ? DT_U8 : DT_I8;
    case 16: return u ? DT_U16 : DT_I16;
    case 32: return u ? DT_U32 : DT_I32;
    case 64: return u ? DT_U64 : DT_I64;
  }
  return -1;
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// ---------------------------------------------------------------- streaming stores
// Trace records are written once and only read back by later kernels / the D2H copy
// long after L2 has cycled: nontemporal stores keep them from thrashing L2/MALL and
// measurably raise the write rate of multi-record epilogues (tools/probe_store2.hip).
typedef int tk_v4i __attribute__((ext_vector_type(4)));

template <int kBytes>
__device__ __forceinline__ void store_nt(void* dst, const void* src) {
  if constexpr (kBytes == 16) {
    tk_v4i v;
    __builtin_memcpy(&v, src, 16);
    __builtin_nontemporal_store(v, reinterpret_cast<tk_v4i*>(dst));
  } else if constexpr (kBytes == 4) {
    uint32_t v;
    __builtin_memcpy(&v, src, 4);
    __builtin_nontemporal_store(v, reinterpret_cast<uint32_t*>(dst));
  } else {
    static_assert(kBytes == 1, "16, 4 or 1 bytes");
    __builtin_nontemporal_store(*reinterpret_cast<const uint8_t*>(src), reinterpret_cast<uint8_t*>(dst));
  }
}

// ---------------------------------------------------------------- fixed point (device)
// q_multiply_shift general form, q = 31 (src/target/intrin_rule.cc:166-195):
//   y = (int64(x) << ls) * m;  y += 1 << (30 + rs);  y >>= 31 + rs;  int32(y)
// (x << ls) * m == (x * m) << ls modulo 2^64, so the exact 62-bit product is
// formed first and shifted with wrap-around.
__device__ __forceinline__ int32_t qms_upward(int32_t x, int32_t m, int32_t shift) {
  int ls = shift > 0 ? shift : 0;
  int rs = shift > 0 ? 0 : -shift;
  unsigned long long y = (unsigned long long)((long long)x * (long long)m);
  y <<= ls;
  int total = rs + 31;
  y += 1ULL << (total - 1);
  return (int32_t)((long long)y >> total);
}

// power-of-two special case, all int32 (intrin_rule.cc:223-237); shift = s.
__device__ __forceinline__ int32_t qms_pow2(int32_t x, int32_t shift) {
  int e = shift - 1;
  if (e > 0) return (int32_t)((uint32_t)x << e);
  int k = -e;
  int32_t r = (int32_t)((uint32_t)x + (1u << (k - 1)));
  return r >> k;
}

// FixedPointMultiplyToNearest (src/relay/qnn/utils.cc:59-109)
__device__ __forceinline__ int32_t qms_tonearest(int32_t x, int32_t m, int32_t shift) {
  int ls = shift > 0 ? shift : 0;
  int rs = shift > 0 ? 0 : -shift;
  unsigned long long y = (unsigned long long)((long long)x * (long long)m);
  y <<= ls;
  int total = rs + 31;
  unsigned long long pos = 1ULL << (total - 1);
  y += ((long long)y >= 0) ? pos : pos - 1;
  return (int32_t)((long long)y >> total);
}

// ---------------------------------------------------------------- requantize
// RequantizeLowerInt (src/relay/qnn/op/requantize.cc:195-273):
//   t = int32(x) - zp_in;  t = FPM(t);  t = zp_out + t;  clip+cast unless out is int32.
struct RqParams {
  int32_t mode, multiplier, shift, zp_in, zp_out;
  const int32_t* ms;
  const int32_t* ss;
  const int32_t* zps;
  int32_t inner, C;
  int64_t qmin, qmax;
  int32_t clip_out;
};

__device__ __forceinline__ int32_t rq_apply(int32_t t, int c, const RqParams& p) {
  int32_t zp = p.zps ? p.zps[c] : p.zp_in;
  t = (int32_t)((uint32_t)t - (uint32_t)zp);
  switch (p.mode) {
    case TK_RQ_IDENTITY: break;
    case TK_RQ_TENSOR_POW2: t = qms_pow2(t, p.shift); break;
    case TK_RQ_TENSOR_UPWARD: t = qms_upward(t, p.multiplier, p.shift); break;
    case TK_RQ_TENSOR_TONEAREST: t = qms_tonearest(t, p.multiplier, p.shift); break;
    case TK_RQ_AXIS_UPWARD: t = qms_upward(t, p.ms[c], p.ss[c]); break;
    case TK_RQ_AXIS_TONEAREST: t = qms_tonearest(t, p.ms[c], p.ss[c]); break;
  }
  t = (int32_t)((uint32_t)p.zp_out + (uint32_t)t);
  return t;
}

}  // namespace tk
