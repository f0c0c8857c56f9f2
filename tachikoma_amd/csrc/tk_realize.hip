// Kernels for the ops a relay.quantize-realized graph runs beside the QNN contractions
// (src/relay/quantize/realize.cc): the int32 shift/add/clip chain that
// moves activations between scales, the float32 input quantize (multiply, round, clip, cast),
// and the float32 layers the quantizer leaves unquantized (the skipped first conv, the
// dequantize, global_avg_pool2d, the classifier dense).
//
// Float contractions accumulate in float32 from 0 in a fixed order — (c, r, s) for conv, k for
// dense, row-major (h, w) for the pool — with one rounding per multiply and per add
// (plain * and + under `fp contract(off)`: no FMA), so results are reproducible run to run and
// bit-identical to the test oracle (oracle/realize_ref.py), which fixes the same order.
// All of these are HBM-bound or small; the int8 contractions of the realized graph run on the
// MFMA path (tk_gemm.hip) with zero zero points.
#include <cmath>
#include <limits>

#include "tk_common.h"

// hipcc contracts a*b+c into FMA by default (the __fmul_rn/__fadd_rn helpers included, once
// inlined); the fixed order above means one rounding per multiply and per add
#pragma clang fp contract(off)

namespace tk {

constexpr int kEwBlock = 256;

static inline int ew_grid(int64_t items) {
  int64_t g = (items + kEwBlock - 1) / kEwBlock;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, 256 * 16));
}

// ---------------------------------------------------------------- elementwise
// One kernel per (type, op): x op rhs with rhs a scalar or a same-shape tensor.
template <typename T> struct Wide { using U = T; };
template <> struct Wide<int8_t> { using U = uint8_t; };
template <> struct Wide<int16_t> { using U = uint16_t; };
template <> struct Wide<int32_t> { using U = uint32_t; };
template <> struct Wide<int64_t> { using U = uint64_t; };

template <typename T, int OP>
__device__ __forceinline__ T ew_apply(T x, T r, const tk_ewise_attrs& a) {
  if constexpr (std::is_floating_point<T>::value) {
    if constexpr (OP == TK_EW_ADD) return x + r;
    if constexpr (OP == TK_EW_MULTIPLY) return x * r;
    if constexpr (OP == TK_EW_ROUND) return roundf(x);  // llvm.round: halves away from zero
    if constexpr (OP == TK_EW_CLIP) return fminf(fmaxf(x, (float)a.lo), (float)a.hi);
    if constexpr (OP == TK_EW_RELU) return fmaxf(x, 0.0f);
    return x;
  } else {
    using U = typename Wide<T>::U;
    if constexpr (OP == TK_EW_ADD) return (T)((U)x + (U)r);  // wraps like the reference's int32 add
    if constexpr (OP == TK_EW_MULTIPLY) return (T)((U)x * (U)r);
    if constexpr (OP == TK_EW_LEFT_SHIFT) return (T)((U)x << (r & (sizeof(T) * 8 - 1)));
    if constexpr (OP == TK_EW_RIGHT_SHIFT) return (T)(x >> (r & (sizeof(T) * 8 - 1)));  // arithmetic
    if constexpr (OP == TK_EW_RELU) return x > 0 ? x : (T)0;
    if constexpr (OP == TK_EW_FIXED_POINT_MULTIPLY) {
      // tir.q_multiply_shift(x, m, 31, s), intrin_rule.cc:166-250.  The power-of-two special
      // case m == 1<<30 (:223-237) shifts and rounds in x's own dtype (x << e, or
      // (x + (1 << (k-1))) >> k, int64 for an int64 x); the general form computes in int64 and
      // casts the result to int32 (QMultiplyShift, :166-195)
      int64_t v = (int64_t)x;
      const int s = a.shift;
      if (a.multiplier == (1 << 30)) {
        const int e = s - 1;
        if (e > 0) return (T)((U)x << e);
        const int k = -e;
        return (T)((T)((U)x + ((U)1 << (k - 1))) >> k);
      }
      const int ls = s > 0 ? s : 0, rs = s > 0 ? 0 : -s;
      if (ls) v = (int64_t)((uint64_t)v << ls);
      v = (int64_t)((uint64_t)v * (uint64_t)(int64_t)a.multiplier);
      const int total = 31 + rs;
      v = (int64_t)((uint64_t)v + (1ull << (total - 1)));
      v >>= total;
      return (T)(int32_t)v;
    }
    return x;
  }
}

template <typename T, int OP>
__global__ __launch_bounds__(kEwBlock) void ewise_kernel(const T* __restrict__ x, const T* __restrict__ rt,
                                                         T rs, T* __restrict__ y, int64_t n, tk_ewise_attrs a) {
  constexpr int V = 16 / sizeof(T) >= 4 ? 4 : 16 / sizeof(T);
  const int64_t nv = n / V;
  const int64_t stride = (int64_t)gridDim.x * kEwBlock;
  for (int64_t v = blockIdx.x * (int64_t)kEwBlock + threadIdx.x; v < nv; v += stride) {
    T in[V], rv[V], out[V];
    __builtin_memcpy(in, x + v * V, sizeof(in));
    if (rt) __builtin_memcpy(rv, rt + v * V, sizeof(rv));
#pragma unroll
    for (int j = 0; j < V; ++j) out[j] = ew_apply<T, OP>(in[j], rt ? rv[j] : rs, a);
    __builtin_memcpy(y + v * V, out, sizeof(out));
  }
  for (int64_t i = nv * V + blockIdx.x * (int64_t)kEwBlock + threadIdx.x; i < n; i += stride)
    y[i] = ew_apply<T, OP>(x[i], rt ? rt[i] : rs, a);
}

// rhs_kind 3: a per-channel vector along axis 1 (element i takes rhs[(i / inner) % C]), e.g. the
// scale of a batch norm that FoldScaleAxis could not fold into a conv
template <typename T, int OP>
__global__ __launch_bounds__(kEwBlock) void ewise_axis_kernel(const T* __restrict__ x, const T* __restrict__ rt,
                                                              T* __restrict__ y, int64_t n, int64_t inner, int64_t C,
                                                              tk_ewise_attrs a) {
  const int64_t stride = (int64_t)gridDim.x * kEwBlock;
  for (int64_t i = blockIdx.x * (int64_t)kEwBlock + threadIdx.x; i < n; i += stride)
    y[i] = ew_apply<T, OP>(x[i], rt[(i / inner) % C], a);
}

// fixed_point_multiply_per_axis (topi/math.py fixed_point_multiply_per_axis, the per-channel
// requantize of FixedPointMultiplyPerChannel, src/relay/qnn/utils.cc:111-135): element i of
// channel c = (i / inner) % C takes multiplier rhs[c] and shift rhs[C + c], always in
// q_multiply_shift's general int64 form (intrin_rule.cc:166-195, :252-267: no power-of-two case)
__global__ __launch_bounds__(kEwBlock) void fpm_axis_kernel(const int32_t* __restrict__ x,
                                                            const int32_t* __restrict__ ms,
                                                            int32_t* __restrict__ y, int64_t n, int64_t inner,
                                                            int64_t C) {
  const int64_t stride = (int64_t)gridDim.x * kEwBlock;
  for (int64_t i = blockIdx.x * (int64_t)kEwBlock + threadIdx.x; i < n; i += stride) {
    const int64_t c = (i / inner) % C;
    const int32_t m = ms[c], sh = ms[C + c];
    const int ls = sh > 0 ? sh : 0, rs = sh > 0 ? 0 : -sh;
    uint64_t v = (uint64_t)(int64_t)x[i] << ls;
    v *= (uint64_t)(int64_t)m;
    const int total = 31 + rs;
    v += 1ull << (total - 1);
    y[i] = (int32_t)((int64_t)v >> total);
  }
}

template <typename T>
static int launch_ewise_axis(const tk_tensor* x, const tk_tensor* r, tk_tensor* y, const tk_ewise_attrs* a,
                             hipStream_t s) {
  const int64_t n = numel(x), C = x->shape[1], inner = n / (x->shape[0] * C);
  const dim3 grid(ew_grid(n)), block(kEwBlock);
  const T* rt = (const T*)ptr(r);
  if constexpr (std::is_same<T, int32_t>::value) {
    if (a->op == TK_EW_FIXED_POINT_MULTIPLY) {
      hipLaunchKernelGGL(fpm_axis_kernel, grid, block, 0, s, (const int32_t*)ptr(x), rt, (int32_t*)ptr(y), n, inner, C);
      TK_LAUNCH_CHECK();
      return TK_OK;
    }
  }
  switch (a->op) {
    case TK_EW_ADD:
      hipLaunchKernelGGL((ewise_axis_kernel<T, TK_EW_ADD>), grid, block, 0, s, (const T*)ptr(x), rt, (T*)ptr(y), n,
                         inner, C, *a);
      break;
    case TK_EW_MULTIPLY:
      hipLaunchKernelGGL((ewise_axis_kernel<T, TK_EW_MULTIPLY>), grid, block, 0, s, (const T*)ptr(x), rt, (T*)ptr(y),
                         n, inner, C, *a);
      break;
    default:
      set_error("tk_ewise: a per-channel rhs (rhs_kind 3) takes add, multiply or (int32) fixed_point_multiply");
      return TK_ERR_INVALID_ARG;
  }
  TK_LAUNCH_CHECK();
  return TK_OK;
}

template <typename T>
static int launch_ewise(const tk_tensor* x, const tk_tensor* r, tk_tensor* y, const tk_ewise_attrs* a, hipStream_t s) {
  if (a->rhs_kind == 3) return launch_ewise_axis<T>(x, r, y, a, s);
  const int64_t n = numel(x);
  const T* rt = a->rhs_kind == 2 ? (const T*)ptr(r) : nullptr;
  T rs;
  if constexpr (std::is_floating_point<T>::value) rs = (T)a->scalar_f;
  else rs = (T)a->scalar_i;
  const dim3 grid(ew_grid(n / 4 + 1)), block(kEwBlock);
#define TK_EW_CASE(OPC)                                                                                      \
  case OPC:                                                                                                  \
    hipLaunchKernelGGL((ewise_kernel<T, OPC>), grid, block, 0, s, (const T*)ptr(x), rt, rs, (T*)ptr(y), n, *a); \
    break;
  switch (a->op) {
    TK_EW_CASE(TK_EW_ADD)
    TK_EW_CASE(TK_EW_MULTIPLY)
    TK_EW_CASE(TK_EW_RELU)
    case TK_EW_ROUND:
    case TK_EW_CLIP:
      if constexpr (!std::is_floating_point<T>::value) {
        set_error("tk_ewise: round/clip here take float32 (integer clip is tk_clip)");
        return TK_ERR_DTYPE;
      } else {
        if (a->op == TK_EW_ROUND)
          hipLaunchKernelGGL((ewise_kernel<T, TK_EW_ROUND>), grid, block, 0, s, (const T*)ptr(x), rt, rs, (T*)ptr(y), n, *a);
        else
          hipLaunchKernelGGL((ewise_kernel<T, TK_EW_CLIP>), grid, block, 0, s, (const T*)ptr(x), rt, rs, (T*)ptr(y), n, *a);
      }
      break;
    case TK_EW_LEFT_SHIFT:
    case TK_EW_RIGHT_SHIFT:
    case TK_EW_FIXED_POINT_MULTIPLY:
      if constexpr (std::is_floating_point<T>::value) {
        set_error("tk_ewise: shifts and fixed_point_multiply take integer tensors");
        return TK_ERR_DTYPE;
      } else {
        if (a->op == TK_EW_LEFT_SHIFT)
          hipLaunchKernelGGL((ewise_kernel<T, TK_EW_LEFT_SHIFT>), grid, block, 0, s, (const T*)ptr(x), rt, rs, (T*)ptr(y), n, *a);
        else if (a->op == TK_EW_RIGHT_SHIFT)
          hipLaunchKernelGGL((ewise_kernel<T, TK_EW_RIGHT_SHIFT>), grid, block, 0, s, (const T*)ptr(x), rt, rs, (T*)ptr(y), n, *a);
        else
          hipLaunchKernelGGL((ewise_kernel<T, TK_EW_FIXED_POINT_MULTIPLY>), grid, block, 0, s, (const T*)ptr(x), rt, rs,
                             (T*)ptr(y), n, *a);
      }
      break;
    default:
      set_error("tk_ewise: unknown op " + std::to_string(a->op));
      return TK_ERR_INVALID_ARG;
  }
#undef TK_EW_CASE
  TK_LAUNCH_CHECK();
  return TK_OK;
}

int ewise_impl(const tk_tensor* x, const tk_tensor* r, tk_tensor* y, const tk_ewise_attrs* a, hipStream_t s) {
  TK_CHECK_ARG(x && y && a, "null argument");
  TK_CHECK_ARG(compact(x) && compact(y) && numel(x) == numel(y), "bad tensors");
  TK_CHECK_ARG(x->dtype.code == y->dtype.code && x->dtype.bits == y->dtype.bits, "dtype mismatch");
  if (a->rhs_kind == 2) {
    TK_CHECK_ARG(r && compact(r) && numel(r) == numel(x) && r->dtype.bits == x->dtype.bits, "rhs must match the lhs");
  } else if (a->rhs_kind == 3) {
    // fixed_point_multiply: multipliers then shifts, two int32 per channel
    const int64_t per = a->op == TK_EW_FIXED_POINT_MULTIPLY ? 2 : 1;
    TK_CHECK_ARG(x->ndim >= 2 && x->shape[0] > 0 && x->shape[1] > 0 && r && compact(r) &&
                     numel(r) == per * x->shape[1] && r->dtype.code == x->dtype.code && r->dtype.bits == x->dtype.bits,
                 "rhs_kind 3: rhs must hold one value per channel (axis 1) of the lhs (fixed_point_multiply: "
                 "the multipliers, then the shifts)");
  } else {
    TK_CHECK_ARG(a->rhs_kind == 0 || a->rhs_kind == 1, "rhs_kind must be 0, 1, 2 or 3");
  }
  if (is_f32(x)) return launch_ewise<float>(x, r, y, a, s);
  if (is_int(x, 32)) return launch_ewise<int32_t>(x, r, y, a, s);
  if (is_int(x, 64)) return launch_ewise<int64_t>(x, r, y, a, s);
  if (is_int(x, 8)) return launch_ewise<int8_t>(x, r, y, a, s);
  if (is_int(x, 16)) return launch_ewise<int16_t>(x, r, y, a, s);
  set_error("tk_ewise: float32, int8, int16, int32 or int64 tensors only");
  return TK_ERR_DTYPE;
}

// ---------------------------------------------------------------- casts with float32
template <typename Ti, typename To>
__global__ __launch_bounds__(kEwBlock) void fcast_kernel(const Ti* __restrict__ x, To* __restrict__ y, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * kEwBlock;
  for (int64_t i = blockIdx.x * (int64_t)kEwBlock + threadIdx.x; i < n; i += stride) {
    if constexpr (std::is_floating_point<Ti>::value && !std::is_floating_point<To>::value) {
      // fptosi truncates toward zero; the realized graph only casts clipped, rounded values
      y[i] = (To)(int64_t)x[i];
    } else {
      y[i] = (To)x[i];
    }
  }
}

int cast_f32_impl(const tk_tensor* x, tk_tensor* y, hipStream_t s) {
  TK_CHECK_ARG(x && y && compact(x) && compact(y) && numel(x) == numel(y), "bad tensors");
  const int64_t n = numel(x);
  const dim3 grid(ew_grid(n)), block(kEwBlock);
  auto to_int = [&](auto tag) -> int {
    using To = decltype(tag);
    hipLaunchKernelGGL((fcast_kernel<float, To>), grid, block, 0, s, (const float*)ptr(x), (To*)ptr(y), n);
    return TK_OK;
  };
  auto from_int = [&](auto tag) -> int {
    using Ti = decltype(tag);
    hipLaunchKernelGGL((fcast_kernel<Ti, float>), grid, block, 0, s, (const Ti*)ptr(x), (float*)ptr(y), n);
    return TK_OK;
  };
  int rc = TK_ERR_DTYPE;
  if (is_f32(x) && is_f32(y)) {
    TK_HIP(hipMemcpyAsync(ptr(y), ptr(x), nbytes(x), hipMemcpyDeviceToDevice, s));
    return TK_OK;
  } else if (is_f32(x)) {
    if (is_int(y, 8)) rc = to_int(int8_t{});
    else if (is_uint(y, 8)) rc = to_int(uint8_t{});
    else if (is_int(y, 32)) rc = to_int(int32_t{});
    else if (is_int(y, 64)) rc = to_int(int64_t{});
  } else if (is_f32(y)) {
    if (is_int(x, 8)) rc = from_int(int8_t{});
    else if (is_uint(x, 8)) rc = from_int(uint8_t{});
    else if (is_int(x, 32)) rc = from_int(int32_t{});
    else if (is_int(x, 64)) rc = from_int(int64_t{});
  }
  if (rc != TK_OK) {
    set_error("tk_cast: unsupported float cast");
    return rc;
  }
  TK_LAUNCH_CHECK();
  return TK_OK;
}

// ---------------------------------------------------------------- float32 per-channel add
__global__ __launch_bounds__(kEwBlock) void bias_add_f32_kernel(const float* __restrict__ x, const float* __restrict__ b,
                                                                float* __restrict__ y, int64_t n, int32_t inner,
                                                                int32_t C) {
  const int64_t stride = (int64_t)gridDim.x * kEwBlock;
  for (int64_t i = blockIdx.x * (int64_t)kEwBlock + threadIdx.x; i < n; i += stride)
    y[i] = x[i] + b[(i / inner) % C];
}

int bias_add_f32_impl(const tk_tensor* x, const tk_tensor* b, tk_tensor* y, int axis, hipStream_t s) {
  TK_CHECK_ARG(x && b && y && is_f32(x) && is_f32(b) && is_f32(y), "float32 tensors expected");
  TK_CHECK_ARG(compact(x) && compact(b) && compact(y) && numel(x) == numel(y), "bad tensors");
  TK_CHECK_ARG(axis >= 0 && axis < x->ndim, "bad axis");
  int64_t inner = 1;
  for (int d = axis + 1; d < x->ndim; ++d) inner *= x->shape[d];
  const int32_t C = (int32_t)x->shape[axis];
  TK_CHECK_ARG(numel(b) == C, "bias length does not match the axis");
  const int64_t n = numel(x);
  hipLaunchKernelGGL(bias_add_f32_kernel, dim3(ew_grid(n)), dim3(kEwBlock), 0, s, (const float*)ptr(x),
                     (const float*)ptr(b), (float*)ptr(y), n, (int32_t)inner, C);
  TK_LAUNCH_CHECK();
  return TK_OK;
}

// ---------------------------------------------------------------- float32 nn.conv2d (direct)
// One thread per output pixel; a workgroup covers pixels of one (n, o) plane so the weight
// taps are wave-uniform (scalar loads) and the input rows are read coalesced along ow.
struct ConvF32Geom {
  int32_t N, C, H, W, O, Cg, KH, KW, OH, OW, sh, sw, pt, pl, dh, dw, groups;
};

__global__ __launch_bounds__(kEwBlock) void conv2d_f32_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                              float* __restrict__ y, ConvF32Geom g) {
  const int ohw = g.OH * g.OW;
  const int og = g.O / g.groups;
  for (int plane = blockIdx.y; plane < g.N * g.O; plane += gridDim.y) {  // n * O + o
    const int o = plane % g.O, n = plane / g.O;
    const int grp = o / og;
    for (int p = blockIdx.x * kEwBlock + threadIdx.x; p < ohw; p += gridDim.x * kEwBlock) {
      const int oh = p / g.OW, ow = p - (p / g.OW) * g.OW;
      float acc = 0.0f;
      for (int ci = 0; ci < g.Cg; ++ci) {
        const float* xp = x + ((int64_t)n * g.C + grp * g.Cg + ci) * g.H * g.W;
        const float* wp = w + ((int64_t)o * g.Cg + ci) * g.KH * g.KW;
        for (int r = 0; r < g.KH; ++r) {
          const int ih = oh * g.sh - g.pt + r * g.dh;
          for (int s = 0; s < g.KW; ++s) {
            const int iw = ow * g.sw - g.pl + s * g.dw;
            const float v = (ih >= 0 && ih < g.H && iw >= 0 && iw < g.W) ? xp[ih * g.W + iw] : 0.0f;
            const float prod = v * wp[r * g.KW + s];
            acc = acc + prod;
          }
        }
      }
      y[(int64_t)plane * ohw + p] = acc;
    }
  }
}

int conv2d_f32_impl(const tk_tensor* x, const tk_tensor* w, tk_tensor* y, const tk_conv2d_attrs* a, hipStream_t s) {
  TK_CHECK_ARG(x && w && y && a, "null argument");
  TK_CHECK_ARG(is_f32(x) && is_f32(w) && is_f32(y), "float32 tensors expected");
  TK_CHECK_ARG(x->ndim == 4 && w->ndim == 4 && y->ndim == 4 && compact(x) && compact(w) && compact(y), "NCHW/OIHW");
  ConvF32Geom g{};
  g.N = (int32_t)x->shape[0]; g.C = (int32_t)x->shape[1]; g.H = (int32_t)x->shape[2]; g.W = (int32_t)x->shape[3];
  g.O = (int32_t)w->shape[0]; g.Cg = (int32_t)w->shape[1]; g.KH = (int32_t)w->shape[2]; g.KW = (int32_t)w->shape[3];
  g.sh = a->strides[0]; g.sw = a->strides[1]; g.pt = a->padding[0]; g.pl = a->padding[1];
  g.dh = a->dilation[0] ? a->dilation[0] : 1; g.dw = a->dilation[1] ? a->dilation[1] : 1;
  g.groups = a->groups ? a->groups : 1;
  g.OH = (g.H + a->padding[0] + a->padding[2] - g.dh * (g.KH - 1) - 1) / g.sh + 1;
  g.OW = (g.W + a->padding[1] + a->padding[3] - g.dw * (g.KW - 1) - 1) / g.sw + 1;
  TK_CHECK_ARG(g.C == g.Cg * g.groups && g.O % g.groups == 0, "channels / groups mismatch");
  TK_CHECK_ARG(y->shape[0] == g.N && y->shape[1] == g.O && y->shape[2] == g.OH && y->shape[3] == g.OW,
               "output shape mismatch");
  TK_CHECK_ARG((int64_t)g.N * g.O < INT32_MAX && (int64_t)g.OH * g.OW < INT32_MAX, "tensor too large");
  const int ohw = g.OH * g.OW;
  dim3 grid((unsigned)std::min(ew_grid(ohw), 64), (unsigned)std::min(g.N * g.O, 65535));
  hipLaunchKernelGGL(conv2d_f32_kernel, grid, dim3(kEwBlock), 0, s, (const float*)ptr(x), (const float*)ptr(w),
                     (float*)ptr(y), g);
  TK_LAUNCH_CHECK();
  return TK_OK;
}

// ---------------------------------------------------------------- float32 nn.dense
// One workgroup of 64 lanes per output column n, lanes along the batch rows m: the weight row
// is wave-uniform; each lane accumulates its row over k in order.
__global__ __launch_bounds__(64) void dense_f32_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                       float* __restrict__ y, int32_t M, int32_t K, int32_t N) {
  const int col = blockIdx.x;
  const float* wr = w + (int64_t)col * K;
  for (int m = blockIdx.y * 64 + threadIdx.x; m < M; m += gridDim.y * 64) {
    const float* xr = x + (int64_t)m * K;
    float acc = 0.0f;
    for (int k = 0; k < K; ++k) {
      const float prod = xr[k] * wr[k];
      acc = acc + prod;
    }
    y[(int64_t)m * N + col] = acc;
  }
}

int dense_f32_impl(const tk_tensor* x, const tk_tensor* w, tk_tensor* y, hipStream_t s) {
  TK_CHECK_ARG(x && w && y && is_f32(x) && is_f32(w) && is_f32(y), "float32 tensors expected");
  TK_CHECK_ARG(x->ndim == 2 && w->ndim == 2 && y->ndim == 2 && x->shape[1] == w->shape[1] &&
                   y->shape[0] == x->shape[0] && y->shape[1] == w->shape[0],
               "dense shapes");
  const int32_t M = (int32_t)x->shape[0], K = (int32_t)x->shape[1], N = (int32_t)w->shape[0];
  TK_CHECK_ARG(N <= 2147483647 && N > 0 && M > 0, "dense shapes");
  dim3 grid((unsigned)N, (unsigned)std::min(65535, (M + 63) / 64));
  hipLaunchKernelGGL(dense_f32_kernel, grid, dim3(64), 0, s, (const float*)ptr(x), (const float*)ptr(w),
                     (float*)ptr(y), M, K, N);
  TK_LAUNCH_CHECK();
  return TK_OK;
}

// ---------------------------------------------------------------- float32 pools
// global_avg_pool2d: sum over the plane in row-major order, then divide by H*W
// (topi adaptive pool, pooling.h:366-389, float division).
__global__ __launch_bounds__(kEwBlock) void global_avg_f32_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                                  int64_t planes, int32_t hw) {
  const int64_t stride = (int64_t)gridDim.x * kEwBlock;
  for (int64_t p = blockIdx.x * (int64_t)kEwBlock + threadIdx.x; p < planes; p += stride) {
    const float* pl = x + p * hw;
    float acc = 0.0f;
    for (int i = 0; i < hw; ++i) acc = acc + pl[i];
    y[p] = acc / (float)hw;  // correctly rounded (hipcc's default fp32 division)
  }
}

int global_avg_pool_f32_impl(const tk_tensor* x, tk_tensor* y, hipStream_t s) {
  TK_CHECK_ARG(x && y && is_f32(x) && is_f32(y) && x->ndim == 4 && y->ndim == 4, "float32 NCHW expected");
  const int64_t planes = x->shape[0] * x->shape[1];
  TK_CHECK_ARG(numel(y) == planes, "output must be [N,C,1,1]");
  const int32_t hw = (int32_t)(x->shape[2] * x->shape[3]);
  hipLaunchKernelGGL(global_avg_f32_kernel, dim3(ew_grid(planes)), dim3(kEwBlock), 0, s, (const float*)ptr(x),
                     (float*)ptr(y), planes, hw);
  TK_LAUNCH_CHECK();
  return TK_OK;
}

// max_pool2d: padded taps are the float32 lowest value (pooling.h:123, min_value(float32)).
__global__ __launch_bounds__(kEwBlock) void max_pool_f32_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                                int32_t N, int32_t C, int32_t H, int32_t W, int32_t OH,
                                                                int32_t OW, tk_pool2d_attrs a) {
  const int64_t n = (int64_t)N * C * OH * OW;
  const int64_t stride = (int64_t)gridDim.x * kEwBlock;
  const int dh = a.dilation[0] ? a.dilation[0] : 1, dw = a.dilation[1] ? a.dilation[1] : 1;
  for (int64_t i = blockIdx.x * (int64_t)kEwBlock + threadIdx.x; i < n; i += stride) {
    const int ow = (int)(i % OW);
    const int64_t t = i / OW;
    const int oh = (int)(t % OH);
    const float* plane = x + (t / OH) * (int64_t)H * W;
    float m = -std::numeric_limits<float>::max();
    for (int r = 0; r < a.pool_size[0]; ++r) {
      const int ih = oh * a.strides[0] - a.padding[0] + r * dh;
      if (ih < 0 || ih >= H) continue;
      for (int c = 0; c < a.pool_size[1]; ++c) {
        const int iw = ow * a.strides[1] - a.padding[1] + c * dw;
        if (iw < 0 || iw >= W) continue;
        m = fmaxf(m, plane[ih * W + iw]);
      }
    }
    y[i] = m;
  }
}

int max_pool_f32_impl(const tk_tensor* x, tk_tensor* y, const tk_pool2d_attrs* a, hipStream_t s) {
  TK_CHECK_ARG(x && y && a && is_f32(x) && is_f32(y) && x->ndim == 4 && y->ndim == 4, "float32 NCHW expected");
  const int32_t N = (int32_t)x->shape[0], C = (int32_t)x->shape[1], H = (int32_t)x->shape[2], W = (int32_t)x->shape[3];
  const int dh = a->dilation[0] ? a->dilation[0] : 1, dw = a->dilation[1] ? a->dilation[1] : 1;
  const int32_t OH = (H + a->padding[0] + a->padding[2] - dh * (a->pool_size[0] - 1) - 1) / a->strides[0] + 1;
  const int32_t OW = (W + a->padding[1] + a->padding[3] - dw * (a->pool_size[1] - 1) - 1) / a->strides[1] + 1;
  TK_CHECK_ARG(y->shape[0] == N && y->shape[1] == C && y->shape[2] == OH && y->shape[3] == OW, "output shape mismatch");
  const int64_t n = (int64_t)N * C * OH * OW;
  hipLaunchKernelGGL(max_pool_f32_kernel, dim3(ew_grid(n)), dim3(kEwBlock), 0, s, (const float*)ptr(x),
                     (float*)ptr(y), N, C, H, W, OH, OW, *a);
  TK_LAUNCH_CHECK();
  return TK_OK;
}

}  // namespace tk
