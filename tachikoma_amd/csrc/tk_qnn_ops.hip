// The QNN ops of a pre-quantized (frontend-produced) graph beside conv / dense / requantize / add:
// qnn.quantize, qnn.dequantize, qnn.simulated_quantize / _dequantize, qnn.concatenate, qnn.mul,
// qnn.subtract (and qnn.add with broadcasting / per-axis parameters), plus the transpose that
// carries NHWC / HWIO / OHWI / HWOI qnn.conv2d operands to the NCHW / OIHW kernels (SURVEY.md §8(f)
// row 1).
//
// All of them are HBM-bound streaming kernels (a few bytes in and out per element, a handful of
// integer or float32 operations).  Integer steps wrap in int32 exactly where the reference's
// canonicalized Relay is int32; float32 steps are single IEEE operations in the reference's order
// (correctly rounded division, hipcc's default; no FMA contraction).
#include <algorithm>
#include <climits>

#include "tk_common.h"

#pragma clang fp contract(off)

namespace tk {

namespace {

constexpr int kQBlock = 256;

int qgrid(int64_t items) {
  int64_t g = (items + kQBlock - 1) / kQBlock;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, 256 * 8));
}

// channel index of element i along an axis with `inner` elements after it and C entries
__device__ __forceinline__ int chan(int64_t i, int32_t inner, int32_t C) {
  return (int)((i / inner) % C);
}

bool axis_inner(const tk_tensor* t, int axis, int32_t* inner, int32_t* C) {
  if (t->ndim == 0) {
    *inner = 1;
    *C = 1;
    return true;
  }
  const int ax = axis < 0 ? t->ndim + axis : axis;
  if (ax < 0 || ax >= t->ndim) return false;
  int64_t in = 1;
  for (int i = ax + 1; i < t->ndim; ++i) in *= t->shape[i];
  if (in > INT32_MAX || t->shape[ax] > INT32_MAX) return false;
  *inner = (int32_t)in;
  *C = (int32_t)t->shape[ax];
  return true;
}

// a full RqParams (per-axis arrays included) from the ABI struct
RqParams rq_params(const tk_requantize_attrs& a) {
  RqParams p{};
  p.mode = a.mode;
  p.multiplier = a.multiplier;
  p.shift = a.shift;
  p.zp_in = a.input_zero_point;
  p.zp_out = a.output_zero_point;
  p.ms = a.multipliers;
  p.ss = a.shifts;
  p.zps = a.input_zero_points;
  p.inner = 1;
  p.C = 1;
  return p;
}

bool per_axis_mode(int mode) { return mode == TK_RQ_AXIS_UPWARD || mode == TK_RQ_AXIS_TONEAREST; }

template <typename T> struct Lim {
  static constexpr int64_t lo = (int64_t)std::numeric_limits<T>::min();
  static constexpr int64_t hi = (int64_t)std::numeric_limits<T>::max();
};

template <typename F> int dispatch_q(const tk_tensor* t, F&& f) {
  if (is_int(t, 8)) return f((int8_t)0);
  if (is_uint(t, 8)) return f((uint8_t)0);
  if (is_int(t, 16)) return f((int16_t)0);
  if (is_int(t, 32)) return f((int32_t)0);
  set_error("qnn op: dtype must be int8, uint8, int16 or int32");
  return TK_ERR_DTYPE;
}

// any integer dtype (concatenate without requantize moves the bytes as they are)
template <typename F> int dispatch_q_any(const tk_tensor* t, F&& f) {
  switch (dt_of(t)) {
    case DT_I8: return f((int8_t)0);
    case DT_U8: return f((uint8_t)0);
    case DT_I16: return f((int16_t)0);
    case DT_U16: return f((uint16_t)0);
    case DT_I32: return f((int32_t)0);
    case DT_U32: return f((uint32_t)0);
    case DT_I64: return f((int64_t)0);
    case DT_U64: return f((uint64_t)0);
  }
  set_error("qnn.concatenate: integer dtype expected");
  return TK_ERR_DTYPE;
}

}  // namespace

// ---------------------------------------------------------------- qnn.quantize
// QuantizeLower (src/relay/qnn/op/quantize.cc:113-149):
//   Cast(Clip(Add(Round(Divide(x, scale)), Cast(zp, float32)), qmin, qmax), out_dtype)
// Clip's bounds are float32 constants (topi clip, python/tvm/topi/math.py:615-640); the float ->
// int cast is fptosi.  For an int32 output the upper bound float32(2^31 - 1) is 2^31, which the
// reference's x86 cvttss2si turns into INT32_MIN ("integer indefinite"); that is reproduced.
template <typename To>
__global__ __launch_bounds__(kQBlock) void quantize_kernel(const float* __restrict__ x, To* __restrict__ y, int64_t n,
                                                            float scale, const float* __restrict__ scales,
                                                            int32_t zp, const int32_t* __restrict__ zps,
                                                            int32_t inner, int32_t C, float qmin, float qmax) {
  const int64_t stride = (int64_t)gridDim.x * kQBlock;
  for (int64_t i = blockIdx.x * (int64_t)kQBlock + threadIdx.x; i < n; i += stride) {
    const int c = (scales || zps) ? chan(i, inner, C) : 0;
    const float s = scales ? scales[c] : scale;
    const float z = (float)(zps ? zps[c] : zp);
    float v = x[i] / s;
    v = roundf(v);  // llvm.round: halves away from zero
    v = v + z;
    v = v < qmax ? v : qmax;  // max(min(v, qmax), qmin)
    v = v > qmin ? v : qmin;
    if constexpr (sizeof(To) == 4) {
      y[i] = v >= 2147483648.0f ? (To)INT32_MIN : (To)(int32_t)v;
    } else {
      y[i] = (To)(int32_t)v;
    }
  }
}

static bool qparams_geometry(const tk_tensor* t, const tk_qparams_attrs* a, int32_t* inner, int32_t* C) {
  if (!a->scales && !a->zero_points) {
    *inner = 1;
    *C = 1;
    return true;
  }
  return axis_inner(t, a->axis, inner, C);
}

int qnn_quantize_impl(const tk_tensor* x, tk_tensor* y, const tk_qparams_attrs* a, hipStream_t s) {
  TK_CHECK_ARG(x && y && a, "null argument");
  TK_CHECK_ARG(compact(x) && compact(y) && numel(x) == numel(y), "bad tensors");
  TK_CHECK_ARG(is_f32(x), "qnn.quantize: float32 data expected");
  int32_t inner, C;
  if (!qparams_geometry(x, a, &inner, &C)) {
    set_error("tk_qnn_quantize: bad axis");
    return TK_ERR_INVALID_ARG;
  }
  const int64_t n = numel(x);
  return dispatch_q(y, [&](auto tag) -> int {
    using To = decltype(tag);
    hipLaunchKernelGGL((quantize_kernel<To>), dim3(qgrid(n)), dim3(kQBlock), 0, s, (const float*)ptr(x), (To*)ptr(y),
                       n, a->scale, a->scales, a->zero_point, a->zero_points, inner, C, (float)Lim<To>::lo,
                       (float)Lim<To>::hi);
    TK_LAUNCH_CHECK();
    return TK_OK;
  });
}

// ---------------------------------------------------------------- qnn.dequantize
// DequantizeLower (src/relay/qnn/op/dequantize.cc:96-129):
//   Multiply(Cast(Subtract(Cast(x, int32), zp), float32), scale)
template <typename Ti>
__global__ __launch_bounds__(kQBlock) void dequantize_kernel(const Ti* __restrict__ x, float* __restrict__ y, int64_t n,
                                                              float scale, const float* __restrict__ scales,
                                                              int32_t zp, const int32_t* __restrict__ zps,
                                                              int32_t inner, int32_t C) {
  const int64_t stride = (int64_t)gridDim.x * kQBlock;
  for (int64_t i = blockIdx.x * (int64_t)kQBlock + threadIdx.x; i < n; i += stride) {
    const int c = (scales || zps) ? chan(i, inner, C) : 0;
    const int32_t t = (int32_t)((uint32_t)(int32_t)x[i] - (uint32_t)(zps ? zps[c] : zp));
    y[i] = (float)t * (scales ? scales[c] : scale);
  }
}

int qnn_dequantize_impl(const tk_tensor* x, tk_tensor* y, const tk_qparams_attrs* a, hipStream_t s) {
  TK_CHECK_ARG(x && y && a, "null argument");
  TK_CHECK_ARG(compact(x) && compact(y) && numel(x) == numel(y), "bad tensors");
  TK_CHECK_ARG(is_f32(y), "qnn.dequantize: float32 output expected");
  int32_t inner, C;
  if (!qparams_geometry(x, a, &inner, &C)) {
    set_error("tk_qnn_dequantize: bad axis");
    return TK_ERR_INVALID_ARG;
  }
  const int64_t n = numel(x);
  return dispatch_q(x, [&](auto tag) -> int {
    using Ti = decltype(tag);
    hipLaunchKernelGGL((dequantize_kernel<Ti>), dim3(qgrid(n)), dim3(kQBlock), 0, s, (const Ti*)ptr(x),
                       (float*)ptr(y), n, a->scale, a->scales, a->zero_point, a->zero_points, inner, C);
    TK_LAUNCH_CHECK();
    return TK_OK;
  });
}

// ---------------------------------------------------------------- qnn binary ops
// Broadcast geometry over the output (numpy rules, operands right-aligned, up to 6-D): element
// strides of each operand per output dimension (0 where it broadcasts), and for each per-axis
// parameter set the output dimension its channel index is read from (-1: none, or a broadcast
// size-1 axis whose single entry is channel 0).
struct BinGeom {
  int32_t nd;
  int64_t shape[6];
  int64_t ls[6], rs[6];
  int32_t lax, rax, oax;
};

// numpy broadcasting of a and b to y (BroadcastRel): per-dimension element strides, 0 where an
// operand broadcasts; `same` when no operand broadcasts at all
static int bin_geometry(const tk_tensor* a, const tk_tensor* b, const tk_tensor* y, BinGeom* g, bool* same) {
  g->nd = y->ndim;
  *same = a->ndim == y->ndim && b->ndim == y->ndim;
  int64_t sa = 1, sb = 1;
  for (int d = y->ndim - 1; d >= 0; --d) {
    g->shape[d] = y->shape[d];
    const int da = d - (y->ndim - a->ndim), db = d - (y->ndim - b->ndim);
    const int64_t ea = da >= 0 ? a->shape[da] : 1, eb = db >= 0 ? b->shape[db] : 1;
    if ((ea != 1 && ea != y->shape[d]) || (eb != 1 && eb != y->shape[d])) {
      set_error("tk_qnn_binary: operands do not broadcast to the output shape");
      return TK_ERR_SHAPE;
    }
    *same = *same && ea == y->shape[d] && eb == y->shape[d];
    g->ls[d] = ea == 1 ? 0 : sa;
    g->rs[d] = eb == 1 ? 0 : sb;
    sa *= ea;
    sb *= eb;
  }
  return TK_OK;
}

// the output dimension a per-axis parameter set of operand t indexes (its axis, right-aligned)
static int bin_out_axis(const tk_tensor* t, const tk_tensor* y, int axis) {
  if (t->ndim == 0) return -1;
  const int ax = axis < 0 ? t->ndim + axis : axis;
  if (ax < 0 || ax >= t->ndim || t->shape[ax] == 1) return -1;
  return ax + (y->ndim - t->ndim);
}

// element i of the output -> operand offsets and channel indices (the broadcast walk)
template <bool FLAT>
__device__ __forceinline__ void bin_walk(int64_t i, const BinGeom& g, int64_t* ia, int64_t* ib, int* ca, int* cb,
                                         int* co) {
  *ia = i;
  *ib = i;
  *ca = *cb = *co = 0;
  if constexpr (!FLAT) {
    *ia = 0;
    *ib = 0;
    int64_t r = i;
    for (int d = g.nd - 1; d >= 0; --d) {
      const int64_t q = r / g.shape[d];
      const int64_t k = r - q * g.shape[d];
      r = q;
      *ia += k * g.ls[d];
      *ib += k * g.rs[d];
      if (d == g.lax) *ca = (int)k;
      if (d == g.rax) *cb = (int)k;
      if (d == g.oax) *co = (int)k;
    }
  }
}

template <typename T, int OP, bool FLAT>
__global__ __launch_bounds__(kQBlock) void qnn_binary_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                              T* __restrict__ y, int64_t n, BinGeom g, RqParams pa,
                                                              RqParams pb, RqParams po, int32_t zp_c, int32_t up_a,
                                                              int32_t up_b) {
  const int64_t stride = (int64_t)gridDim.x * kQBlock;
  for (int64_t i = blockIdx.x * (int64_t)kQBlock + threadIdx.x; i < n; i += stride) {
    int64_t ia, ib;
    int ca, cb, co;
    bin_walk<FLAT>(i, g, &ia, &ib, &ca, &cb, &co);
    const int32_t x0 = (int32_t)a[ia], x1 = (int32_t)b[ib];
    int32_t o;
    if constexpr (OP == TK_QB_MUL) {
      // mul.cc:77-101 (per-tensor) / :109-152 (per-channel): shifted operands, int32 product,
      // requantized from s_a*s_b with zero point 0
      const int32_t sa = (int32_t)((uint32_t)x0 - (uint32_t)(pa.zps ? pa.zps[ca] : pa.zp_in));
      const int32_t sb = (int32_t)((uint32_t)x1 - (uint32_t)(pb.zps ? pb.zps[cb] : pb.zp_in));
      o = rq_apply((int32_t)((uint32_t)sa * (uint32_t)sb), co, po);
    } else {
      const int32_t ra = up_a ? x0 : rq_apply(x0, ca, pa);
      const int32_t rb = up_b ? x1 : rq_apply(x1, cb, pb);
      if constexpr (OP == TK_QB_ADD) {
        o = (int32_t)((uint32_t)ra + (uint32_t)rb - (uint32_t)zp_c);
      } else {
        o = (int32_t)((uint32_t)ra - (uint32_t)rb + (uint32_t)zp_c);
      }
    }
    y[i] = (T)std::min<int64_t>(std::max<int64_t>(o, Lim<T>::lo), Lim<T>::hi);
  }
}

int qnn_binary_impl(const tk_tensor* a, const tk_tensor* b, tk_tensor* y, const tk_qnn_binary_attrs* at,
                    hipStream_t s) {
  TK_CHECK_ARG(a && b && y && at, "null argument");
  TK_CHECK_ARG(compact(a) && compact(b) && compact(y), "strided tensors are not supported");
  TK_CHECK_ARG(dt_of(a) == dt_of(b) && dt_of(a) == dt_of(y), "dtype mismatch");
  TK_CHECK_ARG(at->op >= TK_QB_ADD && at->op <= TK_QB_MUL, "bad op");
  TK_CHECK_ARG(y->ndim <= 6 && a->ndim <= y->ndim && b->ndim <= y->ndim, "up to 6-D, operands no wider than the output");
  BinGeom g{};
  bool same = false;
  if (bin_geometry(a, b, y, &g, &same) != TK_OK) return TK_ERR_SHAPE;
  auto out_axis = [&](const tk_tensor* t, int axis) { return bin_out_axis(t, y, axis); };
  RqParams pa = rq_params(at->lhs), pb = rq_params(at->rhs), po = rq_params(at->out);
  const bool mul = at->op == TK_QB_MUL;
  const bool axis_a = pa.zps || (!mul && !at->lhs_upcast && per_axis_mode(pa.mode));
  const bool axis_b = pb.zps || (!mul && !at->rhs_upcast && per_axis_mode(pb.mode));
  const bool axis_o = mul && per_axis_mode(po.mode);
  TK_CHECK_ARG(!per_axis_mode(pa.mode) || pa.ms, "per-axis lhs plan needs multipliers");
  TK_CHECK_ARG(!per_axis_mode(pb.mode) || pb.ms, "per-axis rhs plan needs multipliers");
  TK_CHECK_ARG(!axis_o || po.ms, "per-axis output plan needs multipliers");
  g.lax = axis_a ? out_axis(a, at->lhs.axis) : -1;
  g.rax = axis_b ? out_axis(b, at->rhs.axis) : -1;
  g.oax = axis_o ? out_axis(a, at->out.axis) : -1;
  const bool flat = same && !axis_a && !axis_b && !axis_o;
  const int64_t n = numel(y);
  return dispatch_q(y, [&](auto tag) -> int {
    using T = decltype(tag);
    auto go = [&](auto op_tag, auto flat_tag) -> int {
      constexpr int OP = decltype(op_tag)::value;
      constexpr bool FLAT = decltype(flat_tag)::value;
      hipLaunchKernelGGL((qnn_binary_kernel<T, OP, FLAT>), dim3(qgrid(n)), dim3(kQBlock), 0, s, (const T*)ptr(a),
                         (const T*)ptr(b), (T*)ptr(y), n, g, pa, pb, po, at->output_zero_point, at->lhs_upcast,
                         at->rhs_upcast);
      TK_LAUNCH_CHECK();
      return TK_OK;
    };
    using TF = std::true_type;
    using FF = std::false_type;
    switch (at->op) {
      case TK_QB_ADD: return flat ? go(std::integral_constant<int, TK_QB_ADD>{}, TF{})
                                  : go(std::integral_constant<int, TK_QB_ADD>{}, FF{});
      case TK_QB_SUBTRACT: return flat ? go(std::integral_constant<int, TK_QB_SUBTRACT>{}, TF{})
                                       : go(std::integral_constant<int, TK_QB_SUBTRACT>{}, FF{});
      default: return flat ? go(std::integral_constant<int, TK_QB_MUL>{}, TF{})
                           : go(std::integral_constant<int, TK_QB_MUL>{}, FF{});
    }
  });
}

// ---------------------------------------------------------------- qnn.concatenate
// ConcatenateQnnCanonicalize (concatenate.cc:153-221): each input requantized (RequantizeLower, out
// dtype = the input's: clip + cast) unless its params equal the output's, then concatenate.
// One launch per input writes its slab: element i of the input (outer index o, offset r inside
// the input's Ck * inner run) lands at o * (Ctot * inner) + Coff * inner + r.
template <typename T>
__global__ __launch_bounds__(kQBlock) void concat_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n,
                                                          int64_t run, int64_t out_run, int64_t off, RqParams p,
                                                          int32_t rq) {
  const int64_t stride = (int64_t)gridDim.x * kQBlock;
  for (int64_t i = blockIdx.x * (int64_t)kQBlock + threadIdx.x; i < n; i += stride) {
    const int64_t o = i / run;
    const int64_t r = i - o * run;
    T v = x[i];
    if constexpr (sizeof(T) <= 4) {
      if (rq) v = (T)std::min<int64_t>(std::max<int64_t>(rq_apply((int32_t)v, 0, p), Lim<T>::lo), Lim<T>::hi);
    }
    y[o * out_run + off + r] = v;
  }
}

int qnn_concatenate_impl(const tk_tensor* const* xs, int n_in, tk_tensor* y, const tk_concat_attrs* a,
                         hipStream_t s) {
  TK_CHECK_ARG(xs && y && a && n_in >= 1 && n_in <= TK_CONCAT_MAX && a->n == n_in, "bad arguments");
  TK_CHECK_ARG(compact(y) && is_integer(y), "integer output expected");
  const int nd = y->ndim;
  const int ax = a->axis < 0 ? nd + a->axis : a->axis;
  TK_CHECK_ARG(nd >= 1 && ax >= 0 && ax < nd, "bad axis");
  int64_t inner = 1, outer = 1;
  for (int d = ax + 1; d < nd; ++d) inner *= y->shape[d];
  for (int d = 0; d < ax; ++d) outer *= y->shape[d];
  int64_t coff = 0;
  for (int k = 0; k < n_in; ++k) {
    const tk_tensor* x = xs[k];
    TK_CHECK_ARG(x && compact(x) && x->ndim == nd && dt_of(x) == dt_of(y), "inputs must match the output's rank and dtype");
    for (int d = 0; d < nd; ++d)
      TK_CHECK_ARG(d == ax || x->shape[d] == y->shape[d], "inputs differ outside the concatenation axis");
    TK_CHECK_ARG(!a->requant[k] || (!per_axis_mode(a->rq[k].mode) && elem_bytes(y) <= 4),
                 "per-tensor requantize of 8/16/32-bit inputs only");
    coff += x->shape[ax];
  }
  TK_CHECK_ARG(coff == y->shape[ax], "input sizes along the axis do not add up to the output's");
  coff = 0;
  for (int k = 0; k < n_in; ++k) {
    const tk_tensor* x = xs[k];
    const int64_t n = numel(x);
    const int64_t run = x->shape[ax] * inner;
    const RqParams p = rq_params(a->rq[k]);
    if (n > 0) {
      int rc = dispatch_q_any(y, [&](auto tag) -> int {
        using T = decltype(tag);
        hipLaunchKernelGGL((concat_kernel<T>), dim3(qgrid(n)), dim3(kQBlock), 0, s, (const T*)ptr(x), (T*)ptr(y), n,
                           run, y->shape[ax] * inner, coff * inner, p, a->requant[k]);
        TK_LAUNCH_CHECK();
        return TK_OK;
      });
      if (rc) return rc;
    }
    coff += x->shape[ax];
  }
  (void)outer;
  return TK_OK;
}

// ---------------------------------------------------------------- transpose
struct TransGeom {
  int32_t nd;
  int64_t shape[6];   // output shape
  int64_t src[6];     // input element stride of each output dimension
};

template <typename T>
__global__ __launch_bounds__(kQBlock) void transpose_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n,
                                                             TransGeom g) {
  const int64_t stride = (int64_t)gridDim.x * kQBlock;
  for (int64_t i = blockIdx.x * (int64_t)kQBlock + threadIdx.x; i < n; i += stride) {
    int64_t r = i, si = 0;
    for (int d = g.nd - 1; d >= 0; --d) {
      const int64_t q = r / g.shape[d];
      si += (r - q * g.shape[d]) * g.src[d];
      r = q;
    }
    y[i] = x[si];
  }
}

int transpose_impl(const tk_tensor* x, tk_tensor* y, const tk_transpose_attrs* a, hipStream_t s) {
  TK_CHECK_ARG(x && y && a, "null argument");
  TK_CHECK_ARG(compact(x) && compact(y) && x->ndim == a->ndim && y->ndim == a->ndim && a->ndim >= 1 && a->ndim <= 6,
               "bad tensors");
  TK_CHECK_ARG(elem_bytes(x) == elem_bytes(y) && x->dtype.code == y->dtype.code, "dtype mismatch");
  TransGeom g{};
  g.nd = a->ndim;
  int64_t st[6];
  st[a->ndim - 1] = 1;
  for (int d = a->ndim - 2; d >= 0; --d) st[d] = st[d + 1] * x->shape[d + 1];
  int seen = 0;
  for (int k = 0; k < a->ndim; ++k) {
    const int p = a->perm[k];
    TK_CHECK_ARG(p >= 0 && p < a->ndim && !(seen & (1 << p)), "perm is not a permutation");
    seen |= 1 << p;
    TK_CHECK_ARG(y->shape[k] == x->shape[p], "output shape is not the permuted input shape");
    g.shape[k] = y->shape[k];
    g.src[k] = st[p];
  }
  const int64_t n = numel(x);
  if (n == 0) return TK_OK;
  auto go = [&](auto tag) -> int {
    using T = decltype(tag);
    hipLaunchKernelGGL((transpose_kernel<T>), dim3(qgrid(n)), dim3(kQBlock), 0, s, (const T*)ptr(x), (T*)ptr(y), n, g);
    TK_LAUNCH_CHECK();
    return TK_OK;
  };
  switch (elem_bytes(x)) {
    case 1: return go((uint8_t)0);
    case 2: return go((uint16_t)0);
    case 4: return go((uint32_t)0);
    case 8: return go((uint64_t)0);
  }
  set_error("tk_transpose: 1, 2, 4 or 8-byte elements");
  return TK_ERR_DTYPE;
}

// ---------------------------------------------------------------- qnn.leaky_relu
// QnnLeakyReluCanonicalize (src/relay/qnn/op/leaky_relu.cc:85-140):
//   data = int32(x);  q = RequantizeOrUpcast(data) at the output params
//   out  = ConvertDtype(Where(Less(data, zp_in), FPM(q, alpha) + FPM(zp_out, 1 - alpha), q))
// FPM = fixed_point_multiply -> tir.q_multiply_shift (intrin_rule.cc:197-250): the int32
// power-of-two branch when the multiplier is 1 << 30, else the int64 QMultiplyShift form.
__device__ __forceinline__ int32_t fpm_tir(int32_t x, int32_t m, int32_t s) {
  return m == (1 << 30) ? qms_pow2(x, s) : qms_upward(x, m, s);
}

template <typename T>
__global__ __launch_bounds__(kQBlock) void leaky_relu_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n,
                                                              RqParams rq, int32_t upcast, int32_t zp_in,
                                                              int32_t zp_out, int32_t am, int32_t as, int32_t zm,
                                                              int32_t zs) {
  const int32_t scaled_z = fpm_tir(zp_out, zm, zs);  // FPM(zp_out, 1 - alpha): a constant
  const int64_t stride = (int64_t)gridDim.x * kQBlock;
  for (int64_t i = blockIdx.x * (int64_t)kQBlock + threadIdx.x; i < n; i += stride) {
    const int32_t d = (int32_t)x[i];
    const int32_t q = upcast ? d : rq_apply(d, 0, rq);
    const int32_t add = (int32_t)((uint32_t)fpm_tir(q, am, as) + (uint32_t)scaled_z);
    int32_t o = d < zp_in ? add : q;
    o = o < (int32_t)Lim<T>::lo ? (int32_t)Lim<T>::lo : o > (int32_t)Lim<T>::hi ? (int32_t)Lim<T>::hi : o;
    y[i] = (T)o;
  }
}

static bool pow2_shift_ok(int32_t m, int32_t s) { return !(m == (1 << 30) && s == 1); }

int qnn_leaky_relu_impl(const tk_tensor* x, tk_tensor* y, const tk_leaky_relu_attrs* a, hipStream_t s) {
  TK_CHECK_ARG(x && y && a, "null argument");
  TK_CHECK_ARG(compact(x) && compact(y) && numel(x) == numel(y) && dt_of(x) == dt_of(y), "bad tensors");
  TK_CHECK_ARG(is_int8ish(x), "qnn.leaky_relu: int8 or uint8 data expected");
  TK_CHECK_ARG(a->upcast || !per_axis_mode(a->rq.mode), "qnn.leaky_relu: per-tensor requantize only");
  // (q_multiply_shift's power-of-two branch with shift 1 needs a rounding factor 1 << -1, which
  // the reference's compiler rejects: alpha == 0 or 1 does not build there either)
  TK_CHECK_ARG(pow2_shift_ok(a->alpha_multiplier, a->alpha_shift) && pow2_shift_ok(a->zp_multiplier, a->zp_shift),
               "qnn.leaky_relu: alpha 0 or 1 (fixed_point_multiply by 1.0) is not buildable in the reference");
  const RqParams rq = rq_params(a->rq);
  const int64_t n = numel(x);
  auto go = [&](auto tag) -> int {
    using T = decltype(tag);
    hipLaunchKernelGGL((leaky_relu_kernel<T>), dim3(qgrid(n)), dim3(kQBlock), 0, s, (const T*)ptr(x), (T*)ptr(y), n,
                       rq, a->upcast, a->input_zero_point, a->output_zero_point, a->alpha_multiplier, a->alpha_shift,
                       a->zp_multiplier, a->zp_shift);
    TK_LAUNCH_CHECK();
    return TK_OK;
  };
  return is_int(x, 8) ? go((int8_t)0) : go((uint8_t)0);
}

// ---------------------------------------------------------------- qnn unary ops (table lookup)
// take(table, reinterpret<uint8>(x), mode="fast") (python/tvm/relay/qnn/op/canonicalizations.py:
// 157-160): 16 bytes per thread and step, the table in LDS.
__global__ __launch_bounds__(kQBlock) void lookup_kernel(const uint8_t* __restrict__ x, uint8_t* __restrict__ y,
                                                          int64_t n, const uint8_t* __restrict__ table) {
  __shared__ uint8_t t[256];
  t[threadIdx.x] = table[threadIdx.x];  // kQBlock == 256
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * kQBlock;
  const int64_t n16 = n / 16;
  for (int64_t i = blockIdx.x * (int64_t)kQBlock + threadIdx.x; i < n16; i += stride) {
    uint4 v = reinterpret_cast<const uint4*>(x)[i];
    uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      w[k] = (uint32_t)t[w[k] & 0xFF] | ((uint32_t)t[(w[k] >> 8) & 0xFF] << 8) |
             ((uint32_t)t[(w[k] >> 16) & 0xFF] << 16) | ((uint32_t)t[w[k] >> 24] << 24);
    reinterpret_cast<uint4*>(y)[i] = make_uint4(w[0], w[1], w[2], w[3]);
  }
  for (int64_t i = n16 * 16 + blockIdx.x * (int64_t)kQBlock + threadIdx.x; i < n; i += stride) y[i] = t[x[i]];
}

int qnn_lookup_impl(const tk_tensor* x, tk_tensor* y, const void* table, hipStream_t s) {
  static_assert(kQBlock == 256, "one table entry per thread");
  TK_CHECK_ARG(x && y && table, "null argument");
  TK_CHECK_ARG(compact(x) && compact(y) && numel(x) == numel(y) && is_int8ish(x) && is_int8ish(y), "bad tensors");
  TK_CHECK_ARG(((uintptr_t)ptr(x) | (uintptr_t)ptr(y)) % 16 == 0, "qnn lookup: 16-byte aligned buffers expected");
  const int64_t n = numel(x);
  hipLaunchKernelGGL(lookup_kernel, dim3(qgrid((n + 15) / 16)), dim3(kQBlock), 0, s, (const uint8_t*)ptr(x),
                     (uint8_t*)ptr(y), n, (const uint8_t*)table);
  TK_LAUNCH_CHECK();
  return TK_OK;
}

// ---------------------------------------------------------------- qnn.conv2d_transpose
// int16 operand shifts (legalizations.py:97-130) and nn.conv2d_transpose (topi conv2d_transpose_nchw,
// python/tvm/topi/nn/conv2d_transpose.py:79-140: dilate by the stride, pad by k - 1 - pad (+ the
// output padding), the kernel flipped): an output pixel (y, x) gathers input pixels iy with
// y + pt - r = sh * iy for each kernel row r (likewise columns), products in int32, wrapping sums.
// A direct gather kernel (one output element per thread): transpose convolutions are not on the
// ResNet-50 trace path; the operands stay in L2 for these shapes.
template <typename Ti, typename Tw>
__global__ __launch_bounds__(kQBlock) void conv2d_transpose_kernel(
    const Ti* __restrict__ x, const Tw* __restrict__ w, int32_t* __restrict__ y, int64_t n_out, int C, int H, int W,
    int O, int OH, int OW, int KH, int KW, int sh, int sw, int pt, int pl, int groups, int32_t zx, int32_t zw,
    const int32_t* __restrict__ zws) {
  const int og = O / groups, cg = C / groups;
  const int64_t stride = (int64_t)gridDim.x * kQBlock;
  for (int64_t i = blockIdx.x * (int64_t)kQBlock + threadIdx.x; i < n_out; i += stride) {
    const int ox = (int)(i % OW);
    const int oy = (int)((i / OW) % OH);
    const int o = (int)((i / ((int64_t)OW * OH)) % O);
    const int64_t nb = i / ((int64_t)OW * OH * O);
    const int g = o / og, oo = o - g * og;
    const int16_t kz = (int16_t)(zws ? zws[oo] : zw);
    uint32_t acc = 0;
    for (int c = g * cg; c < (g + 1) * cg; ++c) {
      const Ti* xc = x + ((nb * C + c) * H) * (int64_t)W;
      const Tw* wc = w + (((int64_t)c * og + oo) * KH) * KW;
      for (int r = 0; r < KH; ++r) {
        const int ty = oy + pt - r;
        if (ty < 0 || ty % sh) continue;
        const int iy = ty / sh;
        if (iy >= H) continue;
        for (int q = 0; q < KW; ++q) {
          const int tx = ox + pl - q;
          if (tx < 0 || tx % sw) continue;
          const int ix = tx / sw;
          if (ix >= W) continue;
          const int16_t d = (int16_t)((int16_t)xc[(int64_t)iy * W + ix] - (int16_t)zx);
          const int16_t k = (int16_t)((int16_t)wc[r * KW + q] - kz);
          acc += (uint32_t)((int32_t)d * (int32_t)k);
        }
      }
    }
    y[i] = (int32_t)acc;
  }
}

int qnn_conv2d_transpose_impl(const tk_tensor* x, const tk_tensor* w, tk_tensor* y, const tk_conv2d_transpose_attrs* a,
                              hipStream_t s) {
  TK_CHECK_ARG(x && w && y && a, "null argument");
  TK_CHECK_ARG(compact(x) && compact(w) && compact(y) && x->ndim == 4 && w->ndim == 4 && y->ndim == 4, "4-D tensors");
  TK_CHECK_ARG(is_int8ish(x) && is_int8ish(w) && is_int(y, 32), "int8/uint8 operands, int32 output");
  const int N = (int)x->shape[0], C = (int)x->shape[1], H = (int)x->shape[2], W = (int)x->shape[3];
  const int og = (int)w->shape[1], KH = (int)w->shape[2], KW = (int)w->shape[3];
  const int groups = a->groups;
  TK_CHECK_ARG(groups >= 1 && C % groups == 0 && w->shape[0] == C, "weight (C, O/groups, KH, KW) for the data's C");
  const int O = og * groups;
  const int sh = a->strides[0], sw = a->strides[1];
  TK_CHECK_ARG(sh >= 1 && sw >= 1 && a->output_padding[0] >= 0 && a->output_padding[0] < sh &&
               a->output_padding[1] >= 0 && a->output_padding[1] < sw, "strides / output padding");
  const int OH = (H - 1) * sh + KH - a->padding[0] - a->padding[2] + a->output_padding[0];
  const int OW = (W - 1) * sw + KW - a->padding[1] - a->padding[3] + a->output_padding[1];
  TK_CHECK_ARG(y->shape[0] == N && y->shape[1] == O && y->shape[2] == OH && y->shape[3] == OW,
               "output shape (N, O, (H-1)*s + K - pads + output_padding, ...) expected");
  const int64_t n = numel(y);
  auto go = [&](auto tx, auto tw) -> int {
    using Ti = decltype(tx);
    using Tw = decltype(tw);
    hipLaunchKernelGGL((conv2d_transpose_kernel<Ti, Tw>), dim3(qgrid(n)), dim3(kQBlock), 0, s, (const Ti*)ptr(x),
                       (const Tw*)ptr(w), (int32_t*)ptr(y), n, C, H, W, O, OH, OW, KH, KW, sh, sw, a->padding[0],
                       a->padding[1], groups, a->input_zero_point, a->kernel_zero_point, a->kernel_zero_points);
    TK_LAUNCH_CHECK();
    return TK_OK;
  };
  if (is_int(x, 8)) return is_int(w, 8) ? go((int8_t)0, (int8_t)0) : go((int8_t)0, (uint8_t)0);
  return is_int(w, 8) ? go((uint8_t)0, (int8_t)0) : go((uint8_t)0, (uint8_t)0);
}

// ---------------------------------------------------------------- simulated (de)quantize
// topi.nn.simulated_quantize / simulated_dequantize (python/tvm/topi/nn/qnn.py:40-190), float32 in
// and out.  The dtype code is read from device memory (a graph may compute it); every thread reads
// the same word.  Float steps are single IEEE operations in topi's order: x / scale, llvm.round,
// + float32(zp), min(., float32(qmax)), max(., float32(qmin)) -- TIR's binary-op type matching casts
// the int32 zero point and the integer bounds to float32 (an int32 qmax of 2^31 - 1 becomes 2^31).
__global__ __launch_bounds__(kQBlock) void sim_quantize_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                               int64_t n, const int32_t* __restrict__ code,
                                                               const float* __restrict__ scales, int32_t ns,
                                                               const int32_t* __restrict__ zps, int32_t nz,
                                                               int32_t inner, int32_t C) {
  const int32_t c0 = *code;
  const bool on = c0 >= 1 && c0 <= 3;
  const float qmin = c0 == 1 ? -128.0f : c0 == 2 ? 0.0f : -2147483648.0f;
  const float qmax = c0 == 1 ? 127.0f : c0 == 2 ? 255.0f : 2147483648.0f;
  const int64_t stride = (int64_t)gridDim.x * kQBlock;
  for (int64_t i = blockIdx.x * (int64_t)kQBlock + threadIdx.x; i < n; i += stride) {
    float v = x[i];
    if (on) {
      const int c = chan(i, inner, C);
      v = v / scales[c % ns];
      v = roundf(v);  // llvm.round: halves away from zero
      v = v + (float)zps[c % nz];
      v = v < qmax ? v : qmax;
      v = v > qmin ? v : qmin;
    }
    y[i] = v;
  }
}

__global__ __launch_bounds__(kQBlock) void sim_dequantize_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                                 int64_t n, const int32_t* __restrict__ code,
                                                                 const float* __restrict__ scales, int32_t ns,
                                                                 const int32_t* __restrict__ zps, int32_t nz,
                                                                 int32_t inner, int32_t C) {
  const int32_t c0 = *code;
  const bool on = c0 >= 1 && c0 <= 3;
  const int64_t stride = (int64_t)gridDim.x * kQBlock;
  for (int64_t i = blockIdx.x * (int64_t)kQBlock + threadIdx.x; i < n; i += stride) {
    float v = x[i];
    if (on) {
      const int c = chan(i, inner, C);
      v = (v - (float)zps[c % nz]) * scales[c % ns];
    }
    y[i] = v;
  }
}

int qnn_simulated_impl(bool quant, const tk_tensor* x, tk_tensor* y, const tk_simq_attrs* a, hipStream_t s) {
  const char* what = quant ? "qnn.simulated_quantize" : "qnn.simulated_dequantize";
  TK_CHECK_ARG(x && y && a, "null argument");
  TK_CHECK_ARG(compact(x) && compact(y) && numel(x) == numel(y), "bad tensors");
  if (!is_f32(x) || !is_f32(y)) {
    set_error(std::string(what) + ": float32 data and output expected");
    return TK_ERR_DTYPE;
  }
  if (!a->dtype_code || !a->scales || !a->zero_points || a->n_scales < 1 || a->n_zero_points < 1) {
    set_error(std::string(what) + ": dtype code, scales and zero points are required device arrays");
    return TK_ERR_INVALID_ARG;
  }
  int32_t inner, C;
  if (x->ndim < 1 || !axis_inner(x, a->axis, &inner, &C)) {
    set_error(std::string(what) + ": bad axis");
    return TK_ERR_INVALID_ARG;
  }
  const int64_t n = numel(x);
  hipLaunchKernelGGL(quant ? sim_quantize_kernel : sim_dequantize_kernel, dim3(qgrid(n)), dim3(kQBlock), 0, s,
                     (const float*)ptr(x), (float*)ptr(y), n, a->dtype_code, a->scales, a->n_scales, a->zero_points,
                     a->n_zero_points, inner, C);
  TK_LAUNCH_CHECK();
  return TK_OK;
}

// ---------------------------------------------------------------- float-compute requantize
// RequantizeLowerFP<Bits> (src/relay/qnn/op/requantize.cc:293-373) for compute_dtype float32 /
// float64, with the non-SSE4.1 rounding forms of :127-173 (the MRT llvm target has no -mcpu).
// Every step is one IEEE operation in F (this file compiles with fp contract off); the float ->
// int casts reproduce x86-64's cvtt* instructions, which the reference's LLVM fptosi lowers to:
// truncation, INT_MIN of the target width for NaN / out-of-range input.
struct RqFp {
  int32_t rounding, scaled;
  double m;
  const double* ms;
  int32_t zp_in;
  const int32_t* zps;
  int32_t zp_out;
};

template <typename F> struct FpInt;                 // Cast(.., Int(Bits))
template <> struct FpInt<float> { using T = int32_t; };
template <> struct FpInt<double> { using T = int64_t; };

template <typename I, typename F>
__device__ __forceinline__ I fptosi_x86(F v) {
  constexpr F lim = sizeof(I) == 4 ? (F)2147483648.0 : (F)9223372036854775808.0;
  return (v >= -lim && v < lim) ? (I)v : std::numeric_limits<I>::min();  // NaN fails both compares
}

template <typename F>
__device__ __forceinline__ F fp_upward(F t) {  // requantize.cc:154-172
  using I = typename FpInt<F>::T;
  const F biased = t + (F)0.5;
  const F bf = (F)fptosi_x86<I>(biased);
  const F r = (biased == bf || biased >= (F)0) ? bf : bf - (F)1;
  return __builtin_isfinite(t) ? r : t;
}

template <typename F>
__device__ __forceinline__ F fp_tonearest(F t) {  // requantize.cc:129-146
  using I = typename FpInt<F>::T;
  const F mult = t < (F)0 ? (F)-1 : (F)1;
  const F biased = t + (F)0.5 * mult;
  const F bm = biased * mult;
  const F r = (F)fptosi_x86<I>(bm) * mult;
  return __builtin_isfinite(t) ? r : t;
}

// one element: int32 input (already cast from the data dtype) -> int32 (before any output clip)
template <typename F>
__device__ __forceinline__ int32_t rq_fp(int32_t x, int c, const RqFp& p) {
  F t = (F)x;
  t = t - (F)(p.zps ? p.zps[c] : p.zp_in);
  if (p.ms) t = t * (F)p.ms[c];
  else if (p.scaled) t = (F)p.m * t;
  t = t + (F)p.zp_out;
  t = p.rounding == TK_ROUND_UPWARD ? fp_upward(t) : fp_tonearest(t);
  return fptosi_x86<int32_t>(t);
}

static RqFp rq_fp_params(const tk_requantize_fp_attrs& a) {
  RqFp p{};
  p.rounding = a.rounding;
  p.scaled = a.scaled;
  p.m = a.multiplier;
  p.ms = a.multipliers;
  p.zp_in = a.input_zero_point;
  p.zps = a.input_zero_points;
  p.zp_out = a.output_zero_point;
  return p;
}

static bool fp_attrs_ok(const tk_requantize_fp_attrs& a) {
  return (a.bits == 32 || a.bits == 64) && (a.rounding == TK_ROUND_UPWARD || a.rounding == TK_ROUND_TONEAREST);
}

template <typename F, typename Tin, typename Tout>
__global__ __launch_bounds__(kQBlock) void requantize_fp_kernel(const Tin* __restrict__ x, Tout* __restrict__ y,
                                                                 int64_t n, RqFp p, int32_t inner, int32_t C,
                                                                 int32_t clip) {
  const int64_t stride = (int64_t)gridDim.x * kQBlock;
  for (int64_t i = blockIdx.x * (int64_t)kQBlock + threadIdx.x; i < n; i += stride) {
    const int c = (p.ms || p.zps) ? chan(i, inner, C) : 0;
    int32_t q = rq_fp<F>((int32_t)x[i], c, p);
    if (clip) q = (int32_t)std::min<int64_t>(std::max<int64_t>(q, Lim<Tout>::lo), Lim<Tout>::hi);
    y[i] = (Tout)q;
  }
}

int requantize_fp_impl(const tk_tensor* x, tk_tensor* y, const tk_requantize_fp_attrs* a, hipStream_t s) {
  TK_CHECK_ARG(x && y && a, "null argument");
  TK_CHECK_ARG(compact(x) && compact(y) && numel(x) == numel(y), "bad tensors");
  if (!fp_attrs_ok(*a)) {
    set_error("tk_requantize_fp: bits must be 32 or 64 and rounding UPWARD or TONEAREST");
    return TK_ERR_INVALID_ARG;
  }
  int32_t inner = 1, C = 1;
  if ((a->multipliers || a->input_zero_points) && !axis_inner(x, a->axis, &inner, &C)) {
    set_error("tk_requantize_fp: bad axis");
    return TK_ERR_INVALID_ARG;
  }
  const RqFp p = rq_fp_params(*a);
  const int64_t n = numel(x);
  const int clip = !is_int(y, 32);
  return dispatch_q(x, [&](auto ti) -> int {
    return dispatch_q(y, [&](auto to) -> int {
      using Tin = decltype(ti);
      using Tout = decltype(to);
      if (a->bits == 32)
        hipLaunchKernelGGL((requantize_fp_kernel<float, Tin, Tout>), dim3(qgrid(n)), dim3(kQBlock), 0, s,
                           (const Tin*)ptr(x), (Tout*)ptr(y), n, p, inner, C, clip);
      else
        hipLaunchKernelGGL((requantize_fp_kernel<double, Tin, Tout>), dim3(qgrid(n)), dim3(kQBlock), 0, s,
                           (const Tin*)ptr(x), (Tout*)ptr(y), n, p, inner, C, clip);
      TK_LAUNCH_CHECK();
      return TK_OK;
    });
  });
}

// qnn.add / subtract / mul with RequantizeLowerFP inner requantizes (int32 results, no clip)
template <typename F, typename T, int OP, bool FLAT>
__global__ __launch_bounds__(kQBlock) void qnn_binary_fp_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                                 T* __restrict__ y, int64_t n, BinGeom g, RqFp pa,
                                                                 RqFp pb, RqFp po, int32_t zp_c, int32_t up_a,
                                                                 int32_t up_b) {
  const int64_t stride = (int64_t)gridDim.x * kQBlock;
  for (int64_t i = blockIdx.x * (int64_t)kQBlock + threadIdx.x; i < n; i += stride) {
    int64_t ia, ib;
    int ca, cb, co;
    bin_walk<FLAT>(i, g, &ia, &ib, &ca, &cb, &co);
    const int32_t x0 = (int32_t)a[ia], x1 = (int32_t)b[ib];
    int32_t o;
    if constexpr (OP == TK_QB_MUL) {
      const int32_t sa = (int32_t)((uint32_t)x0 - (uint32_t)(pa.zps ? pa.zps[ca] : pa.zp_in));
      const int32_t sb = (int32_t)((uint32_t)x1 - (uint32_t)(pb.zps ? pb.zps[cb] : pb.zp_in));
      o = rq_fp<F>((int32_t)((uint32_t)sa * (uint32_t)sb), co, po);
    } else {
      const int32_t ra = up_a ? x0 : rq_fp<F>(x0, ca, pa);
      const int32_t rb = up_b ? x1 : rq_fp<F>(x1, cb, pb);
      if constexpr (OP == TK_QB_ADD) {
        o = (int32_t)((uint32_t)ra + (uint32_t)rb - (uint32_t)zp_c);
      } else {
        o = (int32_t)((uint32_t)ra - (uint32_t)rb + (uint32_t)zp_c);
      }
    }
    y[i] = (T)std::min<int64_t>(std::max<int64_t>(o, Lim<T>::lo), Lim<T>::hi);
  }
}

int qnn_binary_fp_impl(const tk_tensor* a, const tk_tensor* b, tk_tensor* y, const tk_qnn_binary_fp_attrs* at,
                       hipStream_t s) {
  TK_CHECK_ARG(a && b && y && at, "null argument");
  TK_CHECK_ARG(compact(a) && compact(b) && compact(y), "strided tensors are not supported");
  TK_CHECK_ARG(dt_of(a) == dt_of(b) && dt_of(a) == dt_of(y), "dtype mismatch");
  TK_CHECK_ARG(at->op >= TK_QB_ADD && at->op <= TK_QB_MUL, "bad op");
  TK_CHECK_ARG(y->ndim <= 6 && a->ndim <= y->ndim && b->ndim <= y->ndim, "up to 6-D, operands no wider than the output");
  const bool mul = at->op == TK_QB_MUL;
  const int bits = mul ? at->out.bits : at->lhs.bits;
  TK_CHECK_ARG(fp_attrs_ok(mul ? at->out : at->lhs) && (mul || fp_attrs_ok(at->rhs)) &&
               (mul || at->rhs.bits == bits), "bits must be 32 or 64 on every side, rounding UPWARD or TONEAREST");
  BinGeom g{};
  bool same = false;
  if (bin_geometry(a, b, y, &g, &same) != TK_OK) return TK_ERR_SHAPE;
  const RqFp pa = rq_fp_params(at->lhs), pb = rq_fp_params(at->rhs), po = rq_fp_params(at->out);
  const bool axis_a = pa.zps || (!mul && !at->lhs_upcast && pa.ms);
  const bool axis_b = pb.zps || (!mul && !at->rhs_upcast && pb.ms);
  const bool axis_o = mul && po.ms;
  g.lax = axis_a ? bin_out_axis(a, y, at->lhs.axis) : -1;
  g.rax = axis_b ? bin_out_axis(b, y, at->rhs.axis) : -1;
  g.oax = axis_o ? bin_out_axis(a, y, at->out.axis) : -1;
  const bool flat = same && !axis_a && !axis_b && !axis_o;
  const int64_t n = numel(y);
  return dispatch_q(y, [&](auto tag) -> int {
    using T = decltype(tag);
    auto go = [&](auto f_tag, auto op_tag, auto flat_tag) -> int {
      using F = decltype(f_tag);
      constexpr int OP = decltype(op_tag)::value;
      constexpr bool FLAT = decltype(flat_tag)::value;
      hipLaunchKernelGGL((qnn_binary_fp_kernel<F, T, OP, FLAT>), dim3(qgrid(n)), dim3(kQBlock), 0, s,
                         (const T*)ptr(a), (const T*)ptr(b), (T*)ptr(y), n, g, pa, pb, po, at->output_zero_point,
                         at->lhs_upcast, at->rhs_upcast);
      TK_LAUNCH_CHECK();
      return TK_OK;
    };
    auto by_op = [&](auto f_tag) -> int {
      using TF = std::true_type;
      using FF = std::false_type;
      switch (at->op) {
        case TK_QB_ADD: return flat ? go(f_tag, std::integral_constant<int, TK_QB_ADD>{}, TF{})
                                    : go(f_tag, std::integral_constant<int, TK_QB_ADD>{}, FF{});
        case TK_QB_SUBTRACT: return flat ? go(f_tag, std::integral_constant<int, TK_QB_SUBTRACT>{}, TF{})
                                         : go(f_tag, std::integral_constant<int, TK_QB_SUBTRACT>{}, FF{});
        default: return flat ? go(f_tag, std::integral_constant<int, TK_QB_MUL>{}, TF{})
                             : go(f_tag, std::integral_constant<int, TK_QB_MUL>{}, FF{});
      }
    };
    return bits == 32 ? by_op(0.0f) : by_op(0.0);
  });
}

}  // namespace tk

extern "C" {

int tk_qnn_quantize(const tk_tensor* data, tk_tensor* out, const tk_qparams_attrs* attrs, void* stream) {
  return tk::qnn_quantize_impl(data, out, attrs, tk::as_stream(stream));
}
int tk_qnn_dequantize(const tk_tensor* data, tk_tensor* out, const tk_qparams_attrs* attrs, void* stream) {
  return tk::qnn_dequantize_impl(data, out, attrs, tk::as_stream(stream));
}
int tk_qnn_binary(const tk_tensor* lhs, const tk_tensor* rhs, tk_tensor* out, const tk_qnn_binary_attrs* attrs,
                  void* stream) {
  return tk::qnn_binary_impl(lhs, rhs, out, attrs, tk::as_stream(stream));
}
int tk_qnn_concatenate(const tk_tensor* const* inputs, int n, tk_tensor* out, const tk_concat_attrs* attrs,
                       void* stream) {
  return tk::qnn_concatenate_impl(inputs, n, out, attrs, tk::as_stream(stream));
}
int tk_transpose(const tk_tensor* data, tk_tensor* out, const tk_transpose_attrs* attrs, void* stream) {
  return tk::transpose_impl(data, out, attrs, tk::as_stream(stream));
}
int tk_qnn_leaky_relu(const tk_tensor* data, tk_tensor* out, const tk_leaky_relu_attrs* attrs, void* stream) {
  return tk::qnn_leaky_relu_impl(data, out, attrs, tk::as_stream(stream));
}
int tk_qnn_lookup(const tk_tensor* data, tk_tensor* out, const void* table, void* stream) {
  return tk::qnn_lookup_impl(data, out, table, tk::as_stream(stream));
}
int tk_qnn_conv2d_transpose(const tk_tensor* data, const tk_tensor* weight, tk_tensor* out,
                            const tk_conv2d_transpose_attrs* attrs, void* stream) {
  return tk::qnn_conv2d_transpose_impl(data, weight, out, attrs, tk::as_stream(stream));
}
int tk_qnn_simulated_quantize(const tk_tensor* data, tk_tensor* out, const tk_simq_attrs* attrs, void* stream) {
  return tk::qnn_simulated_impl(true, data, out, attrs, tk::as_stream(stream));
}
int tk_qnn_simulated_dequantize(const tk_tensor* data, tk_tensor* out, const tk_simq_attrs* attrs, void* stream) {
  return tk::qnn_simulated_impl(false, data, out, attrs, tk::as_stream(stream));
}
int tk_requantize_fp(const tk_tensor* data, tk_tensor* out, const tk_requantize_fp_attrs* attrs, void* stream) {
  return tk::requantize_fp_impl(data, out, attrs, tk::as_stream(stream));
}
int tk_qnn_binary_fp(const tk_tensor* lhs, const tk_tensor* rhs, tk_tensor* out, const tk_qnn_binary_fp_attrs* attrs,
                     void* stream) {
  return tk::qnn_binary_fp_impl(lhs, rhs, out, attrs, tk::as_stream(stream));
}

}  // extern "C"
