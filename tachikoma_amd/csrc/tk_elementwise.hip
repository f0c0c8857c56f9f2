// Wavefront-level integer elementwise / pooling kernels for gfx950.
//
// All of these are HBM-bound streaming kernels: 16-byte vector loads per lane
// where the element type allows, grid-stride loops sized to ~8 workgroups per CU.
// Semantics follow the canonicalised Relay ops the reference runs on the CPU
// (SURVEY.md Appendix A); every function cites the reference lowering it mirrors.
#include <algorithm>
#include <climits>

#include "tk_common.h"

namespace tk {

// float32 variants of the shared ops (relay.quantize-realized graphs, tk_realize.hip)
int cast_f32_impl(const tk_tensor* x, tk_tensor* y, hipStream_t s);
int bias_add_f32_impl(const tk_tensor* x, const tk_tensor* b, tk_tensor* y, int axis, hipStream_t s);
int global_avg_pool_f32_impl(const tk_tensor* x, tk_tensor* y, hipStream_t s);
int max_pool_f32_impl(const tk_tensor* x, tk_tensor* y, const tk_pool2d_attrs* a, hipStream_t s);

constexpr int kBlock = 256;

static inline int grid_for(int64_t work_items) {
  int64_t g = (work_items + kBlock - 1) / kBlock;
  if (g < 1) g = 1;
  if (g > 256 * 8) g = 256 * 8;
  return (int)g;
}

template <int D> struct DTT;
template <> struct DTT<DT_I8> { using T = int8_t; };
template <> struct DTT<DT_U8> { using T = uint8_t; };
template <> struct DTT<DT_I16> { using T = int16_t; };
template <> struct DTT<DT_U16> { using T = uint16_t; };
template <> struct DTT<DT_I32> { using T = int32_t; };
template <> struct DTT<DT_U32> { using T = uint32_t; };
template <> struct DTT<DT_I64> { using T = int64_t; };
template <> struct DTT<DT_U64> { using T = uint64_t; };

template <typename T> __device__ __forceinline__ int64_t tmin() { return (int64_t)std::numeric_limits<T>::min(); }
template <typename T> __device__ __forceinline__ int64_t tmax() { return (int64_t)std::numeric_limits<T>::max(); }

// dispatch helper: calls f(DTT<D>{}) for the runtime dtype id (generic lambdas)
template <typename F> static int dispatch_int(int dt, F&& f) {
  switch (dt) {
    case DT_I8: return f(DTT<DT_I8>{});
    case DT_U8: return f(DTT<DT_U8>{});
    case DT_I16: return f(DTT<DT_I16>{});
    case DT_U16: return f(DTT<DT_U16>{});
    case DT_I32: return f(DTT<DT_I32>{});
    case DT_U32: return f(DTT<DT_U32>{});
    case DT_I64: return f(DTT<DT_I64>{});
    case DT_U64: return f(DTT<DT_U64>{});
  }
  set_error("unsupported integer dtype");
  return TK_ERR_DTYPE;
}

// Position along a broadcast axis: element i sits in channel (i / inner) % C.
struct AxisWalker {
  int32_t inner, C;
  int64_t q;
  int32_t r, c;
  __device__ __forceinline__ void seek(int64_t i) {
    q = i / inner;
    r = (int32_t)(i - q * inner);
    c = (int32_t)(q % C);
  }
  __device__ __forceinline__ void next() {
    if (++r == inner) {
      r = 0;
      if (++c == C) c = 0;
    }
  }
};

// ---------------------------------------------------------------- requantize
// (RqParams / rq_apply live in tk_common.h: the fused conv epilogue uses them too)

template <typename Tin, typename Tout, int VEC>
__global__ __launch_bounds__(kBlock) void requantize_kernel(const Tin* __restrict__ x, Tout* __restrict__ y,
                                                            int64_t n, RqParams p) {
  int64_t nvec = n / VEC;
  int64_t stride = (int64_t)gridDim.x * kBlock;
  AxisWalker w{p.inner, p.C};
  for (int64_t v = blockIdx.x * (int64_t)kBlock + threadIdx.x; v < nvec; v += stride) {
    Tin in[VEC];
    Tout out[VEC];
    __builtin_memcpy(in, x + v * VEC, sizeof(in));
    w.seek(v * VEC);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      int32_t t = rq_apply((int32_t)in[j], w.c, p);
      if (p.clip_out) t = (int32_t)min(max((int64_t)t, p.qmin), p.qmax);
      out[j] = (Tout)t;
      w.next();
    }
    __builtin_memcpy(y + v * VEC, out, sizeof(out));
  }
  // tail
  int64_t tail0 = nvec * VEC;
  for (int64_t i = tail0 + blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += stride) {
    w.seek(i);
    int32_t t = rq_apply((int32_t)x[i], w.c, p);
    if (p.clip_out) t = (int32_t)min(max((int64_t)t, p.qmin), p.qmax);
    y[i] = (Tout)t;
  }
}

static int axis_geometry(const tk_tensor* t, int axis, int32_t* inner, int32_t* C) {
  if (t->ndim == 0) {
    *inner = 1;
    *C = 1;
    return TK_OK;
  }
  int ax = axis < 0 ? t->ndim + axis : axis;
  if (ax < 0 || ax >= t->ndim) return TK_ERR_INVALID_ARG;
  int64_t in = 1;
  for (int i = ax + 1; i < t->ndim; ++i) in *= t->shape[i];
  if (in > INT32_MAX) return TK_ERR_UNSUPPORTED;
  *inner = (int32_t)in;
  *C = (int32_t)t->shape[ax];
  return TK_OK;
}

template <typename Tin, typename Tout>
static int launch_requantize(const tk_tensor* x, tk_tensor* y, const RqParams& p, hipStream_t s) {
  int64_t n = numel(x);
  constexpr int VEC = 16 / sizeof(Tin) > 0 ? (int)(16 / sizeof(Tin)) : 1;
  int64_t items = n / VEC + 1;
  hipLaunchKernelGGL((requantize_kernel<Tin, Tout, VEC>), dim3(grid_for(items)), dim3(kBlock), 0, s,
                     (const Tin*)ptr(x), (Tout*)ptr(y), n, p);
  TK_LAUNCH_CHECK();
  return TK_OK;
}

int requantize_impl(const tk_tensor* x, tk_tensor* y, const tk_requantize_attrs* a, hipStream_t s) {
  TK_CHECK_ARG(x && y && a, "null argument");
  TK_CHECK_ARG(compact(x) && compact(y), "strided tensors are not supported");
  TK_CHECK_ARG(numel(x) == numel(y), "shape mismatch");
  TK_CHECK_ARG(is_integer(x) && is_integer(y), "integer tensors required");
  RqParams p{};
  p.mode = a->mode;
  p.multiplier = a->multiplier;
  p.shift = a->shift;
  p.zp_in = a->input_zero_point;
  p.zp_out = a->output_zero_point;
  p.ms = a->multipliers;
  p.ss = a->shifts;
  p.zps = a->input_zero_points;
  if (axis_geometry(x, a->axis, &p.inner, &p.C) != TK_OK) {
    set_error("tk_requantize: bad axis");
    return TK_ERR_INVALID_ARG;
  }
  if ((p.mode == TK_RQ_AXIS_UPWARD || p.mode == TK_RQ_AXIS_TONEAREST) && (!p.ms || !p.ss)) {
    set_error("tk_requantize: per-axis mode needs device multipliers/shifts");
    return TK_ERR_INVALID_ARG;
  }
  int dti = dt_of(x), dto = dt_of(y);
  p.clip_out = !(dto == DT_I32);
  switch (dto) {
    case DT_I8: p.qmin = -128; p.qmax = 127; break;
    case DT_U8: p.qmin = 0; p.qmax = 255; break;
    case DT_I16: p.qmin = -32768; p.qmax = 32767; break;
    case DT_U16: p.qmin = 0; p.qmax = 65535; break;
    case DT_I32: p.qmin = INT32_MIN; p.qmax = INT32_MAX; break;
    default: set_error("tk_requantize: unsupported out dtype"); return TK_ERR_DTYPE;
  }
#define RQ_OUT(TI)                                                   \
  switch (dto) {                                                     \
    case DT_I8: return launch_requantize<TI, int8_t>(x, y, p, s);    \
    case DT_U8: return launch_requantize<TI, uint8_t>(x, y, p, s);   \
    case DT_I16: return launch_requantize<TI, int16_t>(x, y, p, s);  \
    case DT_U16: return launch_requantize<TI, uint16_t>(x, y, p, s); \
    case DT_I32: return launch_requantize<TI, int32_t>(x, y, p, s);  \
  }
  switch (dti) {
    case DT_I8: RQ_OUT(int8_t); break;
    case DT_U8: RQ_OUT(uint8_t); break;
    case DT_I16: RQ_OUT(int16_t); break;
    case DT_U16: RQ_OUT(uint16_t); break;
    case DT_I32: RQ_OUT(int32_t); break;
  }
#undef RQ_OUT
  set_error("tk_requantize: unsupported dtype combination");
  return TK_ERR_DTYPE;
}

// ---------------------------------------------------------------- bias_add
// nn.bias_add / broadcast add of a vector along `axis` (int32 wraps like LLVM add).
template <typename T, int VEC>
__global__ __launch_bounds__(kBlock) void bias_add_kernel(const T* __restrict__ x, const T* __restrict__ b,
                                                          T* __restrict__ y, int64_t n, int32_t inner, int32_t C) {
  int64_t nvec = n / VEC;
  int64_t stride = (int64_t)gridDim.x * kBlock;
  AxisWalker w{inner, C};
  for (int64_t v = blockIdx.x * (int64_t)kBlock + threadIdx.x; v < nvec; v += stride) {
    T in[VEC], out[VEC];
    __builtin_memcpy(in, x + v * VEC, sizeof(in));
    w.seek(v * VEC);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      using U = typename std::make_unsigned<T>::type;
      out[j] = (T)((U)in[j] + (U)b[w.c]);
      w.next();
    }
    __builtin_memcpy(y + v * VEC, out, sizeof(out));
  }
  for (int64_t i = nvec * VEC + blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += stride) {
    w.seek(i);
    using U = typename std::make_unsigned<T>::type;
    y[i] = (T)((U)x[i] + (U)b[w.c]);
  }
}

int bias_add_impl(const tk_tensor* x, const tk_tensor* b, tk_tensor* y, int axis, hipStream_t s) {
  TK_CHECK_ARG(x && b && y, "null argument");
  if (is_f32(x)) return bias_add_f32_impl(x, b, y, axis, s);
  TK_CHECK_ARG(compact(x) && compact(y) && compact(b), "strided tensors are not supported");
  TK_CHECK_ARG(dt_of(x) == dt_of(b) && dt_of(x) == dt_of(y), "dtype mismatch");
  TK_CHECK_ARG(numel(x) == numel(y), "shape mismatch");
  int32_t inner, C;
  if (axis_geometry(x, axis, &inner, &C) != TK_OK || numel(b) != C) {
    set_error("tk_bias_add: bias length does not match the axis");
    return TK_ERR_SHAPE;
  }
  int64_t n = numel(x);
  return dispatch_int(dt_of(x), [&](auto tag) -> int {
    using T = typename decltype(tag)::T;
    constexpr int VEC = 16 / sizeof(T);
    hipLaunchKernelGGL((bias_add_kernel<T, VEC>), dim3(grid_for(n / VEC + 1)), dim3(kBlock), 0, s,
                       (const T*)ptr(x), (const T*)ptr(b), (T*)ptr(y), n, inner, C);
    TK_LAUNCH_CHECK();
    return TK_OK;
  });
}

// ---------------------------------------------------------------- clip
template <typename T, int VEC>
__global__ __launch_bounds__(kBlock) void clip_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n, T lo,
                                                      T hi) {
  int64_t nvec = n / VEC;
  int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t v = blockIdx.x * (int64_t)kBlock + threadIdx.x; v < nvec; v += stride) {
    T in[VEC];
    __builtin_memcpy(in, x + v * VEC, sizeof(in));
#pragma unroll
    for (int j = 0; j < VEC; ++j) in[j] = max(min(in[j], hi), lo);
    __builtin_memcpy(y + v * VEC, in, sizeof(in));
  }
  for (int64_t i = nvec * VEC + blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += stride)
    y[i] = max(min(x[i], hi), lo);
}

int clip_impl(const tk_tensor* x, tk_tensor* y, int64_t lo, int64_t hi, hipStream_t s) {
  TK_CHECK_ARG(x && y, "null argument");
  TK_CHECK_ARG(compact(x) && compact(y) && dt_of(x) == dt_of(y) && numel(x) == numel(y), "bad tensors");
  int64_t n = numel(x);
  return dispatch_int(dt_of(x), [&](auto tag) -> int {
    using T = typename decltype(tag)::T;
    constexpr int VEC = 16 / sizeof(T);
    hipLaunchKernelGGL((clip_kernel<T, VEC>), dim3(grid_for(n / VEC + 1)), dim3(kBlock), 0, s, (const T*)ptr(x),
                       (T*)ptr(y), n, (T)lo, (T)hi);
    TK_LAUNCH_CHECK();
    return TK_OK;
  });
}

// ---------------------------------------------------------------- cast
template <typename Ti, typename To>
__global__ __launch_bounds__(kBlock) void cast_kernel(const Ti* __restrict__ x, To* __restrict__ y, int64_t n) {
  int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += stride) y[i] = (To)x[i];
}

int cast_impl(const tk_tensor* x, tk_tensor* y, hipStream_t s) {
  TK_CHECK_ARG(x && y && compact(x) && compact(y) && numel(x) == numel(y), "bad tensors");
  if (is_f32(x) || is_f32(y)) return cast_f32_impl(x, y, s);
  TK_CHECK_ARG(is_integer(x) && is_integer(y), "integer or float32 casts only");
  int64_t n = numel(x);
  return dispatch_int(dt_of(x), [&](auto ti) -> int {
    return dispatch_int(dt_of(y), [&](auto to) -> int {
      using Ti = typename decltype(ti)::T;
      using To = typename decltype(to)::T;
      hipLaunchKernelGGL((cast_kernel<Ti, To>), dim3(grid_for(n)), dim3(kBlock), 0, s, (const Ti*)ptr(x),
                         (To*)ptr(y), n);
      TK_LAUNCH_CHECK();
      return TK_OK;
    });
  });
}

// ---------------------------------------------------------------- qnn.add
// QnnAddCanonicalize (src/relay/qnn/op/add.cc:40-96): a' = RQ(a) or int32(a), b' likewise,
// o = a' + b' - zp_c (int32), clip to the input dtype, cast.
template <typename T>
__global__ __launch_bounds__(kBlock) void qnn_add_kernel(const T* __restrict__ a, const T* __restrict__ b,
                                                         T* __restrict__ y, int64_t n, RqParams pa, RqParams pb,
                                                         int32_t zp_c, int32_t up_a, int32_t up_b) {
  int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += stride) {
    int32_t x0 = (int32_t)a[i], x1 = (int32_t)b[i];
    int32_t ra = up_a ? x0 : rq_apply(x0, 0, pa);
    int32_t rb = up_b ? x1 : rq_apply(x1, 0, pb);
    int32_t o = (int32_t)((uint32_t)ra + (uint32_t)rb);
    o = (int32_t)((uint32_t)o - (uint32_t)zp_c);
    int64_t c = min(max((int64_t)o, tmin<T>()), tmax<T>());
    y[i] = (T)c;
  }
}

static RqParams rq_from_attrs(const tk_requantize_attrs& a) {
  RqParams p{};
  p.mode = a.mode;
  p.multiplier = a.multiplier;
  p.shift = a.shift;
  p.zp_in = a.input_zero_point;
  p.zp_out = a.output_zero_point;
  p.inner = 1;
  p.C = 1;
  return p;
}

int qnn_add_impl(const tk_tensor* a, const tk_tensor* b, tk_tensor* y, const tk_qnn_add_attrs* at, hipStream_t s) {
  TK_CHECK_ARG(a && b && y && at, "null argument");
  TK_CHECK_ARG(numel(a) == numel(b) && numel(a) == numel(y), "qnn.add: only same-shape operands are supported");
  TK_CHECK_ARG(dt_of(a) == dt_of(b) && dt_of(a) == dt_of(y), "dtype mismatch");
  TK_CHECK_ARG(at->lhs.mode <= TK_RQ_TENSOR_TONEAREST && at->rhs.mode <= TK_RQ_TENSOR_TONEAREST,
               "qnn.add: per-tensor parameters only");
  int64_t n = numel(a);
  RqParams pa = rq_from_attrs(at->lhs), pb = rq_from_attrs(at->rhs);
  return dispatch_int(dt_of(a), [&](auto tag) -> int {
    using T = typename decltype(tag)::T;
    hipLaunchKernelGGL((qnn_add_kernel<T>), dim3(grid_for(n)), dim3(kBlock), 0, s, (const T*)ptr(a), (const T*)ptr(b),
                       (T*)ptr(y), n, pa, pb, at->output_zero_point, at->lhs_upcast, at->rhs_upcast);
    TK_LAUNCH_CHECK();
    return TK_OK;
  });
}

// ---------------------------------------------------------------- pooling (NCHW)
struct PoolGeom {
  int32_t N, C, H, W, OH, OW, kh, kw, sh, sw, pt, pl, pb, pr, dh, dw, include_pad;
};

// nn.max_pool2d: padded taps are the dtype minimum (include/tvm/topi/nn/pooling.h:123).
template <typename T>
__global__ __launch_bounds__(kBlock) void max_pool_kernel(const T* __restrict__ x, T* __restrict__ y, PoolGeom g) {
  int64_t n = (int64_t)g.N * g.C * g.OH * g.OW;
  int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += stride) {
    int ow = (int)(i % g.OW);
    int64_t t = i / g.OW;
    int oh = (int)(t % g.OH);
    int64_t nc = t / g.OH;
    const T* plane = x + nc * (int64_t)g.H * g.W;
    T m = (T)tmin<T>();
    for (int r = 0; r < g.kh; ++r) {
      int ih = oh * g.sh - g.pt + r * g.dh;
      if (ih < 0 || ih >= g.H) continue;
      for (int c = 0; c < g.kw; ++c) {
        int iw = ow * g.sw - g.pl + c * g.dw;
        if (iw < 0 || iw >= g.W) continue;
        T v = plane[ih * g.W + iw];
        m = v > m ? v : m;
      }
    }
    y[i] = m;
  }
}

__device__ __forceinline__ int64_t truncdiv64(int64_t a, int64_t b) { return a / b; }  // C++ '/' truncates

// nn.avg_pool2d on integers: window sum in the input dtype (wraps), truncdiv by the count
// (include/tvm/topi/nn/pooling.h:560-650).
template <typename T>
__global__ __launch_bounds__(kBlock) void avg_pool_kernel(const T* __restrict__ x, T* __restrict__ y, PoolGeom g) {
  int64_t n = (int64_t)g.N * g.C * g.OH * g.OW;
  int64_t stride = (int64_t)gridDim.x * kBlock;
  using U = typename std::make_unsigned<T>::type;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += stride) {
    int ow = (int)(i % g.OW);
    int64_t t = i / g.OW;
    int oh = (int)(t % g.OH);
    int64_t nc = t / g.OH;
    const T* plane = x + nc * (int64_t)g.H * g.W;
    U sum = 0;
    for (int r = 0; r < g.kh; ++r) {
      int ih = oh * g.sh - g.pt + r * g.dh;
      if (ih < 0 || ih >= g.H) continue;
      for (int c = 0; c < g.kw; ++c) {
        int iw = ow * g.sw - g.pl + c * g.dw;
        if (iw < 0 || iw >= g.W) continue;
        sum = (U)(sum + (U)plane[ih * g.W + iw]);
      }
    }
    int64_t cnt = 1;
    int dims[2][6] = {{oh, g.sh, g.kh, g.dh, g.H, g.pt}, {ow, g.sw, g.kw, g.dw, g.W, g.pl}};
    int tails[2] = {g.pb, g.pr};
    for (int d = 0; d < 2; ++d) {
      int o = dims[d][0], st = dims[d][1], k = dims[d][2], dl = dims[d][3], dim = dims[d][4], ph = dims[d][5];
      int start = o * st - ph;
      int end = start + (k - 1) * dl;
      if (g.include_pad) {
        end = min(end, dim + tails[d] - 1);
        cnt *= (end - start) / dl + 1;
      } else {
        int jumps = (dl - 1 - start) / dl;
        jumps = max(jumps, 0);
        end = min(end, dim - 1);
        cnt *= (end - (start + dl * jumps)) / dl + 1;
      }
    }
    if (!g.include_pad) cnt = max(cnt, (int64_t)1);
    int64_t sv = (int64_t)(T)sum;
    y[i] = (T)truncdiv64(sv, (int64_t)(T)cnt);
  }
}

// global_avg_pool2d: one wave per (n, c) plane (adaptive pool 1x1, pooling.h:366-389).
template <typename T>
__global__ __launch_bounds__(kBlock) void global_avg_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                            int64_t planes, int32_t hw) {
  using U = typename std::make_unsigned<T>::type;
  int lane = threadIdx.x & 63;
  int64_t wave = (blockIdx.x * (int64_t)kBlock + threadIdx.x) >> 6;
  int64_t nwaves = ((int64_t)gridDim.x * kBlock) >> 6;
  for (int64_t p = wave; p < planes; p += nwaves) {
    const T* plane = x + p * hw;
    U s = 0;
    for (int i = lane; i < hw; i += 64) s = (U)(s + (U)plane[i]);
    for (int off = 32; off > 0; off >>= 1) s = (U)(s + (U)__shfl_xor(s, off));
    if (lane == 0) {
      int64_t sv = (int64_t)(T)s;
      y[p] = (T)truncdiv64(sv, (int64_t)(T)hw);
    }
  }
}

static int pool_geom(const tk_tensor* x, const tk_tensor* y, const tk_pool2d_attrs* a, PoolGeom* g) {
  if (x->ndim != 4 || y->ndim != 4) return TK_ERR_SHAPE;
  g->N = (int32_t)x->shape[0];
  g->C = (int32_t)x->shape[1];
  g->H = (int32_t)x->shape[2];
  g->W = (int32_t)x->shape[3];
  g->kh = a->pool_size[0]; g->kw = a->pool_size[1];
  g->sh = a->strides[0]; g->sw = a->strides[1];
  g->pt = a->padding[0]; g->pl = a->padding[1]; g->pb = a->padding[2]; g->pr = a->padding[3];
  g->dh = a->dilation[0] ? a->dilation[0] : 1; g->dw = a->dilation[1] ? a->dilation[1] : 1;
  g->include_pad = a->count_include_pad;
  g->OH = (g->H + g->pt + g->pb - g->dh * (g->kh - 1) - 1) / g->sh + 1;
  g->OW = (g->W + g->pl + g->pr - g->dw * (g->kw - 1) - 1) / g->sw + 1;
  if (y->shape[0] != g->N || y->shape[1] != g->C || y->shape[2] != g->OH || y->shape[3] != g->OW) return TK_ERR_SHAPE;
  return TK_OK;
}

int max_pool_impl(const tk_tensor* x, tk_tensor* y, const tk_pool2d_attrs* a, hipStream_t s) {
  TK_CHECK_ARG(x && y && a, "bad arguments");
  if (is_f32(x)) return max_pool_f32_impl(x, y, a, s);
  TK_CHECK_ARG(dt_of(x) == dt_of(y), "bad arguments");
  PoolGeom g;
  if (pool_geom(x, y, a, &g)) { set_error("tk_max_pool2d: shape mismatch"); return TK_ERR_SHAPE; }
  int64_t n = (int64_t)g.N * g.C * g.OH * g.OW;
  return dispatch_int(dt_of(x), [&](auto tag) -> int {
    using T = typename decltype(tag)::T;
    hipLaunchKernelGGL((max_pool_kernel<T>), dim3(grid_for(n)), dim3(kBlock), 0, s, (const T*)ptr(x), (T*)ptr(y), g);
    TK_LAUNCH_CHECK();
    return TK_OK;
  });
}

// nn.max_pool2d of an 8-bit tensor read from its conv shadow ([C/16][N*H*W][16], uint8
// stored xor 0x80, so signed byte order = value order): one thread per (16 channels,
// output pixel) with lanes along the output row, 16-byte tap loads, the record written
// NCHW and, for a following MFMA conv, the output shadow written directly.
__global__ __launch_bounds__(kBlock) void max_pool_shadow_kernel(const uint8_t* __restrict__ sin, uint8_t* __restrict__ y,
                                                                 uint8_t* __restrict__ sout, PoolGeom g, int G,
                                                                 uint32_t xr) {
  const int64_t pin = (int64_t)g.N * g.H * g.W, pout = (int64_t)g.N * g.OH * g.OW;
  const int64_t total = (int64_t)G * pout;
  for (int64_t t = blockIdx.x * (int64_t)kBlock + threadIdx.x; t < total; t += (int64_t)gridDim.x * kBlock) {
    const int64_t q = t % pout;  // output pixel (n, oh, ow)
    const int grp = (int)(t / pout);
    const int ow = (int)(q % g.OW);
    const int64_t r = q / g.OW;
    const int oh = (int)(r % g.OH);
    const int n = (int)(r / g.OH);
    int8_t m[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) m[j] = -128;
    for (int kh = 0; kh < g.kh; ++kh) {
      const int ih = oh * g.sh - g.pt + kh * g.dh;
      if (ih < 0 || ih >= g.H) continue;
      for (int kw = 0; kw < g.kw; ++kw) {
        const int iw = ow * g.sw - g.pl + kw * g.dw;
        if (iw < 0 || iw >= g.W) continue;
        int8_t v[16];
        __builtin_memcpy(v, sin + ((int64_t)grp * pin + ((int64_t)n * g.H + ih) * g.W + iw) * 16, 16);
#pragma unroll
        for (int j = 0; j < 16; ++j) m[j] = v[j] > m[j] ? v[j] : m[j];
      }
    }
    const int cvalid = g.C - grp * 16;
    uint8_t sh[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      sh[j] = j < cvalid ? (uint8_t)m[j] : 0;  // padded channels of the shadow stay 0
      if (j < cvalid)
        y[(((int64_t)n * g.C + grp * 16 + j) * g.OH + oh) * g.OW + ow] = (uint8_t)((uint8_t)m[j] ^ (uint8_t)xr);
    }
    if (sout) __builtin_memcpy(sout + ((int64_t)grp * pout + q) * 16, sh, 16);
  }
}

int max_pool_shadow_impl(const tk_tensor* x, const void* x_shadow, tk_tensor* y, const tk_pool2d_attrs* a,
                         void* y_shadow, hipStream_t s) {
  TK_CHECK_ARG(x && y && a && x_shadow && dt_of(x) == dt_of(y) && is_int8ish(x), "bad arguments");
  PoolGeom g;
  if (pool_geom(x, y, a, &g)) { set_error("tk_max_pool2d_shadow: shape mismatch"); return TK_ERR_SHAPE; }
  const int G = (g.C + 15) / 16;
  const int64_t units = (int64_t)G * g.N * g.OH * g.OW;
  hipLaunchKernelGGL(max_pool_shadow_kernel, dim3(grid_for(units)), dim3(kBlock), 0, s, (const uint8_t*)x_shadow,
                     (uint8_t*)ptr(y), (uint8_t*)y_shadow, g, G, is_uint(x, 8) ? 0x80u : 0u);
  TK_LAUNCH_CHECK();
  return TK_OK;
}

int avg_pool_impl(const tk_tensor* x, tk_tensor* y, const tk_pool2d_attrs* a, hipStream_t s) {
  TK_CHECK_ARG(x && y && a && dt_of(x) == dt_of(y), "bad arguments");
  PoolGeom g;
  if (pool_geom(x, y, a, &g)) { set_error("tk_avg_pool2d: shape mismatch"); return TK_ERR_SHAPE; }
  int64_t n = (int64_t)g.N * g.C * g.OH * g.OW;
  return dispatch_int(dt_of(x), [&](auto tag) -> int {
    using T = typename decltype(tag)::T;
    hipLaunchKernelGGL((avg_pool_kernel<T>), dim3(grid_for(n)), dim3(kBlock), 0, s, (const T*)ptr(x), (T*)ptr(y), g);
    TK_LAUNCH_CHECK();
    return TK_OK;
  });
}

int global_avg_pool_impl(const tk_tensor* x, tk_tensor* y, hipStream_t s) {
  TK_CHECK_ARG(x && y && x->ndim == 4 && y->ndim == 4, "bad arguments");
  if (is_f32(x)) return global_avg_pool_f32_impl(x, y, s);
  TK_CHECK_ARG(dt_of(x) == dt_of(y), "bad arguments");
  TK_CHECK_ARG(y->shape[0] == x->shape[0] && y->shape[1] == x->shape[1] && y->shape[2] == 1 && y->shape[3] == 1,
               "output must be [N,C,1,1]");
  int64_t planes = x->shape[0] * x->shape[1];
  int32_t hw = (int32_t)(x->shape[2] * x->shape[3]);
  return dispatch_int(dt_of(x), [&](auto tag) -> int {
    using T = typename decltype(tag)::T;
    hipLaunchKernelGGL((global_avg_kernel<T>), dim3(grid_for(planes * 64)), dim3(kBlock), 0, s, (const T*)ptr(x),
                       (T*)ptr(y), planes, hw);
    TK_LAUNCH_CHECK();
    return TK_OK;
  });
}

int copy_impl(const tk_tensor* x, tk_tensor* y, hipStream_t s) {
  TK_CHECK_ARG(x && y && nbytes(x) == nbytes(y), "size mismatch");
  TK_HIP(hipMemcpyAsync(ptr(y), ptr(x), nbytes(x), hipMemcpyDeviceToDevice, s));
  return TK_OK;
}

// ---------------------------------------------------------------- records to host memory
// One launch copies up to kHostCopyMax device buffers into pinned host memory (a node's trace
// records; tk_module_run_graph's copies).  Host destinations are 8-byte aligned (NDArray-list
// payloads); each buffer is copied as an 8-byte head (to reach 16-byte destination alignment),
// 16-byte nontemporal stores from two 8-byte loads, and a byte tail.  64-128 workgroups of such a
// kernel write pinned memory at ~55 GB/s (profiles/r03b_probe_d2h.jsonl, kernel_wg128), about the
// SDMA engines' rate, and as a graph kernel node it needs no per-copy host call.
constexpr int kHostCopyMax = 6;
struct HostCopies {
  const uint8_t* src[kHostCopyMax];
  uint8_t* dst[kHostCopyMax];
  int64_t bytes[kHostCopyMax];
  int n;
};

__global__ __launch_bounds__(256) void host_copy_kernel(HostCopies c) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (int b = 0; b < c.n; ++b) {
    const uint8_t* src = c.src[b];
    uint8_t* dst = c.dst[b];
    int64_t n = c.bytes[b];
    const int64_t head = (int64_t)((16 - ((uintptr_t)dst & 15)) & 15) < n ? (int64_t)((16 - ((uintptr_t)dst & 15)) & 15) : n;
    for (int64_t i = t; i < head; i += stride) dst[i] = src[i];
    const int64_t n16 = (n - head) / 16;
    const uint64_t* s8 = reinterpret_cast<const uint64_t*>(src + head);
    tk_v4i* d16 = reinterpret_cast<tk_v4i*>(dst + head);
    if (((uintptr_t)(src + head) & 7) == 0) {
      for (int64_t i = t; i < n16; i += stride) {
        const uint64_t a = __builtin_nontemporal_load(s8 + 2 * i), bb = __builtin_nontemporal_load(s8 + 2 * i + 1);
        __builtin_nontemporal_store(tk_v4i{(int)(uint32_t)a, (int)(uint32_t)(a >> 32), (int)(uint32_t)bb, (int)(uint32_t)(bb >> 32)},
                                    d16 + i);
      }
    } else {
      for (int64_t i = t; i < n16 * 16; i += stride) dst[head + i] = src[head + i];
    }
    for (int64_t i = head + n16 * 16 + t; i < n; i += stride) dst[i] = src[i];
  }
}

int host_copy_impl(const void* const* src, void* const* dst, const int64_t* bytes, int n, hipStream_t s) {
  TK_CHECK_ARG(n >= 0 && n <= kHostCopyMax, "host copy: too many buffers");
  HostCopies c{};
  int64_t total = 0;
  int k = 0;
  for (int i = 0; i < n; ++i) {
    if (!dst[i] || bytes[i] <= 0) continue;
    c.src[k] = (const uint8_t*)src[i];
    c.dst[k] = (uint8_t*)dst[i];
    c.bytes[k] = bytes[i];
    total += bytes[i];
    ++k;
  }
  c.n = k;
  if (!k) return TK_OK;
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(128, (total / 16 + 255) / 256));
  hipLaunchKernelGGL(host_copy_kernel, dim3(grid), dim3(256), 0, s, c);
  TK_LAUNCH_CHECK();
  return TK_OK;
}

// ---------------------------------------------------------------- trace image pack
// Packed trace capture (tk_module_run_graph's default): a chunk's records are gathered from their
// own device buffers into a device mirror of the trace image's records section, at their final
// (NDArray-list, any-alignment) offsets, so that the chunk leaves for host memory as ONE contiguous
// SDMA copy (host-issued copies of whole chunks run at 57.0 GB/s, per-record copies at 56.0 and
// graph memcpy nodes at 54.0-54.6, profiles/r04c_copyprobe.jsonl).  One thread writes one 16-byte
// aligned chunk of the mirror: whole chunks from two aligned 16-byte source loads and a funnel
// shift, partial chunks (next to a header) byte by byte, header bytes left as they are.  Record
// buffers must be 16-byte aligned and readable in whole 16-byte chunks (torch allocations are).
struct PackRec {
  const uint8_t* src;
  int64_t dst;        // offset in the mirror
  int64_t bytes;
  int64_t first_blk;  // first workgroup of this record in the launch
};

__device__ __forceinline__ uint32_t funnel(uint32_t lo, uint32_t hi, uint32_t r) {
  return r ? __builtin_amdgcn_alignbyte(hi, lo, r) : lo;
}

__global__ __launch_bounds__(256) void pack_records_kernel(const PackRec* __restrict__ recs, int nrec,
                                                           uint8_t* __restrict__ mirror) {
  int lo = 0, hi = nrec - 1;
  const int64_t b = blockIdx.x;
  while (lo < hi) {  // the record whose workgroups include b
    const int mid = (lo + hi + 1) >> 1;
    if (recs[mid].first_blk <= b) lo = mid;
    else hi = mid - 1;
  }
  const PackRec r = recs[lo];
  const int64_t a0 = r.dst & ~(int64_t)15;  // first 16-byte chunk touching the payload
  const int64_t a = a0 + ((b - r.first_blk) * 256 + threadIdx.x) * 16;
  const int64_t end = r.dst + r.bytes;
  if (a >= end) return;
  if (a >= r.dst && a + 16 <= end) {
    const int64_t so = a - r.dst;  // source offset of the chunk's first byte
    const int64_t base = so & ~(int64_t)15;
    const uint32_t s = (uint32_t)(so - base);
    tk_v4i v0 = __builtin_nontemporal_load(reinterpret_cast<const tk_v4i*>(r.src + base));
    tk_v4i out;
    if (s == 0) {
      out = v0;
    } else {
      tk_v4i v1 = __builtin_nontemporal_load(reinterpret_cast<const tk_v4i*>(r.src + base + 16));
      const uint32_t w[8] = {(uint32_t)v0.x, (uint32_t)v0.y, (uint32_t)v0.z, (uint32_t)v0.w,
                             (uint32_t)v1.x, (uint32_t)v1.y, (uint32_t)v1.z, (uint32_t)v1.w};
      const uint32_t q = s >> 2, rb = s & 3;
      uint32_t o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        // w[k + q] / w[k + q + 1] through selects (no dynamic register indexing)
        const uint32_t x0 = q == 0 ? w[k] : q == 1 ? w[k + 1] : q == 2 ? w[k + 2] : w[k + 3];
        const uint32_t x1 = q == 0 ? w[k + 1] : q == 1 ? w[k + 2] : q == 2 ? w[k + 3] : w[k + 4];
        o[k] = funnel(x0, x1, rb);
      }
      out = tk_v4i{(int)o[0], (int)o[1], (int)o[2], (int)o[3]};
    }
    *reinterpret_cast<tk_v4i*>(mirror + a) = out;
  } else {
    const int64_t from = a > r.dst ? a : r.dst;
    const int64_t to = a + 16 < end ? a + 16 : end;
    for (int64_t i = from; i < to; ++i) mirror[i] = r.src[i - r.dst];
  }
}

int pack_records_impl(const void* table, int nrec, int64_t blocks, void* mirror, hipStream_t s) {
  TK_CHECK_ARG(table && mirror && nrec > 0 && blocks > 0, "bad arguments");
  hipLaunchKernelGGL(pack_records_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const PackRec*)table, nrec,
                     (uint8_t*)mirror);
  TK_LAUNCH_CHECK();
  return TK_OK;
}

// ---------------------------------------------------------------- nn.pad
// One thread per output element (its index decomposed over up to 6 dimensions, innermost first):
// inside the data's range it copies data[i - before], else writes the pad value.
struct PadGeom {
  int32_t ndim;
  int64_t out_shape[6], in_shape[6], before[6];
};

template <typename T>
__global__ __launch_bounds__(kBlock) void pad_kernel(const T* __restrict__ x, T* __restrict__ y, int64_t n, PadGeom g,
                                                     T value) {
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += stride) {
    int64_t r = i, src = 0, pitch = 1;
    bool inside = true;
    for (int d = g.ndim - 1; d >= 0; --d) {
      const int64_t c = r % g.out_shape[d] - g.before[d];
      r /= g.out_shape[d];
      inside = inside && c >= 0 && c < g.in_shape[d];
      src += c * pitch;
      pitch *= g.in_shape[d];
    }
    y[i] = inside ? x[src] : value;
  }
}

int pad_impl(const tk_tensor* x, tk_tensor* y, const tk_pad_attrs* a, hipStream_t s) {
  TK_CHECK_ARG(x && y && a && compact(x) && compact(y), "bad arguments");
  TK_CHECK_ARG(x->ndim == y->ndim && x->ndim >= 1 && x->ndim <= 6 && x->dtype.code == y->dtype.code &&
                   x->dtype.bits == y->dtype.bits && x->dtype.lanes == 1,
               "pad: same dtype, 1-6 dimensions");
  PadGeom g{};
  g.ndim = x->ndim;
  for (int d = 0; d < x->ndim; ++d) {
    TK_CHECK_ARG(a->before[d] >= 0 && a->after[d] >= 0 && y->shape[d] == x->shape[d] + a->before[d] + a->after[d],
                 "pad: output shape must be the padded input shape");
    g.out_shape[d] = y->shape[d];
    g.in_shape[d] = x->shape[d];
    g.before[d] = a->before[d];
  }
  const int64_t n = numel(y);
  if (n == 0) return TK_OK;
  auto launch = [&](auto tag, auto value) -> int {
    using T = decltype(tag);
    hipLaunchKernelGGL((pad_kernel<T>), dim3(grid_for(n)), dim3(kBlock), 0, s, (const T*)ptr(x), (T*)ptr(y), n, g,
                       (T)value);
    TK_LAUNCH_CHECK();
    return TK_OK;
  };
  if (is_f32(x)) return launch(float{}, (float)a->value_f);
  switch (x->dtype.bits) {
    case 8: return launch(uint8_t{}, (uint8_t)a->value_i);
    case 16: return launch(uint16_t{}, (uint16_t)a->value_i);
    case 32: return launch(uint32_t{}, (uint32_t)a->value_i);
    case 64: return launch(uint64_t{}, (uint64_t)a->value_i);
  }
  set_error("pad: unsupported dtype");
  return TK_ERR_INVALID_ARG;
}

// ---------------------------------------------------------------- digest
// Order-aware, parallel 64-bit digest: Σ_i mix(word_i ^ (i · φ)) mod 2^64 over
// little-endian 8-byte words (tail zero-padded).  Host twin: trace_format.digest_bytes.
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(kBlock) void digest_kernel(const uint8_t* __restrict__ p, int64_t nbytes,
                                                         unsigned long long* out) {
  int64_t nw = (nbytes + 7) / 8;
  int64_t stride = (int64_t)gridDim.x * kBlock;
  uint64_t acc = 0;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < nw; i += stride) {
    uint64_t w = 0;
    if ((i + 1) * 8 <= nbytes) {
      __builtin_memcpy(&w, p + i * 8, 8);
    } else {
      for (int b = 0; i * 8 + b < nbytes; ++b) w |= (uint64_t)p[i * 8 + b] << (8 * b);
    }
    acc += mix64(w ^ ((uint64_t)i * 0x9E3779B97F4A7C15ULL));
  }
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)acc);
}

int digest_impl(const void* data, int64_t nbytes, uint64_t* out, hipStream_t s) {
  TK_CHECK_ARG(out && (data || nbytes == 0), "null argument");
  TK_HIP(hipMemsetAsync(out, 0, 8, s));
  if (nbytes == 0) return TK_OK;
  hipLaunchKernelGGL(digest_kernel, dim3(grid_for((nbytes + 7) / 8)), dim3(kBlock), 0, s, (const uint8_t*)data, nbytes,
                     (unsigned long long*)out);
  TK_LAUNCH_CHECK();
  return TK_OK;
}

// ---------------------------------------------------------------- tachikoma composite post-ops
// The float32 post-op chain of a legalized tachikoma.qnn.conv2d / .dense composite
// (tachikoma.py:1262-1276; tachikoma_json_runtime.cc:142-185), see tk_postops_attrs.  Every
// operation is rounded on its own (__fmul_rn / __fadd_rn: no contraction into FMAs), so the
// result is a fixed function of the inputs that oracle/tachikoma_ref.py restates.
template <typename Tout, typename Tsum>
__global__ __launch_bounds__(kBlock) void postops_kernel(const int32_t* __restrict__ acc, const Tsum* __restrict__ sum_src,
                                                         Tout* __restrict__ y, int64_t n, int32_t inner, int32_t C,
                                                         tk_postops_attrs a) {
  const float lo = (float)std::numeric_limits<Tout>::min(), hi = (float)std::numeric_limits<Tout>::max();
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  for (int64_t i = blockIdx.x * (int64_t)kBlock + threadIdx.x; i < n; i += stride) {
    const int c = (int)((i / inner) % C);
    float t = __fadd_rn((float)acc[i], a.bias[c]);
    t = __fmul_rn(t, a.o_scl[a.n_scales == 1 ? 0 : c]);
    t = __fmul_rn(fminf(fmaxf(t, a.clip_lo), a.clip_hi), a.act_scl);
    if (sum_src) t = __fadd_rn(__fmul_rn(a.sum_scl, (float)sum_src[i]), t);
    t = __fadd_rn(t, a.dst_zp);
    t = fminf(fmaxf(__builtin_rintf(t), lo), hi);  // round half to even, saturate
    y[i] = (Tout)(int)t;
  }
}

int postops_impl(const tk_tensor* acc, const tk_tensor* sum_src, tk_tensor* y, const tk_postops_attrs* a,
                 hipStream_t s) {
  TK_CHECK_ARG(acc && y && a && a->bias && a->o_scl, "null argument");
  TK_CHECK_ARG(is_int(acc, 32) && is_int8ish(y), "acc must be int32, out int8/uint8");
  TK_CHECK_ARG(compact(acc) && compact(y) && numel(acc) == numel(y), "shape mismatch");
  TK_CHECK_ARG(!sum_src || (is_int8ish(sum_src) && compact(sum_src) && numel(sum_src) == numel(y)),
               "sum source must be int8/uint8 shaped like the output");
  int32_t inner, C;
  TK_CHECK_ARG(axis_geometry(acc, a->axis, &inner, &C) == TK_OK, "bad axis");
  TK_CHECK_ARG(a->n_scales == 1 || a->n_scales == C, "o_scl must be per-tensor or per-channel");
  const int64_t n = numel(y);
  if (n == 0) return TK_OK;
  const int grid = grid_for(n);
  const bool yu = is_uint(y, 8);
  auto go = [&](auto tout, auto tsum) {
    using To = decltype(tout);
    using Ts = decltype(tsum);
    hipLaunchKernelGGL((postops_kernel<To, Ts>), dim3(grid), dim3(kBlock), 0, s, (const int32_t*)ptr(acc),
                       sum_src ? (const Ts*)ptr(sum_src) : nullptr, (To*)ptr(y), n, inner, C, *a);
  };
  const bool su = sum_src && is_uint(sum_src, 8);
  if (yu) {
    if (su) go(uint8_t{}, uint8_t{}); else go(uint8_t{}, int8_t{});
  } else {
    if (su) go(int8_t{}, uint8_t{}); else go(int8_t{}, int8_t{});
  }
  TK_LAUNCH_CHECK();
  return TK_OK;
}

}  // namespace tk
