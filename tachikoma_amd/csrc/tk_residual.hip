// Fused residual join for gfx950: qnn.add [-> clip] on 8-bit NCHW tensors.
//
// qnn.add canonicalises to  o = RQ(a) + RQ(b) - zp_c ; clip+cast to the input dtype
// (src/relay/qnn/op/add.cc:40-96, op_common.h:169-207), where RQ is a per-tensor
// requantize to int32 or a plain upcast.  With 8-bit operands RQ has 256 possible
// inputs, so each workgroup tabulates RQ for both operands in LDS once (computed with
// the same rq_apply the requantize kernel uses, hence bit-exact by construction) and
// the element loop is two table lookups, an add and two clamps: the kernel is a pure
// HBM stream of 2 bytes in, 2 bytes out (+ the shadow) per element.
//
// Tile = 64 channels x PT pixels of one image.  Records are stored NCHW with
// kV-byte vectors (16 when HW % 16 == 0, else 4 or 1); when the next MFMA conv
// reads this output, the final bytes are also staged in LDS and re-emitted as its
// int8 shadow [C_pad16/16][N·HW][16] (tk_conv2d_make_shadow layout), 16 B per store.
#include <algorithm>

#include "tk_common.h"

namespace tk {

namespace {

constexpr int kThreads = 256;
constexpr int kCT = 64;     // channels per tile
constexpr int kPTMax = 256; // pixels per tile
constexpr int kLdsStride = kPTMax + 4;

struct AddBlockArgs {
  const uint8_t* a;
  const uint8_t* b;
  uint8_t* add_out;
  uint8_t* clip_out;  // null: no clip record
  uint8_t* shadow;    // null: no shadow copy
  int32_t N, C, HW, PT, tiles_per_image;
  int32_t is_u8, zp_c, has_clip, clip_lo, clip_hi, cpad;
  RqParams pa, pb;
  int32_t up_a, up_b;
};

template <int kV>
__global__ __launch_bounds__(kThreads) void add_block_kernel(AddBlockArgs g) {
  __shared__ int32_t lut_a[256];
  __shared__ int32_t lut_b[256];
  __shared__ uint8_t tile[kCT * kLdsStride];

  const int tid = threadIdx.x;
  {
    // RequantizeOrUpcast of every representable 8-bit value (op_common.h:186-200)
    int32_t x = g.is_u8 ? tid : (int32_t)(int8_t)(uint8_t)tid;
    lut_a[tid] = g.up_a ? x : rq_apply(x, 0, g.pa);
    lut_b[tid] = g.up_b ? x : rq_apply(x, 0, g.pb);
  }
  __syncthreads();

  const int n = blockIdx.z;
  const int c0 = blockIdx.y * kCT;
  const int p0 = blockIdx.x * g.PT;
  const int tmin = g.is_u8 ? 0 : -128, tmax = g.is_u8 ? 255 : 127;
  const int vec_per_row = g.PT / kV;
  const int nvec = kCT * vec_per_row;
  const bool want_shadow = g.shadow != nullptr;

  for (int v = tid; v < nvec; v += kThreads) {
    int cl = v / vec_per_row;
    int pl = (v - cl * vec_per_row) * kV;
    int c = c0 + cl, p = p0 + pl;
    if (c >= g.C || p >= g.HW) continue;  // HW % kV == 0: vectors never straddle the plane
    int64_t off = ((int64_t)n * g.C + c) * g.HW + p;
    uint8_t va[kV], vb[kV], vo[kV], vc[kV];
    __builtin_memcpy(va, g.a + off, kV);
    __builtin_memcpy(vb, g.b + off, kV);
#pragma unroll
    for (int j = 0; j < kV; ++j) {
      int32_t o = (int32_t)((uint32_t)lut_a[va[j]] + (uint32_t)lut_b[vb[j]] - (uint32_t)g.zp_c);
      o = min(max(o, tmin), tmax);
      vo[j] = (uint8_t)o;
      vc[j] = (uint8_t)min(max(o, g.clip_lo), g.clip_hi);
    }
    store_nt<kV>(g.add_out + off, vo);
    if (g.has_clip) store_nt<kV>(g.clip_out + off, vc);
    if (want_shadow) {
      const uint8_t* last = g.has_clip ? vc : vo;
#pragma unroll
      for (int j = 0; j < kV; ++j) tile[cl * kLdsStride + pl + j] = last[j];
    }
  }
  if (!want_shadow) return;
  __syncthreads();

  // shadow: one 16-channel chunk of one pixel per item (lanes along pixels: contiguous)
  const int chunks = kCT / 16;
  const int items = chunks * g.PT;
  const uint8_t xr = g.is_u8 ? 0x80 : 0;
  for (int it = tid; it < items; it += kThreads) {
    int pl = it % g.PT;
    int ch = it / g.PT;
    int p = p0 + pl;
    int cbase = c0 + ch * 16;
    if (p >= g.HW || cbase >= g.cpad) continue;
    uint8_t out[16];
#pragma unroll
    for (int j = 0; j < 16; ++j)
      out[j] = (cbase + j < g.C) ? (uint8_t)(tile[(ch * 16 + j) * kLdsStride + pl] ^ xr) : 0;
    __builtin_memcpy(g.shadow + ((int64_t)(cbase >> 4) * g.N * g.HW + (int64_t)n * g.HW + p) * 16, out, 16);
  }
}

RqParams add_rq(const tk_requantize_attrs& a) {
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

}  // namespace

int add_block_impl(const tk_tensor* a, const tk_tensor* b, tk_tensor* const* outs, int n_outs,
                   const tk_add_block_attrs* at, void* shadow, hipStream_t s) {
  TK_CHECK_ARG(a && b && outs && at, "null argument");
  TK_CHECK_ARG(n_outs == 1 + (at->has_clip ? 1 : 0), "outs = {add, [clip]}");
  TK_CHECK_ARG(is_int8ish(a) && dt_of(a) == dt_of(b), "qnn.add block: 8-bit operands of one dtype");
  TK_CHECK_ARG(compact(a) && compact(b), "compact tensors only");
  int64_t total = numel(a);
  TK_CHECK_ARG(numel(b) == total, "qnn.add block: only same-shape operands are supported");
  for (int i = 0; i < n_outs; ++i)
    TK_CHECK_ARG(outs[i] && dt_of(outs[i]) == dt_of(a) && numel(outs[i]) == total && compact(outs[i]),
                 "outputs must match the operands");
  const tk_qnn_add_attrs& ad = at->add;
  TK_CHECK_ARG(ad.lhs.mode <= TK_RQ_TENSOR_TONEAREST && ad.rhs.mode <= TK_RQ_TENSOR_TONEAREST,
               "qnn.add: per-tensor parameters only");
  if (total == 0) return TK_OK;

  AddBlockArgs g{};
  g.a = (const uint8_t*)ptr(a);
  g.b = (const uint8_t*)ptr(b);
  g.add_out = (uint8_t*)ptr(outs[0]);
  g.clip_out = at->has_clip ? (uint8_t*)ptr(outs[1]) : nullptr;
  g.shadow = (uint8_t*)shadow;
  g.is_u8 = is_uint(a, 8);
  int64_t lo = g.is_u8 ? 0 : -128, hi = g.is_u8 ? 255 : 127;
  g.has_clip = at->has_clip;
  g.clip_lo = (int32_t)std::max<int64_t>(at->has_clip ? at->clip_min : lo, lo);
  g.clip_hi = (int32_t)std::min<int64_t>(at->has_clip ? at->clip_max : hi, hi);
  g.zp_c = ad.output_zero_point;
  g.pa = add_rq(ad.lhs);
  g.pb = add_rq(ad.rhs);
  g.up_a = ad.lhs_upcast;
  g.up_b = ad.rhs_upcast;

  int64_t N, C, HW;
  if (shadow) {
    TK_CHECK_ARG(a->ndim == 4, "shadow output needs NCHW operands");
    N = a->shape[0];
    C = a->shape[1];
    HW = a->shape[2] * a->shape[3];
  } else {
    // no layout needed: view the tensor as rows of the longest power-of-4 length dividing it
    int64_t L = 4096;
    while (total % L) L /= 4;
    N = 1;
    C = total / L;
    HW = L;
    if (C > (int64_t)kCT * 65535) {  // keep gridDim.y in range with a 2-level split
      N = C / kCT;
      while (C % N) --N;
      C /= N;
    }
  }
  TK_CHECK_ARG(N <= 65535 && (C + kCT - 1) / kCT <= 65535 && HW <= INT32_MAX, "tensor too large");
  g.N = (int32_t)N;
  g.C = (int32_t)C;
  g.HW = (int32_t)HW;
  g.cpad = (int32_t)((C + 15) / 16 * 16);
  g.PT = (int32_t)std::min<int64_t>(kPTMax, (HW + 15) / 16 * 16);
  g.tiles_per_image = (int32_t)((HW + g.PT - 1) / g.PT);
  dim3 grid(g.tiles_per_image, (unsigned)((C + kCT - 1) / kCT), (unsigned)N);
  if (HW % 16 == 0)
    hipLaunchKernelGGL(add_block_kernel<16>, grid, dim3(kThreads), 0, s, g);
  else if (HW % 4 == 0)
    hipLaunchKernelGGL(add_block_kernel<4>, grid, dim3(kThreads), 0, s, g);
  else
    hipLaunchKernelGGL(add_block_kernel<1>, grid, dim3(kThreads), 0, s, g);
  TK_LAUNCH_CHECK();
  return TK_OK;
}

}  // namespace tk
