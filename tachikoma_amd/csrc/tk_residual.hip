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
// Work unit = 16 channels (one shadow group) x kV consecutive pixels of one image
// (kV = 16 when HW % 16 == 0, else 4 or 1), lanes along the pixels: every load and
// record store of a wave covers 64·kV contiguous bytes of one channel plane.  When
// the next MFMA conv reads this output, the unit's final 16 x kV bytes are transposed
// in registers (v_perm_b32) into kV 16-byte shadow chunks [C_pad16/16][N·HW][16]
// (tk_conv2d_make_shadow layout); channels >= C are written as 0.
#include <algorithm>

#include "tk_common.h"

namespace tk {

namespace {

constexpr int kThreads = 256;

struct AddBlockArgs {
  const uint8_t* a;
  const uint8_t* b;
  uint8_t* add_out;
  uint8_t* clip_out;  // null: no clip record
  uint8_t* shadow;    // null: no shadow copy
  int32_t N, C, HW, G;  // G = channel groups of 16
  int32_t is_u8, zp_c, has_clip, clip_lo, clip_hi;
  RqParams pa, pb;
  int32_t up_a, up_b;
};

// byte k of each of w0..w3, packed little-endian into one dword
__device__ __forceinline__ uint32_t gather_byte(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3, int k) {
  const uint32_t sel = (uint32_t)k | ((uint32_t)(k + 4) << 8) | 0x0c0c0000u;
  const uint32_t lo = __builtin_amdgcn_perm(w1, w0, sel);  // {w0.k, w1.k, 0, 0}
  const uint32_t hi = __builtin_amdgcn_perm(w3, w2, sel);  // {w2.k, w3.k, 0, 0}
  return __builtin_amdgcn_perm(hi, lo, 0x05040100u);       // {w0.k, w1.k, w2.k, w3.k}
}

template <int kV>
__global__ __launch_bounds__(kThreads) void add_block_kernel(AddBlockArgs g) {
  constexpr int kW = kV >= 4 ? kV / 4 : 1;  // dwords per channel row of the unit
  __shared__ int32_t lut_a[256];
  __shared__ int32_t lut_b[256];
  const int tid = threadIdx.x;
  {
    // RequantizeOrUpcast of every representable 8-bit value (op_common.h:186-200)
    int32_t x = g.is_u8 ? tid : (int32_t)(int8_t)(uint8_t)tid;
    lut_a[tid] = g.up_a ? x : rq_apply(x, 0, g.pa);
    lut_b[tid] = g.up_b ? x : rq_apply(x, 0, g.pb);
  }
  __syncthreads();

  const int tmin = g.is_u8 ? 0 : -128, tmax = g.is_u8 ? 255 : 127;
  const int units_per_plane = g.HW / kV;
  const int64_t units = (int64_t)g.N * g.G * units_per_plane;
  const uint32_t xr = g.is_u8 ? 0x80808080u : 0u;
  for (int64_t u = (int64_t)blockIdx.x * kThreads + tid; u < units; u += (int64_t)gridDim.x * kThreads) {
    const int pu = (int)(u % units_per_plane);
    const int64_t rest = u / units_per_plane;
    const int grp = (int)(rest % g.G);
    const int n = (int)(rest / g.G);
    const int p = pu * kV;
    uint32_t last[16][kW];
    const uint8_t* __restrict__ pa = g.a;
    const uint8_t* __restrict__ pb = g.b;
    // 4 channel rows per batch: all 8 loads are issued before the first use (the record
    // stores cannot alias the operands), so each wave pays the load latency 4x, not 16x
#pragma unroll
    for (int j0 = 0; j0 < 16; j0 += 4) {
      uint8_t va[4][kV], vb[4][kV];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int c = min(grp * 16 + j0 + jj, g.C - 1);  // clamped: rows >= C are loaded but not used
        const int64_t off = ((int64_t)n * g.C + c) * g.HW + p;
        __builtin_memcpy(va[jj], pa + off, kV);
        __builtin_memcpy(vb[jj], pb + off, kV);
      }
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int j = j0 + jj;
        const int c = grp * 16 + j;
#pragma unroll
        for (int w = 0; w < kW; ++w) last[j][w] = 0;
        if (c >= g.C) continue;
        const int64_t off = ((int64_t)n * g.C + c) * g.HW + p;
        uint8_t vo[kV], vc[kV];
#pragma unroll
        for (int q = 0; q < kV; ++q) {
          int32_t o = (int32_t)((uint32_t)lut_a[va[jj][q]] + (uint32_t)lut_b[vb[jj][q]] - (uint32_t)g.zp_c);
          o = min(max(o, tmin), tmax);
          vo[q] = (uint8_t)o;
          vc[q] = (uint8_t)min(max(o, g.clip_lo), g.clip_hi);
        }
        store_nt<kV>(g.add_out + off, vo);
        if (g.has_clip) store_nt<kV>(g.clip_out + off, vc);
        __builtin_memcpy(&last[j][0], g.has_clip ? vc : vo, kV);
      }
    }
    if (!g.shadow) continue;
    // 16 channels x kV pixels -> kV chunks of 16 channel bytes
    uint8_t* dst = g.shadow + ((int64_t)grp * g.N * g.HW + (int64_t)n * g.HW + p) * 16;
#pragma unroll
    for (int q = 0; q < kV; ++q) {
      uint32_t o4[4];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        if constexpr (kV == 1)
          o4[d] = (last[4 * d][0] & 0xFF) | ((last[4 * d + 1][0] & 0xFF) << 8) | ((last[4 * d + 2][0] & 0xFF) << 16) |
                  ((last[4 * d + 3][0] & 0xFF) << 24);
        else
          o4[d] = gather_byte(last[4 * d][q >> 2], last[4 * d + 1][q >> 2], last[4 * d + 2][q >> 2],
                              last[4 * d + 3][q >> 2], q & 3);
      }
      // uint8 data is stored xor 0x80; padded channels (>= C) stay 0
      const int cvalid = g.C - grp * 16;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        uint32_t m = 0;
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) m |= (4 * d + bb < cvalid ? 0xFFu : 0u) << (8 * bb);
        o4[d] = (o4[d] ^ xr) & m;
      }
      *reinterpret_cast<tk_v4i*>(dst + q * 16) = tk_v4i{(int)o4[0], (int)o4[1], (int)o4[2], (int)o4[3]};
    }
  }
}

// Small planes (16·HW <= 16 KB, C % 16 == 0): the 16 channel rows of one image's
// channel group are one contiguous 16·HW-byte block in NCHW, and consecutive blocks
// are adjacent, so a workgroup streams K whole blocks (~16 KB) with flat 16-byte
// vectors (no plane-length constraint), parks the final bytes in LDS and re-reads
// them per pixel for the shadow.
constexpr int kPlaneLds = 16384;

__global__ __launch_bounds__(kThreads) void add_block_plane_kernel(AddBlockArgs g, int K) {
  __shared__ int32_t lut_a[256];
  __shared__ int32_t lut_b[256];
  __shared__ __attribute__((aligned(16))) uint8_t tile[kPlaneLds];
  const int tid = threadIdx.x;
  {
    int32_t x = g.is_u8 ? tid : (int32_t)(int8_t)(uint8_t)tid;
    lut_a[tid] = g.up_a ? x : rq_apply(x, 0, g.pa);
    lut_b[tid] = g.up_b ? x : rq_apply(x, 0, g.pb);
  }
  __syncthreads();
  const int tmin = g.is_u8 ? 0 : -128, tmax = g.is_u8 ? 255 : 127;
  const int blk = 16 * g.HW;
  const int64_t nblocks = (int64_t)g.N * g.G;
  const int64_t nsuper = (nblocks + K - 1) / K;
  const uint8_t* __restrict__ pa = g.a;
  const uint8_t* __restrict__ pb = g.b;
  for (int64_t sb = blockIdx.x; sb < nsuper; sb += gridDim.x) {
    const int64_t b0 = sb * K;
    const int nb = (int)min<int64_t>(K, nblocks - b0);
    const int64_t base = b0 * blk;
    const int nvec = nb * blk / 16;
    for (int v = tid; v < nvec; v += kThreads) {
      uint8_t va[16], vb[16], vo[16], vc[16];
      __builtin_memcpy(va, pa + base + 16 * v, 16);
      __builtin_memcpy(vb, pb + base + 16 * v, 16);
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        int32_t o = (int32_t)((uint32_t)lut_a[va[q]] + (uint32_t)lut_b[vb[q]] - (uint32_t)g.zp_c);
        o = min(max(o, tmin), tmax);
        vo[q] = (uint8_t)o;
        vc[q] = (uint8_t)min(max(o, g.clip_lo), g.clip_hi);
      }
      store_nt<16>(g.add_out + base + 16 * v, vo);
      if (g.has_clip) store_nt<16>(g.clip_out + base + 16 * v, vc);
      if (g.shadow) {
        // element-wise select: a pointer chosen between two local arrays would force both
        // into scratch memory
        uint8_t vs[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) vs[q] = g.has_clip ? vc[q] : vo[q];
        __builtin_memcpy(tile + 16 * v, vs, 16);
      }
    }
    if (!g.shadow) continue;
    __syncthreads();
    const uint8_t xr = g.is_u8 ? 0x80 : 0;
    for (int it = tid; it < nb * g.HW; it += kThreads) {
      const int bl = it / g.HW;
      const int pix = it - bl * g.HW;
      const int64_t gb = b0 + bl;
      const int n = (int)(gb / g.G), grp = (int)(gb - (int64_t)n * g.G);
      uint8_t out[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) out[j] = tile[bl * blk + j * g.HW + pix] ^ xr;
      __builtin_memcpy(g.shadow + ((int64_t)grp * g.N * g.HW + (int64_t)n * g.HW + pix) * 16, out, 16);
    }
    __syncthreads();
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
  // max(min(x, a_max), a_min) (topi/math.py:634-638): a_min wins when a_min > a_max
  g.clip_hi = (int32_t)std::max<int64_t>(std::min<int64_t>(at->has_clip ? at->clip_max : hi, hi), g.clip_lo);
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
  } else if (total % 1024 == 0) {
    // no layout needed: flat view as 1-KB blocks
    N = 1;
    HW = 64;
    C = total / 64;
  } else {
    // odd sizes: rows of the longest power-of-4 length <= 4096 dividing the tensor
    int64_t L = 4096;
    while (total % L) L /= 4;
    N = 1;
    C = total / L;
    HW = L;
  }
  TK_CHECK_ARG(HW <= INT32_MAX && C <= INT32_MAX && N <= INT32_MAX, "tensor too large");
  g.N = (int32_t)N;
  g.C = (int32_t)C;
  g.HW = (int32_t)HW;
  g.G = (int32_t)((C + 15) / 16);
  if (C % 16 == 0 && 16 * HW <= kPlaneLds) {
    // ~16 KB per workgroup iteration, fewer when that would leave < 2048 workgroups
    const int64_t nblocks = N * g.G;
    const int K = (int)std::max<int64_t>(1, std::min<int64_t>(kPlaneLds / (16 * HW), nblocks / 2048));
    const int64_t nsuper = (nblocks + K - 1) / K;
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(nsuper, 256 * 16));
    hipLaunchKernelGGL(add_block_plane_kernel, dim3(grid), dim3(kThreads), 0, s, g, K);
    TK_LAUNCH_CHECK();
    return TK_OK;
  }
  const int kv = HW % 16 == 0 ? 16 : HW % 4 == 0 ? 4 : 1;
  const int64_t units = N * g.G * (HW / kv);
  const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((units + kThreads - 1) / kThreads, 256 * 16));
  if (kv == 16)
    hipLaunchKernelGGL(add_block_kernel<16>, dim3(grid), dim3(kThreads), 0, s, g);
  else if (kv == 4)
    hipLaunchKernelGGL(add_block_kernel<4>, dim3(grid), dim3(kThreads), 0, s, g);
  else
    hipLaunchKernelGGL(add_block_kernel<1>, dim3(grid), dim3(kThreads), 0, s, g);
  TK_LAUNCH_CHECK();
  return TK_OK;
}

}  // namespace tk
