// Dense layer blocks with a small batch on the matrix cores: qnn.dense -> nn.bias_add ->
// qnn.requantize [-> clip] of [B, K] x [U, K]^T with B <= a few hundred (the classifier heads;
// dense blocks run as 1x1 conv blocks over [B, K, 1, 1], device_module._dense_as_conv).
//
// The im2col conv tiles (64 rows x 128 columns) leave such a layer 16 tiles for 256 CUs and need
// split-K with a second reduce launch: ResNet-50's 2048 -> 1000 classifier took 23.7 us for 2 MB of
// weights (profiles/r03fin3_layers_rocprof.txt).  Here one launch covers it: a workgroup owns a
// 32-unit x 64-sample tile, its eight waves split K eight ways and stream their A (packed weight)
// and B (input shadow) fragments straight from global memory into registers -- all of a wave's
// loads in one batch for ResNet-50's K = 2048, so the launch costs about one memory round trip --
// (every byte feeds MFMAs directly, LDS staging buys nothing), the partial tiles meet in LDS and the
// workgroup writes every record of the block from there: 32 tiles for ResNet-50's head.  (Four
// waves over two 32-sample tiles each measured 9.0 us in the network, profiles/r04j_layers_rocprof.txt.)
// Bound: the weight bytes (HBM) and the per-CU load rate; v_mfma_i32_32x32x32_i8.
#include <algorithm>

#include "tk_conv.h"

namespace tk {

namespace {

constexpr int kDenseSteps = 8;   // K = 32 steps whose fragments are loaded before their MFMAs
constexpr int kDenseWaves = 8;   // K split eight ways inside the workgroup: every wave's loads in one batch

// A workgroup owns 32 units x CTD * 32 samples; wave w reduces K steps [w * per, (w + 1) * per)
// for all of its CTD column tiles (one weight fragment feeds CTD MFMAs).
template <int CTD>
__global__ __launch_bounds__(64 * kDenseWaves) void dense_tile_kernel(GemmArgs g, int32_t ksteps) {
  __shared__ int32_t part[4][32][CTD * 32 + 1];  // [wave pair][unit row][sample col], +1 against conflicts
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r0 = blockIdx.x * 32, c0 = blockIdx.y * (CTD * 32);
  const int rl = lane & 31, h = lane >> 5;
  const int per = (ksteps + kDenseWaves - 1) / kDenseWaves;
  const int s0 = wave * per, s1 = min(ksteps, s0 + per);
  const int8_t* arow = g.A + (int64_t)(r0 + rl) * g.lda + 16 * h;  // packed rows exist up to rows_pad
  const int8_t* bcol[CTD];
  bool col_ok[CTD];
#pragma unroll
  for (int j = 0; j < CTD; ++j) {
    const int col = c0 + j * 32 + rl;
    col_ok[j] = col < g.N;
    bcol[j] = g.B + (int64_t)(col_ok[j] ? col : 0) * 16 + (int64_t)h * g.in_pix * 16;
  }
  const int64_t bstep = 2 * g.in_pix * 16;  // two 16-channel groups per K step
  v16i acc[CTD];
#pragma unroll
  for (int j = 0; j < CTD; ++j) acc[j] = v16i{0};
  for (int s = s0; s < s1; s += kDenseSteps) {
    v4i a[kDenseSteps], b[kDenseSteps][CTD];
#pragma unroll
    for (int k = 0; k < kDenseSteps; ++k) {
      if (s + k < s1) {
        a[k] = __builtin_nontemporal_load(reinterpret_cast<const v4i*>(arow + (int64_t)(s + k) * 32));
#pragma unroll
        for (int j = 0; j < CTD; ++j)
          b[k][j] = col_ok[j] ? ldg(reinterpret_cast<const v4i*>(bcol[j] + (int64_t)(s + k) * bstep)) : v4i{0, 0, 0, 0};
      }
    }
#pragma unroll
    for (int k = 0; k < kDenseSteps; ++k)
      if (s + k < s1) {
#pragma unroll
        for (int j = 0; j < CTD; ++j) acc[j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[k], b[k][j], acc[j], 0, 0, 0);
      }
  }
  // the eight partial tiles meet in LDS: waves 4..7 store, waves 0..3 add theirs and store the pair
  // sums, then every thread sums the four pairs of its outputs.  C/D layout: register q holds row
  // (q & 3) + 8 * (q >> 2) + 4 * h, column rl of the wave's tile j.
  const int pw = wave & 3;
  if (wave >= 4) {
#pragma unroll
    for (int j = 0; j < CTD; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) part[pw][(q & 3) + 8 * (q >> 2) + 4 * h][j * 32 + rl] = acc[j][q];
  }
  __syncthreads();
  if (wave < 4) {
#pragma unroll
    for (int j = 0; j < CTD; ++j)
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        int32_t& slot = part[pw][(q & 3) + 8 * (q >> 2) + 4 * h][j * 32 + rl];
        slot = (int32_t)((uint32_t)slot + (uint32_t)acc[j][q]);
      }
  }
  __syncthreads();
  // epilogue: thread t owns sample c0 + t / 8 and units r0 + 4 (t % 8) .. + 3 (consecutive in the
  // [B, U] records: 16-byte int32 stores)
  const int t = threadIdx.x;
  const int j = t >> 3, i0 = (t & 7) * 4;
  const int b = c0 + j;
  if (j >= CTD * 32 || b >= g.N) return;
  int32_t v[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int i = i0 + e;
    uint32_t x = (uint32_t)part[0][i][j] + (uint32_t)part[1][i][j] + (uint32_t)part[2][i][j] + (uint32_t)part[3][i][j];
    // zero-point folding with zA = 0 (the weight side): out = acc - zB * RA[unit]
    const int u = min(r0 + i, g.M - 1);
    x -= (uint32_t)g.zB * (uint32_t)g.RA[u];
    v[e] = (int32_t)x;
  }
  const int u0 = r0 + i0;
  const int64_t off = (int64_t)b * g.M + u0;
  const bool full = u0 + 3 < g.M && (off & 3) == 0;
  auto put32 = [&](int32_t* dst, const int32_t* w) {
    if (full) {
      *reinterpret_cast<v4i*>(dst + off) = v4i{w[0], w[1], w[2], w[3]};
    } else {
      for (int e = 0; e < 4; ++e)
        if (u0 + e < g.M) dst[off + e] = w[e];
    }
  };
  auto put8 = [&](uint8_t* dst, const int32_t* w) {
    for (int e = 0; e < 4; ++e)
      if (u0 + e < g.M) dst[off + e] = (uint8_t)w[e];
  };
  put32(g.C, v);
  if (!g.bias_out) return;  // a plain contraction (no block)
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = (int32_t)((uint32_t)v[e] + (uint32_t)g.bias[min(u0 + e, g.M - 1)]);
  put32(g.bias_out, v);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int32_t q = rq_apply(v[e], min(u0 + e, g.M - 1), g.rq);
    v[e] = (int32_t)min(max((int64_t)q, g.rq.qmin), g.rq.qmax);
  }
  put8(g.rq_out, v);
  if (g.has_clip) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = min(max(v[e], g.clip_lo), g.clip_hi);
    put8(g.clip_out, v);
  }
  if (g.shadow_out) {
    // the next MFMA layer's shadow [units / 16][B][16] (padded units of the last group as 0)
    for (int e = 0; e < 4; ++e) {
      const int u = u0 + e;
      if (u < g.M) g.shadow_out[((int64_t)(u >> 4) * g.N + b) * 16 + (u & 15)] = (uint8_t)((uint32_t)v[e] ^ g.shadow_xor);
      else if (u < g.shadow_cpad) g.shadow_out[((int64_t)(u >> 4) * g.N + b) * 16 + (u & 15)] = 0;
    }
  }
}

}  // namespace

bool conv_dense_applies(const ConvGeom& g, const GemmArgs& ga) {
  // (K steps of 32 bytes cover exactly the shadow's channel groups: cin_pad % 32 == 0)
  return g.H == 1 && g.W == 1 && g.KH == 1 && g.KW == 1 && g.OH == 1 && g.OW == 1 && ga.zA == 0 && !ga.zA_vec &&
         !ga.RB && !ga.has_add && g.cin_pad % 32 == 0 && g.N <= 1024;
}

int conv_dense_run(const ConvGeom& g, const GemmArgs& ga, hipStream_t s) {
  TK_CHECK_ARG(conv_dense_applies(g, ga), "dense tile kernel: not a [B, K] x [U, K]^T block with zero weight zero point");
  TK_CHECK_ARG(ga.RA || ga.zB == 0, "dense tile kernel: weight sums needed for the input zero point");
  TK_CHECK_ARG(ga.k_pad <= ga.lda && (int64_t)(g.O + 31) / 32 * 32 <= g.rows_pad, "dense tile kernel: packed weight rows");
  // two 32-sample column tiles per workgroup (one weight fragment per two MFMAs) unless the batch
  // fits one
  if (g.N > 32) {
    const dim3 grid((unsigned)((g.O + 31) / 32), (unsigned)((g.N + 63) / 64));
    hipLaunchKernelGGL(dense_tile_kernel<2>, grid, dim3(64 * kDenseWaves), 0, s, ga, (int32_t)(g.cin_pad / 32));
  } else {
    const dim3 grid((unsigned)((g.O + 31) / 32), 1u);
    hipLaunchKernelGGL(dense_tile_kernel<1>, grid, dim3(64 * kDenseWaves), 0, s, ga, (int32_t)(g.cin_pad / 32));
  }
  TK_LAUNCH_CHECK();
  return TK_OK;
}

}  // namespace tk
