// Dense layer blocks with a small batch on the matrix cores: qnn.dense -> nn.bias_add ->
// qnn.requantize [-> clip] of [B, K] x [U, K]^T with B <= a few hundred (the classifier heads;
// dense blocks run as 1x1 conv blocks over [B, K, 1, 1], device_module._dense_as_conv).
//
// The im2col conv tiles (64 rows x 128 columns) leave such a layer 16 tiles for 256 CUs: round 3's
// split-K im2col run took ResNet-50's 2048 -> 1000 classifier 23.7 us for 2 MB of weights
// (profiles/r03fin3_layers_rocprof.txt).  Here a workgroup owns a 32-unit x 64-sample tile (one
// weight fragment feeds two MFMAs) over a slice of K; its four waves split the slice and stream
// their A (packed weight) and B (input shadow) fragments straight from global memory into
// registers (every byte feeds MFMAs directly, LDS staging buys nothing) and their partial tiles
// meet in LDS.  With one slice (small grids of long K excepted) the workgroup writes every record
// of the block from there; ResNet-50's head has 32 tiles, so K is cut into 8 slices (256
// workgroups, the per-CU load rate of 32 CUs was the bound: 9.0 us with 64 workgroups, 10.3 with
// 32, profiles/r04j_layers_rocprof.txt, r04l) whose raw sums go to scratch, and a second, elementwise
// launch sums them and runs the epilogue.  v_mfma_i32_32x32x32_i8.
#include <algorithm>

#include "tk_conv.h"

namespace tk {

namespace {

constexpr int kDenseSteps = 8;     // K = 32 steps whose fragments are loaded before their MFMAs
constexpr int kDenseMaxSlices = 8; // K slices of a split run (its scratch: slices x [B, U] int32)

// zero-point fold, bias_add, requantize, clip and the next layer's shadow of sample b, units
// u0 .. u0 + 3 (v: the contraction sums)
__device__ __forceinline__ void dense_epilogue(const GemmArgs& g, int b, int u0, int32_t* v) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    // zero-point folding with zA = 0 (the weight side): out = acc - zB * RA[unit]
    const int u = min(u0 + e, g.M - 1);
    v[e] = (int32_t)((uint32_t)v[e] - (uint32_t)g.zB * (uint32_t)g.RA[u]);
  }
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
    if (full) {  // (4-aligned in a [B, U] record: one dword)
      *reinterpret_cast<uint32_t*>(dst + off) = ((uint32_t)w[0] & 0xFFu) | (((uint32_t)w[1] & 0xFFu) << 8) |
                                                (((uint32_t)w[2] & 0xFFu) << 16) | ((uint32_t)w[3] << 24);
    } else {
      for (int e = 0; e < 4; ++e)
        if (u0 + e < g.M) dst[off + e] = (uint8_t)w[e];
    }
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
    // the next MFMA layer's shadow [units / 16][B][16] (padded units of the last group as 0): the
    // 4 units (u0 % 4 == 0) are 4 bytes of one 16-byte chunk, one dword store
    uint32_t word = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (u0 + e < g.M) word |= (((uint32_t)v[e] ^ g.shadow_xor) & 0xFFu) << (8 * e);
    if (u0 < g.shadow_cpad)
      *reinterpret_cast<uint32_t*>(g.shadow_out + ((int64_t)(u0 >> 4) * g.N + b) * 16 + (u0 & 15)) = word;
  }
}

// grid (unit tiles, sample tiles, K slices); slice z = K steps [z * kper, (z + 1) * kper); wave w
// of the workgroup takes a quarter of the slice.  SPLIT: raw sums to part[z][B][U]; else the
// block epilogue.
template <int CTD, bool SPLIT, int W = 4>
__global__ __launch_bounds__(64 * W) void dense_tile_kernel(GemmArgs g, int32_t ksteps, int32_t kper, int32_t* part) {
  __shared__ int32_t red[W][32][CTD * 32 + 1];  // [wave][unit row][sample col], +1 against conflicts
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r0 = blockIdx.x * 32, c0 = blockIdx.y * (CTD * 32);
  const int rl = lane & 31, h = lane >> 5;
  const int z0 = blockIdx.z * kper, z1 = min(ksteps, z0 + kper);
  const int per = (z1 - z0 + W - 1) / W;
  const int s0 = z0 + wave * per, s1 = min(z1, s0 + per);
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
  // C/D layout: register q holds row (q & 3) + 8 * (q >> 2) + 4 * h, column rl of the tile j
#pragma unroll
  for (int j = 0; j < CTD; ++j)
#pragma unroll
    for (int q = 0; q < 16; ++q) red[wave][(q & 3) + 8 * (q >> 2) + 4 * h][j * 32 + rl] = acc[j][q];
  __syncthreads();
  // thread t (< 256) owns samples c0 + t / 8 (+ 32 for CTD = 2) and units r0 + 4 (t % 8) .. + 3
  // (consecutive in the [B, U] records: 16-byte int32 stores)
  const int t = threadIdx.x;
  if (t >= 256) return;
  const int i0 = (t & 7) * 4, u0 = r0 + i0;
#pragma unroll
  for (int jj = 0; jj < CTD; ++jj) {
    const int jc = (t >> 3) + 32 * jj, b = c0 + jc;
    if (b >= g.N) continue;
    int32_t v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      uint32_t x = 0;
#pragma unroll
      for (int w = 0; w < W; ++w) x += (uint32_t)red[w][i0 + e][jc];
      v[e] = (int32_t)x;
    }
    if constexpr (SPLIT) {
      int32_t* dst = part + ((int64_t)blockIdx.z * g.N + b) * g.M + u0;
      if (u0 + 3 < g.M && ((((int64_t)blockIdx.z * g.N + b) * g.M + u0) & 3) == 0) {
        *reinterpret_cast<v4i*>(dst) = v4i{v[0], v[1], v[2], v[3]};
      } else {
        for (int e = 0; e < 4; ++e)
          if (u0 + e < g.M) dst[e] = v[e];
      }
    } else {
      dense_epilogue(g, b, u0, v);
    }
  }
}

// the split run's second launch: thread per (sample, 4 units), the slices' sums + the epilogue
// (units up to the shadow's padded channel count, whose shadow bytes are written as 0; 64-thread
// blocks so that the ~16k threads of a classifier head spread over the CUs, every slice's sums
// loaded in one batch of 16-byte loads)
__global__ __launch_bounds__(64) void dense_slices_epilogue_kernel(GemmArgs g, int32_t slices, const int32_t* part) {
  const int per_row = (max(g.M, g.shadow_out ? (int)g.shadow_cpad : 0) + 3) / 4;
  const int64_t groups = (int64_t)g.N * per_row;
  const int64_t i = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= groups) return;
  const int b = (int)(i / per_row), u0 = (int)(i - (int64_t)b * per_row) * 4;
  uint32_t v[4] = {0, 0, 0, 0};
  if (g.M % 4 == 0 && u0 < g.M) {
    v4i s[kDenseMaxSlices];
#pragma unroll
    for (int z = 0; z < kDenseMaxSlices; ++z)
      if (z < slices) s[z] = ldg(reinterpret_cast<const v4i*>(part + ((int64_t)z * g.N + b) * g.M + u0));
#pragma unroll
    for (int z = 0; z < kDenseMaxSlices; ++z)
      if (z < slices)
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] += (uint32_t)s[z][e];
  } else {
    for (int z = 0; z < slices; ++z) {
      const int32_t* src = part + ((int64_t)z * g.N + b) * g.M + u0;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (u0 + e < g.M) v[e] += (uint32_t)src[e];
    }
  }
  int32_t w[4] = {(int32_t)v[0], (int32_t)v[1], (int32_t)v[2], (int32_t)v[3]};
  dense_epilogue(g, b, u0, w);
}

}  // namespace

bool conv_dense_applies(const ConvGeom& g, const GemmArgs& ga) {
  // (K steps of 32 bytes cover exactly the shadow's channel groups: cin_pad % 32 == 0)
  return g.H == 1 && g.W == 1 && g.KH == 1 && g.KW == 1 && g.OH == 1 && g.OW == 1 && ga.zA == 0 && !ga.zA_vec &&
         !ga.RB && !ga.has_add && g.cin_pad % 32 == 0 && g.N <= 1024;
}

int64_t conv_dense_scratch_bytes(const ConvGeom& g) {
  // a split run's K-slice sums (dense geometry only; conv_dense_applies checks the rest)
  return g.H == 1 && g.W == 1 && g.KH == 1 && g.KW == 1 && g.cin_pad % 32 == 0 && g.N <= 1024
             ? (int64_t)kDenseMaxSlices * g.N * g.O * 4 : 0;
}

int conv_dense_run(const ConvGeom& g, const GemmArgs& ga, void* scratch, hipStream_t s) {
  TK_CHECK_ARG(conv_dense_applies(g, ga), "dense tile kernel: not a [B, K] x [U, K]^T block with zero weight zero point");
  TK_CHECK_ARG(ga.RA || ga.zB == 0, "dense tile kernel: weight sums needed for the input zero point");
  TK_CHECK_ARG(ga.k_pad <= ga.lda && (int64_t)(g.O + 31) / 32 * 32 <= g.rows_pad, "dense tile kernel: packed weight rows");
  const int ksteps = g.cin_pad / 32;
  // one launch where 32-sample tiles give the chip >= 48 workgroups: eight waves split K (every
  // wave's loads in one batch for K <= 2048)
  {
    const unsigned ut1 = (unsigned)((g.O + 31) / 32), st1 = (unsigned)((g.N + 31) / 32);
    if ((int64_t)ut1 * st1 >= 48 || !scratch) {
      hipLaunchKernelGGL((dense_tile_kernel<1, false, 8>), dim3(ut1, st1, 1u), dim3(512), 0, s, ga, ksteps, ksteps,
                         (int32_t*)nullptr);
      TK_LAUNCH_CHECK();
      return TK_OK;
    }
  }
  const int ctd = g.N > 32 ? 2 : 1;
  const unsigned ut = (unsigned)((g.O + 31) / 32), st = (unsigned)((g.N + 32 * ctd - 1) / (32 * ctd));
  // K slices: enough workgroups for the chip, >= 8 K steps (2 per wave) per slice
  int slices = scratch ? (int)std::min<int64_t>({(int64_t)kDenseMaxSlices, std::max<int64_t>(1, 256 / ((int64_t)ut * st)),
                                                 std::max(1, ksteps / 8)})
                       : 1;
  const int kper = (ksteps + slices - 1) / slices;
  slices = (ksteps + kper - 1) / kper;
  int32_t* part = static_cast<int32_t*>(scratch);
  const dim3 grid(ut, st, (unsigned)slices);
  if (slices > 1) {
    if (ctd == 2) hipLaunchKernelGGL((dense_tile_kernel<2, true>), grid, dim3(256), 0, s, ga, ksteps, kper, part);
    else hipLaunchKernelGGL((dense_tile_kernel<1, true>), grid, dim3(256), 0, s, ga, ksteps, kper, part);
    TK_LAUNCH_CHECK();
    const int64_t groups = (int64_t)g.N * ((std::max(g.O, ga.shadow_out ? (int)ga.shadow_cpad : 0) + 3) / 4);
    hipLaunchKernelGGL(dense_slices_epilogue_kernel, dim3((unsigned)((groups + 63) / 64)), dim3(64), 0, s, ga, slices,
                       (const int32_t*)part);
  } else if (ctd == 2) {
    hipLaunchKernelGGL((dense_tile_kernel<2, false>), grid, dim3(256), 0, s, ga, ksteps, kper, part);
  } else {
    hipLaunchKernelGGL((dense_tile_kernel<1, false>), grid, dim3(256), 0, s, ga, ksteps, kper, part);
  }
  TK_LAUNCH_CHECK();
  return TK_OK;
}

}  // namespace tk
