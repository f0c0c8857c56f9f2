// int8 x int8 -> int32 contractions on the gfx950 matrix cores.
//
// qnn.conv2d is an implicit GEMM   C[cout][p] = Σ_k W'[cout][k] · X'[p][k]
// and qnn.dense a plain GEMM        C[m][n]    = Σ_k D'[m][k]   · W'[n][k]
// both computed by one MFMA kernel (v_mfma_i32_32x32x32_i8) over operands whose
// reduction axis is contiguous:
//   * weights are packed once to [Cout][KH][KW][Cin_pad] (Cin_pad = Cin rounded
//     to 16, K rounded to 64; padding bytes are 0, uint8 stored xor 0x80),
//   * conv activations are read from an NHWC int8 "shadow" of the NCHW tensor,
//     gathered per 16-byte chunk (one tap, 16 channels) straight into LDS.
// The zero points are folded exactly (modulo 2^32, like the reference's int32
// accumulation) with row sums:
//   Σ(a-za)(w-zw) = Σ a'w - za·Σw - zw·Σa' + K·za·zw
// where out-of-bounds taps hold a' = za on real channels (they contribute 0,
// python/tvm/relay/qnn/op/legalizations.py:195-226 pads with zeros after the shift).
// The epilogue writes int32 NCHW directly (lanes run along pixels: coalesced).
#include <algorithm>
#include <climits>
#include <cstring>

#include "tk_common.h"

namespace tk {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

constexpr int kBK = 64;          // bytes of K per stage
constexpr int kGemmThreads = 256;

struct GemmArgs {
  const int8_t* A;     // [rowsA_pad][lda]
  const int8_t* B;     // plain: [rowsB_pad][ldb]; im2col: NHWC shadow [N][H][W][cin_pad]
  int32_t* C;
  int32_t M, N;        // real rows of A / rows of B (pixels for conv)
  int32_t lda, ldb;    // row pitch in bytes (plain), K_pad
  int32_t k_pad;       // multiple of kBK
  int32_t k_eff;       // real reduction length (for the K·zA·zB term)
  // zero-point folding: out = acc - zB[j]*RA[i] - zA[i]*RB[j] + k_eff*zA[i]*zB[j]
  int32_t zA, zB;
  const int32_t* zA_vec;  // per row of A (optional)
  const int32_t* zB_vec;  // per row of B (optional)
  const int32_t* RA;      // row sums of A (needed when zB != 0)
  const int32_t* RB;      // row sums of B (needed when zA != 0)
  // im2col geometry (conv)
  int32_t H, W, cin_pad, KH, KW, sh, sw, pt, pl, dh, dw, OH, OW;
  uint32_t fill;                  // za replicated 4x: out-of-bounds taps (padded channels multiply w = 0)
  int32_t taps;                   // KH*KW
  // output addressing
  int32_t out_nchw;    // 1: C[(p/HW)*M*HW + i*HW + p%HW]; 0: C[i*N + j]
  int32_t ldc;         // row-major pitch (elements) when !out_nchw
};

// LDS tile [rows][64 B], 16-byte chunk c of row r stored at chunk c ^ ((r >> 2) & 3):
// the 16-lane groups of ds_read_b128 then hit 16 distinct bank slots.
__device__ __forceinline__ int lds_off(int row, int chunk) { return row * kBK + ((chunk ^ ((row >> 2) & 3)) << 4); }

template <int MT, bool kIm2col>
__global__ __launch_bounds__(kGemmThreads) void gemm_i8_kernel(GemmArgs g) {
  constexpr int BM = 64 * MT;   // rows of A per block (2 waves along M, MT 32-row tiles each)
  constexpr int BN = 128;       // rows of B per block (2 waves along N, 2 32-col tiles each)
  constexpr int A_CHUNKS = BM * kBK / 16 / kGemmThreads;  // 16-byte loads per thread per stage
  constexpr int B_CHUNKS = BN * kBK / 16 / kGemmThreads;
  __shared__ __attribute__((aligned(16))) int8_t smem[2 * (BM + BN) * kBK];
  int8_t* As = smem;
  int8_t* Bs = smem + 2 * BM * kBK;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * BM;
  const int n0 = blockIdx.x * BN;
  const int kc = tid & 3;  // this thread's 16-byte chunk within a K stage

  // ---- per-thread im2col state for the B rows it loads
  int b_img[B_CHUNKS], b_ih0[B_CHUNKS], b_iw0[B_CHUNKS];
  bool b_valid[B_CHUNKS];
#pragma unroll
  for (int t = 0; t < B_CHUNKS; ++t) {
    int row = (tid >> 2) + t * (kGemmThreads / 4);
    int p = n0 + row;
    b_valid[t] = p < g.N;
    if (kIm2col) {
      int pp = b_valid[t] ? p : 0;
      int hw = g.OH * g.OW;
      int img = pp / hw;
      int rem = pp - img * hw;
      int oh = rem / g.OW;
      int ow = rem - oh * g.OW;
      b_img[t] = img;
      b_ih0[t] = oh * g.sh - g.pt;
      b_iw0[t] = ow * g.sw - g.pl;
    }
  }

  v4i ra[A_CHUNKS], rb[B_CHUNKS];

  auto load_stage = [&](int k0) {
#pragma unroll
    for (int t = 0; t < A_CHUNKS; ++t) {
      int row = (tid >> 2) + t * (kGemmThreads / 4);
      ra[t] = *reinterpret_cast<const v4i*>(g.A + (int64_t)(m0 + row) * g.lda + k0 + kc * 16);
    }
    if (!kIm2col) {
#pragma unroll
      for (int t = 0; t < B_CHUNKS; ++t) {
        int row = (tid >> 2) + t * (kGemmThreads / 4);
        rb[t] = *reinterpret_cast<const v4i*>(g.B + (int64_t)(n0 + row) * g.ldb + k0 + kc * 16);
      }
    } else {
      int kg = k0 + kc * 16;
      int tap = kg / g.cin_pad;
      int c0 = kg - tap * g.cin_pad;
      int kh = tap / g.KW;
      int kw = tap - kh * g.KW;
      bool tap_ok = tap < g.taps;
      const uint32_t fill = g.fill;
#pragma unroll
      for (int t = 0; t < B_CHUNKS; ++t) {
        int ih = b_ih0[t] + kh * g.dh;
        int iw = b_iw0[t] + kw * g.dw;
        if (b_valid[t] && tap_ok) {
          if (ih >= 0 && ih < g.H && iw >= 0 && iw < g.W) {
            const int8_t* src = g.B + (((int64_t)b_img[t] * g.H + ih) * g.W + iw) * g.cin_pad + c0;
            rb[t] = *reinterpret_cast<const v4i*>(src);
          } else {
            rb[t] = v4i{(int)fill, (int)fill, (int)fill, (int)fill};
          }
        } else {
          rb[t] = v4i{0, 0, 0, 0};
        }
      }
    }
  };

  auto store_stage = [&](int buf) {
    int8_t* a = As + buf * BM * kBK;
    int8_t* b = Bs + buf * BN * kBK;
#pragma unroll
    for (int t = 0; t < A_CHUNKS; ++t) {
      int row = (tid >> 2) + t * (kGemmThreads / 4);
      *reinterpret_cast<v4i*>(a + lds_off(row, kc)) = ra[t];
    }
#pragma unroll
    for (int t = 0; t < B_CHUNKS; ++t) {
      int row = (tid >> 2) + t * (kGemmThreads / 4);
      *reinterpret_cast<v4i*>(b + lds_off(row, kc)) = rb[t];
    }
  };

  v16i acc[MT][2];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = v16i{0};

  const int nk = g.k_pad / kBK;
  load_stage(0);
  store_stage(0);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) load_stage((kt + 1) * kBK);  // issue early, land under the MFMAs
    const int8_t* a = As + buf * BM * kBK;
    const int8_t* b = Bs + buf * BN * kBK;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int chunk = 2 * ks + (lane >> 5);
      v4i af[MT], bf[2];
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        int row = wm * 32 * MT + i * 32 + (lane & 31);
        af[i] = *reinterpret_cast<const v4i*>(a + lds_off(row, chunk));
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        int row = wn * 64 + j * 32 + (lane & 31);
        bf[j] = *reinterpret_cast<const v4i*>(b + lds_off(row, chunk));
      }
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store_stage(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: zero-point folding + store
  const int hw = g.OH * g.OW;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = n0 + wn * 64 + j * 32 + (lane & 31);
    if (col >= g.N) continue;
    const uint32_t zb = g.zB_vec ? (uint32_t)g.zB_vec[col] : (uint32_t)g.zB;
    const uint32_t rbj = g.RB ? (uint32_t)g.RB[col] : 0u;
    int64_t base;
    if (g.out_nchw) {
      int img = col / hw;
      int pix = col - img * hw;
      base = (int64_t)img * g.M * hw + pix;
    } else {
      base = col;
    }
#pragma unroll
    for (int i = 0; i < MT; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm * 32 * MT + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row >= g.M) continue;
        const uint32_t za = g.zA_vec ? (uint32_t)g.zA_vec[row] : (uint32_t)g.zA;
        const uint32_t rai = g.RA ? (uint32_t)g.RA[row] : 0u;
        uint32_t v = (uint32_t)acc[i][j][r];
        v = v - zb * rai - za * rbj + (uint32_t)g.k_eff * za * zb;
        int64_t off = g.out_nchw ? base + (int64_t)row * hw : (int64_t)row * g.ldc + base;
        g.C[off] = (int32_t)v;
      }
    }
  }
}

// ---------------------------------------------------------------- operand preparation

// pack OIHW (int8/uint8) -> [Cout_rows][k_pad], k = (kh*KW + kw)*cin_pad + c ; row sums over real taps.
// groups == 1 only (grouped convs take the direct kernel).
__global__ __launch_bounds__(256) void pack_weight_kernel(const int8_t* __restrict__ w, int8_t* __restrict__ packed,
                                                          int32_t* __restrict__ sums, int Cout, int Cin, int KH, int KW,
                                                          int cin_pad, int k_pad, int xor_u8) {
  int o = blockIdx.x;
  int8_t* dst = packed + (int64_t)o * k_pad;
  int32_t s = 0;
  for (int k = threadIdx.x; k < k_pad; k += blockDim.x) {
    int tap = k / cin_pad;
    int c = k - tap * cin_pad;
    int8_t v = 0;
    if (o < Cout && tap < KH * KW && c < Cin) {
      int kh = tap / KW, kw = tap - (tap / KW) * KW;
      uint8_t raw = (uint8_t)w[(((int64_t)o * Cin + c) * KH + kh) * KW + kw];
      v = (int8_t)(xor_u8 ? (raw ^ 0x80) : raw);
      s += v;
    }
    dst[k] = v;
  }
  __shared__ int32_t red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0 && o < Cout) sums[o] = red[0];
}

// NCHW int8/uint8 -> NHWC [N][H][W][cin_pad]; padded channels 0; uint8 xor 0x80.
// One thread per (pixel, 16-channel chunk); lanes run along pixels so each channel
// plane read is a contiguous 64-byte span.
__global__ __launch_bounds__(256) void shadow_kernel(const uint8_t* __restrict__ x, uint8_t* __restrict__ y, int N,
                                                     int C, int HW, int cin_pad, int xor_u8) {
  int chunks = cin_pad / 16;
  int64_t total = (int64_t)N * HW * chunks;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += stride) {
    int64_t q = t / HW;          // (n, chunk)
    int pix = (int)(t - q * HW);
    int chunk = (int)(q % chunks);
    int n = (int)(q / chunks);
    uint8_t v[16];
    const uint8_t* src = x + ((int64_t)n * C) * HW + pix;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      int c = chunk * 16 + j;
      uint8_t b = 0;
      if (c < C) b = xor_u8 ? (uint8_t)(src[(int64_t)c * HW] ^ 0x80) : src[(int64_t)c * HW];
      v[j] = b;
    }
    __builtin_memcpy(y + ((int64_t)n * HW + pix) * cin_pad + chunk * 16, v, 16);
  }
}

// dense data [M][K] -> [M_rows][k_pad] (zero padded, uint8 xor 0x80) + row sums.
__global__ __launch_bounds__(256) void pad_rows_kernel(const uint8_t* __restrict__ x, int8_t* __restrict__ y,
                                                       int32_t* __restrict__ sums, int M, int K, int k_pad, int xor_u8) {
  int m = blockIdx.x;
  int32_t s = 0;
  for (int k = threadIdx.x; k < k_pad; k += blockDim.x) {
    int8_t v = 0;
    if (m < M && k < K) {
      uint8_t raw = x[(int64_t)m * K + k];
      v = (int8_t)(xor_u8 ? (raw ^ 0x80) : raw);
      s += v;
    }
    y[(int64_t)m * k_pad + k] = v;
  }
  __shared__ int32_t red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if (threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0 && m < M && sums) sums[m] = red[0];
}

// Σ over the real taps/channels of the (zero-point-filled) patch of every output pixel:
// only needed when the kernel zero point is non-zero.
__global__ __launch_bounds__(256) void patch_sum_kernel(const int8_t* __restrict__ shadow, int32_t* __restrict__ out,
                                                        GemmArgs g, int Cin) {
  int64_t total = g.N;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int8_t zpa = (int8_t)(g.fill & 0xFF);
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < total; p += stride) {
    int hw = g.OH * g.OW;
    int img = (int)(p / hw);
    int rem = (int)(p - (int64_t)img * hw);
    int oh = rem / g.OW, ow = rem - (rem / g.OW) * g.OW;
    int32_t s = 0;
    for (int kh = 0; kh < g.KH; ++kh) {
      int ih = oh * g.sh - g.pt + kh * g.dh;
      for (int kw = 0; kw < g.KW; ++kw) {
        int iw = ow * g.sw - g.pl + kw * g.dw;
        if (ih < 0 || ih >= g.H || iw < 0 || iw >= g.W) {
          s += (int32_t)zpa * Cin;
        } else {
          const int8_t* src = shadow + (((int64_t)img * g.H + ih) * g.W + iw) * g.cin_pad;
          for (int c = 0; c < Cin; ++c) s += src[c];
        }
      }
    }
    out[p] = s;
  }
}

// Direct (VALU) grouped / depthwise / tiny-channel convolution on NCHW int8/uint8.
// out[n][o][oh][ow] = Σ_{c in group(o), r, s} (a - za)(w - zw[o]); padded taps contribute 0.
template <typename Tx, typename Tw>
__global__ __launch_bounds__(256) void direct_conv_kernel(const Tx* __restrict__ x, const Tw* __restrict__ w,
                                                          int32_t* __restrict__ y, int N, int C, int H, int W, int O,
                                                          int OH, int OW, int KH, int KW, int sh, int sw, int pt, int pl,
                                                          int dh, int dw, int groups, int32_t za, int32_t zw,
                                                          const int32_t* __restrict__ zw_vec) {
  int64_t total = (int64_t)N * O * OH * OW;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int cg = C / groups, og = O / groups;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += stride) {
    int ow = (int)(i % OW);
    int64_t t = i / OW;
    int oh = (int)(t % OH);
    t /= OH;
    int o = (int)(t % O);
    int n = (int)(t / O);
    int g = o / og;
    int32_t zwo = zw_vec ? zw_vec[o] : zw;
    uint32_t acc = 0;
    for (int c = 0; c < cg; ++c) {
      int ci = g * cg + c;
      const Tx* plane = x + ((int64_t)n * C + ci) * H * W;
      const Tw* wk = w + (((int64_t)o * cg + c) * KH) * KW;
      for (int r = 0; r < KH; ++r) {
        int ih = oh * sh - pt + r * dh;
        if (ih < 0 || ih >= H) continue;
        for (int s = 0; s < KW; ++s) {
          int iw = ow * sw - pl + s * dw;
          if (iw < 0 || iw >= W) continue;
          int32_t a = (int32_t)plane[ih * W + iw] - za;
          int32_t b = (int32_t)wk[r * KW + s] - zwo;
          acc += (uint32_t)(a * b);
        }
      }
    }
    y[i] = (int32_t)acc;
  }
}

// ---------------------------------------------------------------- host wrappers

struct ConvGeom {
  int N, C, H, W, O, KH, KW, OH, OW, cin_pad, k_pad, k_eff, rows_pad;
};

static int conv_geom(const tk_tensor* data, const tk_tensor* weight, const tk_conv2d_attrs* a, ConvGeom* g) {
  if (data->ndim != 4 || weight->ndim != 4) return TK_ERR_SHAPE;
  g->N = (int)data->shape[0];
  g->C = (int)data->shape[1];
  g->H = (int)data->shape[2];
  g->W = (int)data->shape[3];
  g->O = (int)weight->shape[0];
  g->KH = (int)weight->shape[2];
  g->KW = (int)weight->shape[3];
  int groups = a ? a->groups : 1;
  if (groups < 1 || g->C % groups || g->O % groups || weight->shape[1] * groups != g->C) return TK_ERR_SHAPE;
  if (a) {
    int dh = a->dilation[0], dw = a->dilation[1];
    g->OH = (g->H + a->padding[0] + a->padding[2] - dh * (g->KH - 1) - 1) / a->strides[0] + 1;
    g->OW = (g->W + a->padding[1] + a->padding[3] - dw * (g->KW - 1) - 1) / a->strides[1] + 1;
  }
  g->cin_pad = (g->C + 15) / 16 * 16;
  int k = g->KH * g->KW * g->cin_pad;
  g->k_pad = (k + kBK - 1) / kBK * kBK;
  g->k_eff = g->KH * g->KW * g->C;
  g->rows_pad = (g->O + 127) / 128 * 128;
  return TK_OK;
}

static bool use_mfma_conv(const ConvGeom& g, int groups) { return groups == 1 && g.O >= 16 && g.C >= 3; }

int64_t conv_packed_weight_bytes(const tk_tensor* weight, int groups) {
  if (!weight || weight->ndim != 4 || groups != 1) return 0;
  int O = (int)weight->shape[0], C = (int)weight->shape[1], KH = (int)weight->shape[2], KW = (int)weight->shape[3];
  int cin_pad = (C + 15) / 16 * 16;
  int64_t k_pad = ((int64_t)KH * KW * cin_pad + kBK - 1) / kBK * kBK;
  int64_t rows = (O + 127) / 128 * 128;
  return rows * k_pad;
}

int conv_pack_weight(const tk_tensor* weight, int groups, void* packed, int32_t* sums, hipStream_t s) {
  TK_CHECK_ARG(weight && packed && sums && weight->ndim == 4 && groups == 1, "bad arguments");
  TK_CHECK_ARG(is_int8ish(weight), "weight must be int8/uint8");
  int O = (int)weight->shape[0], C = (int)weight->shape[1], KH = (int)weight->shape[2], KW = (int)weight->shape[3];
  int cin_pad = (C + 15) / 16 * 16;
  int k_pad = (KH * KW * cin_pad + kBK - 1) / kBK * kBK;
  int rows = (O + 127) / 128 * 128;
  hipLaunchKernelGGL(pack_weight_kernel, dim3(rows), dim3(256), 0, s, (const int8_t*)ptr(weight), (int8_t*)packed, sums,
                     O, C, KH, KW, cin_pad, k_pad, (int)is_uint(weight, 8));
  TK_LAUNCH_CHECK();
  return TK_OK;
}

int64_t conv_shadow_bytes(const tk_tensor* data) {
  if (!data || data->ndim != 4) return 0;
  int64_t cin_pad = (data->shape[1] + 15) / 16 * 16;
  return data->shape[0] * data->shape[2] * data->shape[3] * cin_pad;
}

int nchw_to_nhwc_impl(const tk_tensor* data, void* shadow, hipStream_t s) {
  TK_CHECK_ARG(data && shadow && data->ndim == 4 && is_int8ish(data), "data must be 4-D int8/uint8");
  int N = (int)data->shape[0], C = (int)data->shape[1], HW = (int)(data->shape[2] * data->shape[3]);
  int cin_pad = (C + 15) / 16 * 16;
  int64_t total = (int64_t)N * HW * (cin_pad / 16);
  int grid = (int)std::min<int64_t>((total + 255) / 256, 2048);
  hipLaunchKernelGGL(shadow_kernel, dim3(std::max(grid, 1)), dim3(256), 0, s, (const uint8_t*)ptr(data),
                     (uint8_t*)shadow, N, C, HW, cin_pad, (int)is_uint(data, 8));
  TK_LAUNCH_CHECK();
  return TK_OK;
}

static inline uint32_t rep4(int v) {
  uint32_t b = (uint8_t)(int8_t)v;
  return b | (b << 8) | (b << 16) | (b << 24);
}

int conv2d_prepared_impl(const tk_tensor* data, const void* shadow, const tk_tensor* weight, const void* packed,
                         const int32_t* sums, tk_tensor* out, const tk_conv2d_attrs* a, void* workspace_patch,
                         hipStream_t s) {
  TK_CHECK_ARG(data && weight && out && a, "null argument");
  TK_CHECK_ARG(is_int8ish(data) && is_int8ish(weight) && is_int(out, 32), "dtypes: int8/uint8 in, int32 out");
  ConvGeom g;
  if (conv_geom(data, weight, a, &g) != TK_OK) {
    set_error("tk_qnn_conv2d: bad shapes");
    return TK_ERR_SHAPE;
  }
  TK_CHECK_ARG(out->ndim == 4 && out->shape[0] == g.N && out->shape[1] == g.O && out->shape[2] == g.OH &&
                   out->shape[3] == g.OW,
               "output shape mismatch");
  TK_CHECK_ARG(a->strides[0] > 0 && a->strides[1] > 0 && a->dilation[0] > 0 && a->dilation[1] > 0, "bad strides");
  int64_t P = (int64_t)g.N * g.OH * g.OW;
  TK_CHECK_ARG(P < INT32_MAX && (int64_t)g.N * g.O * g.OH * g.OW < INT32_MAX * 2LL, "tensor too large");
  if (!use_mfma_conv(g, a->groups)) {
    // grouped / depthwise / tiny channel counts: direct VALU kernel on NCHW
    int64_t total = (int64_t)g.N * g.O * g.OH * g.OW;
    int grid = (int)std::max<int64_t>(1, std::min<int64_t>((total + 255) / 256, 8192));
#define TK_DIRECT(TX, TW)                                                                                      \
  hipLaunchKernelGGL((direct_conv_kernel<TX, TW>), dim3(grid), dim3(256), 0, s, (const TX*)ptr(data),               \
                     (const TW*)ptr(weight), (int32_t*)ptr(out), g.N, g.C, g.H, g.W, g.O, g.OH, g.OW, g.KH, g.KW,    \
                     a->strides[0], a->strides[1], a->padding[0], a->padding[1], a->dilation[0], a->dilation[1],     \
                     a->groups, a->input_zero_point, a->kernel_zero_point, a->kernel_zero_points)
    bool du = is_uint(data, 8), wu = is_uint(weight, 8);
    if (du && wu) TK_DIRECT(uint8_t, uint8_t);
    else if (du) TK_DIRECT(uint8_t, int8_t);
    else if (wu) TK_DIRECT(int8_t, uint8_t);
    else TK_DIRECT(int8_t, int8_t);
#undef TK_DIRECT
    TK_LAUNCH_CHECK();
    return TK_OK;
  }
  TK_CHECK_ARG(shadow && packed && sums, "MFMA conv needs shadow, packed weight and weight sums");
  int du = is_uint(data, 8), wu = is_uint(weight, 8);
  TK_CHECK_ARG(!(wu && a->kernel_zero_points), "per-channel zero points with uint8 weights are not supported");
  int32_t za = a->input_zero_point - (du ? 128 : 0);
  int32_t zw = a->kernel_zero_point - (wu ? 128 : 0);
  GemmArgs ga{};
  ga.A = (const int8_t*)packed;
  ga.B = (const int8_t*)shadow;
  ga.C = (int32_t*)ptr(out);
  ga.M = g.O;
  ga.N = (int32_t)P;
  ga.lda = g.k_pad;
  ga.ldb = g.cin_pad;
  ga.k_pad = g.k_pad;
  ga.k_eff = g.k_eff;
  // operand A = weights (zero point zw), operand B = activations (zero point za)
  ga.zA = zw;
  ga.zA_vec = nullptr;
  ga.zB = za;
  ga.zB_vec = nullptr;
  ga.RA = sums;
  ga.RB = nullptr;
  ga.H = g.H; ga.W = g.W; ga.cin_pad = g.cin_pad; ga.KH = g.KH; ga.KW = g.KW;
  ga.sh = a->strides[0]; ga.sw = a->strides[1]; ga.pt = a->padding[0]; ga.pl = a->padding[1];
  ga.dh = a->dilation[0]; ga.dw = a->dilation[1]; ga.OH = g.OH; ga.OW = g.OW;
  ga.taps = g.KH * g.KW;
  ga.fill = rep4(za);
  ga.out_nchw = 1;
  ga.ldc = 0;
  if (zw != 0 || a->kernel_zero_points) {
    TK_CHECK_ARG(workspace_patch, "non-zero kernel zero point needs a patch-sum workspace");
    int32_t* ps = (int32_t*)workspace_patch;
    int grid = (int)std::max<int64_t>(1, std::min<int64_t>((P + 255) / 256, 4096));
    hipLaunchKernelGGL(patch_sum_kernel, dim3(grid), dim3(256), 0, s, (const int8_t*)shadow, ps, ga, g.C);
    TK_LAUNCH_CHECK();
    ga.RB = ps;
    ga.zA_vec = a->kernel_zero_points;
  }
  dim3 grid((unsigned)((P + 127) / 128), (unsigned)((g.O + 127) / 128));
  if (g.O <= 64) {
    grid.y = (unsigned)((g.O + 63) / 64);
    hipLaunchKernelGGL((gemm_i8_kernel<1, true>), grid, dim3(kGemmThreads), 0, s, ga);
  } else {
    hipLaunchKernelGGL((gemm_i8_kernel<2, true>), grid, dim3(kGemmThreads), 0, s, ga);
  }
  TK_LAUNCH_CHECK();
  return TK_OK;
}

int64_t conv2d_workspace_bytes(const tk_tensor* data, const tk_tensor* weight, const tk_conv2d_attrs* a) {
  if (!a) return -1;
  ConvGeom g;
  if (conv_geom(data, weight, a, &g) != TK_OK) return -1;
  if (!use_mfma_conv(g, a->groups)) return 0;
  int64_t packed = conv_packed_weight_bytes(weight, 1);
  int64_t sums = (int64_t)g.rows_pad * 4;
  int64_t shadow = conv_shadow_bytes(data);
  int64_t patch = (int64_t)g.N * g.OH * g.OW * 4;
  auto al = [](int64_t v) { return (v + 255) / 256 * 256; };
  return al(packed) + al(sums) + al(shadow) + al(patch);
}

int conv2d_impl(const tk_tensor* data, const tk_tensor* weight, tk_tensor* out, const tk_conv2d_attrs* a,
                void* workspace, hipStream_t s) {
  TK_CHECK_ARG(data && weight && out && a, "null argument");
  ConvGeom g;
  if (conv_geom(data, weight, a, &g) != TK_OK) {
    set_error("tk_qnn_conv2d: bad shapes");
    return TK_ERR_SHAPE;
  }
  if (!use_mfma_conv(g, a->groups))
    return conv2d_prepared_impl(data, nullptr, weight, nullptr, nullptr, out, a, nullptr, s);
  TK_CHECK_ARG(workspace, "workspace required (tk_qnn_conv2d_workspace_bytes)");
  auto al = [](int64_t v) { return (v + 255) / 256 * 256; };
  char* ws = (char*)workspace;
  void* packed = ws;
  ws += al(conv_packed_weight_bytes(weight, 1));
  int32_t* sums = (int32_t*)ws;
  ws += al((int64_t)g.rows_pad * 4);
  void* shadow = ws;
  ws += al(conv_shadow_bytes(data));
  void* patch = ws;
  int rc = conv_pack_weight(weight, 1, packed, sums, s);
  if (rc) return rc;
  rc = nchw_to_nhwc_impl(data, shadow, s);
  if (rc) return rc;
  return conv2d_prepared_impl(data, shadow, weight, packed, sums, out, a, patch, s);
}

// ---------------------------------------------------------------- dense
int64_t dense_workspace_bytes(const tk_tensor* data, const tk_tensor* weight) {
  if (!data || !weight || data->ndim != 2 || weight->ndim != 2) return -1;
  int64_t M = data->shape[0], K = data->shape[1], Nn = weight->shape[0];
  int64_t k_pad = (K + kBK - 1) / kBK * kBK;
  int64_t mrows = (M + 127) / 128 * 128, nrows = (Nn + 127) / 128 * 128;
  auto al = [](int64_t v) { return (v + 255) / 256 * 256; };
  return al(mrows * k_pad) + al(nrows * k_pad) + al(mrows * 4) + al(nrows * 4);
}

int dense_impl(const tk_tensor* data, const tk_tensor* weight, tk_tensor* out, const tk_dense_attrs* a,
               void* workspace, hipStream_t s) {
  TK_CHECK_ARG(data && weight && out && a && workspace, "null argument");
  TK_CHECK_ARG(data->ndim == 2 && weight->ndim == 2 && out->ndim == 2, "dense expects 2-D tensors");
  TK_CHECK_ARG(is_int8ish(data) && is_int8ish(weight) && is_int(out, 32), "dtypes: int8/uint8 in, int32 out");
  int M = (int)data->shape[0], K = (int)data->shape[1], Nn = (int)weight->shape[0];
  TK_CHECK_ARG(weight->shape[1] == K && out->shape[0] == M && out->shape[1] == Nn, "shape mismatch");
  int k_pad = (K + kBK - 1) / kBK * kBK;
  int mrows = (M + 127) / 128 * 128, nrows = (Nn + 127) / 128 * 128;
  auto al = [](int64_t v) { return (v + 255) / 256 * 256; };
  char* ws = (char*)workspace;
  int8_t* dpad = (int8_t*)ws;
  ws += al((int64_t)mrows * k_pad);
  int8_t* wpad = (int8_t*)ws;
  ws += al((int64_t)nrows * k_pad);
  int32_t* dsum = (int32_t*)ws;
  ws += al((int64_t)mrows * 4);
  int32_t* wsum = (int32_t*)ws;
  int du = is_uint(data, 8), wu = is_uint(weight, 8);
  TK_CHECK_ARG(!(wu && a->kernel_zero_points), "per-unit zero points with uint8 weights are not supported");
  hipLaunchKernelGGL(pad_rows_kernel, dim3(mrows), dim3(256), 0, s, (const uint8_t*)ptr(data), dpad, dsum, M, K, k_pad, du);
  hipLaunchKernelGGL(pad_rows_kernel, dim3(nrows), dim3(256), 0, s, (const uint8_t*)ptr(weight), wpad, wsum, Nn, K, k_pad,
                     wu);
  TK_LAUNCH_CHECK();
  int32_t za = a->input_zero_point - (du ? 128 : 0);
  int32_t zw = a->kernel_zero_point - (wu ? 128 : 0);
  GemmArgs ga{};
  ga.A = dpad;
  ga.B = wpad;
  ga.C = (int32_t*)ptr(out);
  ga.M = M;
  ga.N = Nn;
  ga.lda = k_pad;
  ga.ldb = k_pad;
  ga.k_pad = k_pad;
  ga.k_eff = K;
  ga.zA = za;              // operand A = data
  ga.zB = zw;              // operand B = weights
  ga.zB_vec = a->kernel_zero_points;
  ga.RA = dsum;
  ga.RB = wsum;
  ga.out_nchw = 0;
  ga.ldc = Nn;
  dim3 grid((unsigned)((Nn + 127) / 128), (unsigned)((M + 127) / 128));
  hipLaunchKernelGGL((gemm_i8_kernel<2, false>), grid, dim3(kGemmThreads), 0, s, ga);
  TK_LAUNCH_CHECK();
  return TK_OK;
}

}  // namespace tk
