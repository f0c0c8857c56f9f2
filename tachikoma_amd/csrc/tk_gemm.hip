// int8 x int8 -> int32 contractions on the gfx950 matrix cores.
//
// qnn.conv2d is an implicit GEMM   C[cout][p] = Σ_k W'[cout][k] · X'[p][k]
// and qnn.dense a plain GEMM        C[m][n]    = Σ_k D'[m][k]   · W'[n][k]
// both computed by one MFMA kernel (v_mfma_i32_32x32x32_i8) over operands whose
// reduction axis is contiguous:
//   * weights are packed once to [Cout][KH][KW][Cin_pad] (Cin_pad = Cin rounded
//     to 16, K rounded to 64; padding bytes are 0, uint8 stored xor 0x80),
//   * conv activations are read from a channel-blocked int8 "shadow" of the NCHW tensor,
//     gathered per 16-byte chunk (one tap, 16 channels) straight into LDS.
// The zero points are folded exactly (modulo 2^32, like the reference's int32
// accumulation) with row sums:
//   Σ(a-za)(w-zw) = Σ a'w - za·Σw - zw·Σa' + K·za·zw
// where out-of-bounds taps hold a' = za on real channels (they contribute 0,
// python/tvm/relay/qnn/op/legalizations.py:195-226 pads with zeros after the shift).
// The epilogue writes int32 NCHW directly (lanes run along pixels: coalesced).
#include <algorithm>
#include <cstdio>
#include <mutex>
#include <type_traits>
#include <climits>
#include <cstdlib>
#include <cstring>

#include "tk_conv.h"

namespace tk {

// Writes one element of every output of a fused block.  Mirrors, per element:
// nn.bias_add (int32 wrap), RequantizeLowerInt + clip/cast to the out dtype
// (src/relay/qnn/op/requantize.cc:195-273), then clip (python/tvm/topi/math.py:615-640).
template <bool kBlock>
__device__ __forceinline__ void epilogue_store(const GemmArgs& g, int64_t off, int ch, int64_t pix, uint32_t v) {
  g.C[off] = (int32_t)v;
  if (!kBlock) return;
  int32_t b = (int32_t)(v + (uint32_t)g.bias[ch]);
  g.bias_out[off] = b;
  int32_t q = rq_apply(b, ch, g.rq);
  q = (int32_t)min(max((int64_t)q, g.rq.qmin), g.rq.qmax);
  g.rq_out[off] = (uint8_t)q;
  int32_t last = q;
  if (g.has_clip) {
    last = min(max(q, g.clip_lo), g.clip_hi);
    g.clip_out[off] = (uint8_t)last;
  }
  if (g.shadow_out) {
    g.shadow_out[((int64_t)(ch >> 4) * g.N + pix) * 16 + (ch & 15)] = (uint8_t)((uint32_t)last ^ g.shadow_xor);
    if (ch == g.M - 1)  // the padded channels of the last group are written as 0
      for (int c2 = ch + 1; c2 < g.shadow_cpad; ++c2) g.shadow_out[((int64_t)(c2 >> 4) * g.N + pix) * 16 + (c2 & 15)] = 0;
  }
}

__device__ __forceinline__ uint32_t pack4(const int32_t* x) {
  return (uint32_t)(x[0] & 0xFF) | ((uint32_t)(x[1] & 0xFF) << 8) | ((uint32_t)(x[2] & 0xFF) << 16) |
         ((uint32_t)x[3] << 24);
}


// record stores (nontemporal: see store_nt in tk_common.h)
template <int V>
__device__ __forceinline__ void st_i32(int32_t* dst, const int32_t* v, bool nt) {
  if constexpr (V == 4) {
    if (nt) __builtin_nontemporal_store(v4i{v[0], v[1], v[2], v[3]}, reinterpret_cast<v4i*>(dst));
    else *reinterpret_cast<v4i*>(dst) = v4i{v[0], v[1], v[2], v[3]};
  } else {
    *dst = v[0];  // partial lines: let L2 merge them
  }
}

template <int V>
__device__ __forceinline__ void st_i8(uint8_t* dst, const int32_t* v, bool nt) {
  if constexpr (V == 4) {
    if (nt) __builtin_nontemporal_store(pack4(v), reinterpret_cast<uint32_t*>(dst));
    else *reinterpret_cast<uint32_t*>(dst) = pack4(v);
  } else {
    *dst = (uint8_t)v[0];
  }
}

// V consecutive columns of one row after zero-point folding: stores each record as
// soon as it is complete, transforming v in place (conv → bias_add → requantize →
// clip); mirrors nn.bias_add (int32 wrap), RequantizeLowerInt + clip/cast
// (src/relay/qnn/op/requantize.cc:195-273) and clip (python/tvm/topi/math.py:615-640).

// Column constants of a dense block (channel = column), loaded once per thread.
__device__ __forceinline__ EpiRow col_consts(const GemmArgs& g, int col) {
  EpiRow c{};
  const int ch = min(col, g.N - 1);
  c.bias = g.bias[ch];
  const bool axis = g.rq.mode >= TK_RQ_AXIS_UPWARD;
  c.m = axis ? g.rq.ms[ch] : g.rq.multiplier;
  c.s = axis ? g.rq.ss[ch] : g.rq.shift;
  c.zp = g.rq.zps ? g.rq.zps[ch] : g.rq.zp_in;
  return c;
}

template <int V, bool kBlock>
__device__ __forceinline__ void epi_apply(const GemmArgs& g, const EpiRow& r, int32_t* v, int64_t off, bool st,
                                          int col, uint32_t resid, const int32_t* lut, const EpiRow* cc) {
  if (st && !(g.ablate & 8)) st_i32<V>(g.C + off, v, g.nt);
  if (!kBlock) return;
  const int qmin = (int)g.rq.qmin, qmax = (int)g.rq.qmax;
  if (g.ch_is_row) {
#pragma unroll
    for (int q = 0; q < V; ++q) v[q] = (int32_t)((uint32_t)v[q] + (uint32_t)r.bias);
    if (st && !(g.ablate & 16)) st_i32<V>(g.bias_out + off, v, g.nt);
    const int mode = g.rq.mode;
    if (mode == TK_RQ_AXIS_UPWARD || mode == TK_RQ_TENSOR_UPWARD) {
      if (r.s <= -2) {
        // right shift >= 2: the rounding constant 2^(30+rs) has a zero low word, so
        // (x·m + 2^(30+rs)) >> (31+rs) only needs the high word of x·m (v_mul_hi_i32)
        const int sh2 = -r.s - 1;
        const uint32_t rnd = 1u << (sh2 - 1);
#pragma unroll
        for (int q = 0; q < V; ++q)
          v[q] = (int32_t)((uint32_t)__mulhi((int32_t)((uint32_t)v[q] - (uint32_t)r.zp), r.m) + rnd) >> sh2;
      } else {
#pragma unroll
        for (int q = 0; q < V; ++q) v[q] = qms_upward((int32_t)((uint32_t)v[q] - (uint32_t)r.zp), r.m, r.s);
      }
    } else if (mode == TK_RQ_TENSOR_POW2) {
#pragma unroll
      for (int q = 0; q < V; ++q) v[q] = qms_pow2((int32_t)((uint32_t)v[q] - (uint32_t)r.zp), r.s);
    } else if (mode == TK_RQ_IDENTITY) {
#pragma unroll
      for (int q = 0; q < V; ++q) v[q] = (int32_t)((uint32_t)v[q] - (uint32_t)r.zp);
    } else {
#pragma unroll
      for (int q = 0; q < V; ++q) v[q] = qms_tonearest((int32_t)((uint32_t)v[q] - (uint32_t)r.zp), r.m, r.s);
    }
#pragma unroll
    for (int q = 0; q < V; ++q) v[q] = min(max((int32_t)((uint32_t)g.rq.zp_out + (uint32_t)v[q]), qmin), qmax);
  } else {
    // channel = column (dense blocks): per-column constants from registers
#pragma unroll
    for (int q = 0; q < V; ++q) v[q] = (int32_t)((uint32_t)v[q] + (uint32_t)cc[q].bias);
    if (st && !(g.ablate & 16)) st_i32<V>(g.bias_out + off, v, g.nt);
    const int mode = g.rq.mode;
#pragma unroll
    for (int q = 0; q < V; ++q) {
      const int32_t t = rq_core((int32_t)((uint32_t)v[q] - (uint32_t)cc[q].zp), mode, cc[q].m, cc[q].s);
      v[q] = min(max((int32_t)((uint32_t)g.rq.zp_out + (uint32_t)t), qmin), qmax);
    }
  }
  if (st && !(g.ablate & 32)) st_i8<V>(g.rq_out + off, v, g.nt);
  if (g.has_add) {
    // qnn.add (src/relay/qnn/op/add.cc:40-96): RQ(block) + RQ(residual) - zp_out, clip to the dtype
    const int tlo = (int)g.rq.qmin, thi = (int)g.rq.qmax;
#pragma unroll
    for (int q = 0; q < V; ++q) {
      const uint32_t rb = (resid >> (8 * q)) & 0xFFu;
      const int32_t o = (int32_t)((uint32_t)lut[v[q] & 0xFF] + (uint32_t)lut[256 + rb] - (uint32_t)g.add_zp);
      v[q] = min(max(o, tlo), thi);
    }
    if (st) st_i8<V>(g.add_out + off, v, g.nt);
  }
  if (g.has_clip) {
#pragma unroll
    for (int q = 0; q < V; ++q) v[q] = min(max(v[q], g.clip_lo), g.clip_hi);
    if (st && !(g.ablate & 64)) st_i8<V>(g.clip_out + off, v, g.nt);
  }
}


// LDS tile [rows][64 B], 16-byte chunk c of row r stored at chunk c ^ ((r >> 2) & 3):
// the 16-lane groups of ds_read_b128 then hit 16 distinct bank slots.
__device__ __forceinline__ int lds_off(int row, int chunk) { return row * kBK + ((chunk ^ ((row >> 2) & 3)) << 4); }

// Same for stages of SBK = 64 or 128 bytes per row.  128-byte rows: chunk c of row r at
// chunk c ^ ((r >> 1) & 7) (two rows per 256-byte bank period, 8 row pairs per 16 lanes).
template <int SBK>
__device__ __forceinline__ int lds_off_w(int row, int chunk) {
  if constexpr (SBK == 64) return lds_off(row, chunk);
  else return row * SBK + ((chunk ^ ((row >> 1) & 7)) << 4);
}


// XCD-aware tile order: workgroup L runs on XCD L % 8, so XCD x takes the N tiles x, x+8,
// x+16, ... and for each of them all M tiles back to back: the workgroups that share an
// N tile (the same im2col B rows) run close together on one XCD and hit its L2.
__device__ __forceinline__ void tile_of(const GemmArgs& g, int& mt, int& nt) {
  const int L = blockIdx.x;
  if (!g.xcd_order) {  // plain order (N tiles fastest), for A/B measurements
    mt = L / g.ntiles8;
    nt = L - mt * g.ntiles8;
    return;
  }
  const int local = L >> 3;
  mt = local % g.mtiles;
  if (g.xcd_order == 2) {  // contiguous N-tile chunks per XCD (A/B: adjacent tiles share an L2)
    nt = (L & 7) * (g.ntiles8 >> 3) + local / g.mtiles;
    return;
  }
  nt = (local / g.mtiles) * 8 + (L & 7);
}

// kMode: 0 = whole K + epilogue; 1 = split-K partial (raw accumulators to g.ws);
//        2 = sum the split-K partials of this tile + epilogue (no main loop).


// kWide (im2col LDS-DMA path): 128-byte K stages instead of 64, i.e. half the
// barrier-separated steps of long reductions (each step pays a fixed LDS / barrier / address
// latency that the 1-2 workgroups per CU of the small-grid layers cannot hide).
// BN = 256 (image tiles of 65..256 pixels, conv blocks only): each wave owns 4 32-col tiles, and a
// tile's 64 channels x one image are one contiguous run of every NCHW record (see the flat
// epilogue): on 14x14 planes such runs store 2x faster than 128-column tiles that cross images
// (tools/probe_store3.hip, profiles/r02j_store_patterns.txt).
template <int MT, bool kIm2col, bool kBlock, int kMode = 0, int kRing = 3, bool kWide = false, int BN = 128>
__global__ __launch_bounds__(kGemmThreads, BN == 256 ? (kWide ? 1 : 2)
                                           : MT == 1 ? (kWide ? (kRing == 3 ? 2 : 1) : kRing == 3 ? 4 : kRing == 4 ? 3 : 2)
                                                     : (kWide ? 1 : 2)) void
gemm_i8_kernel(GemmArgs g) {
  static_assert(!kWide || (kIm2col && (MT == 1 || (kBlock && kMode == 0 && kRing == 3))), "wide stages: im2col");
  static_assert(BN == 128 || (BN == 256 && MT == 1 && kIm2col && kBlock && kMode == 0), "256-column tiles: conv blocks");
  constexpr int BM = 64 * MT;   // rows of A per block (2 waves along M, MT 32-row tiles each)
  constexpr int NJ = BN / 64;   // 32-col tiles per wave (2 waves along N)
  constexpr int kStr = BN + 4;  // dwords per LDS row of the epilogue tile (breaks the 64-bank period)
  constexpr int kFlat = BM * BN / 1024;  // 4-element groups per thread of the flat epilogue
  // 4-column epilogues: kLPR lanes per tile row (4 columns each), kRPI rows per pass, kRows passes
  constexpr int kLPR = BN / 4, kRPI = kGemmThreads / kLPR, kRows = BM / kRPI;
  constexpr int A_CHUNKS = BM * kBK / 16 / kGemmThreads;  // 16-byte loads per thread per stage (plain path)
  constexpr int B_CHUNKS = BN * kBK / 16 / kGemmThreads;
  constexpr int SBK = kWide ? 2 * kBK : kBK;              // K bytes per stage
  constexpr int CPR = SBK / 16;                           // 16-byte chunks per stage row
  constexpr int RPP = kGemmThreads / CPR;                 // stage rows per pass of all threads
  constexpr int A_DMA = BM / RPP, B_DMA = BN / RPP;       // LDS-DMA loads per thread per stage
  constexpr int kStageBytes = (BM + BN) * SBK;
  // kRing: LDS-DMA stages of the im2col path (kRing - 1 in flight); the plain path double-buffers
  constexpr int kStage = (kIm2col ? kRing : 2) * kStageBytes;
  constexpr int kEpi = BM * kStr * 4 + BM * (int)sizeof(EpiRow) + (kBlock ? 512 * 4 + 16 : 0);  // + flat sink slot
  __shared__ __attribute__((aligned(16))) int8_t smem[kStage > kEpi ? kStage : kEpi];
  __shared__ int s_fast;  // tile-uniform: every row's requantize takes the mul_hi form (shift <= -2)
  int8_t* As = smem;
  int8_t* Bs = smem + 2 * BM * kBK;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  [[maybe_unused]] const int abl = g.ablate;
  if (kBlock && tid == 0) s_fast = 1;  // visible after the first barrier; only cleared later
  int mtile, ntile;
  tile_of(g, mtile, ntile);
  if (ntile >= g.ntiles) return;  // padding of the N-tile count to a multiple of 8
  const int m0 = mtile * BM;
  const int n0 = ntile * g.tcols;
  // per-row epilogue constants (threads < BM, one row each), loaded up front: they land
  // during the main loop
  // (raw loads from a dummy word where an array is absent: the per-row/scalar choice is
  // made at the epilogue, so no path waits for the loads here)
  EpiRow row_pre{};
  const bool rq_axis = g.rq.mode >= TK_RQ_AXIS_UPWARD;
  if (kMode != 1 && tid < BM) {
    const int row = min(m0 + tid, g.M - 1);
    auto raw = [&](const int32_t* p, bool use) { return ldg(use ? p + row : tk_zero_words); };
    row_pre.ra = (uint32_t)raw(g.RA, g.RA != nullptr);
    row_pre.za = (uint32_t)raw(g.zA_vec, g.zA_vec != nullptr);
    if (kBlock && g.ch_is_row) {
      row_pre.bias = raw(g.bias, true);
      row_pre.m = raw(g.rq.ms, rq_axis);
      row_pre.s = raw(g.rq.ss, rq_axis);
      row_pre.zp = raw(g.rq.zps, g.rq.zps != nullptr);
    }
  }
  // residual bytes of every row this thread writes (4-column and flat epilogue paths).  kNR
  // loads, every one issued (a thread with nothing to join reads the zero words), so that the
  // counted waits below know them: on the LDS-DMA path they go out right after the prologue's
  // stages -- the stage waits let them stay in flight, the epilogue stores its conv / bias_add /
  // requantize records before it needs them -- because in the network the residual is a record
  // written several kernels earlier and comes from HBM behind the CU's stores (the 56x56
  // expands ran 115 us with a cached residual and 153 us with a cold one, r05w); elsewhere
  // they are issued here, before the main loop.
  static_assert(kFlat == kRows, "one residual word per 4-element group");
  constexpr int kNR = kBlock && kMode != 1 ? kFlat : 0;
  constexpr bool kLateResid = kNR > 0 && kIm2col && kMode != 2;
  uint32_t resid_pre[kFlat > kRows ? kFlat : kRows];
  auto issue_resid = [&]() __attribute__((always_inline)) {
    if constexpr (kNR > 0) {
      const uint32_t* zw = reinterpret_cast<const uint32_t*>(tk_zero_words);
      const int hw = g.OH * g.OW;
      if (g.has_add && g.ipt) {
        // flat epilogue: 4 consecutive elements of an image run per group (see there)
        const int run = min(BM, g.M - m0) * hw;
#pragma unroll
        for (int k = 0; k < kFlat; ++k) {
          const int gi = tid + kGemmThreads * k;
          const int kk = gi / (16 * hw), f = (gi - kk * 16 * hw) * 4;
          const int img = n0 / hw + kk;
          const bool ok = kk < g.ipt && img < g.N / hw && f < run;
          resid_pre[k] = ldg(ok ? reinterpret_cast<const uint32_t*>(g.add_res + ((int64_t)img * g.M + m0) * hw + f) : zw);
        }
      } else if (g.has_add && g.vecw >= 4) {
        const int col = n0 + (tid % kLPR) * 4;
        const int img = col / hw;
        const int64_t cbase = (int64_t)img * g.M * hw + (col - img * hw);
#pragma unroll
        for (int k = 0; k < kRows; ++k) {
          const int row = m0 + tid / kLPR + kRPI * k;
          const bool ok = col < g.N && row < g.M;
          resid_pre[k] = ldg(reinterpret_cast<const uint32_t*>(g.add_res + (ok ? cbase + (int64_t)row * hw : 0)));
        }
      } else {
#pragma unroll
        for (int k = 0; k < kNR; ++k) resid_pre[k] = ldg(zw);
      }
    }
  };
  if constexpr (!kLateResid) issue_resid();
  const int kc = tid & 3;  // this thread's 16-byte chunk within a K stage

  // ---- per-thread im2col state for the B rows it loads
  int b_img[B_DMA], b_ih0[B_DMA], b_iw0[B_DMA];
  bool b_valid[B_DMA];
#pragma unroll
  for (int t = 0; t < B_DMA; ++t) {
    int row = tid / CPR + t * RPP;
    int p = n0 + row;
    b_valid[t] = p < g.N && row < g.tcols;
    if (kIm2col) {
      const uint32_t pp = b_valid[t] ? p : 0;
      const int hw = g.OH * g.OW;
      const int img = g.mg_hw ? (int)(((uint64_t)pp * g.mg_hw) >> 40) : (int)(pp / (uint32_t)hw);
      const uint32_t rem = pp - img * hw;
      const int oh = g.mg_ow ? (int)(((uint64_t)rem * g.mg_ow) >> 40) : (int)(rem / (uint32_t)g.OW);
      const int ow = rem - oh * g.OW;
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
#pragma unroll
    for (int t = 0; t < B_CHUNKS; ++t) {
      int row = (tid >> 2) + t * (kGemmThreads / 4);
      rb[t] = *reinterpret_cast<const v4i*>(g.B + (int64_t)(n0 + row) * g.ldb + k0 + kc * 16);
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

  v16i acc[MT][NJ];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = v16i{0};

  // partial tiles live in g.ws in register order: v4i r4 of fragment (i, j) of thread tid
  constexpr int kTileInts = MT * 2 * 16 * kGemmThreads;
  const int64_t tile = (int64_t)mtile * g.ntiles + ntile;
  if constexpr (kMode == 2) {
    // sum the partial tiles; two splits' loads are issued together (MT = 1: 16 x 16 B
    // in flight per lane) so the reduction pays the L2 latency once per pair
    constexpr int kPair = MT == 1 ? 2 : 1;
    auto add_tile = [&](const v4i* t) {
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r4 = 0; r4 < 4; ++r4) {
            const v4i u = t[(i * 2 + j) * 4 + r4];
            acc[i][j][4 * r4] += u.x;
            acc[i][j][4 * r4 + 1] += u.y;
            acc[i][j][4 * r4 + 2] += u.z;
            acc[i][j][4 * r4 + 3] += u.w;
          }
    };
    int sp = 0;
    for (; sp + kPair <= g.splits; sp += kPair) {
      v4i t[kPair][MT * 2 * 4];
#pragma unroll
      for (int p = 0; p < kPair; ++p) {
        const v4i* src = reinterpret_cast<const v4i*>(g.ws + (tile * g.splits + sp + p) * kTileInts);
#pragma unroll
        for (int f = 0; f < MT * 2 * 4; ++f) t[p][f] = src[f * kGemmThreads + tid];
      }
#pragma unroll
      for (int p = 0; p < kPair; ++p) add_tile(t[p]);
    }
    for (; sp < g.splits; ++sp) {
      const v4i* src = reinterpret_cast<const v4i*>(g.ws + (tile * g.splits + sp) * kTileInts);
      v4i t[MT * 2 * 4];
#pragma unroll
      for (int f = 0; f < MT * 2 * 4; ++f) t[f] = src[f * kGemmThreads + tid];
      add_tile(t);
    }
  }
  int kt0 = 0, nk = g.k_pad / SBK;
  if constexpr (kMode == 1) {
    kt0 = blockIdx.z * g.kper;
    nk = min(nk, kt0 + g.kper);
  }
  // MFMAs of one staged K step (2 x K=32) from LDS
  // every fragment of the stage is read before the first MFMA: one LDS round trip per
  // stage instead of one per K=32 half (small grids run 1-2 workgroups per CU, so the
  // LDS latency is not hidden by other waves)
  constexpr int KS = SBK / 32;  // K = 32 MFMA steps per stage
  struct Frags {
    v4i a[KS][MT], b[KS][NJ];
  };
  auto read_frags = [&](const int8_t* a, const int8_t* b, Frags& f) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int chunk = 2 * ks + (lane >> 5);
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        int row = wm * 32 * MT + i * 32 + (lane & 31);
        f.a[ks][i] = *reinterpret_cast<const v4i*>(a + lds_off_w<SBK>(row, chunk));
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        int row = wn * (BN / 2) + j * 32 + (lane & 31);
        f.b[ks][j] = *reinterpret_cast<const v4i*>(b + lds_off_w<SBK>(row, chunk));
      }
    }
  };
  auto mfma_frags = [&](const Frags& f) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(f.a[ks][i], f.b[ks][j], acc[i][j], 0, 0, 0);
  };
  auto mma_stage = [&](const int8_t* a, const int8_t* b) {
    Frags f;
    read_frags(a, b, f);
    __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead of the MFMAs (the scheduler interleaves them)
    mfma_frags(f);
  };

  if constexpr (kMode != 2 && kIm2col) {
#ifdef TK_ABLATION_BUILD
    const int ablate = __builtin_amdgcn_readfirstlane(g.ablate);  // profiling builds only
#else
    constexpr int ablate = 0;  // the main-loop ablation branches compile away
#endif
    // ---- LDS-DMA pipeline (conv): a kRing-stage ring filled by global_load_lds_dwordx4 with
    // kRing - 1 stages in flight across the barrier (counted vmcnt + raw s_barrier).
    // The LDS image is lane-linear (lane l of a wave-instruction lands at base + 16 l =
    // row l/4, slot l%4), so the bank swizzle of lds_off goes on the SOURCE: slot s of row r
    // holds chunk s ^ ((r >> 2) & 3), i.e. lane l loads chunk (l & 3) ^ ((l >> 4) & 3).
    // Out-of-bounds taps read a row of the input zero point; rows past N and K padding
    // (whose weights are 0) read it too.
    // (wide: 8 rows of 128 B per wave-instruction, slot s of row r holds chunk s ^ ((r >> 1) & 7))
    const int cl = kWide ? ((lane & 7) ^ ((4 * wave + (lane >> 4)) & 7)) : ((lane & 3) ^ ((lane >> 4) & 3));
    const int8_t* fill_src = reinterpret_cast<const int8_t*>(tk_fill_rows.v + 16 * (g.fill & 0xFFu));
    const int wave_u = __builtin_amdgcn_readfirstlane(wave);
    const int8_t* a_src[A_DMA];
#pragma unroll
    for (int t = 0; t < A_DMA; ++t)
      a_src[t] = g.A + (int64_t)(m0 + tid / CPR + t * RPP) * g.lda + kt0 * SBK + cl * 16;
    const int nst = nk - kt0;
    auto pipeline = [&](auto&& issue) {
#pragma unroll
      for (int st = 0; st < kRing - 1; ++st)
        if (st < nst) issue(st);
      if constexpr (kLateResid) {
        // younger than the prologue's stages (see there): the counted stage waits below let the
        // kNR residual loads stay in flight only if they are issued after every prologue DMA, so
        // the scheduler may not move them across (the plain loads and the LDS-DMAs are otherwise
        // independent to it)
        __builtin_amdgcn_sched_barrier(0);
        issue_resid();
        __builtin_amdgcn_sched_barrier(0);
      }
      int cur = 0, nxt = kRing - 1;  // ring slots of stage it and of stage it + kRing - 1
      // one step: retire stage it (A_DMA + B_DMA LDS-DMAs per thread and stage) with `pending`
      // later stages still in flight, barrier (stage it visible to all waves; the slot read in
      // step it-1 is free), fragments of stage it first so that their LDS latency overlaps the
      // next issue, then the MFMAs
      // extra: the residual loads still allowed in flight (steps retiring a prologue stage)
      auto step = [&](int it, int pending, int extra) __attribute__((always_inline)) {
        if (extra) wait_vm_any(pending * (A_DMA + B_DMA) + extra);
        else wait_vm(pending * (A_DMA + B_DMA));
        if (ablate & 4096) {
        } else if (ablate & 1024) asm volatile("s_barrier" ::: "memory");
        else lds_barrier();
        const int8_t* a = smem + cur * kStageBytes;
        Frags f;
        if (!(ablate & 2048)) read_frags(a, a + BM * SBK, f);
        __builtin_amdgcn_sched_barrier(0);
        if (it + kRing - 1 < nst) {
          issue(nxt);
          nxt = nxt == kRing - 1 ? 0 : nxt + 1;
        }
        __builtin_amdgcn_sched_barrier(0);
        if (!(ablate & 512)) mfma_frags(f);
        cur = cur == kRing - 1 ? 0 : cur + 1;
      };
      // steady state with a compile-time wait count, then the last kRing - 2 stages
      const int steady = nst - (kRing - 2);
      constexpr int kLate = kLateResid ? kNR : 0;
      int it = 0;
      for (; it < steady && it < kRing - 1; ++it) step(it, kRing - 2, kLate);
      for (; it < steady; ++it) step(it, kRing - 2, 0);
      for (; it < nst; ++it) step(it, nst - 1 - it, it < kRing - 1 ? kLate : 0);
    };
    auto issue_a = [&](int8_t* sa) {
#pragma unroll
      for (int t = 0; t < A_DMA; ++t) {
        if (!(ablate & 128))
          __builtin_amdgcn_global_load_lds((const void*)a_src[t], (void*)(sa + ((RPP / 4) * wave_u + RPP * t) * SBK),
                                           16, 0, 0);
        a_src[t] += SBK;
      }
    };
    if (kWide || g.unitap) {
      // lane-constant part of the source (pixel + the lane's channel group) and the taps
      // that are in bounds for the lane's rows; the stage part (channel group, tap) is uniform
      const int8_t* lane_base[B_DMA];
      uint64_t tmask[B_DMA];
#pragma unroll
      for (int t = 0; t < B_DMA; ++t) {
        const int64_t pix = ((int64_t)b_img[t] * g.H + b_ih0[t]) * g.W + b_iw0[t];
        lane_base[t] = g.B + (pix + (int64_t)cl * g.in_pix) * 16;
        uint32_t rows = 0, cols = 0;
        for (int kh = 0; kh < g.KH; ++kh) {
          const int ih = b_ih0[t] + kh * g.dh;
          rows |= (uint32_t)(ih >= 0 && ih < g.H) << kh;
        }
        for (int kw = 0; kw < g.KW; ++kw) {
          const int iw = b_iw0[t] + kw * g.dw;
          cols |= (uint32_t)(iw >= 0 && iw < g.W) << kw;
        }
        uint64_t m = 0;
        for (int kh = 0; kh < g.KH; ++kh)
          if ((rows >> kh) & 1) m |= (uint64_t)cols << (kh * g.KW);
        tmask[t] = b_valid[t] ? m : 0;
      }
      int cg, kh, kw;  // uniform: channel group of the stage's first chunk, tap
      {
        const int k0 = kt0 * SBK;
        const int tap = k0 / g.cin_pad;
        cg = (k0 - tap * g.cin_pad) >> 4;
        kh = tap / g.KW;
        kw = tap - kh * g.KW;
      }
      const int64_t grp_bytes = g.in_pix * 16;
      const int64_t row_bytes = (int64_t)g.dh * g.W * 16;
      const int KW = g.KW, cgroups = g.cgroups, dw16 = g.dw * 16;
      int tap = kh * KW + kw;
      int64_t soff = cg * grp_bytes + kh * row_bytes + (int64_t)kw * dw16;
      pipeline([&](int slot) {
        int8_t* sa = smem + slot * kStageBytes;
        issue_a(sa);
        int8_t* sb = sa + BM * SBK;
        const bool grp_ok = cg + cl < cgroups;  // K padding of a 1x1 conv with cin_pad % 64 != 0
#pragma unroll
        for (int t = 0; t < B_DMA; ++t) {
          const bool ok = ((tmask[t] >> tap) & 1) && grp_ok;
          const int8_t* src = ok ? lane_base[t] + soff : fill_src;
          if (!(ablate & 256))
            __builtin_amdgcn_global_load_lds((const void*)src, (void*)(sb + ((RPP / 4) * wave_u + RPP * t) * SBK),
                                             16, 0, 0);
        }
        cg += CPR;
        soff += CPR * grp_bytes;
        if (cg >= cgroups) {
          cg = 0;
          ++tap;
          if (++kw == KW) kw = 0, ++kh;
          soff = kh * row_bytes + (int64_t)kw * dw16;
        }
      });
    } else if constexpr (!kWide) {
      // general walk: the thread's chunk is (tap, channel offset c0) with the taps in
      // (kh, kw) order; advanced 64 bytes per stage without divisions
      int c0, kh, kw;
      {
        const int kg = kt0 * kBK + cl * 16;
        const int tap = kg / g.cin_pad;
        c0 = kg - tap * g.cin_pad;
        kh = tap / g.KW;
        kw = tap - kh * g.KW;
      }
      int b_pix[B_CHUNKS];
#pragma unroll
      for (int t = 0; t < B_CHUNKS; ++t) b_pix[t] = (b_img[t] * g.H + b_ih0[t]) * g.W + b_iw0[t];
      pipeline([&](int slot) {
        int8_t* sa = smem + slot * kStageBytes;
        issue_a(sa);
        int8_t* sb = sa + BM * kBK;
        const bool tap_ok = kh < g.KH;
        const int dy = kh * g.dh, dx = kw * g.dw;
        const int64_t plane = (int64_t)(c0 >> 4) * g.in_pix;
#pragma unroll
        for (int t = 0; t < B_CHUNKS; ++t) {
          const int ih = b_ih0[t] + dy;
          const int iw = b_iw0[t] + dx;
          const bool inb = ih >= 0 && ih < g.H && iw >= 0 && iw < g.W;
          const int8_t* src = g.B + (plane + b_pix[t] + dy * g.W + dx) * 16;
          src = (b_valid[t] && tap_ok && inb) ? src : fill_src;
          if (!(ablate & 256))
            __builtin_amdgcn_global_load_lds((const void*)src, (void*)(sb + (16 * wave_u + 64 * t) * kBK), 16, 0, 0);
        }
        c0 += kBK;
        while (c0 >= g.cin_pad) {
          c0 -= g.cin_pad;
          if (++kw == g.KW) kw = 0, ++kh;
        }
      });
    }
  }
  if constexpr (kMode != 2 && !kIm2col) {
  load_stage(kt0 * kBK);
  store_stage(0);
  __syncthreads();

  for (int kt = kt0; kt < nk; ++kt) {
    const int buf = (kt - kt0) & 1;
    if (kt + 1 < nk) load_stage((kt + 1) * kBK);  // issue early, land under the MFMAs
    mma_stage(As + buf * BM * kBK, Bs + buf * BN * kBK);
    if (kt + 1 < nk) store_stage(buf ^ 1);
    __syncthreads();
  }
  }  // plain path
  // every load issued so far (LDS-DMA stages, the row constants) has landed: a wait the
  // compiler sees (the ring's counted waits are inline asm), so that it does not add
  // conservative vmcnt(0) waits before the epilogue's LDS reads.  The late residual loads (the
  // youngest, see issue_resid) may stay in flight: vmcnt(kNR)
  if constexpr (kLateResid) {
    __builtin_amdgcn_s_waitcnt(0x0F70 | (kNR & 15) | ((kNR >> 4) << 14));
  } else {
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  }
  if constexpr (kMode == 1) {
    v4i* dst = reinterpret_cast<v4i*>(g.ws + (tile * gridDim.z + blockIdx.z) * kTileInts);
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4)
          dst[((i * 2 + j) * 4 + r4) * kGemmThreads + tid] =
              v4i{acc[i][j][4 * r4], acc[i][j][4 * r4 + 1], acc[i][j][4 * r4 + 2], acc[i][j][4 * r4 + 3]};
    return;
  }

  // ---- epilogue: the whole BM x BN accumulator tile is staged through LDS.
  //  (1) every wave dumps its raw accumulators to LDS [row][col]; threads < BM stage their
  //      row's constants (bias, multiplier, shift, zero points, fold term) next to it;
  //  (2) every thread owns fixed columns (4 consecutive ones when the plane length is a
  //      multiple of 4, else 1) and walks rows: per row, zero-point folding, then each record
  //      is stored as soon as it is complete.  The lanes of a wave run along the columns, so
  //      every store instruction writes whole 128-byte lines of one or two rows (int32: 16 B
  //      per lane, int8: 4 B per lane); the final int8 values go back to the LDS slot;
  //  (3) the shadow for the next conv: each item gathers 16 channels of one pixel (a wave
  //      reads 64 consecutive columns per row: conflict-free) into a 16 B store; the lanes'
  //      stores are contiguous (channel-blocked layout).
  if (g.ablate & 4) return;
  int32_t* tileI = reinterpret_cast<int32_t*>(smem);
  EpiRow* rowc = reinterpret_cast<EpiRow*>(smem + BM * kStr * 4);
  int32_t* lut = reinterpret_cast<int32_t*>(smem + BM * kStr * 4 + BM * sizeof(EpiRow));  // [2][256]
  const int hw = g.OH * g.OW;
  const bool zb_vec = g.zB_vec != nullptr, has_rb = g.RB != nullptr;
  const bool simple_fold = !zb_vec && !has_rb;
  lds_barrier();  // staging buffers are free
  if (tid < BM) {
    EpiRow r = row_pre;
    if (!g.RA) r.ra = 0;
    if (!g.zA_vec) r.za = (uint32_t)g.zA;
    if (kBlock && g.ch_is_row) {
      if (!rq_axis) r.m = g.rq.multiplier, r.s = g.rq.shift;
      if (!g.rq.zps) r.zp = g.rq.zp_in;
    }
    r.fold = (uint32_t)g.k_eff * r.za * (uint32_t)g.zB - (uint32_t)g.zB * r.ra;
    if (kBlock && g.ch_is_row && r.s > -2) s_fast = 0;
    rowc[tid] = r;
  }
  if (kBlock && g.has_add) {
    // RequantizeOrUpcast of every 8-bit value of both qnn.add operands (op_common.h:186-200)
    const int32_t x = g.rq.qmin == 0 ? tid : (int32_t)(int8_t)(uint8_t)tid;
    lut[tid] = g.add_up_b ? x : rq_tensor(x, g.add_pb);
    lut[256 + tid] = g.add_up_r ? x : rq_tensor(x, g.add_pr);
  }
#pragma unroll
  for (int i = 0; i < MT; ++i) {
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int lc = wn * (BN / 2) + j * 32 + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int lr = wm * 32 * MT + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        tileI[lr * kStr + lc] = acc[i][j][r];
      }
    }
  }
  lds_barrier();

  bool done = false;
  if constexpr (kBlock) {
    if (g.ipt && (BN == 256 || !(g.ablate & 0x7F))) {
      // ---- flat epilogue (image-aligned tiles, planes of 1..64 pixels): for image kk of the
      // tile, its channels m0.. and all OH*OW pixels are one contiguous run of the NCHW
      // records, `run` elements long.  Group gi = 4 consecutive elements of one run: b128
      // stores of the int32 records and b32 stores of the 8-bit ones, contiguous across lanes
      // (whole 128-byte lines), each element gathered from its (row, column) slot of the tile.
      done = true;
      const int hw = g.OH * g.OW;
      const int run = min(BM, g.M - m0) * hw;
      const int img0 = n0 / hw, nimg = g.N / hw;
      const uint32_t n4 = g.out_elems * 4u;
      const auto r_conv = rec_rsrc(g.C, n4), r_bias = rec_rsrc(g.bias_out, n4);
      const auto r_rq = rec_rsrc(g.rq_out, g.out_elems);
      const auto r_add = rec_rsrc(g.add_out, g.has_add ? g.out_elems : 0u);
      const auto r_clip = rec_rsrc(g.clip_out, g.has_clip ? g.out_elems : 0u);
      const int32_t qmin = (int32_t)g.rq.qmin, qmax = (int32_t)g.rq.qmax, zpo = g.rq.zp_out;
      const int32_t add_zp = g.add_zp, clip_lo = g.clip_lo, clip_hi = g.clip_hi;
      const bool has_add = g.has_add, has_clip = g.has_clip;
      const int mode = g.rq.mode;
      const int ipt = g.ipt, Mrows = g.M;  // (the lambda must not reference g: that forces it to scratch)
      // x / hw as (x * mg) >> 40, exact for x * hw < 2^40 (x here < 2^16)
      const uint64_t mg = ((1ull << 40) + (uint64_t)hw - 1) / (uint64_t)hw;
      auto groups = [&](auto fast_c, auto rowu_c) __attribute__((always_inline)) {
        constexpr bool FAST = decltype(fast_c)::value;
        // ROWU (hw % 4 == 0): a group's 4 elements lie in one row, 16-byte aligned in LDS: one
        // b128 read of the tile, one row of constants
        constexpr bool ROWU = decltype(rowu_c)::value;
#pragma unroll
        for (int k = 0; k < kFlat; ++k) {
          const int gi = tid + kGemmThreads * k;
          const int kk = (int)((((uint64_t)(gi >> 4)) * mg) >> 40), f = (gi - kk * 16 * hw) * 4;
          if (!(kk < ipt && img0 + kk < nimg && f < run)) continue;  // past a run or the tile's images
          const uint32_t o = (uint32_t)(((img0 + kk) * Mrows + m0) * hw + f);
          const int r0 = (int)(((uint64_t)f * mg) >> 40), p0 = f - r0 * hw;
          int slot[4];
          EpiRow rr[4];
          v4u v;
          if constexpr (ROWU) {
            slot[0] = r0 * kStr + kk * hw + p0;
            rr[0] = rowc[r0];
#pragma unroll
            for (int e = 1; e < 4; ++e) slot[e] = slot[0] + e, rr[e] = rr[0];
            v = *reinterpret_cast<const v4u*>(tileI + slot[0]);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              int re = r0, pe = p0 + e;
#pragma unroll
              for (int w = 0; w < 3; ++w)  // one row change per group when hw >= 4, up to 3 below
                if (pe >= hw) pe -= hw, ++re;
              slot[e] = re * kStr + kk * hw + pe;
              rr[e] = rowc[re];
              v[e] = (uint32_t)tileI[slot[e]];
            }
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += rr[e].fold;
          if (!TK_ABL(2)) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v), r_conv, o * 4u, 0, kAuxNT);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += (uint32_t)rr[e].bias;
          if (!TK_ABL(2)) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v), r_bias, o * 4u, 0, kAuxNT);
          int32_t q[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int32_t t = (int32_t)(v[e] - (uint32_t)rr[e].zp);
            int32_t y;
            if constexpr (FAST) {
              const int sh2 = -rr[e].s - 1;
              y = (int32_t)((uint32_t)__mulhi(t, rr[e].m) + (1u << (sh2 - 1))) >> sh2;
            } else {
              y = rq_core(t, mode, rr[e].m, rr[e].s);
            }
            q[e] = clamp_i32((int32_t)((uint32_t)zpo + (uint32_t)y), qmin, qmax);
          }
          if (!TK_ABL(2)) __builtin_amdgcn_raw_buffer_store_b32(pack4u(q[0], q[1], q[2], q[3]), r_rq, o, 0, kAuxNT);
          if (has_add) {
            // qnn.add (src/relay/qnn/op/add.cc:40-96): RQ(block) + RQ(residual) - zp_out
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const uint32_t rb = (resid_pre[k] >> (8 * e)) & 0xFFu;
              q[e] = clamp_i32(TK_ABL(8192) ? q[e] + (int32_t)rb - add_zp : lut[q[e] & 0xFF] + lut[256 + rb] - add_zp,
                               qmin, qmax);
            }
            if (!TK_ABL(16384 | 2)) __builtin_amdgcn_raw_buffer_store_b32(pack4u(q[0], q[1], q[2], q[3]), r_add, o, 0, kAuxNT);
          }
          if (has_clip) {
#pragma unroll
            for (int e = 0; e < 4; ++e) q[e] = clamp_i32(q[e], clip_lo, clip_hi);
            if (!TK_ABL(2)) __builtin_amdgcn_raw_buffer_store_b32(pack4u(q[0], q[1], q[2], q[3]), r_clip, o, 0, kAuxNT);
          }
          if constexpr (ROWU) {
            *reinterpret_cast<v4i*>(tileI + slot[0]) = v4i{q[0], q[1], q[2], q[3]};
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) tileI[slot[e]] = q[e];
          }
        }
      };
      // Lean form for planes of >= 16 pixels, hw % 4 == 0 (the 14x14 256-column tiles, 8x8): the
      // group -> (image, row, column) walk advances incrementally (256 groups = 1024 elements per
      // step: dr rows + dp columns, at most one image wrap since an image run holds >= 256
      // groups), one b128 LDS read of the 4 values and one row of constants per group, the
      // residual join / clip decided at compile time.  The epilogue is VALU-issue-bound at the 1-2
      // waves per SIMD of these launches (profiles/r02m_flat_epilogue_ablations.txt).
      // XR (hw % 4 != 0, the 7x7 stage): a group may cross into the next row; its elements then
      // take that row's constants (per-element selects) and four b32 tile reads.
      auto lean = [&](auto fast_c, auto add_c, auto clip_c, auto xr_c) __attribute__((always_inline)) {
        constexpr bool FAST = decltype(fast_c)::value, ADD = decltype(add_c)::value, CLIP = decltype(clip_c)::value;
        constexpr bool XR = decltype(xr_c)::value;
        const int runG = 16 * hw;             // 4-element groups per image run (BM = 64 rows)
        const int dr = 1024 / hw, dp = 1024 - dr * hw;
        // walk state of a group; its LDS slot is read unconditionally (in bounds of the epilogue
        // area for every lane), lanes past a run store out of range and write back to the sink
        int fg = tid, kk = 0;                  // group within the image run (tid < 256 <= runG)
        int r0 = (int)(((uint64_t)(4 * fg) * mg) >> 40);
        int p0 = 4 * fg - r0 * hw;
        auto slot_of = [&]() __attribute__((always_inline)) { return r0 * kStr + kk * hw + p0; };
        // element e of a group starting at column p0 lies in the next row when p0 + e >= hw
        auto load = [&](int sl, int r, int p, v4u& v, EpiRow& ra, EpiRow& rb) __attribute__((always_inline)) {
          if constexpr (XR) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = (uint32_t)tileI[sl + e + (p + e >= hw ? kStr - hw : 0)];
            ra = rowc[r];
            rb = rowc[min(r + 1, BM - 1)];
          } else {
            v = *reinterpret_cast<const v4u*>(tileI + sl);
            ra = rowc[r];
          }
        };
        // software pipeline by one group: group k+1's tile values and row constants are read
        // from LDS before group k's arithmetic and stores
        int sl = slot_of();
        v4u vn;
        EpiRow rn, rn1;
        load(sl, r0, p0, vn, rn, rn1);
#pragma unroll
        for (int k = 0; k < kFlat; ++k) {
          const bool ok = kk < ipt && img0 + kk < nimg && 4 * fg < run;
          const uint32_t o = (uint32_t)(((img0 + kk) * Mrows + m0) * hw + 4 * fg) | (ok ? 0u : kOffDrop);
          int32_t* wslot = ok ? tileI + sl : lut + 512;
          const int pc = p0;                   // this group's first column
          v4u v = vn;
          const EpiRow rr = rn, rr1 = rn1;
          if (k + 1 < kFlat) {
            fg += kGemmThreads;
            r0 += dr;
            p0 += dp;
            if (p0 >= hw) p0 -= hw, ++r0;
            if (fg >= runG) fg -= runG, ++kk, r0 -= BM;
            sl = slot_of();
            load(sl, r0, p0, vn, rn, rn1);
          }
          // per-element row constants (XR: elements past the row end take the next row's)
          uint32_t fold[4], zp[4];
          int32_t bias[4], m[4], sh[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const bool nx = XR && pc + e >= hw;
            fold[e] = nx ? rr1.fold : rr.fold;
            bias[e] = nx ? rr1.bias : rr.bias;
            zp[e] = nx ? (uint32_t)rr1.zp : (uint32_t)rr.zp;
            m[e] = nx ? rr1.m : rr.m;
            sh[e] = nx ? rr1.s : rr.s;
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += fold[e];
          if (!TK_ABL(2)) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v), r_conv, o * 4u, 0, kAuxNT);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += (uint32_t)bias[e];
          if (!TK_ABL(2)) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v), r_bias, o * 4u, 0, kAuxNT);
          int32_t q[4];
          if constexpr (FAST) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int sh2 = -sh[e] - 1;
              q[e] = clamp_i32(zpo + ((int32_t)((uint32_t)__mulhi((int32_t)(v[e] - zp[e]), m[e]) + (1u << (sh2 - 1))) >> sh2),
                               qmin, qmax);
            }
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              q[e] = clamp_i32((int32_t)((uint32_t)zpo + (uint32_t)rq_core((int32_t)(v[e] - zp[e]), mode, m[e], sh[e])),
                               qmin, qmax);
          }
          if (!TK_ABL(2)) __builtin_amdgcn_raw_buffer_store_b32(pack4u(q[0], q[1], q[2], q[3]), r_rq, o, 0, kAuxNT);
          if constexpr (ADD) {
            // qnn.add (src/relay/qnn/op/add.cc:40-96): RQ(block) + RQ(residual) - zp_out
            const uint32_t res = resid_pre[k];
#pragma unroll
            for (int e = 0; e < 4; ++e)
              q[e] = clamp_i32(lut[q[e] & 0xFF] + lut[256 + ((res >> (8 * e)) & 0xFFu)] - add_zp, qmin, qmax);
            if (!TK_ABL(2)) __builtin_amdgcn_raw_buffer_store_b32(pack4u(q[0], q[1], q[2], q[3]), r_add, o, 0, kAuxNT);
          }
          if constexpr (CLIP) {
#pragma unroll
            for (int e = 0; e < 4; ++e) q[e] = clamp_i32(q[e], clip_lo, clip_hi);
            if (!TK_ABL(2)) __builtin_amdgcn_raw_buffer_store_b32(pack4u(q[0], q[1], q[2], q[3]), r_clip, o, 0, kAuxNT);
          }
          if constexpr (XR) {
#pragma unroll
            for (int e = 0; e < 4; ++e) wslot[e + (ok && pc + e >= hw ? kStr - hw : 0)] = q[e];
          } else {
            *reinterpret_cast<v4i*>(wslot) = v4i{q[0], q[1], q[2], q[3]};
          }
        }
      };
      auto lean_fast = [&](auto fast_c, auto xr_c) __attribute__((always_inline)) {
        using T = std::true_type;
        using F = std::false_type;
        if (has_add) {
          if (has_clip) lean(fast_c, T{}, T{}, xr_c);
          else lean(fast_c, T{}, F{}, xr_c);
        } else {
          if (has_clip) lean(fast_c, F{}, T{}, xr_c);
          else lean(fast_c, F{}, F{}, xr_c);
        }
      };
      const bool fastrq = s_fast && (mode == TK_RQ_AXIS_UPWARD || mode == TK_RQ_TENSOR_UPWARD);
      if (TK_ABL(65536)) {
      } else if (hw % 4 == 0 && hw >= 16 && !TK_ABL(32768)) {
        if (fastrq) lean_fast(std::true_type{}, std::false_type{});
        else lean_fast(std::false_type{}, std::false_type{});
      } else if (hw >= 16 && !TK_ABL(32768 | 131072)) {
        if (fastrq) lean_fast(std::true_type{}, std::true_type{});
        else lean_fast(std::false_type{}, std::true_type{});
      } else if (hw % 4 == 0 && !TK_ABL(32768)) {
        if (fastrq) groups(std::true_type{}, std::true_type{});
        else groups(std::false_type{}, std::true_type{});
      } else {
        if (fastrq) groups(std::true_type{}, std::false_type{});
        else groups(std::false_type{}, std::false_type{});
      }
    } else if (g.fast_epi && simple_fold && s_fast && !(g.ablate & 0x7D)) {
      // ---- fast path (tile-uniform): 4 consecutive columns x rows (tid>>5) + 8k, every
      // record through a buffer descriptor (masked lanes get an out-of-range offset),
      // requantize in the mul_hi form: ((x - zp)·m + 2^(sh2-1)) >> sh2 over the high word
      done = true;
      const int c4 = (tid % kLPR) * 4;
      const int col = n0 + c4;
      const bool colok = col < g.N;
      const int img = col / hw;
      const uint32_t cbase = (uint32_t)img * (uint32_t)g.M * (uint32_t)hw + (uint32_t)(col - img * hw);
      const uint32_t n4 = g.out_elems * 4u;
      const auto r_conv = rec_rsrc(g.C, n4), r_bias = rec_rsrc(g.bias_out, n4);
      const auto r_rq = rec_rsrc(g.rq_out, g.out_elems);
      const auto r_add = rec_rsrc(g.add_out, g.has_add ? g.out_elems : 0u);
      const auto r_clip = rec_rsrc(g.clip_out, g.has_clip ? g.out_elems : 0u);
      const int32_t qmin = (int32_t)g.rq.qmin, qmax = (int32_t)g.rq.qmax, zpo = g.rq.zp_out;
      // kernel arguments the row loop needs, held in registers: read through `g` after a
      // store, the compiler reloads them (s_load + lgkmcnt(0), which also drains the LDS reads)
      const int32_t add_zp = g.add_zp, clip_lo = g.clip_lo, clip_hi = g.clip_hi;
      const bool want_shadow = g.shadow_out != nullptr;
      uint32_t offs[kRows];
#pragma unroll
      for (int k = 0; k < kRows; ++k) {
        const int row = m0 + tid / kLPR + kRPI * k;
        offs[k] = (colok && row < g.M) ? cbase + (uint32_t)row * (uint32_t)hw : kOffDrop;
      }
      auto rows = [&](auto add_c, auto clip_c, auto aux_c) __attribute__((always_inline)) {
        constexpr bool ADD = decltype(add_c)::value, CLIP = decltype(clip_c)::value;
        constexpr int AUX = decltype(aux_c)::value;
        if constexpr (ADD) {
          if (!TK_ABL(262144 | 2 | 8192 | 16384)) {
            // residual join: every row's conv / bias_add / requantize records first (3 kRows
            // stores), then the joins, whose residual words (issue_resid) land under those stores
            int32_t qs[kRows][4];
#pragma unroll
            for (int k = 0; k < kRows; ++k) {
              const int lr = tid / kLPR + kRPI * k;
              const EpiRow r = rowc[lr];
              const v4i t = *reinterpret_cast<const v4i*>(tileI + lr * kStr + c4);
              const uint32_t o = offs[k];
              v4u v = __builtin_bit_cast(v4u, t) + r.fold;
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v), r_conv, o * 4u, 0, AUX);
              v += (uint32_t)r.bias;
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v), r_bias, o * 4u, 0, AUX);
              const int sh2 = -r.s - 1;
              const uint32_t rnd = 1u << (sh2 - 1);
#pragma unroll
              for (int e = 0; e < 4; ++e)
                qs[k][e] = clamp_i32(zpo + ((int32_t)((uint32_t)__mulhi((int32_t)(v[e] - (uint32_t)r.zp), r.m) + rnd) >> sh2),
                                     qmin, qmax);
              __builtin_amdgcn_raw_buffer_store_b32(pack4u(qs[k][0], qs[k][1], qs[k][2], qs[k][3]), r_rq, o, 0, AUX);
            }
#pragma unroll
            for (int k = 0; k < kRows; ++k) {
              const int lr = tid / kLPR + kRPI * k;
              const uint32_t o = offs[k];
              int32_t q[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                // qnn.add (src/relay/qnn/op/add.cc:40-96): RQ(block) + RQ(residual) - zp_out
                const uint32_t rb = (resid_pre[k] >> (8 * e)) & 0xFFu;
                q[e] = clamp_i32(lut[qs[k][e] & 0xFF] + lut[256 + rb] - add_zp, qmin, qmax);
              }
              __builtin_amdgcn_raw_buffer_store_b32(pack4u(q[0], q[1], q[2], q[3]), r_add, o, 0, AUX);
              if constexpr (CLIP) {
#pragma unroll
                for (int e = 0; e < 4; ++e) q[e] = clamp_i32(q[e], clip_lo, clip_hi);
                __builtin_amdgcn_raw_buffer_store_b32(pack4u(q[0], q[1], q[2], q[3]), r_clip, o, 0, AUX);
              }
              if (want_shadow) *reinterpret_cast<v4i*>(tileI + lr * kStr + c4) = v4i{q[0], q[1], q[2], q[3]};
            }
            return;
          }
        }
#pragma unroll
        for (int k = 0; k < kRows; ++k) {
          const int lr = tid / kLPR + kRPI * k;
          const EpiRow r = rowc[lr];
          int32_t* slot = tileI + lr * kStr + c4;
          const v4i t = *reinterpret_cast<const v4i*>(slot);
          const uint32_t o = offs[k];
          if (TK_ABL(262144)) {
            // profiling: every record stored with no epilogue arithmetic (store side alone)
            const uint32_t b8 = pack4u(t.x, t.y, t.z, t.w);
            __builtin_amdgcn_raw_buffer_store_b128(t, r_conv, o * 4u, 0, AUX);
            __builtin_amdgcn_raw_buffer_store_b128(t, r_bias, o * 4u, 0, AUX);
            __builtin_amdgcn_raw_buffer_store_b32(b8, r_rq, o, 0, AUX);
            if constexpr (ADD) __builtin_amdgcn_raw_buffer_store_b32(b8 ^ resid_pre[k], r_add, o, 0, AUX);
            if constexpr (CLIP) __builtin_amdgcn_raw_buffer_store_b32(b8, r_clip, o, 0, AUX);
            continue;
          }
          // int32 wrap-around arithmetic in unsigned lanes (the reference accumulates mod 2^32)
          v4u v = __builtin_bit_cast(v4u, t) + r.fold;
          if (!TK_ABL(2)) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v), r_conv, o * 4u, 0, AUX);
          v += (uint32_t)r.bias;
          if (!TK_ABL(2)) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v), r_bias, o * 4u, 0, AUX);
          const int sh2 = -r.s - 1;
          const uint32_t rnd = 1u << (sh2 - 1);
          int32_t q[4];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            q[e] = clamp_i32(zpo + ((int32_t)((uint32_t)__mulhi((int32_t)(v[e] - (uint32_t)r.zp), r.m) + rnd) >> sh2),
                             qmin, qmax);
          if (!TK_ABL(2)) __builtin_amdgcn_raw_buffer_store_b32(pack4u(q[0], q[1], q[2], q[3]), r_rq, o, 0, AUX);
          if constexpr (ADD) {
            // qnn.add (src/relay/qnn/op/add.cc:40-96): RQ(block) + RQ(residual) - zp_out
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const uint32_t rb = (resid_pre[k] >> (8 * e)) & 0xFFu;
              q[e] = clamp_i32(TK_ABL(8192) ? q[e] + (int32_t)rb - add_zp : lut[q[e] & 0xFF] + lut[256 + rb] - add_zp,
                               qmin, qmax);
            }
            if (!TK_ABL(16384 | 2)) __builtin_amdgcn_raw_buffer_store_b32(pack4u(q[0], q[1], q[2], q[3]), r_add, o, 0, AUX);
          }
          if constexpr (CLIP) {
#pragma unroll
            for (int e = 0; e < 4; ++e) q[e] = clamp_i32(q[e], clip_lo, clip_hi);
            if (!TK_ABL(2)) __builtin_amdgcn_raw_buffer_store_b32(pack4u(q[0], q[1], q[2], q[3]), r_clip, o, 0, AUX);
          }
          if (want_shadow) *reinterpret_cast<v4i*>(slot) = v4i{q[0], q[1], q[2], q[3]};
        }
      };
      using T = std::true_type;
      using F = std::false_type;
      // always_inline: the epilogue lambdas must not become calls, which would take the address
      // of g and copy every kernel argument to scratch (a 4x slowdown measured)
      auto dispatch = [&](auto aux_c) __attribute__((always_inline)) {
        if (g.has_add) {
          if (g.has_clip) rows(T{}, T{}, aux_c);
          else rows(T{}, F{}, aux_c);
        } else {
          if (g.has_clip) rows(F{}, T{}, aux_c);
          else rows(F{}, F{}, aux_c);
        }
      };
      if (g.fast_epi == 2) dispatch(std::integral_constant<int, 0>{});
      else dispatch(std::integral_constant<int, kAuxNT>{});
    }
  }
  // zero-point folding of V columns: acc - zB[col]*RA[row] - zA[row]*RB[col] + K*zA[row]*zB[col]
  auto fold = [&](int32_t* v, const EpiRow& r, int col, int V) {
    if (simple_fold) {
      for (int q = 0; q < V; ++q) v[q] = (int32_t)((uint32_t)v[q] + r.fold);
    } else {
      for (int q = 0; q < V; ++q) {
        const int cq = min(col + q, g.N - 1);
        const uint32_t zb = zb_vec ? (uint32_t)g.zB_vec[cq] : (uint32_t)g.zB;
        const uint32_t rb = has_rb ? (uint32_t)g.RB[cq] : 0u;
        v[q] = (int32_t)((uint32_t)v[q] - zb * r.ra - r.za * rb + (uint32_t)g.k_eff * r.za * zb);
      }
    }
  };
  const bool store_on = !(g.ablate & 2);
  if (done) {
  } else if (g.vecw >= 4) {
    // 4 consecutive columns x rows (tid>>5) + 8k (BN = 256: (tid>>6) + 4k); the 4 never straddle
    // an image plane
    const int c4 = (tid % kLPR) * 4;
    const int col = n0 + c4;
    const bool colok = col < g.N;
    int64_t cbase, rstride;
    if (g.out_nchw) {
      const int img = col / hw;
      cbase = (int64_t)img * g.M * hw + (col - img * hw);
      rstride = hw;
    } else {
      cbase = col;
      rstride = g.ldc;
    }
    EpiRow cc[4] = {};
    if (kBlock && !g.ch_is_row)
      for (int q = 0; q < 4; ++q) cc[q] = col_consts(g, col + q);
#pragma unroll
    for (int k = 0; k < kRows; ++k) {
      const int lr = tid / kLPR + kRPI * k;
      const int row = m0 + lr;
      const EpiRow r = rowc[lr];
      const bool ok = colok && row < g.M;
      const int64_t off = cbase + (int64_t)row * rstride;
      const uint32_t resid = (kBlock && g.has_add) ? resid_pre[k] : 0u;
      int32_t* slot = tileI + lr * kStr + c4;
      const v4i t = *reinterpret_cast<const v4i*>(slot);
      int32_t v[4] = {t.x, t.y, t.z, t.w};
      fold(v, r, col, 4);
      epi_apply<4, kBlock>(g, r, v, off, store_on && ok, col, resid, lut, cc);
      if (kBlock && g.shadow_out) *reinterpret_cast<v4i*>(slot) = v4i{v[0], v[1], v[2], v[3]};
    }
  } else if (BN == 128) {
    // one column x rows (tid>>7) + 2k (planes whose length is not a multiple of 4)
    const int lc = tid & (BN - 1);
    const int col = n0 + lc;
    const bool colok = col < g.N;
    EpiRow cc1{};
    if (kBlock && !g.ch_is_row) cc1 = col_consts(g, col);
    int64_t cbase = col, rstride = g.ldc;
    if (g.out_nchw) {
      const int img = col / hw;
      cbase = (int64_t)img * g.M * hw + (col - img * hw);
      rstride = hw;
    }
#pragma unroll 4
    for (int k = 0; k < BM / 2; ++k) {
      const int lr = (tid >> 7) + 2 * k;
      const int row = m0 + lr;
      const EpiRow r = rowc[lr];
      const bool ok = colok && row < g.M;
      const int64_t off = cbase + (int64_t)row * rstride;
      uint32_t resid = 0;
      if (kBlock && g.has_add && ok) resid = g.add_res[off];
      int32_t* slot = tileI + lr * kStr + lc;
      int32_t v[1] = {*slot};
      fold(v, r, col, 1);
      epi_apply<1, kBlock>(g, r, v, off, store_on && ok, col, resid, lut, &cc1);
      if (kBlock && g.shadow_out) *slot = v[0];
    }
  }
  if (kBlock && g.shadow_out && !(g.ablate & 1)) {
    lds_barrier();
    constexpr int kItems = (BM / 16) * BN;
#pragma unroll
    for (int it0 = 0; it0 < kItems; it0 += kGemmThreads) {
      const int it = it0 + tid;
      const int lc = it & (BN - 1);
      const int grp = it / BN;
      const int col = n0 + lc;
      const int ch0 = m0 + grp * 16;
      if (col < g.N && lc < g.tcols && ch0 < g.shadow_cpad) {
        uint32_t w[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          uint32_t word = 0;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int ch = ch0 + d * 4 + q;
            uint32_t b = (uint32_t)tileI[(grp * 16 + d * 4 + q) * kStr + lc] ^ g.shadow_xor;
            if (ch >= g.M) b = 0;  // padded channels of a partial group stay zero
            word |= (b & 0xFFu) << (8 * q);
          }
          w[d] = word;
        }
        *reinterpret_cast<v4i*>(g.shadow_out + ((int64_t)(ch0 >> 4) * g.N + col) * 16) =
            v4i{(int)w[0], (int)w[1], (int)w[2], (int)w[3]};
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

// NCHW int8/uint8 -> shadow [cin_pad/16][N*HW][16]; padded channels 0; uint8 xor 0x80.
// One thread per (16-channel chunk, pixel); lanes run along pixels, so each channel
// plane read is a contiguous 64-byte span and the 16-byte stores are contiguous.
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
    __builtin_memcpy(y + ((int64_t)chunk * N * HW + (int64_t)n * HW + pix) * 16, v, 16);
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
          const int64_t pix = ((int64_t)img * g.H + ih) * g.W + iw;
          for (int c = 0; c < Cin; ++c) s += shadow[((int64_t)(c >> 4) * g.in_pix + pix) * 16 + (c & 15)];
        }
      }
    }
    out[p] = s;
  }
}

// Direct (VALU) grouped / depthwise / tiny-channel convolution on NCHW int8/uint8.
// out[n][o][oh][ow] = Σ_{c in group(o), r, s} (a - za)(w - zw[o]); padded taps contribute 0.
template <typename Tx, typename Tw, bool kBlock>
__global__ __launch_bounds__(256) void direct_conv_kernel(const Tx* __restrict__ x, const Tw* __restrict__ w,
                                                          int N, int C, int H, int W, int O,
                                                          int OH, int OW, int KH, int KW, int sh, int sw, int pt, int pl,
                                                          int dh, int dw, int groups, int32_t za, int32_t zw,
                                                          const int32_t* __restrict__ zw_vec, GemmArgs g) {
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
    int grp = o / og;
    int32_t zwo = zw_vec ? zw_vec[o] : zw;
    uint32_t acc = 0;
    for (int c = 0; c < cg; ++c) {
      int ci = grp * cg + c;
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
    int64_t pix = (int64_t)n * OH * OW + (int64_t)oh * OW + ow;
    epilogue_store<kBlock>(g, i, o, pix, acc);
  }
}

// Depthwise 3x3 conv (groups == C == O, the MobileNetV2 layers) with the fused block epilogue.
// One workgroup = one image x 16 channels x a band of BH output rows:
//   * the input band plus halo is staged planar in LDS ([16][rows][cols], bytes, taps outside
//     the image hold the input zero point so they contribute 0, legalizations.py:195-226), the
//     per-channel weights minus their zero point as int32;
//   * lanes run along output columns, V consecutive pixels each, so every record store is a
//     contiguous row segment of an NCHW plane (b128 int32 / b32 int8 when V = 4);
//   * the final 8-bit values are parked in LDS and written to the next conv's channel-blocked
//     shadow as one 16-byte chunk (the 16 channels) per pixel.
// Same arithmetic as direct_conv_kernel / epilogue_store (int32 wrap-around accumulation).
template <typename Tx, typename Tw, int V>
__global__ __launch_bounds__(256) void dw3x3_kernel(const Tx* __restrict__ x, const Tw* __restrict__ w, int C, int H,
                                                    int W, int OH, int OW, int sh, int sw, int pt, int pl, int32_t za,
                                                    int32_t zw, const int32_t* __restrict__ zw_vec, int BH, int bands,
                                                    int Wp, GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) uint8_t dsm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int bid = blockIdx.x;
  const int band = bid % bands;
  bid /= bands;
  const int cgroups = C / 16;
  const int cgrp = bid % cgroups, n = bid / cgroups;
  const int c0 = cgrp * 16;
  const int oh0 = band * BH;
  const int bh = min(BH, OH - oh0);
  const int rows_in = (bh - 1) * sh + 3;
  const int ih0 = oh0 * sh - pt;
  uint8_t* tin = dsm;
  const int tin_bytes = (16 * rows_in * Wp + 15) & ~15;
  int32_t* wts = reinterpret_cast<int32_t*>(dsm + tin_bytes);
  uint8_t* tout = dsm + tin_bytes + 16 * 9 * 4;
  // ---- stage the band: (channel, input row) rows of Wp = W + 8 bytes, input column iw at
  // byte 4 + iw (4-byte aligned interior; the 4-byte halos hold the zero point); one dword
  // per lane (W % 4 == 0, W <= 248), 8 rows per wave at a time so that 8 loads are in flight
  const uint32_t fill4 = 0x01010101u * (uint8_t)za;
  const int nrows = 16 * rows_in;
  const int words = W / 4;
  for (int r0 = wave; r0 < nrows; r0 += 32) {
    uint32_t v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int r = r0 + 4 * u;
      const int c = r / rows_in, lr = r - c * rows_in;
      const int ih = ih0 + lr;
      const bool ok = r < nrows && ih >= 0 && ih < H && lane < words;
      const uint32_t* src = reinterpret_cast<const uint32_t*>(
          reinterpret_cast<const uint8_t*>(x) + (((int64_t)n * C + c0 + c) * H + (ok ? ih : 0)) * W);
      v[u] = ok ? src[lane] : fill4;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int r = r0 + 4 * u;
      if (r < nrows) {
        uint32_t* row = reinterpret_cast<uint32_t*>(tin + r * Wp);
        if (lane < words) row[1 + lane] = v[u];
        else if (lane == words) row[0] = fill4, row[1 + words] = fill4;
      }
    }
  }
  if (tid < 16 * 9) {
    const int c = tid / 9;
    wts[tid] = (int32_t)w[(int64_t)(c0 + c) * 9 + (tid - c * 9)] - (zw_vec ? zw_vec[c0 + c] : zw);
  }
  __syncthreads();
  // ---- 9 taps + epilogue, V pixels of one channel row per item
  const int owv = OW / V;
  const int items = 16 * bh * owv;
  const int qmin = (int)g.rq.qmin, qmax = (int)g.rq.qmax;
  for (int it = tid; it < items; it += 256) {
    const int vv = it % owv;
    const int t = it / owv;
    const int row = t % bh, c = t / bh;
    const int ch = c0 + c;
    int32_t acc[V];
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = 0;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const uint8_t* base = tin + (c * rows_in + row * sh + r) * Wp;
#pragma unroll
      for (int s2 = 0; s2 < 3; ++s2) {
        const int32_t wv = wts[c * 9 + r * 3 + s2];
#pragma unroll
        for (int e = 0; e < V; ++e) {
          const int32_t a = (int32_t)(Tx)base[(vv * V + e) * sw + s2 + 4 - pl] - za;
          acc[e] = (int32_t)((uint32_t)acc[e] + (uint32_t)(a * wv));
        }
      }
    }
    const int oh = oh0 + row, ow = vv * V;
    const int64_t off = (((int64_t)n * C + ch) * OH + oh) * OW + ow;
    int32_t v[V];
#pragma unroll
    for (int e = 0; e < V; ++e) v[e] = acc[e];
    st_i32<V>(g.C + off, v, false);
    const int32_t bias = g.bias[ch];
#pragma unroll
    for (int e = 0; e < V; ++e) v[e] = (int32_t)((uint32_t)v[e] + (uint32_t)bias);
    st_i32<V>(g.bias_out + off, v, false);
#pragma unroll
    for (int e = 0; e < V; ++e) v[e] = min(max(rq_apply(v[e], ch, g.rq), qmin), qmax);
    st_i8<V>(g.rq_out + off, v, false);
    if (g.has_clip) {
#pragma unroll
      for (int e = 0; e < V; ++e) v[e] = min(max(v[e], g.clip_lo), g.clip_hi);
      st_i8<V>(g.clip_out + off, v, false);
    }
#pragma unroll
    for (int e = 0; e < V; ++e) tout[((row * OW) + ow + e) * 16 + c] = (uint8_t)((uint32_t)v[e] ^ g.shadow_xor);
  }
  if (!g.shadow_out) return;
  __syncthreads();
  // ---- shadow: 16 channels of one pixel per 16-byte store, contiguous across lanes
  const int64_t pix0 = ((int64_t)n * OH + oh0) * OW;
  for (int p = tid; p < bh * OW; p += 256)
    *reinterpret_cast<v4i*>(g.shadow_out + ((int64_t)cgrp * g.N + pix0 + p) * 16) =
        *reinterpret_cast<const v4i*>(tout + p * 16);
}

// ---------------------------------------------------------------- host wrappers


// tk_dw.hip: the depthwise 3x3 tile kernel (returns 1 and sets *rc when its plan applies)
int dw_block_try(const tk_tensor* data, const tk_tensor* weight, const ConvGeom& g, const tk_conv2d_attrs* a,
                 const GemmArgs& ga, hipStream_t s, int* rc);

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
  // + the chunked image of a KHxKW > 1 weight for the image-tile kernel (tk_conv_img.hip)
  return rows * k_pad + conv_img_chunked_bytes((int)rows, cin_pad, KH * KW);
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
  return conv_img_pack(weight, (int8_t*)packed + (int64_t)rows * k_pad, rows, cin_pad, s);
}

int64_t conv_shadow_bytes(const tk_tensor* data) {
  if (!data || data->ndim != 4) return 0;
  int64_t cin_pad = (data->shape[1] + 15) / 16 * 16;
  return data->shape[0] * data->shape[2] * data->shape[3] * cin_pad;
}

int make_shadow_impl(const tk_tensor* data, void* shadow, hipStream_t s) {
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


// Validates a fused block and fills the epilogue part of GemmArgs.
static int setup_block(GemmArgs& ga, const BlockIO* b, const tk_tensor* conv_out, int channels, int ch_axis) {
  if (!b) return TK_OK;
  const tk_block_attrs* at = b->attrs;
  TK_CHECK_ARG(at && b->outs && b->bias, "block needs bias, attrs and outputs");
  const int has_add = at->has_add ? 1 : 0;
  TK_CHECK_ARG(b->n_outs == 3 + has_add + (at->has_clip ? 1 : 0), "outs = {conv, bias_add, requantize, [add], [clip]}");
  TK_CHECK_ARG(is_int(b->bias, 32) && numel(b->bias) == channels, "bias must be int32 [channels]");
  const tk_tensor* bo = b->outs[1];
  const tk_tensor* rq = b->outs[2];
  TK_CHECK_ARG(is_int(bo, 32) && numel(bo) == numel(conv_out), "bias_add output must be int32, conv shaped");
  TK_CHECK_ARG(is_int8ish(rq) && numel(rq) == numel(conv_out), "requantize output must be int8/uint8, conv shaped");
  int rq_axis = at->requantize.axis;
  TK_CHECK_ARG(rq_axis == ch_axis || at->requantize.mode <= TK_RQ_TENSOR_TONEAREST,
               "requantize must run along the channel axis to fuse");
  for (int k = 3; k < b->n_outs; ++k)
    TK_CHECK_ARG(b->outs[k]->dtype.code == rq->dtype.code && b->outs[k]->dtype.bits == 8 &&
                     numel(b->outs[k]) == numel(conv_out) && compact(b->outs[k]),
                 "add / clip outputs must match the requantize output");
  if (has_add) {
    const tk_tensor* res = at->residual;
    TK_CHECK_ARG(res && dt_of(res) == dt_of(rq) && numel(res) == numel(conv_out) && compact(res),
                 "residual must match the requantize output (same shape and dtype)");
    TK_CHECK_ARG(at->add.lhs.mode <= TK_RQ_TENSOR_TONEAREST && at->add.rhs.mode <= TK_RQ_TENSOR_TONEAREST,
                 "qnn.add: per-tensor parameters only");
    const tk_requantize_attrs& blk_side = at->block_is_rhs ? at->add.rhs : at->add.lhs;
    const tk_requantize_attrs& res_side = at->block_is_rhs ? at->add.lhs : at->add.rhs;
    auto rqp = [](const tk_requantize_attrs& r) {
      RqParams q{};
      q.mode = r.mode;
      q.multiplier = r.multiplier;
      q.shift = r.shift;
      q.zp_in = r.input_zero_point;
      q.zp_out = r.output_zero_point;
      q.inner = 1;
      q.C = 1;
      return q;
    };
    ga.has_add = 1;
    ga.add_res = (const uint8_t*)ptr(res);
    ga.add_out = (uint8_t*)ptr(b->outs[3]);
    ga.add_pb = rqp(blk_side);
    ga.add_pr = rqp(res_side);
    ga.add_up_b = at->block_is_rhs ? at->add.rhs_upcast : at->add.lhs_upcast;
    ga.add_up_r = at->block_is_rhs ? at->add.lhs_upcast : at->add.rhs_upcast;
    ga.add_zp = at->add.output_zero_point;
  }
  ga.bias = (const int32_t*)ptr(b->bias);
  ga.bias_out = (int32_t*)ptr(bo);
  ga.rq_out = (uint8_t*)ptr(rq);
  ga.clip_out = at->has_clip ? (uint8_t*)ptr(b->outs[3 + has_add]) : nullptr;
  ga.has_clip = at->has_clip;
  bool u8 = is_uint(rq, 8);
  int64_t lo = u8 ? 0 : -128, hi = u8 ? 255 : 127;
  ga.clip_lo = (int32_t)std::max(at->clip_min, lo);
  // clip is max(min(x, a_max), a_min) (topi/math.py:634-638): a_min wins when a_min > a_max, which
  // the kernels' min(max(x, lo), hi) reproduces with hi raised to lo (and clamp_i32 needs lo <= hi)
  ga.clip_hi = (int32_t)std::max<int64_t>(std::min(at->clip_max, hi), ga.clip_lo);
  RqParams& p = ga.rq;
  p.mode = at->requantize.mode;
  p.multiplier = at->requantize.multiplier;
  p.shift = at->requantize.shift;
  p.zp_in = at->requantize.input_zero_point;
  p.zp_out = at->requantize.output_zero_point;
  p.ms = at->requantize.multipliers;
  p.ss = at->requantize.shifts;
  p.zps = at->requantize.input_zero_points;
  p.inner = 1;
  p.C = channels;
  p.qmin = lo;
  p.qmax = hi;
  p.clip_out = 1;
  if ((p.mode == TK_RQ_AXIS_UPWARD || p.mode == TK_RQ_AXIS_TONEAREST) && (!p.ms || !p.ss)) {
    set_error("block: per-axis requantize needs device multipliers/shifts");
    return TK_ERR_INVALID_ARG;
  }
  ga.shadow_out = (uint8_t*)b->shadow_out;
  ga.shadow_cpad = (channels + 15) / 16 * 16;
  ga.shadow_xor = u8 ? 0x80u : 0u;
  return TK_OK;
}

// Tile order (tile_of): on planes of up to 28x28 outputs, each XCD takes a contiguous run of N
// tiles, so the int32 record lines two neighbouring tiles share (rows of 784 B or less) are
// completed in one L2; on larger planes N tiles are striped over the XCDs (the 56x56 stage
// measured 5-7 % faster striped, the 28/14/7 stages 5-11 % faster chunked,
// profiles/r01e_ab_xcd_order.txt).  TK_XCD overrides (0 = plain order).
// Kernel-selection switches (TK_XCD, TK_RING, TK_FASTEPI, ...) exist for A/B measurements
// only: they are read from the environment in the ablation build (build.py --ablation,
// -DTK_ABLATION_BUILD, loaded by the tools through TK_LIB_PATH).  The product library
// compiles them to their defaults, so no variable on a box changes what it runs.

static int xcd_order(int64_t out_hw) {
  const char* e = tune_env("TK_XCD");
  return e ? atoi(e) : (out_hw <= 784 ? 2 : 1);
}

static int nt_stores() {
  const char* e = tune_env("TK_NT");
  return e ? atoi(e) : 1;
}


static int ring_depth() {
  const char* e = tune_env("TK_RING");
  const int r = e ? atoi(e) : 3;
  return r >= 3 && r <= 5 ? r : 3;
}

static int ablate_flags() {
  const char* e = tune_env("TK_ABLATE");
  return e ? atoi(e) : 0;
}

// Split-K plan of an MFMA conv: layers whose tile grid cannot give every CU a workgroup
// (the 7x7 stage at 64 samples) split the reduction so that ~3 workgroups per CU stay
// resident (each split keeps >= 6 k-steps); kper = k-steps per split.
struct SplitPlan {
  int splits, kper;
  int64_t tiles;
};
// 64-row (MT = 1) tiles for conv blocks, except 128-channel layers with K >= 512, where one
// 128-row tile (MT = 2) per N tile measured 7-18% faster (ResNet-50's 28x28 stage: the B
// operand is staged once for both M halves); plain convs use MT = 2 above 64 channels.
// The 256-channel 3x3 layers of the 14x14 stage (K = 2304) also take 128-row tiles while the grid
// keeps >= 192 of them: half the im2col B re-reads per CU, -10 % (profiles/r02q_mt2_ab.txt).
static bool conv_mt1(const ConvGeom& g, bool block) {
  if (g.O <= 64) return true;
  if (!block || tune_env("TK_MT2")) return false;
  if (g.O == 128 && g.k_eff >= 512 && env_int("TK_MT2_128", 1)) return false;
  const int64_t mt2_tiles = ((int64_t)g.N * g.OH * g.OW + 127) / 128 * ((g.O + 127) / 128);
  return !(g.O == 256 && g.k_eff >= 2048 && mt2_tiles >= 192 && env_int("TK_MT2_256", 1));
}

static bool conv_needs_patch(const tk_tensor* weight, const tk_conv2d_attrs* a) {
  return (a->kernel_zero_point - (is_uint(weight, 8) ? 128 : 0)) != 0 || a->kernel_zero_points;
}

static int conv_bn256_ipt(const ConvGeom& g, bool block, bool patch);

// 256-column tiles over the flattened pixel axis (BN = 256, no image alignment) for the short-K,
// >= 256-channel conv blocks on planes of more than 256 pixels (the 56x56 / 28x28 expand and
// downsample layers): each store instruction writes one 1 KB segment of a channel row instead of
// two 512-byte ones (store probe: -10 % on these layers' record writes,
// profiles/r02j_store_patterns.txt "span 64x256").  Off (TK_BN256_ROWS=1 in the ablation build):
// on the kernel the halved occupancy (2 workgroups per CU for 70 KB of LDS) costs more than the
// store pattern gains, the 56x56 expand with its residual join +19 % (profiles/r02s_bn256_rows_ab.txt).
static bool conv_bn256_rows(const ConvGeom& g, bool block, bool patch) {
  const int64_t hw = (int64_t)g.OH * g.OW, P = (int64_t)g.N * hw;
  if (!block || patch || hw <= 256 || hw % 4 != 0 || g.O < 256 || g.k_pad > 256 ||
      P * g.O * 4 >= 0xFFFFFFC0ll || !env_int("TK_BN256_ROWS", 0))
    return false;
  return (P + 255) / 256 * ((g.O + 63) / 64) >= 256;
}

// Images per N tile of a conv block whose planes hold 1..64 pixels (0: plain 128-column
// tiles).  Needs the flat epilogue's preconditions: no per-pixel zero-point patch, a channel
// count that keeps every image run 16-byte aligned, and 32-bit record offsets.
static int conv_image_tiles(const ConvGeom& g, bool block, bool patch) {
  const int64_t hw = (int64_t)g.OH * g.OW;
  if (const int ipt = conv_bn256_ipt(g, block, patch)) return ipt;
  if (!block || patch || hw > 64 || g.O % 4 != 0 || (int64_t)g.N * hw * g.O * 4 >= 0xFFFFFFC0ll ||
      !env_int("TK_IMGTILE", 1))
    return 0;
  return (int)(128 / hw);
}

static int64_t conv_ntiles(const ConvGeom& g, int ipt) {
  return ipt ? ((int64_t)g.N + ipt - 1) / ipt : ((int64_t)g.N * g.OH * g.OW + 127) / 128;
}

// 256-column image tiles (BN = 256) for conv blocks whose planes hold 65..256 pixels (14x14):
// floor(256 / HW) whole images per tile, so that each tile's records are contiguous runs
// (probe: 2x the store rate of 128-column tiles that cross images on 14x14 planes,
// profiles/r02j_store_patterns.txt).  Only where the grid still gives every CU a tile (no
// split-K), with the flat epilogue's preconditions.  Returns images per tile, or 0.
static int conv_bn256_ipt(const ConvGeom& g, bool block, bool patch) {
  const int64_t hw = (int64_t)g.OH * g.OW;
  // short reductions only (the store-bound expand layers): a long K loop at the one or two
  // workgroups per CU of these tiles ran 15-20 % slower than 128-column tiles (3x3 256->256 and
  // 1x1 1024->256 at 14x14, profiles/r02n_bn256_ab.txt)
  if (!block || patch || hw <= 64 || hw > 256 || g.O % 4 != 0 || (int64_t)g.N * hw * g.O * 4 >= 0xFFFFFFC0ll ||
      g.k_pad > env_int("TK_BN256_KMAX", 256) || !env_int("TK_BN256", 1))
    return 0;
  const int ipt = (int)(256 / hw);
  const int64_t tiles = ((int64_t)g.N + ipt - 1) / ipt * ((g.O + 63) / 64);
  return tiles >= 256 ? ipt : 0;
}

// Wide (128-byte) K stages for conv blocks with long reductions on small grids: >= 8 steps of
// 64 bytes, every stage within one tap (cin_pad % 128 == 0), and few enough tiles that the
// 2 workgroups per CU the wide ring's LDS allows hold the whole grid (TK_WIDE_MAX_TILES).
static bool conv_wide(const ConvGeom& g, bool block, int ipt) {
  if (!block || g.KH * g.KW > 64 || g.cin_pad % 128 != 0 || g.k_pad / kBK < 8 ||
      !env_int("TK_WIDE", 1) || !env_int("TK_UNITAP", 1) || tune_env("TK_MT2"))
    return false;
  const int64_t tiles = conv_ntiles(g, ipt) * ((g.O + 63) / 64);
  // (256-column tiles: the wide ring holds one workgroup per CU)
  return tiles <= (conv_bn256_ipt(g, block, false) ? 256 : env_int("TK_WIDE_MAX_TILES", 512));
}

// 128-row tiles with 128-byte K stages (96 KB ring, one workgroup per CU) where the grid fits one
// round: the 14x14 3x3 256-channel layers, -5.5 % (profiles/r02z_wide_mt2_ab.txt)
static bool wide_mt2(const ConvGeom& g, int64_t tiles) {
  return g.KH * g.KW <= 64 && g.cin_pad % 128 == 0 && g.k_pad / kBK >= 8 && tiles <= 256 && env_int("TK_WIDE_MT2", 1);
}

static SplitPlan conv_split_plan(const ConvGeom& g, bool mt1, int ipt, int sbk = kBK) {
  const int64_t tiles = conv_ntiles(g, ipt) * ((g.O + (mt1 ? 63 : 127)) / (mt1 ? 64 : 128));
  const int nk = (int)(g.k_pad / sbk);
  SplitPlan sp{1, nk, tiles};
  // measured: splitting grids of >= 256 tiles (one per CU) loses more to the partial-tile
  // round trip than it gains in latency hiding
  if (!mt1 || tiles >= 256) return sp;
  int want = (int)std::min<int64_t>((768 + tiles - 1) / tiles, nk / 6);
  if (want <= 1) return sp;
  sp.kper = (nk + want - 1) / want;
  sp.splits = (nk + sp.kper - 1) / sp.kper;
  return sp;
}


static inline int64_t al256(int64_t v) { return (v + 255) / 256 * 256; }

int64_t conv_scratch_bytes(const tk_tensor* data, const tk_tensor* weight, const tk_conv2d_attrs* a, int block) {
  if (!a) return -1;
  ConvGeom g;
  if (conv_geom(data, weight, a, &g) != TK_OK) return -1;
  if (!use_mfma_conv(g, a->groups)) return 0;
  int64_t bytes = 0;
  if (conv_needs_patch(weight, a)) bytes += al256((int64_t)g.N * g.OH * g.OW * 4);
  const bool mt1 = conv_mt1(g, block);
  const int ipt = mt1 ? conv_image_tiles(g, block, conv_needs_patch(weight, a)) : 0;
  const bool wide = mt1 && conv_wide(g, block, ipt);
  const SplitPlan sp = conv_split_plan(g, mt1, ipt, wide ? 2 * kBK : kBK);
  int64_t split = sp.splits > 1 ? al256(sp.tiles * sp.splits * (int64_t)(2 * 16 * kGemmThreads) * 4) : 0;
  // a conv block's split-K image-tile plans (3x3) use the same space for their partial records
  if (block && !conv_needs_patch(weight, a)) {
    split = std::max(split, al256(conv_img_split_scratch_bytes(g)));
    split = std::max(split, al256(conv_dense_scratch_bytes(g)));  // the dense head's K-slice sums
  }
  return bytes + split;
}

static int conv2d_run(const tk_tensor* data, const void* shadow, const tk_tensor* weight, const void* packed,
                      const int32_t* sums, tk_tensor* out, const tk_conv2d_attrs* a, void* scratch,
                      const BlockIO* blk, hipStream_t s) {
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
  GemmArgs ga{};
  ga.C = (int32_t*)ptr(out);
  ga.M = g.O;
  ga.N = (int32_t)P;
  ga.OH = g.OH;
  ga.OW = g.OW;
  ga.ch_is_row = 1;
  ga.ablate = ablate_flags();
  ga.nt = nt_stores();
  ga.xcd_order = xcd_order((int64_t)g.OH * g.OW);
  int rc = setup_block(ga, blk, out, g.O, 1);
  if (rc) return rc;
  if (!use_mfma_conv(g, a->groups)) {
    TK_CHECK_ARG(!(blk && blk->attrs->has_add), "residual join needs an MFMA conv block");
    // depthwise 3x3 blocks, every plane size: the tile kernel of tk_dw.hip (TK_DW2=0 in the
    // ablation build keeps the older band / direct kernels below for A/B)
    if (blk && env_int("TK_DW2", 1)) {
      int rc_dw = TK_OK;
      if (dw_block_try(data, weight, g, a, ga, s, &rc_dw)) return rc_dw;
    }
    // depthwise 3x3 blocks: the LDS-staged band kernel (see dw3x3_kernel)
    // (large planes only: on 7x7 / 14x14 planes and strided 28x28 ones the generic kernel measured
    // faster, the band staging does not amortise; MobileNetV2 dw layers 1.2-2x faster otherwise)
    const int64_t ohw = (int64_t)g.OH * g.OW;
    if (blk && a->groups == g.C && g.C == g.O && g.C % 16 == 0 && g.KH == 3 && g.KW == 3 && a->dilation[0] == 1 &&
        a->dilation[1] == 1 && ((a->strides[0] == 1 && ohw >= 784) || ohw >= 3136) && env_int("TK_DW", 1)) {
      const int sh = a->strides[0], sw = a->strides[1];
      // output pixels per workgroup and channel: whole planes up to 1024 pixels, else bands of
      // ~512 (stride 1) / ~256 (stride 2) pixels (measured on MobileNetV2's 112x112 and 56x56 layers)
      const int budget = env_int("TK_DW_BUDGET", sh == 1 ? 512 : 256);
      const int BH = g.OH * g.OW <= 1024 ? g.OH : std::max(1, budget / g.OW);
      const int bands = (g.OH + BH - 1) / BH;
      const int Wp = g.W + 8;  // input row + 4-byte halos (see dw3x3_kernel)
      const int rows_max = (BH - 1) * sh + 3;
      const size_t lds = (size_t)((16 * rows_max * Wp + 15) & ~15) + 16 * 9 * 4 + (size_t)BH * g.OW * 16;
      const bool fits = g.W % 4 == 0 && g.W <= 248 && a->padding[1] <= 4 && (g.OW - 1) * sw + 2 - a->padding[1] < g.W + 4;
      if (lds <= 64 * 1024 && fits) {
        const unsigned grid = (unsigned)((int64_t)g.N * (g.C / 16) * bands);
        const bool v4 = g.OW % 4 == 0;
#define TK_DW(TX, TW)                                                                                              \
  if (v4)                                                                                                          \
    hipLaunchKernelGGL((dw3x3_kernel<TX, TW, 4>), dim3(grid), dim3(256), lds, s, (const TX*)ptr(data),            \
                       (const TW*)ptr(weight), g.C, g.H, g.W, g.OH, g.OW, sh, sw, a->padding[0], a->padding[1],     \
                       a->input_zero_point, a->kernel_zero_point, a->kernel_zero_points, BH, bands, Wp, ga);      \
  else                                                                                                             \
    hipLaunchKernelGGL((dw3x3_kernel<TX, TW, 1>), dim3(grid), dim3(256), lds, s, (const TX*)ptr(data),            \
                       (const TW*)ptr(weight), g.C, g.H, g.W, g.OH, g.OW, sh, sw, a->padding[0], a->padding[1],     \
                       a->input_zero_point, a->kernel_zero_point, a->kernel_zero_points, BH, bands, Wp, ga)
        const bool du = is_uint(data, 8), wu = is_uint(weight, 8);
        if (du && wu) { TK_DW(uint8_t, uint8_t); }
        else if (du) { TK_DW(uint8_t, int8_t); }
        else if (wu) { TK_DW(int8_t, uint8_t); }
        else { TK_DW(int8_t, int8_t); }
#undef TK_DW
        TK_LAUNCH_CHECK();
        return TK_OK;
      }
    }
    // grouped / depthwise / tiny channel counts: direct VALU kernel on NCHW
    int64_t total = (int64_t)g.N * g.O * g.OH * g.OW;
    int grid = (int)std::max<int64_t>(1, std::min<int64_t>((total + 255) / 256, 8192));
#define TK_DIRECT(TX, TW, BLK)                                                                                   \
  hipLaunchKernelGGL((direct_conv_kernel<TX, TW, BLK>), dim3(grid), dim3(256), 0, s, (const TX*)ptr(data),        \
                     (const TW*)ptr(weight), g.N, g.C, g.H, g.W, g.O, g.OH, g.OW, g.KH, g.KW, a->strides[0],          \
                     a->strides[1], a->padding[0], a->padding[1], a->dilation[0], a->dilation[1], a->groups,         \
                     a->input_zero_point, a->kernel_zero_point, a->kernel_zero_points, ga)
#define TK_DIRECT_B(TX, TW) \
  if (blk) TK_DIRECT(TX, TW, true); else TK_DIRECT(TX, TW, false)
    bool du = is_uint(data, 8), wu = is_uint(weight, 8);
    if (du && wu) { TK_DIRECT_B(uint8_t, uint8_t); }
    else if (du) { TK_DIRECT_B(uint8_t, int8_t); }
    else if (wu) { TK_DIRECT_B(int8_t, uint8_t); }
    else { TK_DIRECT_B(int8_t, int8_t); }
#undef TK_DIRECT_B
#undef TK_DIRECT
    TK_LAUNCH_CHECK();
    return TK_OK;
  }
  TK_CHECK_ARG(shadow && packed && sums, "MFMA conv needs shadow, packed weight and weight sums");
  int du = is_uint(data, 8), wu = is_uint(weight, 8);
  TK_CHECK_ARG(!(wu && a->kernel_zero_points), "per-channel zero points with uint8 weights are not supported");
  int32_t za = a->input_zero_point - (du ? 128 : 0);
  int32_t zw = a->kernel_zero_point - (wu ? 128 : 0);
  ga.A = (const int8_t*)packed;
  ga.B = (const int8_t*)shadow;
  ga.lda = g.k_pad;
  ga.ldb = g.cin_pad;
  ga.k_pad = g.k_pad;
  ga.k_eff = g.k_eff;
  // operand A = weights (zero point zw), operand B = activations (zero point za)
  ga.zA = zw;
  ga.zB = za;
  ga.RA = sums;
  ga.H = g.H; ga.W = g.W; ga.cin_pad = g.cin_pad; ga.KH = g.KH; ga.KW = g.KW;
  ga.in_pix = (int64_t)g.N * g.H * g.W;
  ga.sh = a->strides[0]; ga.sw = a->strides[1]; ga.pt = a->padding[0]; ga.pl = a->padding[1];
  ga.dh = a->dilation[0]; ga.dw = a->dilation[1];
  ga.taps = g.KH * g.KW;
  ga.cgroups = g.cin_pad / 16;
  ga.unitap = ga.taps <= 64 && (g.cin_pad % kBK == 0 || ga.taps == 1) && env_int("TK_UNITAP", 1);
  {
    // (p * ceil(2^40 / d)) >> 40 == p / d while p * d < 2^40
    const uint64_t hw = (uint64_t)g.OH * g.OW;
    auto magic = [](uint64_t d, uint64_t pmax) -> uint64_t {
      return pmax * d < (1ull << 40) ? ((1ull << 40) + d - 1) / d : 0;
    };
    ga.mg_hw = magic(hw, (uint64_t)P);
    ga.mg_ow = magic((uint64_t)g.OW, hw);
  }
  ga.fill = rep4(za);
  {
    const uint64_t elems = (uint64_t)P * g.O;
    ga.out_elems = (uint32_t)std::min<uint64_t>(elems, 0xFFFFFFFFull);
    const int mode = blk ? blk->attrs->requantize.mode : -1;
    // record stores are nontemporal (1) only where a plane's int32 rows are whole 128-byte
    // lines (or planes are tiny): measured on ResNet-50, partial-line NT stores (28x28, 14x14
    // planes) run up to 1.9x slower than plain ones, which the L2 merges before write-back
    const int hwp = g.OH * g.OW;
    const int epi = hwp % 32 == 0 || hwp <= 64 ? 1 : 2;
    ga.fast_epi = blk && elems * 4 < 0xFFFFFFC0ull && hwp % 4 == 0 &&
                  (mode == TK_RQ_AXIS_UPWARD || mode == TK_RQ_TENSOR_UPWARD) ? env_int("TK_FASTEPI", epi) : 0;
  }
  ga.out_nchw = 1;
  {
    const int hwv = g.OH * g.OW;  // store vectors must not straddle an image plane
    ga.vecw = hwv % 4 == 0 ? 4 : 1;
  }
  char* sc = (char*)scratch;
  if (conv_needs_patch(weight, a)) {
    TK_CHECK_ARG(sc, "non-zero kernel zero point needs scratch (tk_conv2d_scratch_bytes)");
    int32_t* ps = (int32_t*)sc;
    sc += al256(P * 4);
    int grid = (int)std::max<int64_t>(1, std::min<int64_t>((P + 255) / 256, 4096));
    hipLaunchKernelGGL(patch_sum_kernel, dim3(grid), dim3(256), 0, s, (const int8_t*)shadow, ps, ga, g.C);
    TK_LAUNCH_CHECK();
    ga.RB = ps;
    ga.zA_vec = a->kernel_zero_points;
  }
  if (blk && blk->attrs->algo == kAlgoDense) {
    if (!conv_dense_applies(g, ga)) {
      set_error("tk_qnn_conv2d_block: algo 5 (dense tiles) does not apply to this block; see tk_conv2d_block_algos");
      return TK_ERR_INVALID_ARG;
    }
    return conv_dense_run(g, ga, sc, s);
  }
  if (blk) {
    // whole-image tiles with the patch staged per channel stage (tk_conv_img.hip) where they apply
    const int8_t* chunked = conv_img_chunked_bytes(g.rows_pad, g.cin_pad, g.KH * g.KW)
                                ? (const int8_t*)packed + (int64_t)g.rows_pad * g.k_pad
                                : nullptr;
    int irc = TK_OK;
    if (conv_img_try(g, a, ga, chunked, sc, blk->attrs->algo, s, &irc)) return irc;
    const int algo = blk->attrs->algo;
    if (algo == kAlgoPf2 || algo == kAlgoPf3) {
      if (!conv_pf_applies(g, ga)) {
        set_error("tk_qnn_conv2d_block: algo " + std::to_string(algo) +
                  " (persistent im2col) does not apply to this conv; see tk_conv2d_block_algos");
        return TK_ERR_INVALID_ARG;
      }
      return conv_pf_run(g, ga, algo == kAlgoPf2 ? 2 : 3, s);
    }
  }
  const bool mt1 = conv_mt1(g, blk != nullptr);
  const int ipt = mt1 ? conv_image_tiles(g, blk != nullptr, conv_needs_patch(weight, a)) : 0;
  ga.ipt = ipt;
  const bool bn_rows = mt1 && !ipt && conv_bn256_rows(g, blk != nullptr, conv_needs_patch(weight, a));
  ga.tcols = ipt ? ipt * g.OH * g.OW : bn_rows ? 256 : 128;
  const bool bn256 = bn_rows || (mt1 && conv_bn256_ipt(g, blk != nullptr, conv_needs_patch(weight, a)) != 0);
  ga.ntiles = bn_rows ? (int32_t)((P + 255) / 256) : (int32_t)conv_ntiles(g, ipt);
  ga.ntiles8 = (ga.ntiles + 7) / 8 * 8;
  ga.mtiles = (g.O + (mt1 ? 63 : 127)) / (mt1 ? 64 : 128);
  dim3 grid((unsigned)((int64_t)ga.mtiles * ga.ntiles8));
  const bool wide = mt1 && conv_wide(g, blk != nullptr, ipt);
  const SplitPlan sp = conv_split_plan(g, mt1, ipt, wide ? 2 * kBK : kBK);
  const int ring = ring_depth();
  if (sp.splits > 1) {
    TK_CHECK_ARG(sc, "split-K conv needs scratch (tk_conv2d_scratch_bytes)");
    ga.ws = (int32_t*)sc;
    ga.splits = sp.splits;
    ga.kper = sp.kper;
    dim3 pgrid(grid.x, 1, (unsigned)sp.splits);
    if (wide) hipLaunchKernelGGL((gemm_i8_kernel<1, true, false, 1, 3, true>), pgrid, dim3(kGemmThreads), 0, s, ga);
    else switch (ring) {
      case 4: hipLaunchKernelGGL((gemm_i8_kernel<1, true, false, 1, 4>), pgrid, dim3(kGemmThreads), 0, s, ga); break;
      case 5: hipLaunchKernelGGL((gemm_i8_kernel<1, true, false, 1, 5>), pgrid, dim3(kGemmThreads), 0, s, ga); break;
      default: hipLaunchKernelGGL((gemm_i8_kernel<1, true, false, 1>), pgrid, dim3(kGemmThreads), 0, s, ga);
    }
    TK_LAUNCH_CHECK();
    if (blk) hipLaunchKernelGGL((gemm_i8_kernel<1, true, true, 2>), grid, dim3(kGemmThreads), 0, s, ga);
    else hipLaunchKernelGGL((gemm_i8_kernel<1, true, false, 2>), grid, dim3(kGemmThreads), 0, s, ga);
  } else if (bn256) {
    if (wide) hipLaunchKernelGGL((gemm_i8_kernel<1, true, true, 0, 3, true, 256>), grid, dim3(kGemmThreads), 0, s, ga);
    else hipLaunchKernelGGL((gemm_i8_kernel<1, true, true, 0, 3, false, 256>), grid, dim3(kGemmThreads), 0, s, ga);
  } else if (mt1) {
    if (blk) {
      const unsigned pad = (unsigned)env_int("TK_LDS_PAD", 0);  // profiling: extra LDS per workgroup
      if (wide) switch (ring) {
        case 4: hipLaunchKernelGGL((gemm_i8_kernel<1, true, true, 0, 4, true>), grid, dim3(kGemmThreads), pad, s, ga); break;
        case 5: hipLaunchKernelGGL((gemm_i8_kernel<1, true, true, 0, 5, true>), grid, dim3(kGemmThreads), pad, s, ga); break;
        default: hipLaunchKernelGGL((gemm_i8_kernel<1, true, true, 0, 3, true>), grid, dim3(kGemmThreads), pad, s, ga);
      }
      else switch (ring) {
        case 4: hipLaunchKernelGGL((gemm_i8_kernel<1, true, true, 0, 4>), grid, dim3(kGemmThreads), pad, s, ga); break;
        case 5: hipLaunchKernelGGL((gemm_i8_kernel<1, true, true, 0, 5>), grid, dim3(kGemmThreads), pad, s, ga); break;
        default: hipLaunchKernelGGL((gemm_i8_kernel<1, true, true>), grid, dim3(kGemmThreads), pad, s, ga);
      }
    } else {
      hipLaunchKernelGGL((gemm_i8_kernel<1, true, false>), grid, dim3(kGemmThreads), 0, s, ga);
    }
  } else {
    if (blk && wide_mt2(g, ga.mtiles * (int64_t)ga.ntiles))
      hipLaunchKernelGGL((gemm_i8_kernel<2, true, true, 0, 3, true>), grid, dim3(kGemmThreads), 0, s, ga);
    else if (blk) hipLaunchKernelGGL((gemm_i8_kernel<2, true, true>), grid, dim3(kGemmThreads), 0, s, ga);
    else hipLaunchKernelGGL((gemm_i8_kernel<2, true, false>), grid, dim3(kGemmThreads), 0, s, ga);
  }
  TK_LAUNCH_CHECK();
  return TK_OK;
}

int conv2d_prepared_impl(const tk_tensor* data, const void* shadow, const tk_tensor* weight, const void* packed,
                         const int32_t* sums, tk_tensor* out, const tk_conv2d_attrs* a, void* workspace_patch,
                         hipStream_t s) {
  return conv2d_run(data, shadow, weight, packed, sums, out, a, workspace_patch, nullptr, s);
}

int conv2d_block_impl(const tk_tensor* data, const void* shadow, const tk_tensor* weight, const void* packed,
                      const int32_t* sums, const tk_tensor* bias, tk_tensor* const* outs, int n_outs,
                      const tk_block_attrs* attrs, void* patch, void* shadow_out, hipStream_t s) {
  TK_CHECK_ARG(outs && n_outs >= 3 && outs[0], "block needs outputs");
  BlockIO b{bias, outs, n_outs, attrs, shadow_out};
  return conv2d_run(data, shadow, weight, packed, sums, outs[0], attrs ? &attrs->conv : nullptr, patch, &b, s);
}

// what the image-tile planner reads of a block's launch arguments (see conv2d_run)
static GemmArgs planner_args(const ConvGeom& g, const tk_tensor* weight, const tk_block_attrs* attrs) {
  static int32_t marker;
  GemmArgs ga{};
  ga.bias_out = &marker;
  ga.has_add = attrs->has_add;
  ga.in_pix = (int64_t)g.N * g.H * g.W;
  ga.zA = attrs->conv.kernel_zero_point - (is_uint(weight, 8) ? 128 : 0);
  ga.zA_vec = attrs->conv.kernel_zero_points;
  ga.RB = conv_needs_patch(weight, &attrs->conv) ? &marker : nullptr;
  return ga;
}

int conv_img_describe(const ConvGeom& g, const tk_conv2d_attrs* a, const GemmArgs& ga, bool have_chunked, int algo,
                      char* buf, int len);

int conv2d_block_algo_info_impl(const tk_tensor* data, const tk_tensor* weight, const tk_block_attrs* attrs, int algo,
                                char* buf, int len) {
  TK_CHECK_ARG(data && weight && attrs && buf && len > 0, "null argument");
  ConvGeom g;
  if (conv_geom(data, weight, &attrs->conv, &g) != TK_OK) {
    set_error("tk_conv2d_block_algo_info: bad shapes");
    return TK_ERR_SHAPE;
  }
  const GemmArgs ga = planner_args(g, weight, attrs);
  const char* fixed = algo == kAlgoIm2col ? "im2col tiles (64 or 128 rows x 128 or 256 columns, the library's own shape)"
                      : algo == kAlgoPf2  ? "persistent im2col tiles, 2 workgroups per CU"
                      : algo == kAlgoPf3  ? "persistent im2col tiles, 1 workgroup per CU (3-slot ring)"
                      : algo == kAlgoDense ? "dense tiles: 32 units x 64 samples, K split over 8 waves"
                                           : nullptr;
  if (fixed) {
    std::snprintf(buf, (size_t)len, "%s", fixed);
    return TK_OK;
  }
  const int rc = conv_img_describe(g, &attrs->conv, ga,
                                   g.KH * g.KW == 1 || conv_img_chunked_bytes(g.rows_pad, g.cin_pad, g.KH * g.KW), algo,
                                   buf, len);
  if (rc) set_error("tk_conv2d_block_algo_info: algo " + std::to_string(algo) + " is not listed for this block");
  return rc;
}

int conv2d_block_algos_impl(const tk_tensor* data, const tk_tensor* weight, const tk_block_attrs* attrs,
                            int32_t* algos, int max_algos) {
  TK_CHECK_ARG(data && weight && attrs && (algos || max_algos <= 0), "null argument");
  ConvGeom g;
  if (conv_geom(data, weight, &attrs->conv, &g) != TK_OK) {
    set_error("tk_conv2d_block_algos: bad shapes");
    return TK_ERR_SHAPE;
  }
  if (!use_mfma_conv(g, attrs->conv.groups) || !is_int8ish(data) || !is_int8ish(weight)) return 0;
  const GemmArgs ga = planner_args(g, weight, attrs);
  int n = 0;
  // dense blocks (1x1 over [B, K, 1, 1]) with a zero weight zero point: the dense tile kernel first
  if (conv_dense_applies(g, ga)) {
    if (n < max_algos) algos[n] = kAlgoDense;
    ++n;
  }
  if (n < max_algos) algos[n] = kAlgoIm2col;
  ++n;
  n += conv_img_algos(g, &attrs->conv, ga, g.KH * g.KW == 1 || conv_img_chunked_bytes(g.rows_pad, g.cin_pad, g.KH * g.KW),
                      algos && max_algos > n ? algos + n : nullptr, max_algos - n);
  // the persistent im2col kernel, last: it measured slower than the im2col kernel on every
  // ResNet-50 layer (profiles/r03w_find_step_pf.json), so the find step's first candidates stay
  // the image-tile plans; listed where conv2d_run's arguments will meet conv_pf_applies
  {
    const int64_t P = (int64_t)g.N * g.OH * g.OW, hw = (int64_t)g.OH * g.OW;
    const int mode = attrs->requantize.mode;
    const int taps = g.KH * g.KW;
    GemmArgs pa = ga;
    // the same gates (incl. the TK_FASTEPI / TK_UNITAP overrides) as conv2d_run, so that every
    // algo listed here runs there
    const int epi = hw % 32 == 0 || hw <= 64 ? 1 : 2;
    pa.fast_epi = P * g.O * 4 < 0xFFFFFFC0ll && hw % 4 == 0 && (mode == TK_RQ_AXIS_UPWARD || mode == TK_RQ_TENSOR_UPWARD)
                      ? env_int("TK_FASTEPI", epi) : 0;
    pa.unitap = taps <= 64 && (g.cin_pad % kBK == 0 || taps == 1) && env_int("TK_UNITAP", 1);
    pa.ch_is_row = 1;
    pa.out_nchw = 1;
    pa.shadow_out = nullptr;  // (bounded like the records)
    if (conv_pf_applies(g, pa) && (int64_t)(g.O + 15) / 16 * 16 * P < 0xFFFFFF00ll) {
      for (int al : {kAlgoPf2, kAlgoPf3}) {
        if (n < max_algos) algos[n] = al;
        ++n;
      }
    }
  }
  return n;
}

int64_t conv2d_workspace_bytes(const tk_tensor* data, const tk_tensor* weight, const tk_conv2d_attrs* a) {
  if (!a) return -1;
  ConvGeom g;
  if (conv_geom(data, weight, a, &g) != TK_OK) return -1;
  if (!use_mfma_conv(g, a->groups)) return 0;
  int64_t packed = conv_packed_weight_bytes(weight, 1);
  int64_t sums = (int64_t)g.rows_pad * 4;
  int64_t shadow = conv_shadow_bytes(data);
  auto al = [](int64_t v) { return (v + 255) / 256 * 256; };
  return al(packed) + al(sums) + al(shadow) + conv_scratch_bytes(data, weight, a, 0);
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
    return conv2d_run(data, nullptr, weight, nullptr, nullptr, out, a, nullptr, nullptr, s);
  TK_CHECK_ARG(workspace, "workspace required (tk_qnn_conv2d_workspace_bytes)");
  auto al = [](int64_t v) { return (v + 255) / 256 * 256; };
  char* ws = (char*)workspace;
  void* packed = ws;
  ws += al(conv_packed_weight_bytes(weight, 1));
  int32_t* sums = (int32_t*)ws;
  ws += al((int64_t)g.rows_pad * 4);
  void* shadow = ws;
  ws += al(conv_shadow_bytes(data));
  void* scratch = ws;
  int rc = conv_pack_weight(weight, 1, packed, sums, s);
  if (rc) return rc;
  rc = make_shadow_impl(data, shadow, s);
  if (rc) return rc;
  return conv2d_run(data, shadow, weight, packed, sums, out, a, scratch, nullptr, s);
}

// ---------------------------------------------------------------- dense
// Split-K of a dense GEMM (MT = 2 tiles, 128 x 128): classifier heads have a handful of
// tiles and a long K (ResNet-50 fc: 8 tiles, 32 k-steps), so split until ~512 workgroups
// run, keeping >= 2 k-steps per split.
static SplitPlan dense_split_plan(int64_t M, int64_t Nn, int64_t K) {
  const int64_t tiles = ((M + 127) / 128) * ((Nn + 127) / 128);
  const int nk = (int)((K + kBK - 1) / kBK);
  SplitPlan sp{1, nk, tiles};
  if (tiles >= 256) return sp;
  // the reduce pass reads splits sequentially: a few splits already fill the chip
  int want = (int)std::min<int64_t>(std::min<int64_t>((512 + tiles - 1) / tiles, nk / 2), 4);
  if (want <= 1) return sp;
  sp.kper = (nk + want - 1) / want;
  sp.splits = (nk + sp.kper - 1) / sp.kper;
  return sp;
}

int64_t dense_workspace_bytes(const tk_tensor* data, const tk_tensor* weight) {
  if (!data || !weight || data->ndim != 2 || weight->ndim != 2) return -1;
  int64_t M = data->shape[0], K = data->shape[1], Nn = weight->shape[0];
  int64_t k_pad = (K + kBK - 1) / kBK * kBK;
  int64_t mrows = (M + 127) / 128 * 128, nrows = (Nn + 127) / 128 * 128;
  auto al = [](int64_t v) { return (v + 255) / 256 * 256; };
  const SplitPlan sp = dense_split_plan(M, Nn, K);
  const int64_t partial = sp.splits > 1 ? sp.tiles * sp.splits * (int64_t)(2 * 2 * 16 * kGemmThreads) * 4 : 0;
  return al(mrows * k_pad) + al(nrows * k_pad) + al(mrows * 4) + al(nrows * 4) + al(partial);
}

static int dense_run(const tk_tensor* data, const tk_tensor* weight, tk_tensor* out, const tk_dense_attrs* a,
                     void* workspace, const BlockIO* blk, hipStream_t s) {
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
  ws += al((int64_t)nrows * 4);
  int32_t* partial = (int32_t*)ws;
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
  ga.vecw = Nn % 4 == 0 ? 4 : 1;
  ga.ch_is_row = 0;
  TK_CHECK_ARG(!(blk && blk->attrs->has_add), "residual join is supported on conv blocks only");
  int rc = setup_block(ga, blk, out, Nn, 1);
  if (rc) return rc;
  ga.shadow_out = nullptr;
  ga.tcols = 128;
  ga.ntiles = (int32_t)((Nn + 127) / 128);
  ga.ntiles8 = (ga.ntiles + 7) / 8 * 8;
  ga.mtiles = (M + 127) / 128;
  dim3 grid((unsigned)((int64_t)ga.mtiles * ga.ntiles8));
  const SplitPlan sp = dense_split_plan(M, Nn, K);
  if (sp.splits > 1) {
    ga.ws = partial;
    ga.splits = sp.splits;
    ga.kper = sp.kper;
    hipLaunchKernelGGL((gemm_i8_kernel<2, false, false, 1>), dim3(grid.x, 1, sp.splits), dim3(kGemmThreads), 0, s, ga);
    TK_LAUNCH_CHECK();
    if (blk) hipLaunchKernelGGL((gemm_i8_kernel<2, false, true, 2>), grid, dim3(kGemmThreads), 0, s, ga);
    else hipLaunchKernelGGL((gemm_i8_kernel<2, false, false, 2>), grid, dim3(kGemmThreads), 0, s, ga);
  } else if (blk) {
    hipLaunchKernelGGL((gemm_i8_kernel<2, false, true>), grid, dim3(kGemmThreads), 0, s, ga);
  } else {
    hipLaunchKernelGGL((gemm_i8_kernel<2, false, false>), grid, dim3(kGemmThreads), 0, s, ga);
  }
  TK_LAUNCH_CHECK();
  return TK_OK;
}

int dense_impl(const tk_tensor* data, const tk_tensor* weight, tk_tensor* out, const tk_dense_attrs* a,
               void* workspace, hipStream_t s) {
  return dense_run(data, weight, out, a, workspace, nullptr, s);
}

int dense_block_impl(const tk_tensor* data, const tk_tensor* weight, const tk_tensor* bias, tk_tensor* const* outs,
                     int n_outs, const tk_block_attrs* attrs, void* workspace, hipStream_t s) {
  TK_CHECK_ARG(outs && n_outs >= 3 && outs[0] && attrs, "block needs outputs and attrs");
  BlockIO b{bias, outs, n_outs, attrs, nullptr};
  return dense_run(data, weight, outs[0], &attrs->dense, workspace, &b, s);
}

}  // namespace tk
