// Depthwise 3x3 conv blocks: qnn.conv2d (groups == C == O, 3x3, stride 1 or 2, dilation 1) ->
// bias_add -> requantize [-> clip] in one launch, for every plane size (MobileNetV2's seventeen
// depthwise layers: 112x112 down to 7x7, stride 1 and 2) -- the non-MFMA path of BASELINE config 5.
//
// The layer writes ~10-11 bytes of records per output element (int32 conv + int32 bias_add +
// int8 requantize + int8 clip + the next conv's int8 shadow) from 1 input byte and 9 weights per
// channel, so it is HBM-write-bound: the kernel is built around the store pattern.
//   * A workgroup owns a tile = one image x CT = 16 * cbg channels x a band of BH output rows (the
//     whole plane when it is small).  Its records are one contiguous NCHW run per channel -- or, for
//     whole planes, one run for all CT channels -- so the tile is walked as a flat array of 4-element
//     groups, each lane storing 16 bytes (int32 records) / 4 bytes (int8 records) with buffer stores:
//     the whole-line pattern that writes at ~5.3 TB/s in the store probes.
//   * The input rows of the tile's channels (+ the one-row halo, out-of-image rows and columns
//     holding the input zero point) are staged in LDS: row loads of 16 / 8 / 4 bytes, or, for
//     narrow whole planes (14x14, 7x7), 16-byte loads of the tile's contiguous input run placed
//     byte by byte (dw_stage_flat).  A tap row of an output is three bytes there; one
//     v_dot4_i32_i8 against the channel's packed weight row (w0, w1, w2, 0) accumulates the three
//     products -- 3 dot instructions per output instead of 9 multiply-adds on single bytes.  On
//     planes with OW % 4 == 0 a group is 4 outputs of one row whose tap windows are fixed
//     v_alignbyte_b32 shifts of 3 (stride 1) or 4 (stride 2) aligned dwords per tap row; other
//     planes decode each element and read two dwords + one alignbyte per tap row.
//   * Zero points are folded, not subtracted per tap: with out-of-image taps holding za,
//       sum (x - za)(w - zw) = sum x w - zw sum x - za sum w + 9 za zw   (exactly, in int32),
//     the last two terms a per-channel constant, sum x another dot against 0x00010101 (only when a
//     kernel zero point is nonzero).  uint8 operands are staged xor 0x80 (x - 128) with the zero
//     point moved by 128, so every dot is signed x signed (python/tvm/relay/qnn/op/
//     legalizations.py:195-226 defines the arithmetic: int16 operand shifts, int32 accumulation).
//   * Epilogue per element as the other conv-block kernels: bias_add (int32 wrap), RequantizeLowerInt
//     (src/relay/qnn/op/requantize.cc:195-273; the mul_hi form when every right shift is >= 2),
//     clip (python/tvm/topi/math.py:615-640), and the last output's shadow byte into LDS, written
//     after the tile as 16-byte chunks (16 channels of one pixel) contiguous across lanes.
// Parity: tests/test_gpu_ops.py (depthwise blocks vs the oracle) and the MobileNetV2 traces.
#include <algorithm>
#include <cstdint>

#include "tk_conv.h"

namespace tk {

namespace {

constexpr int kDwThreads = 256;
constexpr int kDwPL = 16;  // LDS bytes left of each staged input row (>= the conv's left padding; 16-byte
                           // aligned so that the vector loads of a row land on aligned LDS slots)

// how the 4-element groups of a tile are formed
enum { kDwGen = 0,    // any plane: elements decoded one by one (groups may cross rows and channels)
       kDwRow1 = 1,   // OW % 4 == 0, stride 1, left padding 1: a group is 4 outputs of one row
       kDwRow2 = 2 }; // the same at stride 2

struct DwArgs {
  const uint8_t* x;        // NCHW data (int8, or uint8 staged xor 0x80)
  const uint8_t* w;        // (C, 1, 3, 3) weights (int8 / uint8)
  const int32_t* zw_vec;   // per-channel kernel zero points (NULL: zw)
  int32_t zw;
  int32_t za_s;            // staged input zero point: za, or za - 128 for uint8 data
  uint32_t xor_x, xor_w;   // 0x80 for uint8 data / weights
  int32_t w_u8;            // weights are uint8 (their zero point moves by 128 too)
  int32_t C, H, W, OH, OW, sh, pt, pl;
  int32_t BH, bands, cbg;  // output rows per tile, tiles per plane, 16-channel groups per tile
  int32_t rows_in, Wp;     // staged rows per channel (of Wp bytes, a multiple of 16)
  int32_t vw;              // bytes per staging load: 16, 8, 4, 2 or 1 (divides W)
  int32_t flat;            // whole-plane tiles staged from the planes' flat run (dw_stage_flat)
  int32_t npix;            // N * OH * OW: pixels per channel group of the shadow
  uint32_t m_ow, m_plane, m_plane_last;  // fdiv_u magics of OW and of a tile's pixels (BH / last band)
  uint32_t m_cpr, m_rin;   // fdiv_u magics of the loads per staged row (W / vw) and of rows_in
  int32_t lds_const, lds_tout;  // LDS byte offsets of the channel constants / shadow staging
};

struct DwConst {            // one channel's epilogue constants (32 bytes in LDS)
  uint32_t fold;            // -za' sum w' + 9 za' zw'
  int32_t zwc;              // zw' (the sum-x term's factor)
  int32_t bias, m, s, zp;   // bias_add, requantize multiplier / shift / input zero point
  uint32_t pad0, pad1;
};

__device__ __forceinline__ uint32_t fdiv_u(uint32_t x, uint32_t m) { return __umulhi(x, m); }

// The block epilogue of one 4-element group (values v: the convolution sums), elements in channel
// cc[e] at tile pixel pp[e]; o = the group's first element offset in every record (the 4 are
// contiguous there).  Writes conv, bias_add, requantize [, clip] and the shadow bytes (LDS).
template <bool FAST>
__device__ __forceinline__ void dw_epilogue(const GemmArgs& g, const DwConst* cst, uint8_t* tout, uint32_t plane,
                                            int32_t v[4], const int cc[4], const int pp[4], uint32_t o,
                                            __amdgpu_buffer_rsrc_t r_conv, __amdgpu_buffer_rsrc_t r_bias,
                                            __amdgpu_buffer_rsrc_t r_rq, __amdgpu_buffer_rsrc_t r_clip,
                                            bool clip, bool shadow, bool same_c) {
  const int32_t qmin = (int32_t)g.rq.qmin, qmax = (int32_t)g.rq.qmax, zpo = g.rq.zp_out;
  const int mode = g.rq.mode;
  DwConst k[4];
  k[0] = cst[cc[0]];
#pragma unroll
  for (int e = 1; e < 4; ++e) k[e] = same_c ? k[0] : cst[cc[e]];
  __builtin_amdgcn_raw_buffer_store_b128(v4i{v[0], v[1], v[2], v[3]}, r_conv, o * 4u, 0, 0);
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = (int32_t)((uint32_t)v[e] + (uint32_t)k[e].bias);
  __builtin_amdgcn_raw_buffer_store_b128(v4i{v[0], v[1], v[2], v[3]}, r_bias, o * 4u, 0, 0);
  int32_t q[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int32_t t = (int32_t)((uint32_t)v[e] - (uint32_t)k[e].zp);
    int32_t y;
    if constexpr (FAST) {
      // right shift >= 2: (x·m + 2^(30+rs)) >> (31+rs) only needs the high word of x·m
      const int sh2 = -k[e].s - 1;
      y = (int32_t)((uint32_t)__mulhi(t, k[e].m) + (1u << (sh2 - 1))) >> sh2;
    } else {
      y = rq_core(t, mode, k[e].m, k[e].s);
    }
    q[e] = clamp_i32((int32_t)((uint32_t)zpo + (uint32_t)y), qmin, qmax);
  }
  __builtin_amdgcn_raw_buffer_store_b32(pack4u(q[0], q[1], q[2], q[3]), r_rq, o, 0, 0);
  if (clip) {
#pragma unroll
    for (int e = 0; e < 4; ++e) q[e] = clamp_i32(q[e], g.clip_lo, g.clip_hi);
    __builtin_amdgcn_raw_buffer_store_b32(pack4u(q[0], q[1], q[2], q[3]), r_clip, o, 0, 0);
  }
  if (shadow) {
    // the shadow bytes in the tile's flat order ([channel][pixel]: element f at byte f): one
    // aligned dword per group (a [pixel][16] layout here would put the lanes' bytes 64 bytes apart,
    // a 16-way LDS bank conflict per store); transposed to 16-channel chunks after the tile
    const uint32_t f0 = (uint32_t)cc[0] * plane + (uint32_t)pp[0];
    *reinterpret_cast<uint32_t*>(tout + f0) = pack4u(q[0], q[1], q[2], q[3]) ^ (g.shadow_xor * 0x01010101u);
  }
}

template <int MODE, bool FAST>
__device__ __forceinline__ void dw_walk(const DwArgs& d, const GemmArgs& g, const uint8_t* tin, const uint32_t* wts,
                                        const DwConst* cst, uint8_t* tout, int n, int c0, int oh0, int bh, bool zw,
                                        bool clip, bool shadow) {
  const int tid = threadIdx.x;
  const int CT = 16 * d.cbg;
  const uint32_t plane = (uint32_t)(bh * d.OW);                    // tile elements per channel
  const uint32_t m_plane = bh == d.BH ? d.m_plane : d.m_plane_last;
  const uint32_t m_ow = d.m_ow;
  const uint32_t total = plane * (uint32_t)CT;
  const int Wp = d.Wp, rin = d.rows_in;
  const uint32_t n4 = g.out_elems * 4u;
  const auto r_conv = rec_rsrc(g.C, n4), r_bias = rec_rsrc(g.bias_out, n4);
  const auto r_rq = rec_rsrc(g.rq_out, g.out_elems);
  const auto r_clip = rec_rsrc(g.clip_out, clip ? g.out_elems : 0u);
  // (whole-plane tiles: the CT channel runs are adjacent in memory, so the tile is one run)
  const uint32_t base0 = (uint32_t)(((n * d.C + c0) * d.OH + oh0) * d.OW);
  const uint32_t cstride = (uint32_t)(d.OH * d.OW);
  for (uint32_t f0 = 4u * tid; f0 < total; f0 += 4u * kDwThreads) {
    int32_t v[4];
    int cc[4], pp[4];
    if constexpr (MODE == kDwGen) {
      const int colofs = kDwPL - d.pl, sh = d.sh;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t f = f0 + e;
        const uint32_t c = fdiv_u(f, m_plane);
        const uint32_t rem = f - c * plane;
        const uint32_t r = fdiv_u(rem, m_ow);
        const uint32_t ow = rem - r * (uint32_t)d.OW;
        cc[e] = (int)c;
        pp[e] = (int)rem;
        // tap row t of output (r, ow): bytes [a, a + 3) of the staged row r * sh + t
        const int a0 = ((int)c * rin + (int)r * sh) * Wp + colofs + (int)ow * sh;
        int32_t acc = 0, sx = 0;
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          const int a = a0 + t * Wp;
          const uint32_t* q = reinterpret_cast<const uint32_t*>(tin + (a & ~3));
          const uint32_t win = __builtin_amdgcn_alignbyte(q[1], q[0], (uint32_t)(a & 3));
          acc = __builtin_amdgcn_sdot4((int)win, (int)wts[c * 4 + t], acc, false);
          if (zw) sx = __builtin_amdgcn_sdot4((int)win, 0x00010101, sx, false);
        }
        uint32_t val = (uint32_t)acc + cst[c].fold;
        if (zw) val -= (uint32_t)cst[c].zwc * (uint32_t)sx;
        v[e] = (int32_t)val;
      }
      dw_epilogue<FAST>(g, cst, tout, plane, v, cc, pp, base0 + (uint32_t)cc[0] * cstride + (uint32_t)pp[0], r_conv,
                        r_bias, r_rq, r_clip, clip, shadow, false);
    } else {
      // 4 outputs of one row: channel c, row r, columns ow0 .. ow0 + 3 (ow0 % 4 == 0); with the
      // left padding 1 the first tap byte sits at 3 mod 4, so each tap row is 3 (stride 1) or 4
      // (stride 2) aligned dwords and the windows are fixed byte shifts of them
      constexpr int SH = MODE == kDwRow1 ? 1 : 2;
      const uint32_t c = fdiv_u(f0, m_plane);
      const uint32_t rem = f0 - c * plane;
      const uint32_t r = fdiv_u(rem, m_ow);
      const uint32_t ow0 = rem - r * (uint32_t)d.OW;
      const int al = ((int)c * rin + (int)r * SH) * Wp + (kDwPL - 4) + (int)ow0 * SH;  // = first tap byte - 3
      int32_t acc[4] = {0, 0, 0, 0}, sx[4] = {0, 0, 0, 0};
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const uint32_t* q = reinterpret_cast<const uint32_t*>(tin + al + t * Wp);
        const int wr = (int)wts[c * 4 + t];
        uint32_t win[4];
        if constexpr (SH == 1) {
          const uint32_t d0 = q[0], d1 = q[1], d2 = q[2];
          win[0] = __builtin_amdgcn_alignbyte(d1, d0, 3);
          win[1] = d1;
          win[2] = __builtin_amdgcn_alignbyte(d2, d1, 1);
          win[3] = __builtin_amdgcn_alignbyte(d2, d1, 2);
        } else {
          const uint32_t d0 = q[0], d1 = q[1], d2 = q[2], d3 = q[3];
          win[0] = __builtin_amdgcn_alignbyte(d1, d0, 3);
          win[1] = __builtin_amdgcn_alignbyte(d2, d1, 1);
          win[2] = __builtin_amdgcn_alignbyte(d2, d1, 3);
          win[3] = __builtin_amdgcn_alignbyte(d3, d2, 1);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[e] = __builtin_amdgcn_sdot4((int)win[e], wr, acc[e], false);
          if (zw) sx[e] = __builtin_amdgcn_sdot4((int)win[e], 0x00010101, sx[e], false);
        }
      }
      const uint32_t fold = cst[c].fold;
      const uint32_t zwc = (uint32_t)cst[c].zwc;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        uint32_t val = (uint32_t)acc[e] + fold;
        if (zw) val -= zwc * (uint32_t)sx[e];
        v[e] = (int32_t)val;
        cc[e] = (int)c;
        pp[e] = (int)rem + e;
      }
      dw_epilogue<FAST>(g, cst, tout, plane, v, cc, pp, base0 + c * cstride + rem, r_conv, r_bias, r_rq, r_clip, clip,
                        shadow, true);
    }
  }
}

// Staged input: row (c, rr) = input row ih0 + rr of channel c0 + c at LDS bytes [kDwPL, kDwPL + W)
// of a Wp-byte row; the pads and out-of-image rows hold the staged zero point.  VW-byte loads,
// UNROLL of them in flight per thread before they are written.
template <int VW>
__device__ __forceinline__ void dw_stage_data(const DwArgs& d, uint8_t* tin, int n, int c0, int ih0, int CT) {
  typedef typename std::conditional<VW == 16, v4u, typename std::conditional<VW == 8, uint64_t,
          typename std::conditional<VW == 4, uint32_t, typename std::conditional<VW == 2, uint16_t, uint8_t>::type>::type>::type>::type VT;
  constexpr int UNROLL = VW == 16 ? 4 : VW == 8 ? 6 : 8;
  const int tid = threadIdx.x;
  const int cpr = d.W / VW;                 // loads per row
  const int total = CT * d.rows_in * cpr;   // (rows outside the image keep the zero-point fill)
  const uint32_t xb = d.xor_x;
  const uint8_t* xbase = d.x + (int64_t)(n * d.C + c0) * d.H * d.W;
  for (int k0 = tid; k0 < total; k0 += UNROLL * kDwThreads) {
    VT val[UNROLL];
    int dst[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int k = k0 + u * kDwThreads;
      const int row = (int)fdiv_u((uint32_t)k, d.m_cpr), j = k - row * cpr;
      const int c = (int)fdiv_u((uint32_t)row, d.m_rin), rr = row - c * d.rows_in;
      const int ih = ih0 + rr;
      const bool ok = k < total && ih >= 0 && ih < d.H;
      dst[u] = ok ? row * d.Wp + kDwPL + j * VW : -1;
      if (ok) val[u] = ldg(reinterpret_cast<const VT*>(xbase + ((int64_t)c * d.H + ih) * d.W + j * VW));
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      if (dst[u] < 0) continue;
      VT x = val[u];
      if constexpr (VW == 16) {
        x ^= v4u{xb * 0x01010101u, xb * 0x01010101u, xb * 0x01010101u, xb * 0x01010101u};
      } else if constexpr (VW == 8) {
        x ^= (uint64_t)xb * 0x0101010101010101ull;
      } else if constexpr (VW == 4) {
        x ^= xb * 0x01010101u;
      } else if constexpr (VW == 2) {
        x = (uint16_t)(x ^ (uint16_t)(xb * 0x0101u));
      } else {
        x = (uint8_t)(x ^ (uint8_t)xb);
      }
      *reinterpret_cast<VT*>(tin + dst[u]) = x;
    }
  }
}

// Whole-plane tiles on narrow rows (14x14, 7x7: W % 8 != 0, so row loads would be 2- or 1-byte
// loads, 12+ per thread in a chain of load latencies): the tile's CT input planes are one
// contiguous, 16-byte aligned run of CT * H * W bytes (c0 is a multiple of 16), loaded 16 bytes per
// lane; each byte then goes to its padded LDS row, the position advanced byte by byte.
__device__ __forceinline__ void dw_stage_flat(const DwArgs& d, uint8_t* tin, int n, int c0, int ih0, int CT) {
  constexpr int UNROLL = 4;
  const int tid = threadIdx.x;
  const int HW = d.H * d.W;
  const int nq = CT * HW / 16;
  const v4u* src = reinterpret_cast<const v4u*>(d.x + (int64_t)(n * d.C + c0) * HW);
  const uint32_t xb4 = d.xor_x * 0x01010101u;
  for (int q0 = tid; q0 < nq; q0 += UNROLL * kDwThreads) {
    v4u val[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
      if (q0 + u * kDwThreads < nq) val[u] = ldg(src + q0 + u * kDwThreads);
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int q = q0 + u * kDwThreads;
      if (q >= nq) continue;
      const int idx = 16 * q;
      const int c = idx / HW, rem = idx - c * HW;
      int ih = rem / d.W, iw = rem - ih * d.W;
      int dst = (c * d.rows_in + ih - ih0) * d.Wp + kDwPL + iw;
#pragma unroll
      for (int b = 0; b < 16; ++b) {
        tin[dst] = (uint8_t)((val[u][b >> 2] ^ xb4) >> (8 * (b & 3)));
        ++dst;
        if (++iw == d.W) {
          iw = 0;
          dst += d.Wp - d.W;
          if (++ih == d.H) ih = 0, dst += (d.rows_in - d.H) * d.Wp;
        }
      }
    }
  }
}

template <int MODE>
__global__ __launch_bounds__(kDwThreads, 6) void dw_tile_kernel(DwArgs d, GemmArgs g) {
  extern __shared__ __attribute__((aligned(16))) uint8_t dsm[];
  const int tid = threadIdx.x;
  const int CT = 16 * d.cbg;
  int bid = blockIdx.x;
  const int band = bid % d.bands;
  bid /= d.bands;
  const int cgroups = d.C / CT;
  const int cg = bid % cgroups, n = bid / cgroups;
  const int c0 = cg * CT;
  const int oh0 = band * d.BH;
  const int bh = min(d.BH, d.OH - oh0);
  const int ih0 = oh0 * d.sh - d.pt;
  uint8_t* tin = dsm;
  uint32_t* wts = reinterpret_cast<uint32_t*>(dsm + d.lds_const);      // [CT][4] packed rows
  DwConst* cst = reinterpret_cast<DwConst*>(dsm + d.lds_const + CT * 16);
  uint8_t* tout = dsm + d.lds_tout;
  // ---- this channel's weights and epilogue operands, loaded before the staging so that their
  // latency overlaps it (written to LDS after it)
  const int ch = c0 + min(tid, CT - 1);
  const bool axis = g.rq.mode == TK_RQ_AXIS_UPWARD || g.rq.mode == TK_RQ_AXIS_TONEAREST;
  uint32_t wb[9];
  int32_t zw = d.zw, bias = 0, m = g.rq.multiplier, sft = g.rq.shift, zp = g.rq.zp_in;
  if (tid < CT) {
#pragma unroll
    for (int i = 0; i < 9; ++i) wb[i] = (uint32_t)ldg(d.w + (int64_t)ch * 9 + i);
    if (d.zw_vec) zw = ldg(d.zw_vec + ch);
    bias = ldg(g.bias + ch);
    if (axis) m = ldg(g.rq.ms + ch), sft = ldg(g.rq.ss + ch);
    if (g.rq.zps) zp = ldg(g.rq.zps + ch);
  }
  // ---- every staged byte to the zero point (16-byte stores), then the image's bytes over it
  {
    const uint32_t za4 = 0x01010101u * (uint8_t)d.za_s;
    const int n16 = CT * d.rows_in * d.Wp / 16;
    for (int k = tid; k < n16; k += kDwThreads) reinterpret_cast<v4u*>(tin)[k] = v4u{za4, za4, za4, za4};
    lds_barrier();  // (orders LDS only: the operand loads above stay in flight)
  }
  if (d.flat) dw_stage_flat(d, tin, n, c0, ih0, CT);
  else switch (d.vw) {
    case 16: dw_stage_data<16>(d, tin, n, c0, ih0, CT); break;
    case 8: dw_stage_data<8>(d, tin, n, c0, ih0, CT); break;
    case 4: dw_stage_data<4>(d, tin, n, c0, ih0, CT); break;
    case 2: dw_stage_data<2>(d, tin, n, c0, ih0, CT); break;
    default: dw_stage_data<1>(d, tin, n, c0, ih0, CT); break;
  }
  // ---- per channel: packed weight rows (w0, w1, w2, 0) and the epilogue constants
  int shift_ok = 1;  // this channel's right shift is >= 2 (the mul_hi requantize form applies)
  if (tid < CT) {
    const int32_t zws = d.w_u8 ? zw - 128 : zw;
    int32_t sw = 0;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      uint32_t pk = 0;
#pragma unroll
      for (int s2 = 0; s2 < 3; ++s2) {
        const uint32_t b = (wb[r * 3 + s2] ^ d.xor_w) & 0xFFu;
        sw += (int32_t)(int8_t)b;
        pk |= b << (8 * s2);
      }
      wts[tid * 4 + r] = pk;
    }
    wts[tid * 4 + 3] = 0;
    DwConst k{};
    k.fold = (uint32_t)0 - (uint32_t)d.za_s * (uint32_t)sw + 9u * (uint32_t)d.za_s * (uint32_t)zws;
    k.zwc = zws;
    k.bias = bias;
    k.m = m;
    k.s = sft;
    k.zp = zp;
    cst[tid] = k;
    shift_ok = k.s <= -2;
  }
  const bool fast = __syncthreads_and(shift_ok) && (g.rq.mode == TK_RQ_AXIS_UPWARD || g.rq.mode == TK_RQ_TENSOR_UPWARD);
  const bool zw_any = d.zw_vec || d.w_u8 || d.zw != 0;
  const bool shadow = g.shadow_out != nullptr;
  const bool clip = g.has_clip != 0;
  if (fast) dw_walk<MODE, true>(d, g, tin, wts, cst, tout, n, c0, oh0, bh, zw_any, clip, shadow);
  else dw_walk<MODE, false>(d, g, tin, wts, cst, tout, n, c0, oh0, bh, zw_any, clip, shadow);
  if (!shadow) return;
  __syncthreads();
  // ---- the next conv's shadow: 16 channels of one pixel per 16-byte store, the tile's pixels of
  // each channel group contiguous in [C / 16][N * OH * OW][16]; staged as [channel][pixel] bytes,
  // so 4 pixels of 16 channels are 16 dwords transposed in registers (v_perm_b32)
  const int plane = bh * d.OW;
  const int pix0 = (n * d.OH + oh0) * d.OW;
  if (plane % 4 == 0) {
    const int pq = plane / 4;
    for (int k = tid; k < d.cbg * pq; k += kDwThreads) {
      const int grp = k / pq, p4 = (k - grp * pq) * 4;
      uint32_t in[16];
#pragma unroll
      for (int ch = 0; ch < 16; ++ch) in[ch] = *reinterpret_cast<const uint32_t*>(tout + (grp * 16 + ch) * plane + p4);
      uint8_t* dst = g.shadow_out + ((int64_t)(c0 / 16 + grp) * d.npix + pix0 + p4) * 16;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t o[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const uint32_t lo = __builtin_amdgcn_perm(in[4 * m + 1], in[4 * m], 0x0c0c0000u | ((4u + j) << 8) | (uint32_t)j);
          const uint32_t hi = __builtin_amdgcn_perm(in[4 * m + 3], in[4 * m + 2], 0x00000c0cu | ((uint32_t)j << 16) | ((4u + j) << 24));
          o[m] = lo | hi;
        }
        *reinterpret_cast<v4i*>(dst + j * 16) = v4i{(int)o[0], (int)o[1], (int)o[2], (int)o[3]};
      }
    }
  } else {
    for (int k = tid; k < d.cbg * plane; k += kDwThreads) {
      const int grp = k / plane, p = k - grp * plane;
      uint32_t o[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        uint32_t w = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) w |= (uint32_t)tout[(grp * 16 + 4 * m + b) * plane + p] << (8 * b);
        o[m] = w;
      }
      *reinterpret_cast<v4i*>(g.shadow_out + ((int64_t)(c0 / 16 + grp) * d.npix + pix0 + p) * 16) =
          v4i{(int)o[0], (int)o[1], (int)o[2], (int)o[3]};
    }
  }
}

}  // namespace

// The depthwise tile plan of a conv block, when one applies: every output channel reads only its
// own input channel (groups == C == O), 3x3 taps, stride 1 or 2 on both axes, dilation 1, channel
// counts in whole 16-channel shadow groups, and records that fit 32-bit byte offsets.
int dw_block_try(const tk_tensor* data, const tk_tensor* weight, const ConvGeom& g, const tk_conv2d_attrs* a,
                 const GemmArgs& ga_in, hipStream_t s, int* rc) {
  GemmArgs ga = ga_in;
  const int sh = a->strides[0];
  if (!(a->groups == g.C && g.C == g.O && g.C % 16 == 0 && g.KH == 3 && g.KW == 3 && a->dilation[0] == 1 &&
        a->dilation[1] == 1 && a->strides[1] == sh && (sh == 1 || sh == 2) && a->padding[0] <= 2 &&
        a->padding[1] <= 2 && g.OW >= 2 && ga.bias_out && ga.rq_out))
    return 0;
  if ((int64_t)g.N * g.O * g.OH * g.OW * 4 >= (int64_t)UINT32_MAX || !is_int8ish(data) || !is_int8ish(weight))
    return 0;
  const int OHW = g.OH * g.OW;
  ga.out_elems = (uint32_t)((int64_t)g.N * g.O * OHW);  // every record's elements (buffer-store range)
  DwArgs d{};
  d.x = (const uint8_t*)ptr(data);
  d.w = (const uint8_t*)ptr(weight);
  d.zw_vec = a->kernel_zero_points;
  d.zw = a->kernel_zero_point;
  const bool xu = is_uint(data, 8), wu = is_uint(weight, 8);
  d.xor_x = xu ? 0x80u : 0u;
  d.xor_w = wu ? 0x80u : 0u;
  d.w_u8 = wu;
  d.za_s = xu ? a->input_zero_point - 128 : a->input_zero_point;
  if (d.za_s < -128 || d.za_s > 127) return 0;  // the staged zero point must be a byte value
  d.C = g.C;
  d.H = g.H;
  d.W = g.W;
  d.OH = g.OH;
  d.OW = g.OW;
  d.sh = sh;
  d.pt = a->padding[0];
  d.pl = a->padding[1];
  d.npix = g.N * OHW;
  d.vw = g.W % 16 == 0 ? 16 : g.W % 8 == 0 ? 8 : g.W % 4 == 0 ? 4 : g.W % 2 == 0 ? 2 : 1;
  // row groups (4 outputs of one row, taps from aligned dwords) where the plane allows them
  const int mode = g.OW % 4 == 0 && d.pl == 1 ? (sh == 1 ? kDwRow1 : kDwRow2) : kDwGen;
  // staged row: [kDwPL][W][pads], long enough for the last group's tap dwords
  const int need = std::max(kDwPL + g.W + 4, kDwPL - d.pl + (g.OW - 1) * sh + 16);
  d.Wp = (need + 15) & ~15;
  auto lds_of = [&](int cbg, int BH) {
    const int CT = 16 * cbg;
    const size_t tin = (size_t)CT * ((BH - 1) * sh + 3) * d.Wp + 16;
    return tin + (size_t)CT * 16 + (size_t)CT * sizeof(DwConst) + (size_t)CT * BH * g.OW;
  };
  constexpr size_t kLds = 64 * 1024;
  // tiles: whole planes of up to 1024 pixels, 1, 2 or 4 16-channel groups per tile so that a tile
  // has ~3k outputs (14x14: one group, 1536 tiles at B = 64; 7x7: four); larger planes in bands of
  // ~512 (stride 1) / ~256 (stride 2) output pixels per channel.  (Measured on MobileNetV2 at
  // B = 64: more, smaller tiles -- 14-row bands of the 28x28 planes, 6-row bands of a 14x14 one,
  // two groups on 7x7 -- ran 1-5 us slower per layer; two groups on 14x14 planes 4 us slower.)
  auto band_ok = [&](int bh) { return (bh * g.OW) % 4 == 0 && ((g.OH % bh) * g.OW) % 4 == 0; };
  int cbg = 1, BH = g.OH;
  if (OHW <= 1024 && lds_of(1, g.OH) <= kLds) {
    while (cbg < 4 && 16 * cbg * 2 * OHW <= 4096 && g.C % (32 * cbg) == 0 && lds_of(2 * cbg, g.OH) <= kLds) cbg *= 2;
  } else {
    int bh = std::max(1, std::min(g.OH, (sh == 1 ? 512 : 256) / g.OW));
    // equal bands where a height within [bh / 2, bh] divides the plane (28 rows: 4 x 7, not 9 9 9 1)
    for (int b = bh; b > 0 && 2 * b >= bh; --b)
      if (g.OH % b == 0 && band_ok(b) && lds_of(1, b) <= kLds) {
        bh = b;
        break;
      }
    while (bh > 1 && (lds_of(1, bh) > kLds || !band_ok(bh))) --bh;
    if (!band_ok(bh) || lds_of(1, bh) > kLds) return 0;
    BH = bh;
  }
  d.cbg = cbg;
  d.BH = BH;
  d.bands = (g.OH + BH - 1) / BH;
  d.rows_in = (BH - 1) * sh + 3;
  // x / d as __umulhi(x, ceil(2^32 / d)): exact for x * d < 2^32 (tile indices < 2^16, d <= 2^16)
  auto magic = [](uint32_t v) { return (uint32_t)((0x100000000ull + v - 1) / v); };
  const int last = g.OH - (d.bands - 1) * BH;
  if ((int64_t)16 * cbg * BH * g.OW >= 65536 || g.W / d.vw < 2) return 0;
  d.m_ow = magic((uint32_t)g.OW);
  d.m_plane = magic((uint32_t)(BH * g.OW));
  d.m_plane_last = magic((uint32_t)(last * g.OW));
  d.m_cpr = magic((uint32_t)(g.W / d.vw));
  d.m_rin = magic((uint32_t)d.rows_in);
  // narrow rows of whole-plane tiles whose staged rows cover every input row: the flat staging
  d.flat = d.bands == 1 && d.vw < 8 && d.rows_in - d.pt >= g.H && (reinterpret_cast<uintptr_t>(d.x) & 15) == 0 &&
           env_int("TK_DW_FLAT", 1);
  const int CT = 16 * cbg;
  const size_t tin = (size_t)CT * d.rows_in * d.Wp + 16;
  d.lds_const = (int32_t)tin;
  d.lds_tout = (int32_t)(tin + (size_t)CT * 16 + (size_t)CT * sizeof(DwConst));
  const size_t lds = lds_of(cbg, BH);
  const unsigned grid = (unsigned)((int64_t)g.N * (g.C / CT) * d.bands);
  if (mode == kDwRow1) hipLaunchKernelGGL(dw_tile_kernel<kDwRow1>, dim3(grid), dim3(kDwThreads), lds, s, d, ga);
  else if (mode == kDwRow2) hipLaunchKernelGGL(dw_tile_kernel<kDwRow2>, dim3(grid), dim3(kDwThreads), lds, s, d, ga);
  else hipLaunchKernelGGL(dw_tile_kernel<kDwGen>, dim3(grid), dim3(kDwThreads), lds, s, d, ga);
  *rc = hipGetLastError() == hipSuccess ? TK_OK : TK_ERR_HIP;
  if (*rc) set_error("dw_tile_kernel launch failed");
  return 1;
}

}  // namespace tk
