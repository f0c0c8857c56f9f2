// Weight-stationary 1x1 conv blocks: qnn.conv2d (1x1, stride 1) -> bias_add -> requantize
// [-> qnn.add(residual)] [-> clip] for the store-heavy expand / join layers whose whole weight
// fits in LDS (ResNet-50's 28x28 128->512 and 56x56 64->256 residual expands, MobileNetV2's
// narrow pointwise layers).
//
// Why a third schedule: those layers write 12 bytes of records per output element, and the
// earlier kernels spend a K loop per tile that cannot overlap the previous tile's record stores
// (a CU's loads queue behind its stores; a wave retires only when its stores completed): the
// image-tile kernel re-reads a whole image's input (100 KB on 28x28) once per 32 output channels,
// so on the 28x28 expands K loops and store bursts add up to ~95 us against ~55 us of store
// traffic (profiles/r06c_res28_expand_valu_ab.txt, docs/DESIGN_HISTORY.md).  Here a workgroup
// owns ALL output channels of P pixels of one image: the weights (M x K) and its input slice
// (K x P) are loaded once, at the start, and the rows are then produced in chunks of 32 channels
// -- MFMAs from LDS, staging, the block epilogue -- so the only loads after the prologue are the
// next chunk's residual words, issued before the current chunk's stores.  The MFMAs of chunk c+1
// run while chunk c's stores drain.
//
// LDS: [weights rows32 x K, 16-byte chunks XOR-swizzled by row] [input K/16 x Ppad x 16]
// [staging 32 x (Ppad + 4) int32] [row constants rows32 x 32 B] [add LUTs 2 KB], plus two static
// residual buffers that the chunks alternate (LDS-DMA targets in arrays of their own, so that the
// compiler can tell the epilogue's LDS reads from the outstanding DMA writes: no vmcnt(0) waits).
// vmcnt counts loads and stores in order (gfx9 has no separate store counter): every walk and
// shadow store is issued unconditionally (masked lanes store out of range), so the count of this
// wave's stores after a chunk's residual loads is fixed and the wait for those loads is counted.
//
// Arithmetic: the zero-point fold of conv_pf_kernel (uniform weight zero point, no per-pixel patch
// sums), bias_add, RequantizeLowerInt (src/relay/qnn/op/requantize.cc:195-273), qnn.add
// (src/relay/qnn/op/add.cc:40-96) via the 256-entry LUTs, clip (python/tvm/topi/math.py:615-640);
// parity: tests/test_gpu_ops.py (every algo of tk_conv2d_block_algos).
#include <algorithm>
#include <string>
#include <type_traits>

#include "tk_conv.h"

namespace tk {

namespace {

constexpr int kWsRows = 32;     // output channels per chunk
constexpr int kWsMaxCT = 4;     // 32-column tiles per wave (Ppad <= 512)
constexpr int kWsMaxIt = 8;     // walk iterations per chunk (32 * P / 4 groups over 256 threads)
constexpr int kWsMaxSh = 4;     // shadow iterations per chunk (2 * P pixels over 256 threads)
constexpr int kWsResBytes = kWsMaxIt * kGemmThreads * 4;  // one chunk's residual words
constexpr int kWsLds = 160 * 1024 - 1024 - 2 * kWsResBytes;  // dynamic LDS (the residual buffers are static)

struct WsArgs {
  int32_t P, Ppad, segs;       // pixels per tile (a run of one image's plane), padded to 32; tiles per image
  int32_t tiles, tiles8;       // N * segs; rounded up to 8 (XCD-contiguous tile order)
  int32_t nchunk, rows32;      // 32-row chunks; weight rows staged (nchunk * 32)
  int32_t swz;                 // weight chunk swizzle mask (3 or 7)
  int32_t x_off, t_off, rowc_off, lut_off;  // LDS byte offsets (the weights at 0)
  int32_t ts;                  // staging row pitch (int32)
  int32_t iters, sh_iters;     // walk / shadow iterations per chunk
};

// at most n of this wave's vector-memory instructions outstanding (n <= 63; run-time n)
__device__ __forceinline__ void ws_wait_vm(int n) {
  switch (n) {
#define TK_W(k) \
  case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
#define TK_W8(b) TK_W(b) TK_W(b + 1) TK_W(b + 2) TK_W(b + 3) TK_W(b + 4) TK_W(b + 5) TK_W(b + 6) TK_W(b + 7)
    TK_W8(0) TK_W8(8) TK_W8(16) TK_W8(24) TK_W8(32) TK_W8(40) TK_W8(48) TK_W8(56)
#undef TK_W8
#undef TK_W
    default: asm volatile("s_waitcnt vmcnt(63)" ::: "memory"); break;
  }
}

int ws_lds_bytes(int rows32, int K, int Ppad, WsArgs* h) {
  auto al1k = [](int v) { return (v + 1023) / 1024 * 1024; };
  const int w = al1k(rows32 * K);
  const int x = al1k(K / 16 * Ppad * 16);
  const int t = kWsRows * (Ppad + 4) * 4;
  const int rc = rows32 * (int)sizeof(EpiRow);
  if (h) {
    h->x_off = w;
    h->t_off = w + x;
    h->rowc_off = h->t_off + al1k(t);
    h->lut_off = h->rowc_off + al1k(rc);
    h->ts = Ppad + 4;
  }
  return w + x + al1k(t) + al1k(rc) + 2048;
}

}  // namespace

template <bool ADD, bool CLIP, bool SHADOW, int AUX>
__global__ __launch_bounds__(kGemmThreads, 1) void conv_ws_kernel(GemmArgs g, WsArgs h) {
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  __shared__ __attribute__((aligned(16))) uint32_t s_res0[kWsMaxIt * kGemmThreads];
  __shared__ __attribute__((aligned(16))) uint32_t s_res1[kWsMaxIt * kGemmThreads];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD x (= blockIdx % 8) runs a contiguous run of tiles: an image's segments share one L2, which
  // merges the partial 128-byte lines at their seams before write-back
  const int L = blockIdx.x;
  const int t = (L & 7) * (h.tiles8 >> 3) + (L >> 3);
  if (t >= h.tiles) return;
  const int n = t / h.segs, seg = t - n * h.segs;
  const int hw = g.OH * g.OW, P = h.P, Ppad = h.Ppad, ts = h.ts;
  const int p0 = seg * P;
  const int K = g.k_pad, nck = K / 16;
  const int Mrows = g.M;
  int8_t* const wl = smem;
  int8_t* const xl = smem + h.x_off;
  int32_t* const tileI = reinterpret_cast<int32_t*>(smem + h.t_off);
  EpiRow* const rowc = reinterpret_cast<EpiRow*>(smem + h.rowc_off);
  int32_t* const lut = reinterpret_cast<int32_t*>(smem + h.lut_off);
  const int8_t* fill_src = reinterpret_cast<const int8_t*>(tk_fill_rows.v + 16 * (g.fill & 0xFFu));

  // ---- prologue: the weights and this tile's input slice by LDS-DMA (16-byte slots in lane order;
  // the regions are whole KB, so the slack lanes of a wave's last instruction stay inside them)
  {
    const int wslots = h.rows32 * nck;
    for (int s0 = wave * 64; s0 < wslots; s0 += kGemmThreads) {
      const int s = s0 + lane;
      const int row = s / nck, c = s - row * nck;
      const int8_t* src = s < wslots ? g.A + (int64_t)row * g.lda + ((c ^ (row & h.swz)) << 4) : fill_src;
      __builtin_amdgcn_global_load_lds((const void*)src, (void*)(wl + s0 * 16), 16, 0, 0);
    }
    const int xslots = nck * Ppad;
    const int8_t* xb = g.B + ((int64_t)n * hw + p0) * 16;
    for (int s0 = wave * 64; s0 < xslots; s0 += kGemmThreads) {
      const int s = s0 + lane;
      const int kc = s / Ppad, p = s - kc * Ppad;
      // (K groups past the shadow's cin_pad / 16 multiply zero weights: any bytes do)
      const int8_t* src = s < xslots && p < P && kc < g.cgroups ? xb + ((int64_t)kc * g.in_pix + p) * 16 : fill_src;
      __builtin_amdgcn_global_load_lds((const void*)src, (void*)(xl + s0 * 16), 16, 0, 0);
    }
  }
  // row constants of every row, and the add LUTs
  const bool rq_axis = g.rq.mode >= TK_RQ_AXIS_UPWARD;
  const uint32_t fold_k = (uint32_t)g.k_eff * (uint32_t)g.zA * (uint32_t)g.zB;
  bool shift_ok = true;
  for (int r = tid; r < h.rows32; r += kGemmThreads) {
    const int row = min(r, Mrows - 1);
    EpiRow e{};
    e.ra = (uint32_t)ldg(g.RA + row);
    e.za = (uint32_t)g.zA;
    e.bias = ldg(g.bias + row);
    e.m = rq_axis ? ldg(g.rq.ms + row) : g.rq.multiplier;
    e.s = rq_axis ? ldg(g.rq.ss + row) : g.rq.shift;
    e.zp = g.rq.zps ? ldg(g.rq.zps + row) : g.rq.zp_in;
    e.fold = fold_k - (uint32_t)g.zB * e.ra;
    shift_ok = shift_ok && e.s <= -2;
    rowc[r] = e;
  }
  if (ADD) {
    // RequantizeOrUpcast of every 8-bit value of both qnn.add operands (op_common.h:186-200): the
    // block's own values indexed by value - qmin, the residual's by its raw byte, with the add's
    // - zp_out folded in
    const int32_t xb = (int32_t)g.rq.qmin + tid;
    const int32_t xr = g.rq.qmin == 0 ? tid : (int32_t)(int8_t)(uint8_t)tid;
    lut[tid] = g.add_up_b ? xb : rq_tensor(xb, g.add_pb);
    lut[256 + tid] = (int32_t)((uint32_t)(g.add_up_r ? xr : rq_tensor(xr, g.add_pr)) - (uint32_t)g.add_zp);
  }
  const int32_t* lut_b = lut - (int32_t)g.rq.qmin;

  // ---- the walk's groups (the same for every chunk): group gi = tid + 256 i is 4 consecutive
  // pixels 4 (gi % (P / 4)) of chunk row gi / (P / 4)
  const int q4 = P / 4, iters = h.iters;
  int g_row[kWsMaxIt], g_px[kWsMaxIt];
#pragma unroll
  for (int i = 0; i < kWsMaxIt; ++i) {
    const int gi = tid + kGemmThreads * i;
    const int r = gi / q4;
    g_row[i] = r < kWsRows ? r : -1;  // -1: past the chunk (its stores are dropped)
    g_px[i] = gi - r * q4;
  }
  const uint32_t n4 = g.out_elems * 4u;
  const auto r_conv = rec_rsrc(g.C, n4), r_bias = rec_rsrc(g.bias_out, n4);
  const auto r_rq = rec_rsrc(g.rq_out, g.out_elems);
  const auto r_add = rec_rsrc(g.add_out, ADD ? g.out_elems : 0u);
  const auto r_clip = rec_rsrc(g.clip_out, CLIP ? g.out_elems : 0u);
  const uint32_t shadow_bytes = SHADOW ? (uint32_t)((g.shadow_cpad / 16) * (int64_t)g.N * 16) : 0u;
  const auto r_shadow = rec_rsrc(g.shadow_out, shadow_bytes);
  const uint32_t obase = (uint32_t)n * (uint32_t)Mrows * (uint32_t)hw + (uint32_t)p0;
  // element offset of group i of chunk c (kOffDrop: dropped)
  auto goff = [&](int c, int i) __attribute__((always_inline)) -> uint32_t {
    const int row = c * kWsRows + g_row[i];
    return g_row[i] >= 0 && row < Mrows ? obase + (uint32_t)row * (uint32_t)hw + 4u * (uint32_t)g_px[i] : kOffDrop;
  };
  // chunk c's residual words, by LDS-DMA: word i of thread tid at buf[i * 256 + tid]
  const uint8_t* res_src = g.add_res;
  auto load_res = [&](int c, uint32_t* buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < kWsMaxIt; ++i)
      if (i < iters) {
        const uint32_t o = goff(c, i);
        const void* src = o != kOffDrop ? (const void*)(res_src + o) : (const void*)tk_zero_words;
        __builtin_amdgcn_global_load_lds(src, (void*)(buf + i * kGemmThreads + wave * 64), 4, 0, 0);
      }
  };
  if (ADD) load_res(0, s_res0);
  wait_vm(0);
  const bool fast = __syncthreads_and(shift_ok) && (g.rq.mode == TK_RQ_AXIS_UPWARD || g.rq.mode == TK_RQ_TENSOR_UPWARD);

  // ---- MFMA operands: A = weight row c * 32 + lane % 32, B = pixel column of tile jt; lane / 32
  // selects the 16-byte half of each 32-byte K step
  const int nct = Ppad / 32;
  int jn = 0;
#pragma unroll
  for (int j = 0; j < kWsMaxCT; ++j) jn += wave + 4 * j < nct ? 1 : 0;
  const int kh = lane >> 5;
  const int32_t qmin = (int32_t)g.rq.qmin, qmax = (int32_t)g.rq.qmax, zpo = g.rq.zp_out;
  const int32_t clip_lo = g.clip_lo, clip_hi = g.clip_hi;
  const int mode = g.rq.mode;
  const uint32_t sx4 = g.shadow_xor * 0x01010101u;
  const int cpad = g.shadow_cpad, Npix = g.N;
  constexpr int S = 3 + (ADD ? 1 : 0) + (CLIP ? 1 : 0);  // record stores per walk iteration
  const int after_res = iters * S + (SHADOW ? h.sh_iters : 0);

  auto chunk = [&](auto fast_c, int c, uint32_t* res_cur, uint32_t* res_nxt) __attribute__((always_inline)) {
    constexpr bool FAST = decltype(fast_c)::value;
    {
      v16i acc[kWsMaxCT];
#pragma unroll
      for (int j = 0; j < kWsMaxCT; ++j) acc[j] = v16i{0};
      {
        const int row = c * kWsRows + (lane & 31);
        const int8_t* arow = wl + row * K;
        for (int ks = 0; ks < K / 32; ++ks) {
          const int kc = 2 * ks + kh;
          const v4i a = *reinterpret_cast<const v4i*>(arow + ((kc ^ (row & h.swz)) << 4));
#pragma unroll
          for (int j = 0; j < kWsMaxCT; ++j)
            if (j < jn) {
              const v4i b = *reinterpret_cast<const v4i*>(xl + (kc * Ppad + (wave + 4 * j) * 32 + (lane & 31)) * 16);
              acc[j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[j], 0, 0, 0);
            }
        }
      }
      lds_barrier();  // the previous chunk's walk and shadow pass are done with the staging tile
#pragma unroll
      for (int j = 0; j < kWsMaxCT; ++j)
        if (j < jn) {
          const int col = (wave + 4 * j) * 32 + (lane & 31);
#pragma unroll
          for (int q = 0; q < 16; ++q) tileI[((q & 3) + 8 * (q >> 2) + 4 * kh) * ts + col] = acc[j][q];
        }
      lds_barrier();
      // this chunk's residual words (loaded during the previous chunk) have landed once no more
      // than the previous walk's and shadow pass's stores remain outstanding; then the next chunk's
      // words go out, ahead of this chunk's stores
      if constexpr (ADD) {
        if (c > 0) ws_wait_vm(after_res);
        if (c + 1 < h.nchunk) load_res(c + 1, res_nxt);
      }
      // ---- the block epilogue of the chunk's 32 rows x P pixels
#pragma unroll
      for (int i = 0; i < kWsMaxIt; ++i)
        if (i < iters) {
          const uint32_t o = goff(c, i);
          const int lr = max(g_row[i], 0);
          int32_t* slot = tileI + lr * ts + 4 * g_px[i];
          const EpiRow r = rowc[c * kWsRows + lr];
          v4u v = __builtin_bit_cast(v4u, *reinterpret_cast<const v4i*>(slot)) + r.fold;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v), r_conv, o * 4u, 0, AUX);
          v += (uint32_t)r.bias;
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v), r_bias, o * 4u, 0, AUX);
          int32_t q[4];
          if constexpr (FAST) {
            const int sh2 = -r.s - 1;
            const uint32_t rnd = 1u << (sh2 - 1);
#pragma unroll
            for (int e = 0; e < 4; ++e)
              q[e] = clamp_i32((int32_t)((uint32_t)zpo + (uint32_t)((int32_t)((uint32_t)__mulhi((int32_t)(v[e] - (uint32_t)r.zp), r.m) + rnd) >> sh2)),
                               qmin, qmax);
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              q[e] = clamp_i32((int32_t)((uint32_t)zpo + (uint32_t)rq_core((int32_t)(v[e] - (uint32_t)r.zp), mode, r.m, r.s)),
                               qmin, qmax);
          }
          __builtin_amdgcn_raw_buffer_store_b32(pack4u(q[0], q[1], q[2], q[3]), r_rq, o, 0, AUX);
          if constexpr (ADD) {
            const uint32_t rw = res_cur[i * kGemmThreads + tid];
#pragma unroll
            for (int e = 0; e < 4; ++e)
              q[e] = clamp_i32((int32_t)((uint32_t)lut_b[q[e]] + (uint32_t)lut[256 + ((rw >> (8 * e)) & 0xFFu)]), qmin, qmax);
            __builtin_amdgcn_raw_buffer_store_b32(pack4u(q[0], q[1], q[2], q[3]), r_add, o, 0, AUX);
          }
          if constexpr (CLIP) {
#pragma unroll
            for (int e = 0; e < 4; ++e) q[e] = clamp_i32(q[e], clip_lo, clip_hi);
            __builtin_amdgcn_raw_buffer_store_b32(pack4u(q[0], q[1], q[2], q[3]), r_clip, o, 0, AUX);
          }
          if constexpr (SHADOW) {
            if (g_row[i] >= 0) *reinterpret_cast<v4i*>(slot) = v4i{q[0], q[1], q[2], q[3]};
          }
        }
      if constexpr (SHADOW) {
        // the next conv's shadow: 16 channels of one pixel per 16-byte store
        lds_barrier();
#pragma unroll
        for (int k = 0; k < kWsMaxSh; ++k)
          if (k < h.sh_iters) {
            const int u = tid + kGemmThreads * k;
            const int grp = u / P, px = u - grp * P;
            const int ch0 = c * kWsRows + grp * 16;
            const bool ok = grp < 2 && ch0 < cpad;
            uint32_t w[4];
            if (ok) {
#pragma unroll
              for (int d = 0; d < 4; ++d) {
                const int32_t* tp = tileI + (grp * 16 + d * 4) * ts + px;
                uint32_t word = pack4u((uint32_t)tp[0], (uint32_t)tp[ts], (uint32_t)tp[2 * ts], (uint32_t)tp[3 * ts]) ^ sx4;
                // padded channels of a partial group stay zero
                const int chd = ch0 + d * 4;
                if (chd + 4 > Mrows) {
                  const int keep = max(0, Mrows - chd);
                  word = keep >= 4 ? word : keep == 0 ? 0u : word & ((1u << (8 * keep)) - 1u);
                }
                w[d] = word;
              }
            } else {
              w[0] = w[1] = w[2] = w[3] = 0u;
            }
            const uint32_t off = ok ? (uint32_t)(((ch0 >> 4) * Npix + n * hw + p0 + px) * 16) : 0xFFFFFFF0u;
            __builtin_amdgcn_raw_buffer_store_b128(v4i{(int)w[0], (int)w[1], (int)w[2], (int)w[3]}, r_shadow, off, 0, 0);
          }
      }
    }
  };
  // chunks in pairs: the residual buffers alternate by parity, with distinct arrays per call site
  auto chunks = [&](auto fast_c) __attribute__((always_inline)) {
    for (int c = 0; c < h.nchunk; c += 2) {
      chunk(fast_c, c, s_res0, s_res1);
      if (c + 1 < h.nchunk) chunk(fast_c, c + 1, s_res1, s_res0);
    }
  };
  if (fast) chunks(std::true_type{});
  else chunks(std::false_type{});
}

namespace {
template <bool ADD, bool CLIP, bool SHADOW>
void* ws_kernel_aux(int aux) {
  return aux == kAuxNT ? reinterpret_cast<void*>(conv_ws_kernel<ADD, CLIP, SHADOW, kAuxNT>)
                       : reinterpret_cast<void*>(conv_ws_kernel<ADD, CLIP, SHADOW, 0>);
}
void* ws_kernel(bool add, bool clip, bool shadow, int aux) {
  if (add) {
    if (clip) return shadow ? ws_kernel_aux<true, true, true>(aux) : ws_kernel_aux<true, true, false>(aux);
    return shadow ? ws_kernel_aux<true, false, true>(aux) : ws_kernel_aux<true, false, false>(aux);
  }
  if (clip) return shadow ? ws_kernel_aux<false, true, true>(aux) : ws_kernel_aux<false, true, false>(aux);
  return shadow ? ws_kernel_aux<false, false, true>(aux) : ws_kernel_aux<false, false, false>(aux);
}

// the tiling: P = HW / segs pixels per tile (P % 4 == 0, P <= 512); fewest rounds of tiles over
// the 256 CUs times P (a CU's record bytes), ties to the larger P
bool ws_plan(const ConvGeom& g, const GemmArgs& ga, WsArgs* out) {
  const int hw = g.OH * g.OW;
  const int K = g.k_pad;
  const int nchunk = (g.O + kWsRows - 1) / kWsRows;
  const int rows32 = nchunk * kWsRows;
  if (rows32 > g.rows_pad || K % 64 || K > 512) return false;
  int64_t best = -1;
  WsArgs pick{};
  for (int segs = 1; segs <= hw / 4; ++segs) {
    if (hw % segs) continue;
    const int P = hw / segs;
    if (P % 4 || P > 512 || P < 32) continue;
    const int Ppad = (P + 31) / 32 * 32;
    WsArgs h{};
    if (ws_lds_bytes(rows32, K, Ppad, &h) > kWsLds) continue;
    const int64_t tiles = (int64_t)g.N * segs;
    const int64_t rounds = (tiles + 255) / 256;
    const int64_t cost = rounds * P;
    if (best < 0 || cost < best || (cost == best && P > pick.P)) {
      best = cost;
      h.P = P;
      h.Ppad = Ppad;
      h.segs = segs;
      h.tiles = (int32_t)tiles;
      h.tiles8 = (int32_t)((tiles + 7) / 8 * 8);
      h.nchunk = nchunk;
      h.rows32 = rows32;
      h.swz = (K / 16) % 8 == 0 ? 7 : 3;
      h.iters = (kWsRows * P / 4 + kGemmThreads - 1) / kGemmThreads;
      h.sh_iters = (2 * P + kGemmThreads - 1) / kGemmThreads;
      if (h.iters > kWsMaxIt || h.sh_iters > kWsMaxSh) continue;
      pick = h;
    }
  }
  if (best < 0) return false;
  (void)ga;
  *out = pick;
  return true;
}
}  // namespace

// The weight-stationary kernel's launch arguments (conv2d_run's, before the tile grid) and
// geometry: a 1x1 stride-1 unpadded conv block with the fast epilogue's gates (conv_pf_applies)
// and a tiling whose weights + input slice + staging fit the CU's LDS.
bool conv_ws_applies(const ConvGeom& g, const GemmArgs& ga) {
  WsArgs h;
  return conv_pf_applies(g, ga) && g.KH == 1 && g.KW == 1 && ga.sh == 1 && ga.sw == 1 && ga.pt == 0 && ga.pl == 0 &&
         g.OH == g.H && g.OW == g.W && (int64_t)g.N * g.OH * g.OW * (int64_t)((g.O + 31) / 32 * 32) < 0xFFFFFF00ll &&
         ws_plan(g, ga, &h);
}

int conv_ws_describe(const ConvGeom& g, const GemmArgs& ga, char* buf, int len) {
  WsArgs h;
  if (!ws_plan(g, ga, &h)) return TK_ERR_INVALID_ARG;
  std::snprintf(buf, (size_t)len,
                "weight-stationary 1x1 tiles: all %d channels x %d pixels (%d per image, %d tiles), weights resident "
                "in LDS, %d-row chunks, %.1f KB LDS",
                g.O, h.P, h.segs, h.tiles, kWsRows, ws_lds_bytes(h.rows32, g.k_pad, h.Ppad, nullptr) / 1024.0);
  return TK_OK;
}

int conv_ws_run(const ConvGeom& g, GemmArgs ga, hipStream_t s) {
  WsArgs h;
  if (!ws_plan(g, ga, &h)) {
    set_error("conv weight-stationary kernel: no tiling fits this conv");
    return TK_ERR_INVALID_ARG;
  }
  const int lds = ws_lds_bytes(h.rows32, g.k_pad, h.Ppad, &h);
  // nontemporal record stores only where a tile's channel rows are whole 128-byte lines
  const int aux = ga.fast_epi == 2 || (h.P * 4) % 128 ? 0 : kAuxNT;
  void* k = ws_kernel(ga.has_add, ga.has_clip, ga.shadow_out != nullptr, aux);
  static bool attr_set[16] = {};
  const int ki = (ga.has_add ? 8 : 0) | (ga.has_clip ? 4 : 0) | (ga.shadow_out ? 2 : 0) | (aux ? 1 : 0);
  if (!attr_set[ki]) {
    if (hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, kWsLds) != hipSuccess) {
      set_error("conv weight-stationary kernel: cannot raise its LDS limit");
      return TK_ERR_HIP;
    }
    attr_set[ki] = true;
  }
  void* args[] = {&ga, &h};
  hipError_t e = hipLaunchKernel(k, dim3((unsigned)h.tiles8), dim3(kGemmThreads), args, (size_t)lds, s);
  if (e != hipSuccess) {
    set_error(std::string("conv weight-stationary kernel: launch failed: ") + hipGetErrorString(e));
    return TK_ERR_HIP;
  }
  return TK_OK;
}

}  // namespace tk
