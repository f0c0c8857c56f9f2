// Persistent im2col conv blocks with cross-tile prefetch: qnn.conv2d -> bias_add -> requantize
// [-> qnn.add(residual)] [-> clip] for the large planes (ResNet-50's 56x56 and 28x28 layers), the
// same 64 x 128 tiles and arithmetic as gemm_i8_kernel's fast epilogue (tk_gemm.hip), scheduled
// differently.
//
// Why: a load issued from a CU whose waves are storing waits behind those stores -- an L2 hit
// takes ~1.5 us instead of ~90 ns (tools/probe_ldlat.hip, profiles/r03v_load_latency.txt), so the
// one-tile-per-workgroup kernel pays its operand loads' latency after the previous tile's record
// stores, and K loop and store burst add up on the store-heavy layers.  Here a workgroup walks
// tiles L = blockIdx.x, + gridDim.x, ... (grid = resident workgroups, a multiple of 8 so every
// workgroup stays on one XCD and tile_of's XCD order holds) and issues tile t+1's operands -- the
// residual words, the row constants and the first K stages, all by LDS-DMA -- BEFORE tile t's
// epilogue stores: they are ahead of the stores in the CU's queue and land while the epilogue runs.
//
// LDS, two arrays since the prefetch fills the first while the epilogue reads the second:
// [ring kRing x 12 KB | residual words 8 KB | raw row words] and [tile 64 x 132 int32 | row constants
// | add LUTs]: 70 KB with 2 ring slots (two workgroups per CU), 82 KB with 3 (one).
// vmcnt counts loads and stores in order (gfx9 has no separate store counter): the first K steps of
// a prefetched tile allow this wave's epilogue stores (kStoresPerTile, every one issued
// unconditionally: masked lanes store out of range) to remain outstanding.
//
// Arithmetic: zero-point fold (simple form: uniform weight zero point, no per-pixel patch sums),
// bias_add, RequantizeLowerInt UPWARD (src/relay/qnn/op/requantize.cc:195-273), qnn.add
// (src/relay/qnn/op/add.cc:40-96) via the 256-entry LUTs, clip (python/tvm/topi/math.py:615-640);
// parity: tests/test_gpu_ops.py (every algo of tk_conv2d_block_algos).
#include <algorithm>
#include <string>
#include <type_traits>

#include "tk_conv.h"

namespace tk {

namespace {

constexpr int kBM = 64, kBN = 128, kStr = kBN + 4;
constexpr int kStage = (kBM + kBN) * kBK;               // 12 KB per ring slot
constexpr int kRows = kBM / (kGemmThreads / (kBN / 4));  // 8 rows per thread in the epilogue
constexpr int kTileBytes = kBM * kStr * 4;
constexpr int kResBytes = kRows * kGemmThreads * 4;
constexpr int kRawBytes = 5 * kBM * 4;

// LDS-DMA targets and the epilogue's areas are separate arrays, so that the compiler can tell
// the epilogue's LDS reads from the outstanding prefetch writes (no conservative vmcnt waits)
template <int kRing>
struct PfLds {
  static constexpr int res = kRing * kStage;      // in the DMA array, after the ring
  static constexpr int raw = res + kResBytes;
  static constexpr int dma = raw + kRawBytes;
  static constexpr int rowc = kTileBytes;         // in the epilogue array, after the tile
  static constexpr int lut = rowc + kBM * (int)sizeof(EpiRow);
  static constexpr int epi = lut + 512 * 4;
};

// at most n of this wave's vector-memory instructions outstanding (n <= 63; run-time n)
__device__ __forceinline__ void wait_vm_upto(int n) {
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

__device__ __forceinline__ int pf_lds_off(int row, int chunk) { return row * kBK + ((chunk ^ ((row >> 2) & 3)) << 4); }

}  // namespace

// kRing: LDS-DMA ring slots (2: two workgroups per CU; 3: one); AUX: record store cache policy.
template <int kRing, bool ADD, bool CLIP, bool SHADOW, int AUX>
__global__ __launch_bounds__(kGemmThreads, kRing == 2 ? 2 : 1) void conv_pf_kernel(GemmArgs g) {
  using Lds = PfLds<kRing>;
  __shared__ __attribute__((aligned(16))) int8_t dmem[Lds::dma];
  __shared__ __attribute__((aligned(16))) int8_t emem[Lds::epi];
  __shared__ int s_fast;
  int32_t* tileI = reinterpret_cast<int32_t*>(emem);
  EpiRow* rowc = reinterpret_cast<EpiRow*>(emem + Lds::rowc);
  int32_t* lut = reinterpret_cast<int32_t*>(emem + Lds::lut);
  uint32_t* resw = reinterpret_cast<uint32_t*>(dmem + Lds::res);
  int32_t* raw = reinterpret_cast<int32_t*>(dmem + Lds::raw);  // [5][64]: RA, bias, m, s, zp

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int hw = g.OH * g.OW;
  const int total = g.mtiles * g.ntiles8;
  const int nst = g.k_pad / kBK;
  const bool rq_axis = g.rq.mode >= TK_RQ_AXIS_UPWARD;
  // this wave's vector-memory instructions per epilogue (all issued unconditionally)
  constexpr int kStoresPerTile = kRows * (3 + (ADD ? 1 : 0) + (CLIP ? 1 : 0)) + (SHADOW ? 2 : 0);

  if (ADD) {
    // RequantizeOrUpcast of every 8-bit value of both qnn.add operands (op_common.h:186-200)
    const int32_t x = g.rq.qmin == 0 ? tid : (int32_t)(int8_t)(uint8_t)tid;
    lut[tid] = g.add_up_b ? x : rq_tensor(x, g.add_pb);
    lut[256 + tid] = g.add_up_r ? x : rq_tensor(x, g.add_pr);
  }

  // ---- tile order: tile_of (tk_gemm.hip) for virtual workgroup L; padding tiles are skipped
  auto tile_ok = [&](int L, int& mt, int& nt) __attribute__((always_inline)) {
    const int local = L >> 3;
    mt = local % g.mtiles;
    nt = g.xcd_order == 2 ? (L & 7) * (g.ntiles8 >> 3) + local / g.mtiles : (local / g.mtiles) * 8 + (L & 7);
    if (!g.xcd_order) mt = L / g.ntiles8, nt = L - mt * g.ntiles8;
    return nt < g.ntiles;
  };
  auto next_tile = [&](int L, int& mt, int& nt) __attribute__((always_inline)) {
    while (L < total && !tile_ok(L, mt, nt)) L += gridDim.x;
    return L;
  };

  // ---- LDS-DMA walk state of the tile being loaded (1x1 or unitap taps: every 64-byte stage is
  // one tap and 4 channel groups; lane l loads chunk (l & 3) ^ ((l >> 4) & 3) of its row so that
  // the lane-linear LDS image has lds_off's bank swizzle)
  const int cl = (lane & 3) ^ ((lane >> 4) & 3);
  const int8_t* fill_src = reinterpret_cast<const int8_t*>(tk_fill_rows.v + 16 * (g.fill & 0xFFu));
  const int64_t grp_bytes = g.in_pix * 16;
  const int64_t row_bytes = (int64_t)g.dh * g.W * 16;
  const int dw16 = g.dw * 16;
  const int8_t* a_src;
  const int8_t* lane_base[2];
  uint64_t tmask[2];
  int cg, kh, kw, tap;
  int64_t soff;
  auto setup = [&](int mt, int nt) __attribute__((always_inline)) {
    const int m0 = mt * kBM, n0 = nt * kBN;
    a_src = g.A + (int64_t)(m0 + tid / 4) * g.lda + cl * 16;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int p = n0 + tid / 4 + 64 * t;
      const bool valid = p < g.N;
      const uint32_t pp = valid ? p : 0;
      const int img = g.mg_hw ? (int)(((uint64_t)pp * g.mg_hw) >> 40) : (int)(pp / (uint32_t)hw);
      const uint32_t rem = pp - img * hw;
      const int oh = g.mg_ow ? (int)(((uint64_t)rem * g.mg_ow) >> 40) : (int)(rem / (uint32_t)g.OW);
      const int ow = rem - oh * g.OW;
      const int ih0 = oh * g.sh - g.pt, iw0 = ow * g.sw - g.pl;
      lane_base[t] = g.B + ((((int64_t)img * g.H + ih0) * g.W + iw0) + (int64_t)cl * g.in_pix) * 16;
      uint32_t rows = 0, cols = 0;
      for (int y = 0; y < g.KH; ++y) {
        const int ih = ih0 + y * g.dh;
        rows |= (uint32_t)(ih >= 0 && ih < g.H) << y;
      }
      for (int x = 0; x < g.KW; ++x) {
        const int iw = iw0 + x * g.dw;
        cols |= (uint32_t)(iw >= 0 && iw < g.W) << x;
      }
      uint64_t m = 0;
      for (int y = 0; y < g.KH; ++y)
        if ((rows >> y) & 1) m |= (uint64_t)cols << (y * g.KW);
      tmask[t] = valid ? m : 0;
    }
    cg = kh = kw = tap = 0;
    soff = 0;
  };
  auto issue = [&](int slot) __attribute__((always_inline)) {
    int8_t* sa = dmem + slot * kStage;
    __builtin_amdgcn_global_load_lds((const void*)a_src, (void*)(sa + 16 * wave * kBK), 16, 0, 0);
    a_src += kBK;
    int8_t* sb = sa + kBM * kBK;
    const bool grp_ok = cg + cl < g.cgroups;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const bool ok = ((tmask[t] >> tap) & 1) && grp_ok;
      const int8_t* src = ok ? lane_base[t] + soff : fill_src;
      __builtin_amdgcn_global_load_lds((const void*)src, (void*)(sb + (16 * wave + 64 * t) * kBK), 16, 0, 0);
    }
    cg += 4;
    soff += 4 * grp_bytes;
    if (cg >= g.cgroups) {
      cg = 0;
      ++tap;
      if (++kw == g.KW) kw = 0, ++kh;
      soff = kh * row_bytes + (int64_t)kw * dw16;
    }
  };
  // residual words (the thread's 4 columns x 8 rows, lane-linear per row pass) and the raw row
  // constants of tile (mt, nt), issued ahead of its stages so that the stage waits cover them
  auto issue_side = [&](int mt, int nt) __attribute__((always_inline)) {
    const int m0 = mt * kBM, n0 = nt * kBN;
    if (ADD) {
      const int col = n0 + (tid & 31) * 4;
      const int img = col / hw;
      const int64_t cbase = (int64_t)img * g.M * hw + (col - img * hw);
#pragma unroll
      for (int k = 0; k < kRows; ++k) {
        const int row = m0 + (tid >> 5) + 8 * k;
        const bool ok = col < g.N && row < g.M;
        const int8_t* src = ok ? reinterpret_cast<const int8_t*>(g.add_res) + cbase + (int64_t)row * hw
                               : reinterpret_cast<const int8_t*>(tk_zero_words);
        __builtin_amdgcn_global_load_lds((const void*)src, (void*)(resw + k * kGemmThreads + wave * 64), 4, 0, 0);
      }
    }
    if (wave == 0) {
      const int row = min(m0 + lane, g.M - 1);
      const int32_t* srcs[5] = {g.RA, g.bias, rq_axis ? g.rq.ms : nullptr, rq_axis ? g.rq.ss : nullptr, g.rq.zps};
#pragma unroll
      for (int f = 0; f < 5; ++f) {
        const int32_t* src = srcs[f] ? srcs[f] + row : tk_zero_words;
        __builtin_amdgcn_global_load_lds((const void*)src, (void*)(raw + f * 64), 4, 0, 0);
      }
    }
  };
  auto prologue = [&](int mt, int nt) __attribute__((always_inline)) {
    issue_side(mt, nt);
    setup(mt, nt);
    for (int st = 0; st < kRing - 1 && st < nst; ++st) issue(st);
  };

  int mt, nt;
  int L = next_tile(blockIdx.x, mt, nt);
  if (L >= total) return;
  prologue(mt, nt);
  int stores_after = 0;  // this wave's epilogue stores issued after the prefetched stages
  const uint32_t n4 = g.out_elems * 4u;
  const auto r_conv = rec_rsrc(g.C, n4), r_bias = rec_rsrc(g.bias_out, n4);
  const auto r_rq = rec_rsrc(g.rq_out, g.out_elems);
  const auto r_add = rec_rsrc(g.add_out, ADD ? g.out_elems : 0u);
  const auto r_clip = rec_rsrc(g.clip_out, CLIP ? g.out_elems : 0u);
  const uint32_t shadow_bytes = SHADOW ? (uint32_t)((g.shadow_cpad / 16) * (int64_t)g.N * 16) : 0u;
  const auto r_shadow = rec_rsrc(g.shadow_out, shadow_bytes);
  const int32_t qmin = (int32_t)g.rq.qmin, qmax = (int32_t)g.rq.qmax, zpo = g.rq.zp_out;
  const int32_t add_zp = g.add_zp, clip_lo = g.clip_lo, clip_hi = g.clip_hi;
  const int Mrows = g.M, Ncols = g.N, cpad = g.shadow_cpad;
  const uint32_t sxor = g.shadow_xor;
  const uint32_t fold_k = (uint32_t)g.k_eff * (uint32_t)g.zA * (uint32_t)g.zB;

  while (true) {
    const int m0 = mt * kBM, n0 = nt * kBN;
    // ---- K loop: ring of kRing slots, kRing - 1 stages in flight; stages < kRing - 1 came with
    // the prologue (before the previous epilogue's stores, which may still be outstanding)
    v16i acc[2] = {v16i{0}, v16i{0}};
    int cur = 0, nxt = kRing - 1;
    for (int it = 0; it < nst; ++it) {
      const int pending = min(kRing - 2, nst - 1 - it);
      wait_vm_upto(pending * 3 + (it < kRing - 1 ? stores_after : 0));
      lds_barrier();
      const int8_t* a = dmem + cur * kStage;
      const int8_t* b = a + kBM * kBK;
      v4i fa[2], fb[2][2];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int chunk = 2 * ks + (lane >> 5);
        fa[ks] = *reinterpret_cast<const v4i*>(a + pf_lds_off(wm * 32 + (lane & 31), chunk));
#pragma unroll
        for (int j = 0; j < 2; ++j)
          fb[ks][j] = *reinterpret_cast<const v4i*>(b + pf_lds_off(wn * 64 + j * 32 + (lane & 31), chunk));
      }
      __builtin_amdgcn_sched_barrier(0);
      if (it + kRing - 1 < nst) {
        issue(nxt);
        nxt = nxt == kRing - 1 ? 0 : nxt + 1;
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[ks], fb[ks][j], acc[j], 0, 0, 0);
      cur = cur == kRing - 1 ? 0 : cur + 1;
    }
    // every stage, residual word and raw row word of this tile has landed (the last step's wait
    // left only this wave's older epilogue stores outstanding); stage the tile
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int lc = wn * 64 + j * 32 + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) tileI[(wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * kStr + lc] = acc[j][r];
    }
    if (wave == 0) {
      EpiRow r{};
      r.ra = (uint32_t)raw[lane];
      r.za = (uint32_t)g.zA;
      r.bias = raw[64 + lane];
      r.m = rq_axis ? raw[128 + lane] : g.rq.multiplier;
      r.s = rq_axis ? raw[192 + lane] : g.rq.shift;
      r.zp = g.rq.zps ? raw[256 + lane] : g.rq.zp_in;
      r.fold = fold_k - (uint32_t)g.zB * r.ra;
      rowc[lane] = r;
      const bool fast = __builtin_amdgcn_ballot_w64(r.s > -2) == 0;
      if (lane == 0) s_fast = fast ? 1 : 0;
    }
    uint32_t res[kRows];
#pragma unroll
    for (int k = 0; k < kRows; ++k) res[k] = ADD ? resw[k * kGemmThreads + tid] : 0u;
    lds_barrier();  // tile, row constants and s_fast visible; ring, residual and raw areas free

    // ---- prefetch the next tile (ahead of this tile's stores in the CU's memory queue)
    int mtn = 0, ntn = 0;
    const int Ln = next_tile(L + gridDim.x, mtn, ntn);
    const bool more = Ln < total;
    if (more) prologue(mtn, ntn);
    __builtin_amdgcn_sched_barrier(0);

    // ---- epilogue: 4 consecutive columns x rows (tid >> 5) + 8k, every record through a buffer
    // descriptor (masked lanes store out of range, so every lane issues every store)
    const int c4 = (tid & 31) * 4;
    const int col = n0 + c4;
    const bool colok = col < Ncols;
    const int img = col / hw;
    const uint32_t cbase = (uint32_t)img * (uint32_t)Mrows * (uint32_t)hw + (uint32_t)(col - img * hw);
    const bool fast = s_fast != 0;
    const int mode = g.rq.mode;
    auto rows = [&](auto fast_c) __attribute__((always_inline)) {
      constexpr bool FAST = decltype(fast_c)::value;
#pragma unroll
      for (int k = 0; k < kRows; ++k) {
        const int lr = (tid >> 5) + 8 * k;
        const int row = m0 + lr;
        const uint32_t o = (colok && row < Mrows) ? cbase + (uint32_t)row * (uint32_t)hw : kOffDrop;
        const EpiRow r = rowc[lr];
        int32_t* slot = tileI + lr * kStr + c4;
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
            q[e] = clamp_i32(zpo + ((int32_t)((uint32_t)__mulhi((int32_t)(v[e] - (uint32_t)r.zp), r.m) + rnd) >> sh2),
                             qmin, qmax);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            q[e] = clamp_i32((int32_t)((uint32_t)zpo + (uint32_t)rq_core((int32_t)(v[e] - (uint32_t)r.zp), mode, r.m, r.s)),
                             qmin, qmax);
        }
        __builtin_amdgcn_raw_buffer_store_b32(pack4u(q[0], q[1], q[2], q[3]), r_rq, o, 0, AUX);
        if (ADD) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            q[e] = clamp_i32(lut[q[e] & 0xFF] + lut[256 + ((res[k] >> (8 * e)) & 0xFFu)] - add_zp, qmin, qmax);
          __builtin_amdgcn_raw_buffer_store_b32(pack4u(q[0], q[1], q[2], q[3]), r_add, o, 0, AUX);
        }
        if (CLIP) {
#pragma unroll
          for (int e = 0; e < 4; ++e) q[e] = clamp_i32(q[e], clip_lo, clip_hi);
          __builtin_amdgcn_raw_buffer_store_b32(pack4u(q[0], q[1], q[2], q[3]), r_clip, o, 0, AUX);
        }
        if (SHADOW) *reinterpret_cast<v4i*>(slot) = v4i{q[0], q[1], q[2], q[3]};
      }
    };
    if (fast) rows(std::true_type{});
    else rows(std::false_type{});
    if (SHADOW) {
      // the next conv's shadow: 16 channels of one pixel per 16-byte store (two per thread)
      lds_barrier();
#pragma unroll
      for (int it0 = 0; it0 < 2 * kGemmThreads; it0 += kGemmThreads) {
        const int it = it0 + tid;
        const int lc = it & (kBN - 1), grp = it / kBN;
        const int pcol = n0 + lc, ch0 = m0 + grp * 16;
        uint32_t w[4];
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          uint32_t word = 0;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int ch = ch0 + d * 4 + q;
            uint32_t bt = (uint32_t)tileI[(grp * 16 + d * 4 + q) * kStr + lc] ^ sxor;
            if (ch >= Mrows) bt = 0;  // padded channels of a partial group stay zero
            word |= (bt & 0xFFu) << (8 * q);
          }
          w[d] = word;
        }
        const bool ok = pcol < Ncols && ch0 < cpad;
        const uint32_t off = ok ? (uint32_t)(((ch0 >> 4) * Ncols + pcol) * 16) : 0xFFFFFFF0u;
        __builtin_amdgcn_raw_buffer_store_b128(v4i{(int)w[0], (int)w[1], (int)w[2], (int)w[3]}, r_shadow, off, 0, 0);
      }
    }
    if (!more) break;
    L = Ln, mt = mtn, nt = ntn;
    stores_after = kStoresPerTile;
  }
}

namespace {
template <int kRing, bool ADD, bool CLIP, bool SHADOW>
void* pf_kernel_aux(int aux) {
  return aux == kAuxNT ? reinterpret_cast<void*>(conv_pf_kernel<kRing, ADD, CLIP, SHADOW, kAuxNT>)
                       : reinterpret_cast<void*>(conv_pf_kernel<kRing, ADD, CLIP, SHADOW, 0>);
}
template <int kRing>
void* pf_kernel(bool add, bool clip, bool shadow, int aux) {
  if (add) {
    if (clip) return shadow ? pf_kernel_aux<kRing, true, true, true>(aux) : pf_kernel_aux<kRing, true, true, false>(aux);
    return shadow ? pf_kernel_aux<kRing, true, false, true>(aux) : pf_kernel_aux<kRing, true, false, false>(aux);
  }
  if (clip) return shadow ? pf_kernel_aux<kRing, false, true, true>(aux) : pf_kernel_aux<kRing, false, true, false>(aux);
  return shadow ? pf_kernel_aux<kRing, false, false, true>(aux) : pf_kernel_aux<kRing, false, false, false>(aux);
}

int cu_count() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
  }
  return n;
}
}  // namespace

bool conv_pf_applies(const ConvGeom& g, const GemmArgs& ga) {
  const int64_t hw = (int64_t)g.OH * g.OW;
  return ga.fast_epi != 0 && ga.unitap && ga.RB == nullptr && ga.zB_vec == nullptr && ga.ch_is_row && ga.out_nchw &&
         hw % 4 == 0 && hw > 64 && g.k_pad % kBK == 0 && g.KH * g.KW <= 64 &&
         (int64_t)(g.cin_pad / 16) * ga.in_pix * 16 < (1ll << 40) &&
         (ga.shadow_out == nullptr || (int64_t)(ga.shadow_cpad / 16) * g.N * g.OH * g.OW * 16 < 0xFFFFFF00ll);
}

int conv_pf_run(const ConvGeom& g, GemmArgs ga, int ring, hipStream_t s) {
  ga.ipt = 0;
  ga.tcols = kBN;
  ga.ntiles = (int32_t)(((int64_t)g.N * g.OH * g.OW + kBN - 1) / kBN);
  ga.ntiles8 = (ga.ntiles + 7) / 8 * 8;
  ga.mtiles = (g.O + kBM - 1) / kBM;
  const int64_t tiles8 = (int64_t)ga.mtiles * ga.ntiles8;
  const int per_cu = ring == 2 ? 2 : 1;
  const int grid = (int)std::min<int64_t>(tiles8, (int64_t)per_cu * cu_count() / 8 * 8);
  const int aux = ga.fast_epi == 2 ? 0 : kAuxNT;
  void* k = ring == 2 ? pf_kernel<2>(ga.has_add, ga.has_clip, ga.shadow_out != nullptr, aux)
                      : pf_kernel<3>(ga.has_add, ga.has_clip, ga.shadow_out != nullptr, aux);
  void* args[] = {&ga};
  hipError_t e = hipLaunchKernel(k, dim3((unsigned)std::max(grid, 8)), dim3(kGemmThreads), args, 0, s);
  if (e != hipSuccess) {
    set_error(std::string("conv persistent kernel: launch failed: ") + hipGetErrorString(e));
    return TK_ERR_HIP;
  }
  return TK_OK;
}

}  // namespace tk
