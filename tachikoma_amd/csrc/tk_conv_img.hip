// Image-tile conv blocks: qnn.conv2d (1x1 or 3x3, stride 1 or 2) -> bias_add -> requantize
// [-> qnn.add(residual)] [-> clip] in one launch, for the small planes of a CNN's later stages
// (ResNet-50's 14x14 and 7x7 layers at 64 samples per GPU).
//
// What differs from gemm_i8_kernel (tk_gemm.hip), whose 64x128 im2col tiles gather every input
// pixel once per tap through each CU's LDS-DMA path and end with one store burst:
//   * a workgroup owns R = 32 or 64 output channels x `ipt` WHOLE images, so each of its records
//     is one contiguous NCHW run per image (the store pattern that writes at ~5.3 TB/s on 14x14
//     planes against ~2.4 for image-crossing 128-column tiles, profiles/r02j_store_patterns.txt);
//   * the K loop walks the input channels in stages of CC channels (32 or 64 for 3x3, up to 128
//     for 1x1);
//     each stage brings the patch of those channels for the tile's images -- the output pixels'
//     receptive field incl. the one-pixel halo, out-of-image pixels holding the input zero point --
//     and the R weight rows of all taps of those channels, both by LDS-DMA into one ring slot that
//     all four waves read: every input pixel crosses L2 -> LDS once per stage, not once per tap,
//     and every weight byte once per workgroup, not once per wave (which sank the round-2
//     patch-tile kernel, profiles/r02g_patch_ab.txt);
//   * the 3x3 weights are read from a second, chunked packing [rows][cin_pad/32][9][32] so that a
//     stage's rows are contiguous (CC / 32 consecutive chunks, conv_img_pack); 1x1 weights use the
//     plain packing.  In LDS a weight row of a stage is [CC / 32][taps][32] either way.
// Arithmetic: the same zero-point fold (weights' zero point 0: out = Σ a'w − za·Σw, out-of-bounds
// taps hold a' = za, python/tvm/relay/qnn/op/legalizations.py:195-226), bias_add, RequantizeLowerInt
// (src/relay/qnn/op/requantize.cc:195-273), qnn.add (src/relay/qnn/op/add.cc:40-96) and clip
// (python/tvm/topi/math.py:615-640) as the other conv-block kernels; parity: tests/test_gpu_ops.py.
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "tk_conv.h"

namespace tk {

constexpr int kImgNI = 12;  // most LDS-DMA wave-instructions per wave and stage

// 32-bit LDS byte address of a pointer into the workgroup's LDS (the operand of an asm ds_read)
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// s_waitcnt lgkmcnt(n) for an n known once the K steps are unrolled (0..15)
__device__ __forceinline__ void lgkm_wait(int n) {
  switch (n) {
#define TK_LGKM(k) \
  case k: asm volatile("s_waitcnt lgkmcnt(" #k ")" ::: "memory"); break;
    TK_LGKM(0) TK_LGKM(1) TK_LGKM(2) TK_LGKM(3) TK_LGKM(4) TK_LGKM(5) TK_LGKM(6) TK_LGKM(7) TK_LGKM(8)
    TK_LGKM(9) TK_LGKM(10) TK_LGKM(11) TK_LGKM(12) TK_LGKM(13) TK_LGKM(14)
#undef TK_LGKM
    default: asm volatile("s_waitcnt lgkmcnt(15)" ::: "memory"); break;
  }
}

struct ImgArgs {
  const int8_t* wimg;          // weight rows: chunked packing (3x3) or the plain one (1x1)
  int32_t ldw;                 // bytes per weight row
  int32_t nimg, ipt;           // images of the batch; whole images per workgroup
  int32_t hr, hc, pl;          // patch rows / cols per image; slots per channel group (lead + ipt*hr*hc)
  int32_t lead;                // 3x3: slots ahead of each channel group's pixels (the taps' reach)
  int32_t half;                // 3x3 stride 2 (even W): a row holds its even columns, then its odd ones
                               // (half = W / 2), so a tap's lanes read consecutive slots; 0 = in order
  int32_t ih0, iw0, ls;        // input pixel of patch (0, 0); input pixels per patch pixel (strided 1x1)
  int32_t ps;                  // patch pixels per output pixel (the stride of a 3x3)
  int32_t hw, p, nct;          // output pixels per image and per workgroup; 32-column tiles
  int32_t mtiles, wgs, wgs8;   // channel ranges; workgroups (rounded up to 8)
  int32_t stages, ns;          // cin_pad / CC; ring slots
  int32_t pslots, wslot, sslots, ni, stage_bytes;  // 16-byte LDS slots of a stage: patch, per weight
                                                   // row, all; DMA instructions per wave; ring slot bytes
  int32_t pstep;               // patch source bytes per stage (CC/16 shadow channel groups)
  int32_t tstride;             // int32 pitch of the epilogue staging rows
  int32_t rowc_off, lut_off, res_off;  // LDS byte offsets (the staging tile aliases the ring at 0)
  uint32_t m_pl, m_img, m_hc, m_ws, m_hw, m_ow, m_runq, m_cw;  // fdiv32(x, m_d) == x / d (x, d < 2^16)
  int32_t runq;                // 4-element epilogue groups per image run and pass (R * cw / 4)
  int32_t npass, cw;           // epilogue passes over the tile's columns (npass > 1: one image per
                               // workgroup, cw = hw / npass pixels per pass), or 1 pass of cw = hw
  int32_t skew;                // profiling: first-round workgroups start up to 3 x skew x s_sleep(8) late
  int32_t early_res;           // residual words issued after the prologue's stages (two workgroups
                               // per CU), else during the last K step
  // split K (3x3): MODE 1 workgroups reduce stages [z * stages / ksplit, (z + 1) * stages / ksplit)
  // of their tile and store the raw sums as partial record z (NCHW int32, the conv record's layout,
  // part + z * part_stride); MODE 2 workgroups (their own tiling) sum the ksplit partial records
  // into their accumulators and run the block epilogue
  int32_t ksplit;
  int64_t part_stride;
  int32_t* part;
};

// KT: 1 or 3 taps per axis; WM: 32-row wave groups (R = 32 * WM); CT: 32-column tiles per wave
// (the waves of a row group take columns wn, wn + WN, ...); CC: input channels per K stage (32 or
// 64 for 3x3 -- 64 halves the barrier-separated stages of the 7x7 / 14x14 layers' long K loops;
// 32, 64 or 128 for 1x1: smaller stages for larger planes or two workgroups per CU).
// MODE: 0 = the whole block; 1 = split-K partial sums (no epilogue); 2 = sum the partials + the
// block epilogue (no K loop); 3 = the whole block of a 1x1 join with two workgroups per CU, its
// residual words issued after the prologue's stages (a separate instantiation, so that the stage
// loop of every other kernel is unchanged).
template <int KT, int WM, int CT, int CC, int MODE = 0>
__global__ __launch_bounds__(kGemmThreads, 2) void conv_img_kernel(GemmArgs g, ImgArgs h) {
  extern __shared__ __attribute__((aligned(16))) int8_t smem[];
  __shared__ int s_fast;
  constexpr int R = 32 * WM;
  constexpr int WN = 4 / WM;
  static_assert(CC % 32 == 0 && (KT == 1 || CC <= 64), "3x3 stages hold 32 or 64 channels");
  constexpr int TAPS = KT * KT;
  constexpr int SUB = CC / 32;             // K = 32 MFMA steps per tap and stage
  constexpr int KS = TAPS * SUB;           // K = 32 MFMA steps per stage
  constexpr int WROW = TAPS * CC + 16;     // LDS bytes per weight row: one pad chunk (bank spread)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % WM, wn = wave / WM;
  [[maybe_unused]] const int abl = g.ablate;
  // XCD x runs a contiguous chunk of workgroups; the channel ranges of one patch are adjacent
  const int L = blockIdx.x;
  const int w = (L & 7) * (h.wgs8 >> 3) + (L >> 3);
  if (w >= h.wgs) return;
  if (TK_ABL(1 << 23)) return;  // (ablation build: launch and wave start / end alone)
#ifdef TK_ABLATION_BUILD
  // profiling: stagger the first round's workgroups ((L >> 3) % 4 quarters of h.skew x s_sleep(8))
  // so that CUs are in different phases (K loop / epilogue stores)
  if (h.skew && L < 8 * 256)
    for (int k = 0; k < ((L >> 3) & 3) * h.skew; ++k) __builtin_amdgcn_s_sleep(8);
#endif
  // split K: the ksplit workgroups of a tile are adjacent (same XCD, same input patch in its L2)
  const int S = MODE == 1 ? h.ksplit : 1;
  const int tw = MODE == 1 ? w / S : w;
  const int zs = w - tw * S;
  const int mt = tw % h.mtiles;
  const int img0 = (tw / h.mtiles) * h.ipt;
  const int nimg = min(h.ipt, h.nimg - img0);
  const int m0 = mt * R;
  const int hw = h.hw;
  int32_t* tileI = reinterpret_cast<int32_t*>(smem);  // epilogue staging, over the ring
  EpiRow* rowc = reinterpret_cast<EpiRow*>(smem + h.rowc_off);
  int32_t* lut = reinterpret_cast<int32_t*>(smem + h.lut_off);
  uint32_t* resw = reinterpret_cast<uint32_t*>(smem + h.res_off);
  const int8_t* fill_src = reinterpret_cast<const int8_t*>(tk_fill_rows.v + 16 * (g.fill & 0xFFu));
  const bool has_add = g.has_add;
  const int runq = h.runq;
  const int npass = h.npass, W = h.cw;  // epilogue passes; pixels of a channel row per pass
  const int total = (npass > 1 ? 1 : nimg) * runq;  // epilogue groups per pass
  if (tid == 0) s_fast = 1;       // visible after the first barrier; only cleared at the epilogue

  // ---- residual words of every epilogue group (qnn.add joins), LDS-DMA'd in group order.  With
  // two workgroups per CU (h.early_res) right after the prologue's stages: the stage waits of
  // those stages let them stay in flight, so they land during the K loop -- the residual is a
  // record written several kernels earlier and comes from HBM (profiles/r05ae_residual_cold_per_
  // kernel.txt; the 14x14 joins 45-46 -> 40-41 us) -- while the other workgroup computes.  With
  // one workgroup per CU they would slow its own stage loads (the 28x28 joins: 101.5 -> 112.6 us
  // cached), so there they go out during the last K step, after its barrier (no counted ring wait
  // follows).  Either way the epilogue's full wait covers them.
  auto issue_residual = [&](int c0) __attribute__((always_inline)) {
    for (int q0 = wave * 64; q0 < total; q0 += kGemmThreads) {
      const int gi = q0 + lane;
      const int8_t* src = reinterpret_cast<const int8_t*>(tk_zero_words);
      if (gi < total) {
        const int kk = (int)fdiv32((uint32_t)gi, h.m_runq);
        const int f = (gi - kk * runq) * 4;
        const int r = (int)fdiv32((uint32_t)f, h.m_cw), pp = f - r * W;  // row, pixel of the pass
        src = reinterpret_cast<const int8_t*>(g.add_res) + (uint32_t)(((img0 + kk) * g.M + m0 + r) * hw + c0 + pp);
      }
      __builtin_amdgcn_global_load_lds((const void*)src, (void*)(resw + q0), 4, 0, 0);
    }
  };
  // ---- row constants (threads < R): they land during the K loop
  const bool rq_axis = g.rq.mode >= TK_RQ_AXIS_UPWARD;
  EpiRow row_pre{};
  if (tid < R) {
    const int row = m0 + tid;
    row_pre.ra = (uint32_t)ldg(g.RA + row);
    row_pre.bias = ldg(g.bias + row);
    row_pre.m = ldg(rq_axis ? g.rq.ms + row : tk_zero_words);
    row_pre.s = ldg(rq_axis ? g.rq.ss + row : tk_zero_words);
    row_pre.zp = ldg(g.rq.zps ? g.rq.zps + row : tk_zero_words);
  }

  // ---- LDS-DMA sources of this lane: slot q = (wave + 4k) * 64 + lane of every stage is patch
  // chunk (group q / pl, pixel q % pl) or weight chunk (row, 16-byte chunk) or slack; each source
  // advances by a fixed step per stage (0 for the zero-point fill and the pad chunks)
  // (32-bit arithmetic throughout: one v_mul_hi_u32 per division and 24-bit products -- the 64-bit
  // magic divisions and pointer products cost ~150 v_mad_u64_u32 before the first DMA; the byte
  // offsets below stay under 2^31, img_candidate checks)
  const int ni = h.ni;
  const int8_t* srcs[kImgNI];
  uint32_t steps[kImgNI];
  const int8_t* const pbase = g.B + (int64_t)img0 * g.H * g.W * 16;  // image img0 of channel group 0
  const int8_t* const wbase = h.wimg + (int64_t)m0 * h.ldw;          // weight row m0
  const uint32_t img_px = (uint32_t)(h.hr * h.hc), gstride = (uint32_t)g.in_pix * 16u;
#pragma unroll
  for (int k = 0; k < kImgNI; ++k) {
    srcs[k] = fill_src;
    steps[k] = 0;
    if (k < ni) {
      const uint32_t q = (uint32_t)((wave + 4 * k) * 64 + lane);
      if (q < (uint32_t)h.pslots) {
        const uint32_t grp = fdiv32(q, h.m_pl), pix0 = q - __umul24(grp, (uint32_t)h.pl);
        if (grp < (uint32_t)(CC / 16) && pix0 >= (uint32_t)h.lead) {  // else lead / trailing slack: fill
          const uint32_t pix = pix0 - h.lead;
          const uint32_t kk = fdiv32(pix, h.m_img), r = pix - __umul24(kk, img_px);
          const uint32_t hrow = fdiv32(r, h.m_hc), hcol = r - __umul24(hrow, (uint32_t)h.hc);
          const int ih = h.ih0 + (int)__umul24(hrow, (uint32_t)h.ls);
          const int iw = h.half ? ((int)hcol < h.half ? 2 * (int)hcol : 2 * ((int)hcol - h.half) + 1)
                                : h.iw0 + (int)__umul24(hcol, (uint32_t)h.ls);
          if (img0 + (int)kk < h.nimg && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W) {
            const uint32_t px = __umul24(__umul24(kk, (uint32_t)g.H) + (uint32_t)ih, (uint32_t)g.W) + (uint32_t)iw;
            srcs[k] = pbase + (grp * gstride + px * 16u);
            steps[k] = (uint32_t)h.pstep;
          }
        }
      } else if (q < (uint32_t)h.sslots) {
        const uint32_t wq = q - h.pslots;
        const uint32_t row = fdiv32(wq, h.m_ws), c = wq - __umul24(row, (uint32_t)h.wslot);
        if (c + 1 < (uint32_t)h.wslot) {
          srcs[k] = wbase + (__umul24(row, (uint32_t)h.ldw) + c * 16u);
          steps[k] = TAPS * CC;
        }
      }
    }
  }
  // this split's first stage
  const int st_lo = MODE == 1 ? (int)((int64_t)zs * h.stages / S) : 0;
  if (MODE == 1 && st_lo) {
#pragma unroll
    for (int k = 0; k < kImgNI; ++k) srcs[k] += (int64_t)steps[k] * st_lo;
  }
  auto issue = [&](int slot) __attribute__((always_inline)) {
    int8_t* dst = smem + slot * h.stage_bytes + wave * 1024;
#pragma unroll
    for (int k = 0; k < kImgNI; ++k)
      if (k < ni) {
        if (!TK_ABL(128)) __builtin_amdgcn_global_load_lds((const void*)srcs[k], (void*)(dst + k * 4096), 16, 0, 0);
        srcs[k] += steps[k];
      }
  };

  // ---- fragment addresses: A = weights (row = lane % 32 of this wave's row group), B = patch
  // (column = output pixel of the tile, lane % 32 of each column tile); lane / 32 = 16-byte K half
  int jn = 0;  // column tiles of this wave (wave-uniform)
#pragma unroll
  for (int j = 0; j < CT; ++j) jn += (wn + WN * j < h.nct) ? 1 : 0;
  // 3x3: the patch holds each image's input pixels densely (no halo): lane l's B chunk for tap
  // (kh, kw) sits (kh - 1) * W + kw - 1 slots from its centre pixel, a uniform shift, so the 16
  // lanes of a ds_read_b128 group -- 16 distinct residues of the output column mod 16 -- hit 16
  // distinct 16-byte bank slots (the halo layout cost 3.4-6.5 extra LDS cycles per read,
  // SQ_LDS_BANK_CONFLICT in profiles/r04j_pmc_block.json); taps that fall outside the image take
  // the input zero point: their reads are redirected to the channel group's first lead slot, which
  // the ring fills with it (flg[j]: the column's image edges, bit 0 top, 1 bottom, 2 left, 3 right)
  int boff[CT];
  [[maybe_unused]] uint32_t flg[CT];
#pragma unroll
  for (int j = 0; j < CT; ++j) {
    const uint32_t c = (uint32_t)min((wn + WN * j) * 32 + (lane & 31), h.p - 1);
    const uint32_t kk = fdiv32(c, h.m_hw), r = c - kk * hw;
    const uint32_t oh = fdiv32(r, h.m_ow), ow = r - oh * g.OW;
    boff[j] = (int)(((lane >> 5) * h.pl + h.lead + kk * (h.hr * h.hc) + oh * h.hc * h.ps + ow * (h.half ? 1 : h.ps)) * 16);
    if constexpr (KT == 3) {
      const int ih = (int)oh * h.ps, iw = (int)ow * h.ps;  // the centre tap's input pixel
      flg[j] = (ih == 0 ? 1u : 0u) | (ih + 1 >= g.H ? 2u : 0u) | (iw == 0 ? 4u : 0u) | (iw + 1 >= g.W ? 8u : 0u);
    }
  }
  [[maybe_unused]] const int hb = (lane >> 5) * h.pl * 16;  // lead slot 0 of this lane's channel group
  const int aoff = h.pslots * 16 + (wm * 32 + (lane & 31)) * WROW + (lane >> 5) * 16;
  const int hc = h.hc, pl16 = h.pl * 16;

  v16i acc[CT];
#pragma unroll
  for (int j = 0; j < CT; ++j) acc[j] = v16i{0};
  auto compute_c = [&](const int8_t* base) __attribute__((always_inline)) {
    v4i a[2], b[2][CT];
    auto rd = [&](int ks, int u) __attribute__((always_inline)) {
      const int t = ks / SUB, s = ks - t * SUB, kh = t / KT, kw = t - kh * KT;
      // weight row of the stage: [SUB][TAPS][32] (3x3: CC / 32 consecutive chunks of the chunked
      // packing; 1x1: TAPS = 1, the plain packing's CC channels)
      a[u] = *reinterpret_cast<const v4i*>(base + aoff + (s * TAPS + t) * 32);
      // (stride-2 rows split by column parity: the centre column 2 ow is even slot ow, 2 ow - 1 odd
      // slot half + ow - 1, 2 ow + 1 odd slot half + ow)
      const int dx = KT == 3 && h.half ? (kw == 1 ? 0 : kw == 0 ? h.half - 1 : h.half) : kw - KT / 2;
      const int gs = 2 * s * pl16, bo = ((kh - KT / 2) * hc + dx) * 16;
      // the image edges this tap crosses (a constant once the K loop is unrolled)
      [[maybe_unused]] const uint32_t me =
          KT == 3 ? (kh == 0 ? 1u : 0u) | (kh == 2 ? 2u : 0u) | (kw == 0 ? 4u : 0u) | (kw == 2 ? 8u : 0u) : 0u;
#pragma unroll
      for (int j = 0; j < CT; ++j)
        if (j < jn) {
          int off = boff[j] + bo;
          if constexpr (KT == 3) {
            if (me && (flg[j] & me)) off = hb;
          }
          b[u][j] = *reinterpret_cast<const v4i*>(base + gs + off);
        }
    };
    rd(0, 0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (ks + 1 < KS) rd(ks + 1, (ks + 1) & 1);
      if (!TK_ABL(512)) {
#pragma unroll
        for (int j = 0; j < CT; ++j)
          if (j < jn) {
            acc[j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[ks & 1], b[ks & 1][j], acc[j], 0, 0, 0);
          }
      }
    }
  };

  // The 3x3 K steps with the fragment reads software-pipelined by hand: the
  // compiler's own waits drain every outstanding LDS read (lgkmcnt(0)) before each MFMA pair
  // (DESIGN.md §9), so a wave exposed an LDS round trip about every other step.  Here the reads are
  // inline-asm ds_read_b128 issued D - 1 steps ahead -- every column tile read each step (columns a
  // wave does not own re-read its first tile) so that each step issues exactly NR reads -- and each
  // step waits with a counted lgkmcnt for its own reads only (LDS returns in order), then pins its
  // fragments (an empty "+v" asm per fragment after the wait, and sched_barrier(0)) so no MFMA is
  // scheduled above the wait (cdna_hip_programming.md §5.7, rule 18).
  constexpr int NR = 1 + CT;                  // ds_read_b128 per K step
  constexpr int D = NR * 3 <= 12 ? 3 : 2;     // steps of reads in flight (<= 15 outstanding)
  auto compute_asm = [&](const int8_t* base) __attribute__((always_inline)) {
    const uint32_t lb = lds_u32(base);
    v4i fa[D], fb[D][CT];
    auto rd = [&](int ks, int u) __attribute__((always_inline)) {
      if (TK_ABL(1 << 20)) return;  // (ablation build: no fragment reads, timing only)
      const int t = ks / SUB, s = ks - t * SUB, kh = t / KT, kw = t - kh * KT;
      asm volatile("ds_read_b128 %0, %1" : "=v"(fa[u]) : "v"(lb + (uint32_t)(aoff + (s * TAPS + t) * 32)));
      const int dx = KT == 3 && h.half ? (kw == 1 ? 0 : kw == 0 ? h.half - 1 : h.half) : kw - KT / 2;
      const int gs = 2 * s * pl16, bo = ((kh - KT / 2) * hc + dx) * 16;
      [[maybe_unused]] const uint32_t me =
          KT == 3 ? (kh == 0 ? 1u : 0u) | (kh == 2 ? 2u : 0u) | (kw == 0 ? 4u : 0u) | (kw == 2 ? 8u : 0u) : 0u;
#pragma unroll
      for (int j = 0; j < CT; ++j) {
        const int jj = j < jn ? j : 0;  // (wave-uniform)
        int off = boff[jj] + bo;
        if constexpr (KT == 3) {
          if (me && (flg[jj] & me)) off = hb;
        }
        asm volatile("ds_read_b128 %0, %1" : "=v"(fb[u][j]) : "v"(lb + (uint32_t)(gs + off)));
      }
    };
#pragma unroll
    for (int k = 0; k < D - 1 && k < KS; ++k) rd(k, k);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int u = ks % D;
      if (ks + D - 1 < KS) rd(ks + D - 1, (ks + D - 1) % D);
      lgkm_wait(NR * (min(ks + D - 1, KS - 1) - ks));
      asm volatile("" : "+v"(fa[u]));
#pragma unroll
      for (int j = 0; j < CT; ++j) asm volatile("" : "+v"(fb[u][j]));
      __builtin_amdgcn_sched_barrier(0);
      if (!TK_ABL(512)) {
#pragma unroll
        for (int j = 0; j < CT; ++j)
          if (j < jn) acc[j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[u], fb[u][j], acc[j], 0, 0, 0);
      }
    }
  };
  auto compute = [&](const int8_t* base) __attribute__((always_inline)) {
    if constexpr (KT == 3) {
      if (!TK_ABL(1 << 22)) {  // (ablation build: 1 << 22 runs the compiler-scheduled steps)
        compute_asm(base);
        return;
      }
    }
    compute_c(base);
  };

  // ---- K loop: an ns-slot ring with ns - 1 stages in flight (ns from the plan: as many slots as
  // the LDS holds, since one workgroup per CU has nothing else to hide the L2 -> LDS latency
  // with); after the barrier of stage it, the slot read in step it - 1 is free for stage
  // it + ns - 1
  if (TK_ABL(1 << 24)) return;  // (ablation build: + the prologue: sources, offsets, row constants)
  if constexpr (MODE != 2) {
    const int nst = MODE == 1 ? (int)((int64_t)(zs + 1) * h.stages / S) - st_lo : h.stages, ns = h.ns;
    for (int st = 0; st < ns - 1 && st < nst; ++st) issue(st);
    // the residual words, younger than the prologue's stages: this wave's count of them stays
    // allowed in flight while those stages are retired
    const bool early_res = MODE == 3 && has_add && !TK_ABL(65536);
    const int nres = early_res && total > wave * 64 ? (total - wave * 64 + kGemmThreads - 1) / kGemmThreads : 0;
    if constexpr (MODE == 3) {
      if (early_res) issue_residual(0);
    }
    int cur = 0, nxt = ns - 1;
    for (int it = 0; it < nst; ++it) {
      if (!TK_ABL(1 << 21)) {  // (ablation build: 1 << 21 drops the stage waits, timing only)
        if constexpr (MODE == 3) wait_vm_any(min(ns - 2, nst - 1 - it) * ni + (it < ns - 1 ? nres : 0));
        else wait_vm_any(min(ns - 2, nst - 1 - it) * ni);
        lds_barrier();
      }
      if (it + ns - 1 < nst) {
        issue(nxt);
        nxt = nxt == ns - 1 ? 0 : nxt + 1;
      }
      if ((MODE == 0 || MODE == 3) && has_add && !early_res && it == nst - 1 && !TK_ABL(65536)) issue_residual(0);
      compute(smem + cur * h.stage_bytes);
      cur = cur == ns - 1 ? 0 : cur + 1;
    }
  }
  // the accumulator element (j, q) of this lane: channel row wm * 32 + (q & 3) + 8 (q >> 2) + 4 h
  // of the tile, column (wn + WN j) * 32 + lane % 32 (an image pixel of the tile)
  auto part_ptr = [&](int j, int32_t* base) __attribute__((always_inline)) -> int32_t* {
    const int col = min((wn + WN * j) * 32 + (lane & 31), h.p - 1);
    const uint32_t kk = fdiv32((uint32_t)col, h.m_hw);
    const int pix = col - (int)kk * hw;
    const int img = min(img0 + (int)kk, h.nimg - 1);
    return base + ((int64_t)img * g.M + m0 + wm * 32 + 4 * (lane >> 5)) * hw + pix;
  };
  if constexpr (MODE == 1) {
    // raw sums of this split's stages -> partial record zs (every tile column stored once: columns
    // past the tile's images are skipped)
    int32_t* base = h.part + (int64_t)zs * h.part_stride;
#pragma unroll
    for (int j = 0; j < CT; ++j)
      if (j < jn) {
        const int col = (wn + WN * j) * 32 + (lane & 31);
        const int kk = (int)fdiv32((uint32_t)min(col, h.p - 1), h.m_hw);
        if (col < h.p && img0 + kk < h.nimg) {
          int32_t* o = part_ptr(j, base);
#pragma unroll
          for (int q = 0; q < 16; ++q) o[((q & 3) + 8 * (q >> 2)) * hw] = acc[j][q];
        }
      }
    return;
  }
  if constexpr (MODE == 2) {
    if (has_add && !TK_ABL(65536)) issue_residual(0);
#pragma unroll
    for (int j = 0; j < CT; ++j)
      if (j < jn) {
        const int32_t* o = part_ptr(j, h.part);
        for (int z = 0; z < h.ksplit; ++z) {
#pragma unroll
          for (int q = 0; q < 16; ++q)
            acc[j][q] = (int32_t)((uint32_t)acc[j][q] + (uint32_t)o[(int64_t)z * h.part_stride + ((q & 3) + 8 * (q >> 2)) * hw]);
        }
      }
  }
  wait_vm(0);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0), visible to the compiler
  if (TK_ABL(4)) return;

  // ---- epilogue: stage the tile (rows = channels m0.., columns = the images' pixels) in LDS
  lds_barrier();  // the ring is free
  if (tid < R) {
    EpiRow r = row_pre;
    if (!rq_axis) r.m = g.rq.multiplier, r.s = g.rq.shift;
    if (!g.rq.zps) r.zp = g.rq.zp_in;
    r.fold = (uint32_t)0 - (uint32_t)g.zB * r.ra;  // weights' zero point 0: the fold is -za * rowsum
    if (r.s > -2) s_fast = 0;
    rowc[tid] = r;
  }
  if (has_add) {
    // RequantizeOrUpcast of every 8-bit value of both qnn.add operands (op_common.h:186-200): the
    // block's own values indexed by value - qmin (one v_lshl_add per lookup), the residual's by its
    // raw byte, with the add's - zp_out folded in
    const int32_t xb = (int32_t)g.rq.qmin + tid;
    const int32_t xr = g.rq.qmin == 0 ? tid : (int32_t)(int8_t)(uint8_t)tid;
    lut[tid] = g.add_up_b ? xb : rq_tensor(xb, g.add_pb);
    lut[256 + tid] = (int32_t)((uint32_t)(g.add_up_r ? xr : rq_tensor(xr, g.add_pr)) - (uint32_t)g.add_zp);
  }
  const int ts = h.tstride;
  // columns of the tile staged per pass: [c0, c0 + span)
  const int span = npass > 1 ? W : h.p;
  auto stage = [&](int c0) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < CT; ++j)
      if (j < jn) {
        const int lc = (wn + WN * j) * 32 + (lane & 31) - c0;
        if ((unsigned)lc < (unsigned)span) {
#pragma unroll
          for (int r = 0; r < 16; ++r) tileI[(wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)) * ts + lc] = acc[j][r];
        }
      }
  };

  // group gi = 4 consecutive elements of image run kk = gi / runq (channels m0 .. m0 + R, the W
  // pixels [c0, c0 + W) of each channel row: contiguous NCHW memory when W = hw), element
  // f = 4 (gi % runq) = row r0 (channel m0 + r0), pixel p0.  A thread's groups are 256 apart: the
  // walk advances (r0, p0) and the record / staging offsets by 1024 elements per step, without
  // divisions or products.  W % 4 == 0: a group
  // lies in one channel row (one b128 read of the tile, one row of constants); else (7x7, one pass)
  // it may cross into the next row, whose elements take that row's constants.
  const uint32_t n4 = g.out_elems * 4u;
  const auto r_conv = rec_rsrc(g.C, n4), r_bias = rec_rsrc(g.bias_out, n4);
  const auto r_rq = rec_rsrc(g.rq_out, g.out_elems);
  const auto r_add = rec_rsrc(g.add_out, has_add ? g.out_elems : 0u);
  const auto r_clip = rec_rsrc(g.clip_out, g.has_clip ? g.out_elems : 0u);
  const int32_t qmin = (int32_t)g.rq.qmin, qmax = (int32_t)g.rq.qmax, zpo = g.rq.zp_out;
  const int32_t clip_lo = g.clip_lo, clip_hi = g.clip_hi, add_zp = g.add_zp;
  const int mode = g.rq.mode, Mrows = g.M;
  const int dr = 1024 / W, dp = 1024 - dr * W;
  // the walk's record offset o and staging slot base advance by fixed steps plus a correction
  // for each pixel / row wrap (no per-group products)
  const uint32_t dO = (uint32_t)(dr * hw + dp), dOp = (uint32_t)(hw - W), dOr = (uint32_t)((Mrows - R) * hw);
  const int dB = dr * ts + dp, dBp = ts - W, dBr = W - R * ts;
  const int32_t* lut_b = lut - (int32_t)g.rq.qmin;  // lut_b[q], q in [qmin, qmin + 255]
  const int tile_end = R * ts;  // staging words (a group's reads are clamped below it)
  int c0 = 0;  // first pixel of the current pass
  // nontemporal record stores (plain ones measured no faster, also on multi-pass epilogues:
  // profiles/r03k_img_epilogue_ablations.txt)
  auto st128 = [&](v4u v, __amdgpu_buffer_rsrc_t rsrc, uint32_t off) __attribute__((always_inline)) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, v), rsrc, off, 0, kAuxNT);
  };
  auto st32 = [&](uint32_t v, __amdgpu_buffer_rsrc_t rsrc, uint32_t off) __attribute__((always_inline)) {
    __builtin_amdgcn_raw_buffer_store_b32(v, rsrc, off, 0, kAuxNT);
  };
  auto walk = [&](auto fast_c, auto add_c, auto clip_c, auto rowu_c) __attribute__((always_inline)) {
    constexpr bool FAST = decltype(fast_c)::value, ADD = decltype(add_c)::value, CLIP = decltype(clip_c)::value;
    constexpr bool ROWU = decltype(rowu_c)::value;
    int kk = 0, r0 = (4 * tid) / W, p0 = 4 * tid - r0 * W;
    while (r0 >= R) r0 -= R, ++kk;
    uint32_t on = (uint32_t)(((img0 + kk) * Mrows + m0 + r0) * hw + c0 + p0);
    // software pipeline by one group: the next group's tile values, row constants and residual
    // word are read from LDS before this group's arithmetic and stores (at one or two waves per
    // SIMD nothing else hides the LDS latency); every step reads the next group's slots, also past
    // the last group, whose position (up to W + 4 words beyond the staging tile) is clamped into
    // the tile (values unused)
    auto load = [&](int r, int base, int p, int gi, v4u& v, EpiRow& ra, EpiRow& rb, uint32_t& res)
        __attribute__((always_inline)) {
      if (TK_ABL(1 << 25)) {  // (ablation build: no LDS reads in the walk -- values from registers)
        v = v4u{(uint32_t)base, (uint32_t)gi, 7u, (uint32_t)r};
        ra = rb = row_pre;
        res = 0x01010101u;
        return;
      }
      ra = rowc[min(r, R - 1)];
      if constexpr (ROWU) {
        v = *reinterpret_cast<const v4u*>(tileI + min(base, tile_end - 4));
        rb = ra;
      } else {
        rb = rowc[min(r + 1, R - 1)];
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (uint32_t)tileI[min(base + e + (p + e >= W ? ts - W : 0), tile_end - 1)];
      }
      if constexpr (ADD) res = TK_ABL(32768) ? 0x01010101u : resw[min(gi, total - 1)];
    };
    v4u vn;
    EpiRow ran, rbn;
    uint32_t resn = 0;
    int basen = r0 * ts + kk * W + p0;
    load(r0, basen, p0, tid, vn, ran, rbn, resn);
    for (int gi = tid; gi < total; gi += kGemmThreads) {
      const uint32_t o = on;
      const int base = basen, pc = p0;
      v4u v = vn;
      const EpiRow ra = ran, rb = rbn;
      const uint32_t res = resn;
      // next group: 1024 elements on
      r0 += dr;
      p0 += dp;
      on += dO;
      basen += dB;
      if (p0 >= W) p0 -= W, ++r0, on += dOp, basen += dBp;
      while (r0 >= R) r0 -= R, on += dOr, basen += dBr;
      load(r0, basen, p0, gi + kGemmThreads, vn, ran, rbn, resn);
      uint32_t fold[4], zp[4];
      int32_t bias[4], m[4], sh[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool nx = !ROWU && pc + e >= W;
        fold[e] = nx ? rb.fold : ra.fold;
        bias[e] = nx ? rb.bias : ra.bias;
        zp[e] = nx ? (uint32_t)rb.zp : (uint32_t)ra.zp;
        m[e] = nx ? rb.m : ra.m;
        sh[e] = nx ? rb.s : ra.s;
      }
      if (TK_ABL(262144)) {
        // profiling: every record stored with no epilogue arithmetic (raw accumulators / their low
        // bytes): the store side of the epilogue alone, at the kernel's own occupancy and order
        st128(v, r_conv, o * 4u);
        st128(v, r_bias, o * 4u);
        const uint32_t b8 = pack4u((int32_t)v[0], (int32_t)v[1], (int32_t)v[2], (int32_t)v[3]);
        st32(b8, r_rq, o);
        if constexpr (ADD) st32(b8 ^ res, r_add, o);
        if constexpr (CLIP) st32(b8, r_clip, o);
        continue;
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] += fold[e];
      if (!TK_ABL(2)) st128(v, r_conv, o * 4u);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] += (uint32_t)bias[e];
      if (!TK_ABL(2)) st128(v, r_bias, o * 4u);
      int32_t q[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int32_t t = (int32_t)(v[e] - zp[e]);
        int32_t y;
        if constexpr (FAST) {
          // right shift >= 2: (x·m + 2^(30+rs)) >> (31+rs) only needs the high word of x·m
          const int sh2 = -sh[e] - 1;
          y = (int32_t)((uint32_t)__mulhi(t, m[e]) + (1u << (sh2 - 1))) >> sh2;
        } else {
          y = rq_core(t, mode, m[e], sh[e]);
        }
        q[e] = clamp_i32((int32_t)((uint32_t)zpo + (uint32_t)y), qmin, qmax);
      }
      if (!TK_ABL(2)) st32(pack4u(q[0], q[1], q[2], q[3]), r_rq, o);
      if constexpr (ADD) {
        // qnn.add (src/relay/qnn/op/add.cc:40-96): RQ(block) + RQ(residual) - zp_out
#pragma unroll
        for (int e = 0; e < 4; ++e)
          q[e] = clamp_i32(TK_ABL(8192) ? q[e] + (int32_t)((res >> (8 * e)) & 0xFFu) - add_zp
                                        : (int32_t)((uint32_t)lut_b[q[e]] + (uint32_t)lut[256 + ((res >> (8 * e)) & 0xFFu)]),
                           qmin, qmax);
        if (!TK_ABL(16384 | 2)) st32(pack4u(q[0], q[1], q[2], q[3]), r_add, o);
      }
      if constexpr (CLIP) {
#pragma unroll
        for (int e = 0; e < 4; ++e) q[e] = clamp_i32(q[e], clip_lo, clip_hi);
        if (!TK_ABL(2)) st32(pack4u(q[0], q[1], q[2], q[3]), r_clip, o);
      }
      if constexpr (ROWU) {
        *reinterpret_cast<v4i*>(tileI + base) = v4i{q[0], q[1], q[2], q[3]};
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) tileI[base + e + (pc + e >= W ? ts - W : 0)] = q[e];
      }
    }
  };
  using T = std::true_type;
  using F = std::false_type;
  auto by_rowu = [&](auto fast_c, auto add_c, auto clip_c) __attribute__((always_inline)) {
    if (W % 4 == 0) walk(fast_c, add_c, clip_c, T{});
    else walk(fast_c, add_c, clip_c, F{});
  };
  auto by_clip = [&](auto fast_c, auto add_c) __attribute__((always_inline)) {
    if (g.has_clip) by_rowu(fast_c, add_c, T{});
    else by_rowu(fast_c, add_c, F{});
  };
  auto by_add = [&](auto fast_c) __attribute__((always_inline)) {
    if (has_add) by_clip(fast_c, T{});
    else by_clip(fast_c, F{});
  };
  for (int pass = 0; pass < npass; ++pass) {
    c0 = pass * W;
    if (pass) {
      lds_barrier();  // the previous pass is done with the staging tile and the residual words
      if (has_add && !TK_ABL(65536)) issue_residual(c0);
    }
    stage(c0);
    if (pass && has_add) {
      wait_vm(0);
      __builtin_amdgcn_s_waitcnt(0x0F70);
    }
    lds_barrier();  // (also publishes s_fast and the row constants)
    if (s_fast && (mode == TK_RQ_AXIS_UPWARD || mode == TK_RQ_TENSOR_UPWARD)) by_add(T{});
    else by_add(F{});

    // ---- the next conv's shadow: 16 channels of one pixel per 16-byte store; the pass's columns
    // are the images' pixels in order, so column col is shadow pixel img0 * hw + c0 + col
    if (g.shadow_out && !TK_ABL(1)) {
      lds_barrier();
      const uint32_t sx4 = (uint32_t)g.shadow_xor * 0x01010101u;
      const int pe = npass > 1 ? W : nimg * hw;  // this pass's pixels (the last workgroup may hold fewer images)
#pragma unroll
      for (int grp = 0; grp < R / 16; ++grp)
        for (int col = tid; col < pe; col += kGemmThreads) {
          uint32_t wd[4];
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            const int32_t* t = tileI + (grp * 16 + d * 4) * ts + col;
            wd[d] = pack4u((uint32_t)t[0], (uint32_t)t[ts], (uint32_t)t[2 * ts], (uint32_t)t[3 * ts]) ^ sx4;
          }
          *reinterpret_cast<v4i*>(g.shadow_out +
                                  ((int64_t)((m0 >> 4) + grp) * g.N + (int64_t)img0 * hw + c0 + col) * 16) =
              v4i{(int)wd[0], (int)wd[1], (int)wd[2], (int)wd[3]};
        }
    }
  }
}

// ---------------------------------------------------------------- chunked weight packing
// OIHW (int8, or uint8 stored xor 0x80) -> [rows_pad][cin_pad / 32][taps][32]: a stage of 32 input
// channels is one contiguous run of taps * 32 bytes per row.  Padding rows / channels are 0.
__global__ __launch_bounds__(256) void pack_chunked_kernel(const int8_t* __restrict__ w, int8_t* __restrict__ dst,
                                                           int Cout, int Cin, int taps, int cin_pad, int xor_u8) {
  const int o = blockIdx.x;
  const int row = taps * cin_pad;
  for (int k = threadIdx.x; k < row; k += blockDim.x) {
    const int c32 = k / (taps * 32), rem = k - c32 * taps * 32;
    const int tap = rem >> 5, c = c32 * 32 + (rem & 31);
    int8_t v = 0;
    if (o < Cout && c < Cin) {
      const uint8_t raw = (uint8_t)w[((int64_t)o * Cin + c) * taps + tap];
      v = (int8_t)(xor_u8 ? (raw ^ 0x80) : raw);
    }
    dst[(int64_t)o * row + k] = v;
  }
}

int64_t conv_img_chunked_bytes(int rows_pad, int cin_pad, int taps) {
  return taps > 1 && cin_pad % 32 == 0 ? (int64_t)rows_pad * taps * cin_pad : 0;
}

int conv_img_pack(const tk_tensor* weight, int8_t* dst, int rows_pad, int cin_pad, hipStream_t s) {
  const int O = (int)weight->shape[0], C = (int)weight->shape[1];
  const int taps = (int)(weight->shape[2] * weight->shape[3]);
  if (!conv_img_chunked_bytes(rows_pad, cin_pad, taps)) return TK_OK;
  hipLaunchKernelGGL(pack_chunked_kernel, dim3(rows_pad), dim3(256), 0, s, (const int8_t*)ptr(weight), dst, O, C, taps,
                     cin_pad, (int)is_uint(weight, 8));
  TK_LAUNCH_CHECK();
  return TK_OK;
}

// ---------------------------------------------------------------- plan + launch
namespace {

using ImgKernel = void (*)(GemmArgs, ImgArgs);

template <int KT, int WM, int CC>
ImgKernel img_kernel_cc(int ct) {
  if constexpr (WM == 1 && KT == 1) {  // (3x3 with 7 column tiles per wave spills: not planned)
    if (ct == 7) return conv_img_kernel<KT, WM, 7, CC>;
  }
  return ct == 2 ? conv_img_kernel<KT, WM, 2, CC> : conv_img_kernel<KT, WM, 4, CC>;
}

template <int KT, int WM>
ImgKernel img_kernel(int ct, int cc) {
  if constexpr (KT == 3) {
    return cc == 64 ? img_kernel_cc<3, WM, 64>(ct) : img_kernel_cc<3, WM, 32>(ct);
  } else {
    return cc == 32 ? img_kernel_cc<1, WM, 32>(ct) : cc == 64 ? img_kernel_cc<1, WM, 64>(ct) : img_kernel_cc<1, WM, 128>(ct);
  }
}

// 1x1 joins with two workgroups per CU: residual words issued early (MODE 3)
template <int WM>
ImgKernel img_kernel_early(int ct, int cc) {
  if (cc == 128) return ct == 2 ? conv_img_kernel<1, WM, 2, 128, 3> : conv_img_kernel<1, WM, 4, 128, 3>;
  if (cc == 64) return ct == 2 ? conv_img_kernel<1, WM, 2, 64, 3> : conv_img_kernel<1, WM, 4, 64, 3>;
  return ct == 2 ? conv_img_kernel<1, WM, 2, 32, 3> : conv_img_kernel<1, WM, 4, 32, 3>;
}

// Split-K kernels: the partial pass (MODE 1) and the epilogue pass (MODE 2: one 32-row tiling for
// 1x1 and 3x3 alike -- it has no K loop, so neither the taps nor the stage width matter there)
template <int KT, int WM, int MODE>
ImgKernel img_kernel_split(int ct, int cc) {
  if constexpr (MODE == 2) {
    return ct == 2 ? conv_img_kernel<3, WM, 2, 32, 2> : conv_img_kernel<3, WM, 4, 32, 2>;
  } else {
    if constexpr (KT == 1) {
      if (cc == 128) return ct == 2 ? conv_img_kernel<1, WM, 2, 128, MODE> : conv_img_kernel<1, WM, 4, 128, MODE>;
    }
    if (cc == 64) return ct == 2 ? conv_img_kernel<KT, WM, 2, 64, MODE> : conv_img_kernel<KT, WM, 4, 64, MODE>;
    return ct == 2 ? conv_img_kernel<KT, WM, 2, 32, MODE> : conv_img_kernel<KT, WM, 4, 32, MODE>;
  }
}

struct ImgPlan {
  ImgArgs a;
  size_t lds;
  int kt, wm, ct, cc, occ;
  double cost;
  // split K (ksplit > 1): `a` is the partial pass, `b` the epilogue pass
  int ksplit;
  ImgArgs b;
  size_t lds_b;
  int wm_b, ct_b;
};

uint32_t magic32(uint32_t d) { return (uint32_t)(((1ull << 32) + d - 1) / d); }  // d >= 2

// Most output columns a workgroup holds: 4 waves x 7 column tiles (R = 32), 2 x 4 (R = 64).
constexpr int kImgMaxCols = 4 * 7 * 32;
constexpr int kImgMaxSplit = 4;  // split-K partial records a 3x3 block may need (scratch)

// One candidate tiling (R rows, ipt images per workgroup, CC channels per stage, one or two
// workgroups per CU, the epilogue in npass column passes); false if it does not fit.
// mode: 0 the whole block, 1 / 2 the partial / epilogue pass of a split-K plan over ksplit splits
// (mode 1 needs no epilogue staging, mode 2 no ring)
bool img_candidate(const ConvGeom& g, const GemmArgs& ga, int kt, int st, int R, int ipt, int CC, bool two,
                   int npass, ImgPlan* out, int mode = 0, int ksplit = 1) {
  const int taps = kt * kt;
  const int hw = g.OH * g.OW;
  // several passes: one image per workgroup, each pass a whole number of 4-pixel groups per row
  if (npass > 1 && (ipt != 1 || hw % (4 * npass))) return false;
  const int cw = hw / npass;
  const int p = ipt * hw;
  const int nct = (p + 31) / 32;
  const int wm = R / 32, wn = 4 / wm;
  const int ct_need = (nct + wn - 1) / wn;
  const int ct = ct_need <= 2 ? 2 : ct_need <= 4 ? 4 : ct_need <= 7 ? 7 : 0;
  if (!ct || (ct == 7 && (wm != 1 || kt == 3))) return false;
  ImgArgs x{};
  x.nimg = g.N;
  x.ipt = ipt;
  // 3x3: the images' input pixels, dense, after `lead` slots of slack (reads up to W + 1 slots
  // either side of a pixel land in the slack or a neighbour, and are replaced by the zero point);
  // 1x1: the input pixels the (strided) outputs read
  x.hr = kt == 3 ? g.H : g.OH;
  x.hc = kt == 3 ? g.W : g.OW;
  x.half = kt == 3 && st == 2 && g.W % 2 == 0 ? g.W / 2 : 0;
  x.lead = kt == 3 ? g.W + 1 : 0;
  x.pl = x.lead + ipt * x.hr * x.hc;
  x.ih0 = 0;
  x.iw0 = 0;
  x.ls = kt == 3 ? 1 : st;
  x.ps = kt == 3 ? st : 1;
  x.hw = hw;
  x.p = p;
  x.nct = nct;
  x.mtiles = g.O / R;
  x.wgs = (int32_t)(((int64_t)g.N + ipt - 1) / ipt * x.mtiles);
  x.wgs8 = (x.wgs + 7) / 8 * 8;
  x.stages = g.cin_pad / CC;
  x.ksplit = ksplit;
  if (mode == 1 && x.stages < ksplit) return false;
  x.pslots = CC / 16 * x.pl + x.lead;  // + trailing slack after the last channel group
  x.wslot = taps * CC / 16 + 1;
  x.sslots = x.pslots + R * x.wslot;
  x.ni = ((x.sslots + 63) / 64 + 3) / 4;
  if (x.ni > kImgNI) return false;
  x.stage_bytes = 4 * x.ni * 1024;
  const int64_t pstep = (int64_t)(CC / 16) * ga.in_pix * 16;
  if (pstep >= (1ll << 31)) return false;
  x.pstep = (int32_t)pstep;
  x.npass = npass;
  x.cw = cw;
  x.skew = env_int("TK_IMG_SKEW", 0);
  x.early_res = two ? 1 : 0;
  x.tstride = npass > 1 ? cw + 4 : nct * 32 + 4;
  // ring depth: every slot the LDS budget holds (up to 8, no more than the stages need), at least
  // 3 where there are more than 2 stages and one workgroup per CU.  The budget is the CU's 160 KB, or half of it for two
  // resident workgroups (one's epilogue stores then overlap the other's K loop).
  const size_t res_bytes = ga.has_add && mode != 1 ? ((size_t)(npass > 1 ? cw : p) * R + 255) / 256 * 256 : 0;
  const size_t extra = mode == 1 ? 0 : (size_t)R * sizeof(EpiRow) + 2048 + res_bytes;
  const size_t tile = mode == 1 ? 0 : (size_t)R * x.tstride * 4;
  const int cap = env_int("TK_IMG_NS", 8);
  const size_t budget = (two ? 80 : 160) * 1024 - 64 - extra;
  if (tile > budget) return false;
  size_t ring = 0;
  if (mode != 2) {
    const int kst = mode == 1 ? (x.stages + ksplit - 1) / ksplit : x.stages;  // a split's stages
    x.ns = (int)std::min<size_t>({(size_t)cap, budget / x.stage_bytes, (size_t)kst + 1});
    // one workgroup per CU needs a stage in flight while it computes; two may double-buffer (the
    // other workgroup computes while this one waits)
    if (x.ns < (kst > 2 && !two ? 3 : 2)) return false;
    ring = (size_t)x.ns * x.stage_bytes;
  }
  x.rowc_off = (int32_t)std::max(ring, tile);
  x.lut_off = x.rowc_off + (mode == 1 ? 0 : R * (int)sizeof(EpiRow));  // (the partial pass has no epilogue)
  x.res_off = x.lut_off + (mode == 1 ? 0 : 2048);
  const size_t lds = (size_t)x.res_off + res_bytes;
  if (lds > (two ? 80 : 160) * 1024 - 64) return false;
  x.runq = R * cw / 4;
  // the kernel's 32-bit index arithmetic (fdiv32, 24-bit products): every divisor in [2, 2^16),
  // every dividend below 2^16 (slots, tile columns, epilogue groups and their R * cw pixels), and
  // the input's byte offsets (channel groups of a stage x in_pix x 16) below 2^31 (pstep, above)
  for (int64_t d : {(int64_t)cw, (int64_t)x.pl, (int64_t)x.hr * x.hc, (int64_t)x.hc, (int64_t)x.wslot, (int64_t)hw,
                    (int64_t)g.OW, (int64_t)x.runq})
    if (d < 2 || d >= 65536) return false;
  if ((int64_t)R * cw >= 65536 || p >= 65536 || x.ni * 256 >= 65536 || 9ll * g.cin_pad >= (1ll << 24) ||
      ga.lda >= (1ll << 24))
    return false;
  x.m_cw = magic32(cw);
  x.m_pl = magic32(x.pl);
  x.m_img = magic32((uint32_t)(x.hr * x.hc));
  x.m_hc = magic32(x.hc);
  x.m_ws = magic32(x.wslot);
  x.m_hw = magic32(hw);
  x.m_ow = magic32(g.OW);
  x.m_runq = magic32(x.runq);
  out->a = x;
  out->lds = lds;
  out->kt = kt;
  out->wm = wm;
  out->ct = ct;
  out->cc = CC;
  out->occ = two ? 2 : 1;
  // estimated time per CU (ns): each workgroup's K loop = max(L2 -> LDS bytes at ~55 GB/s per CU,
  // the busiest wave's MFMA cycles at ~2.1 GHz) and epilogue = its record bytes at ~22 GB/s per CU
  // (~5.6 TB/s over 256 CUs), plus ~2 us of load latency per round.  One workgroup per CU runs
  // them back to back; two overlap one's epilogue with the other's K loop.
  const double K = (double)taps * g.cin_pad / (mode == 1 ? ksplit : 1);
  const double bytes = R * K + (double)x.pl * g.cin_pad / (mode == 1 ? ksplit : 1);
  // (mode 2: reading the ksplit partial tiles instead of the K loop; mode 1: storing one)
  const double main_ns = mode == 2 ? (double)ksplit * R * p * 4 / 55.0 : std::max(bytes / 55.0, ct_need * K / 2.1);
  const double epi_ns = mode == 1 ? (double)R * p * 4 / 22.0 : (double)R * p * (ga.has_add ? 12.0 : 10.0) / 22.0;
  const double per_cu = std::ceil(x.wgs / 256.0);
  const double lat = 2000.0;
  out->cost = two && per_cu >= 2 ? per_cu * std::max(main_ns, epi_ns) + lat + std::min(main_ns, epi_ns)
                                 : per_cu * (lat + main_ns + epi_ns);
  out->cost += per_cu * (npass - 1) * 1000.0;  // a store drain + barrier per extra pass
  out->ksplit = 1;
  return true;
}

// The long-K layers on small planes (7x7, 14x14: 3x3, and the 1x1 reduces over 1024-2048 channels)
// are bound by their L2 -> LDS bytes: every workgroup streams its R weight rows of all K plus its
// images' patch, so wide tiles (more images, R = 64) re-read less but leave CUs idle.  Split K
// keeps them: ksplit workgroups per wide tile each reduce a share of the stages into a partial
// record (NCHW int32), and a second pass with small tiles (R = 32, enough workgroups for the
// chip) sums the partials and runs the block epilogue.
bool img_split_candidate(const ConvGeom& g, const GemmArgs& ga, int kt, int st, int R, int ipt, int CC, bool two,
                         int ksplit, ImgPlan* out) {
  ImgPlan pa{}, pb{}, best_b{};
  if (!img_candidate(g, ga, kt, st, R, ipt, CC, two, 1, &pa, 1, ksplit)) return false;
  if (pa.ct > 4) return false;  // (the split kernels are instantiated for 2 and 4 column tiles per wave)
  const int tiles = pa.a.wgs, wgs = tiles * ksplit;
  if (tiles > 256 || wgs > 2048) return false;  // the plain plans already fill the chip
  pa.a.wgs = wgs;
  pa.a.wgs8 = (wgs + 63) / 64 * 64;  // (a multiple of 8 * ksplit: a tile's splits share an XCD)
  // the epilogue pass: 32-row tiles of as many images as keep >= 512 workgroups
  const int hw = g.OH * g.OW;
  bool have_b = false;
  for (int ipt_b = std::max(1, std::min(kImgMaxCols / hw, g.N)); ipt_b >= 1; --ipt_b)
    for (int two_b = 1; two_b >= 0; --two_b)
      if (g.O % 32 == 0 && img_candidate(g, ga, kt, st, 32, ipt_b, 32, two_b, 1, &pb, 2, ksplit) && pb.ct <= 4 &&
          (!have_b || pb.cost < best_b.cost)) {
        best_b = pb;
        have_b = true;
      }
  if (!have_b) return false;
  *out = pa;
  // (pa.cost counted rounds of `tiles` workgroups per CU; the pass runs ksplit times as many)
  out->cost = pa.cost * std::ceil(wgs / 256.0) / std::ceil(tiles / 256.0) + best_b.cost + 1000.0;
  out->ksplit = ksplit;
  out->b = best_b.a;
  out->lds_b = best_b.lds;
  out->wm_b = best_b.wm;
  out->ct_b = best_b.ct;
  return true;
}

}  // namespace

namespace {

std::vector<ImgPlan> img_plans_build(const ConvGeom& g, const tk_conv2d_attrs* a, const GemmArgs& ga,
                                     bool have_chunked);

// Every image-tile plan that applies to the conv block, in enumeration order (R, stage width,
// images per tile, one or two workgroups per CU, then the split-K plans); empty when the kernel
// does not apply.  Memoised per block shape: a 7x7 block enumerates ~1,000 candidates (split
// plans each search an epilogue tiling), and the launch path plans on every call, so without the
// cache each launch spent ~15-20 us of host time before its kernel -- idle GPU time inside the
// find step's event-timed launches, which made every image plan of those blocks look 2x slower.
using ImgPlans = std::shared_ptr<const std::vector<ImgPlan>>;

ImgPlans img_plans(const ConvGeom& g, const tk_conv2d_attrs* a, const GemmArgs& ga, bool have_chunked) {
  // Outside the ablation build tune_env() is compiled to nullptr (tk_conv.h), so every TK_IMG*
  // knob read by img_plans_build / img_candidate / conv_img_split_scratch_bytes is its constant
  // default and the geometry is the whole key.  The ablation build (plans follow TK_IMG_*
  // variables set between calls) keys its cache by the knobs' values too, so that its launches
  // cost a lookup like the product's (re-planning per launch made host time the measurement).
  std::string knobs;
#ifdef TK_ABLATION_BUILD
  for (const char* k : {"TK_IMG", "TK_IMG3", "TK_IMG1", "TK_IMG_MAXHW", "TK_IMG_R", "TK_IMG_IPT", "TK_IMG_CC",
                        "TK_IMG_TWO", "TK_IMG_SPLIT", "TK_IMG_NS", "TK_IMG_SKEW"}) {
    const char* v = tune_env(k);
    knobs += std::string(k) + "=" + (v ? v : "") + ";";
  }
#endif
  const std::array<int64_t, 27> key = {g.N, g.C, g.H, g.W, g.O, g.KH, g.KW, g.OH, g.OW, g.cin_pad, g.k_pad,
                                       g.rows_pad, a->strides[0], a->strides[1], a->padding[0], a->padding[1],
                                       a->padding[2], a->padding[3], a->dilation[0], a->dilation[1],
                                       ga.bias_out != nullptr, ga.RB != nullptr, ga.zA_vec != nullptr, ga.zA,
                                       ga.has_add, ga.in_pix, have_chunked};
  static std::mutex mu;
  static std::map<std::pair<std::array<int64_t, 27>, std::string>, ImgPlans> cache;
  const auto ck = std::make_pair(key, knobs);
  {
    std::lock_guard<std::mutex> lock(mu);
    auto it = cache.find(ck);
    if (it != cache.end()) return it->second;
  }
  ImgPlans plans = std::make_shared<const std::vector<ImgPlan>>(img_plans_build(g, a, ga, have_chunked));
  std::lock_guard<std::mutex> lock(mu);
  if (cache.size() > 4096) cache.clear();
  cache.emplace(ck, plans);
  return plans;
}

std::vector<ImgPlan> img_plans_build(const ConvGeom& g, const tk_conv2d_attrs* a, const GemmArgs& ga,
                                     bool have_chunked) {
  std::vector<ImgPlan> out;
  if (!env_int("TK_IMG", 1) || !ga.bias_out) return out;  // conv blocks only
  if (ga.RB || ga.zA_vec || ga.zA != 0) return out;       // the weights' zero point must be 0
  if (a->dilation[0] != 1 || a->dilation[1] != 1) return out;
  const int st = a->strides[0];
  if (a->strides[1] != st || (st != 1 && st != 2)) return out;
  int kt = 0;
  if (g.KH == 3 && g.KW == 3 && a->padding[0] == 1 && a->padding[1] == 1 && a->padding[2] == 1 && a->padding[3] == 1)
    kt = 3;
  else if (g.KH == 1 && g.KW == 1 && !a->padding[0] && !a->padding[1] && !a->padding[2] && !a->padding[3])
    kt = 1;
  if (!kt || (kt == 3 && !have_chunked)) return out;
  if (kt == 3 && !env_int("TK_IMG3", 1)) return out;
  if (kt == 1 && !env_int("TK_IMG1", 1)) return out;
  const int hw = g.OH * g.OW;
  if (g.cin_pad % 32 || g.O % 32 || hw > env_int("TK_IMG_MAXHW", kImgMaxCols) || hw < 4 ||
      (int64_t)g.N * hw * g.O * 4 >= 0xFFFFFFC0ll)
    return out;
  const int force_r = env_int("TK_IMG_R", 0), force_ipt = env_int("TK_IMG_IPT", 0);
  const int force_cc = env_int("TK_IMG_CC", 0), two_mode = env_int("TK_IMG_TWO", 1);  // 0 never, 2 only
  ImgPlan c{};
  for (int R : {64, 32}) {
    if (g.O % R || (force_r && R != force_r)) continue;
    const int maxcols = R == 32 ? kImgMaxCols : 256;
    for (int CC : {128, 64, 32}) {
      if ((kt == 3 && CC > 64) || g.cin_pad % CC || (force_cc && CC != force_cc)) continue;
      for (int ipt = std::min(maxcols / hw, g.N); ipt >= 1; --ipt) {
        if (force_ipt && ipt != force_ipt) continue;
        for (int two = 0; two < 2; ++two) {
          if ((two && !two_mode) || (!two && two_mode == 2)) continue;
          for (int npass : {1, 2, 4})
            if (img_candidate(g, ga, kt, st, R, ipt, CC, two, npass, &c)) out.push_back(c);
        }
      }
    }
  }
  // split-K plans, after the plain ones so that the plain plans' algo numbers stay put
  if (env_int("TK_IMG_SPLIT", 1) && g.N * (int64_t)g.O * hw * 4 * kImgMaxSplit <= ((int64_t)1 << 31))
    for (int S : {2, 4})
      for (int R : {64, 32}) {
        if (g.O % R || (force_r && R != force_r)) continue;
        const int maxcols = R == 32 ? kImgMaxCols : 256;
        for (int CC : {128, 64, 32}) {
          if ((kt == 3 && CC > 64) || g.cin_pad % CC || (force_cc && CC != force_cc)) continue;
          for (int ipt = std::min(maxcols / hw, g.N); ipt >= 1; --ipt)
            for (int two = 0; two < 2; ++two)
              if (img_split_candidate(g, ga, kt, st, R, ipt, CC, two, S, &c)) out.push_back(c);
        }
      }
  return out;
}

}  // namespace

int conv_img_algos(const ConvGeom& g, const tk_conv2d_attrs* a, const GemmArgs& ga, bool have_chunked,
                   int32_t* algos, int max_algos) {
  const ImgPlans pp = img_plans(g, a, ga, have_chunked);
  const std::vector<ImgPlan>& plans = *pp;
  std::vector<int> order(plans.size());
  for (size_t i = 0; i < order.size(); ++i) order[i] = (int)i;
  std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return plans[x].cost < plans[y].cost; });
  // the find step times the first candidates only: give the split-K plans (whose two-pass cost the
  // model knows least well) 5 of the first 14 places, the plain plans the other 9
  {
    std::vector<int> plain, split, head, rest;
    for (int i : order) (plans[i].ksplit > 1 ? split : plain).push_back(i);
    const size_t ns = std::min<size_t>(split.size(), 5), np = std::min<size_t>(plain.size(), 14 - ns);
    for (size_t i = 0; i < plain.size(); ++i) (i < np ? head : rest).push_back(plain[i]);
    for (size_t i = 0; i < split.size(); ++i) (i < ns ? head : rest).push_back(split[i]);
    std::stable_sort(head.begin(), head.end(), [&](int x, int y) { return plans[x].cost < plans[y].cost; });
    std::stable_sort(rest.begin(), rest.end(), [&](int x, int y) { return plans[x].cost < plans[y].cost; });
    order = head;
    order.insert(order.end(), rest.begin(), rest.end());
  }
  for (int k = 0; k < (int)order.size() && k < max_algos; ++k) algos[k] = kAlgoImg0 + order[k];
  return (int)plans.size();
}

int conv_img_describe(const ConvGeom& g, const tk_conv2d_attrs* a, const GemmArgs& ga, bool have_chunked, int algo,
                      char* buf, int len) {
  const ImgPlans pp = img_plans(g, a, ga, have_chunked);
  const std::vector<ImgPlan>& plans = *pp;
  const int i = algo - kAlgoImg0;
  if (i < 0 || i >= (int)plans.size()) return TK_ERR_INVALID_ARG;
  const ImgPlan& p = plans[i];
  const ImgArgs& x = p.a;
  int n = std::snprintf(buf, (size_t)len, "image tiles %dx%d: %d rows x %d image%s (%d columns), %d-channel stages, "
                        "%d-slot ring, %d workgroup%s per CU, %d epilogue pass%s, %.1f KB LDS",
                        p.kt, p.kt, 32 * p.wm, x.ipt, x.ipt > 1 ? "s" : "", x.p, p.cc, x.ns, p.occ, p.occ > 1 ? "s" : "",
                        x.npass, x.npass > 1 ? "es" : "", p.lds / 1024.0);
  if (p.ksplit > 1 && n >= 0 && n < len)
    std::snprintf(buf + n, (size_t)(len - n), "; split K %d ways (%d workgroups), then an epilogue pass of %d rows x %d "
                  "image%s (%d workgroups)", p.ksplit, x.wgs, 32 * p.wm_b, p.b.ipt, p.b.ipt > 1 ? "s" : "", p.b.wgs);
  return TK_OK;
}

int64_t conv_img_split_scratch_bytes(const ConvGeom& g) {
  // the partial records of a split-K image-tile plan (1x1 and 3x3 blocks)
  if (g.KH != g.KW || (g.KH != 1 && g.KH != 3) || !env_int("TK_IMG_SPLIT", 1)) return 0;
  const int64_t rec = (int64_t)g.N * g.O * g.OH * g.OW * 4;
  return rec * kImgMaxSplit <= ((int64_t)1 << 31) && g.OH * g.OW <= kImgMaxCols ? rec * kImgMaxSplit : 0;
}

static int set_lds(ImgKernel kern, size_t lds, int* rc) {
  if (lds <= 64 * 1024) return 0;
  // dynamic LDS beyond 64 KiB must be allowed per kernel (the static s_fast word counts too)
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    set_error(std::string("conv image-tile kernel: LDS attribute failed: ") + hipGetErrorString(e));
    *rc = TK_ERR_HIP;
    return 1;
  }
  return 0;
}

int conv_img_try(const ConvGeom& g, const tk_conv2d_attrs* a, const GemmArgs& ga, const int8_t* chunked, void* scratch,
                 int algo, hipStream_t s, int* rc) {
  if (algo == kAlgoIm2col || algo == kAlgoPf2 || algo == kAlgoPf3) return 0;
  const ImgPlans pp = img_plans(g, a, ga, chunked != nullptr);
  const std::vector<ImgPlan>& plans = *pp;
  if (plans.empty() && algo == 0) return 0;
  if (plans.empty() || (algo >= kAlgoImg0 && algo - kAlgoImg0 >= (int)plans.size()) ||
      (algo != 0 && algo != kAlgoImg && algo < kAlgoImg0)) {
    set_error("tk_qnn_conv2d_block: algo " + std::to_string(algo) + " does not apply to this conv (" +
              std::to_string(plans.size()) + " image-tile plans; see tk_conv2d_block_algos)");
    *rc = TK_ERR_INVALID_ARG;
    return 1;
  }
  ImgPlan best = plans[0];
  if (algo >= kAlgoImg0) {
    best = plans[algo - kAlgoImg0];
  } else {
    // the library's own choice: the cheapest plain plan (split plans are the find step's to pick)
    for (const ImgPlan& p : plans)
      if (p.ksplit == 1 && p.cost < best.cost) best = p;
  }
  const int kt = best.kt;
  best.a.wimg = kt == 3 ? chunked : ga.A;
  best.a.ldw = kt == 3 ? 9 * g.cin_pad : ga.lda;
  if (best.ksplit > 1) {
    if (!scratch) {
      set_error("tk_qnn_conv2d_block: split-K image-tile plan needs scratch (tk_conv2d_scratch_bytes)");
      *rc = TK_ERR_INVALID_ARG;
      return 1;
    }
    const int64_t stride = (int64_t)g.N * g.O * g.OH * g.OW;
    best.a.part = best.b.part = static_cast<int32_t*>(scratch);
    best.a.part_stride = best.b.part_stride = stride;
    best.a.ksplit = best.b.ksplit = best.ksplit;
    ImgKernel ka = kt == 3 ? (best.wm == 2 ? img_kernel_split<3, 2, 1>(best.ct, best.cc)
                                           : img_kernel_split<3, 1, 1>(best.ct, best.cc))
                           : (best.wm == 2 ? img_kernel_split<1, 2, 1>(best.ct, best.cc)
                                           : img_kernel_split<1, 1, 1>(best.ct, best.cc));
    ImgKernel kb = img_kernel_split<3, 1, 2>(best.ct_b, 32);
    if (best.wm_b != 1) {
      set_error("conv image-tile split-K: epilogue pass must use 32-row tiles");
      *rc = TK_ERR_INVALID_ARG;
      return 1;
    }
    if (set_lds(ka, best.lds, rc) || set_lds(kb, best.lds_b, rc)) return 1;
    hipLaunchKernelGGL(ka, dim3((unsigned)best.a.wgs8), dim3(kGemmThreads), best.lds, s, ga, best.a);
    hipLaunchKernelGGL(kb, dim3((unsigned)best.b.wgs8), dim3(kGemmThreads), best.lds_b, s, ga, best.b);
  } else {
    best.a.ksplit = 1;
    const bool early = kt == 1 && ga.has_add && best.a.early_res && best.ct != 7;
    ImgKernel kern = kt == 3 ? (best.wm == 2 ? img_kernel<3, 2>(best.ct, best.cc) : img_kernel<3, 1>(best.ct, best.cc))
                   : early   ? (best.wm == 2 ? img_kernel_early<2>(best.ct, best.cc) : img_kernel_early<1>(best.ct, best.cc))
                             : (best.wm == 2 ? img_kernel<1, 2>(best.ct, best.cc) : img_kernel<1, 1>(best.ct, best.cc));
    if (set_lds(kern, best.lds, rc)) return 1;
    hipLaunchKernelGGL(kern, dim3((unsigned)best.a.wgs8), dim3(kGemmThreads), best.lds, s, ga, best.a);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string("conv image-tile kernel: launch failed: ") + hipGetErrorString(e));
    *rc = TK_ERR_HIP;
    return 1;
  }
  *rc = TK_OK;
  return 1;
}

}  // namespace tk
