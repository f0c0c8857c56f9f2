// Definitions shared by the MFMA conv-block kernels (tk_gemm.hip: im2col / patch kernels and
// the host dispatch; tk_conv_img.hip: image-tile kernel): kernel arguments, the fused block
// epilogue's per-row constants, device helpers and the host-side conv geometry.
#pragma once

#include <cstdlib>

#include "tk_common.h"

namespace tk {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef uint32_t v4u __attribute__((ext_vector_type(4)));

constexpr int kBK = 64;          // bytes of K per stage
constexpr int kGemmThreads = 256;


struct GemmArgs {
  const int8_t* A;     // [rowsA_pad][lda]
  const int8_t* B;     // plain: [rowsB_pad][ldb]; im2col: shadow [cin_pad/16][N*H*W][16]
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
  int64_t in_pix;                 // N*H*W of the input: pixels per channel group of the shadow
  uint32_t fill;                  // za replicated 4x: out-of-bounds taps (padded channels multiply w = 0)
  int32_t taps;                   // KH*KW
  // output addressing
  int32_t out_nchw;    // 1: C[(p/HW)*M*HW + i*HW + p%HW]; 0: C[i*N + j]
  int32_t ldc;         // row-major pitch (elements) when !out_nchw
  // fused block epilogue (bias_add -> requantize -> clip), see BlockEpi
  int32_t* bias_out;
  uint8_t* rq_out;
  uint8_t* clip_out;
  uint8_t* shadow_out;  // shadow [shadow_cpad/16][N][16] of the last output (conv blocks)
  const int32_t* bias;
  RqParams rq;
  int32_t has_clip, clip_lo, clip_hi, shadow_cpad;
  uint32_t shadow_xor;  // 0x80 when the block output is uint8 (shadow stores int8 = u8 ^ 0x80)
  int32_t ch_is_row;    // channel index = row (conv: Cout) or column (dense: units)
  int32_t vecw;         // epilogue store vector (4 or 1 elements): divides the plane / row length
  // split-K (small grids): kMode 1 writes raw partial tiles for k-steps [z*kper, (z+1)*kper) to ws,
  // kMode 2 sums `splits` of them and runs the epilogue
  int32_t* ws;
  int32_t splits, kper;
  // tile grid: 1-D launch of mtiles * ntiles8 workgroups (ntiles rounded up to 8), see tile_of
  int32_t mtiles, ntiles, ntiles8, xcd_order;
  // residual join (conv blocks): add = RQ(requantize) + RQ(residual) - zp, via 256-entry LUTs
  int32_t has_add, add_zp, add_up_b, add_up_r;
  const uint8_t* add_res;
  uint8_t* add_out;
  RqParams add_pb, add_pr;
  // lean im2col walk (unitap): every 64-byte K stage lies in one tap (cin_pad % 64 == 0, or a
  // 1x1 conv), so the stage's source offset is uniform and each lane only tests its row's
  // tap bitmask (taps <= 64); cgroups = cin_pad / 16
  int32_t unitap, cgroups;
  // p / (OH*OW) and p / OW as (p * magic) >> 40 (0: plain division), exact for p * d < 2^40
  uint64_t mg_hw, mg_ow;
  // fast block epilogue (conv blocks, 4-column vectors, requantize UPWARD): every record
  // byte offset fits 32 bits, so stores go through buffer descriptors; 1 = nontemporal
  // record stores, 2 = plain ones
  int32_t fast_epi;
  uint32_t out_elems;   // N * M: elements of each record
  int32_t nt;           // nontemporal record stores
  // image-aligned N tiles (conv blocks with planes of <= 64 pixels): a tile holds ipt whole
  // images (tcols = ipt * OH*OW of its 128 columns are used), so that for every image the
  // tile's 64 channels x OH*OW pixels are one contiguous NCHW run: see the flat epilogue
  int32_t ipt, tcols;
  int32_t ablate;       // profiling only (TK_ABLATE env): 1 skip shadow, 2 skip stores, 4 skip epilogue,
                       // 32768 flat epilogue without the lean groups, 65536 skip the flat groups,
                       // 131072 flat epilogue without the lean row-crossing groups (hw % 4 != 0),
                       // 8192 residual join without the LUTs, 16384 skip the add record,
                       // (image-tile kernel: 32768 residual words not read from LDS, 65536 residual
                       // words not loaded, 262144 records stored with no epilogue arithmetic),
                       // 8/16/32/64 skip the conv / bias_add / requantize / clip record,
                       // 128/256 skip the A / B LDS-DMA loads, 512 skip the MFMAs, 1024 main-loop
                       // barrier without the lgkmcnt(0) drain, 2048 skip the fragment reads, 4096 skip
                       // the main-loop barrier (timing skeletons only: results are garbage)
};


// Per-row constants of the fused epilogue (one output channel per row for conv
// blocks), staged once per tile in LDS: 32 bytes, read back with two ds_read_b128.
struct EpiRow {
  uint32_t fold;  // K·zA·zB − zB·RA[row]: the whole zero-point correction when zB and RB are uniform/absent
  uint32_t ra, za;
  int32_t bias, m, s, zp, pad;
};


// requantize core of one element (mode is uniform; used where constants vary per element)
__device__ __forceinline__ int32_t rq_core(int32_t t, int mode, int32_t m, int32_t sh) {
  switch (mode) {
    case TK_RQ_IDENTITY: return t;
    case TK_RQ_TENSOR_POW2: return qms_pow2(t, sh);
    case TK_RQ_TENSOR_TONEAREST:
    case TK_RQ_AXIS_TONEAREST: return qms_tonearest(t, m, sh);
    default: return qms_upward(t, m, sh);
  }
}


// 16-byte rows of every byte value: the LDS-DMA source of out-of-bounds im2col taps
// (the input zero point) and of padding rows (0); constant-initialised in device memory.
struct FillRows {
  uint8_t v[256 * 16];
  constexpr FillRows() : v{} {
    for (int i = 0; i < 256 * 16; ++i) v[i] = (uint8_t)(i >> 4);
  }
};
// (static: each translation unit's code object holds its own copy)
static __device__ FillRows tk_fill_rows{};
static __device__ int32_t tk_zero_words[4] = {0, 0, 0, 0};


// Ablation switches of the profiling build (g.ablate, see GemmArgs::ablate); compiled out of
// the product library.  Needs a local `abl` copy of g.ablate (lambdas must not touch g).
#ifdef TK_ABLATION_BUILD
#define TK_ABL(flag) (abl & (flag))
#else
#define TK_ABL(flag) 0
#endif


// Workgroup barrier that only drains this wave's LDS traffic.  __syncthreads() also waits
// vmcnt(0), i.e. for every outstanding global store of the epilogue to complete, which
// serialises the store latency once per barrier; the epilogue's barriers only order LDS.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }


// load through a global-address-space pointer (struct members are generic pointers: flat
// loads would wait on both vmcnt and lgkmcnt)
template <typename T>
__device__ __forceinline__ T ldg(const T* p) {
  return *(const __attribute__((address_space(1))) T*)p;
}


// per-tensor requantize core (no per-channel arrays): the qnn.add operand tables
__device__ __forceinline__ int32_t rq_tensor(int32_t t, const RqParams& p) {
  t = (int32_t)((uint32_t)t - (uint32_t)p.zp_in);
  switch (p.mode) {
    case TK_RQ_TENSOR_POW2: t = qms_pow2(t, p.shift); break;
    case TK_RQ_TENSOR_UPWARD: t = qms_upward(t, p.multiplier, p.shift); break;
    case TK_RQ_TENSOR_TONEAREST: t = qms_tonearest(t, p.multiplier, p.shift); break;
    default: break;
  }
  return (int32_t)((uint32_t)p.zp_out + (uint32_t)t);
}


// ---- fast conv-block epilogue helpers
// buffer descriptor of a record (uniform base and size): stores at offsets >= bytes are
// dropped by the range check, which masks the tile edges without branches
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rec_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, 0x00020000);
}
constexpr int kAuxNT = 2;  // cache policy: nontemporal
constexpr uint32_t kOffDrop = 0x3FFFFFF0u;  // element offset of a masked lane (x4 + 15 stays out of range)

__device__ __forceinline__ uint32_t pack4u(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  // low bytes of a, b, c, d -> one dword (two v_perm_b32 + v_or)
  const uint32_t lo = __builtin_amdgcn_perm(b, a, 0x0c0c0400u);
  const uint32_t hi = __builtin_amdgcn_perm(d, c, 0x04000c0cu);
  return lo | hi;
}

// min(max(x, lo), hi) in one v_med3_i32 (the compiler only forms it for constant bounds); needs
// lo <= hi, which setup_block guarantees for the clip bounds (see there) and the dtype ranges are
__device__ __forceinline__ int32_t clamp_i32(int32_t x, int32_t lo, int32_t hi) {
  int32_t r;
  asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(x), "v"(lo), "v"(hi));
  return r;
}

// counted wait for this wave's global loads (vmcnt immediate): at most n outstanding
__device__ __forceinline__ void wait_vm(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
    case 24: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// the same for any count up to 40 (a count known only at run time: the image-tile kernel's
// DMA instructions per stage, plus its residual words on the plans that issue them early);
// larger counts wait for everything
__device__ __forceinline__ void wait_vm_any(int n) {
  switch (n) {
#define TK_WVM(k) \
  case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    TK_WVM(1) TK_WVM(2) TK_WVM(3) TK_WVM(4) TK_WVM(5) TK_WVM(6) TK_WVM(7) TK_WVM(8) TK_WVM(9) TK_WVM(10)
    TK_WVM(11) TK_WVM(12) TK_WVM(13) TK_WVM(14) TK_WVM(15) TK_WVM(16) TK_WVM(17) TK_WVM(18) TK_WVM(19) TK_WVM(20)
    TK_WVM(21) TK_WVM(22) TK_WVM(23) TK_WVM(24) TK_WVM(25) TK_WVM(26) TK_WVM(27) TK_WVM(28) TK_WVM(29) TK_WVM(30)
    TK_WVM(31) TK_WVM(32) TK_WVM(33) TK_WVM(34) TK_WVM(35) TK_WVM(36) TK_WVM(37) TK_WVM(38) TK_WVM(39) TK_WVM(40)
#undef TK_WVM
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}


__device__ __forceinline__ uint32_t fdiv40(uint32_t x, uint64_t mg) { return (uint32_t)(((uint64_t)x * mg) >> 40); }
// x / d as one v_mul_hi_u32 with m = ceil(2^32 / d) (magic32): exact whenever x * d < 2^32, which
// x, d < 2^16 guarantees (m * d = 2^32 + e, e < d, so the error x * e / (d * 2^32) stays below 1 / d)
__device__ __forceinline__ uint32_t fdiv32(uint32_t x, uint32_t m) { return __umulhi(x, m); }


struct ConvGeom {
  int N, C, H, W, O, KH, KW, OH, OW, cin_pad, k_pad, k_eff, rows_pad;
};


// Block outputs (NULL `b` = plain conv/dense writing only the int32 contraction).
struct BlockIO {
  const tk_tensor* bias;
  tk_tensor* const* outs;  // conv, bias_add, requantize, [clip]
  int n_outs;
  const tk_block_attrs* attrs;
  void* shadow_out;
};


#ifdef TK_ABLATION_BUILD
static const char* tune_env(const char* name) { return getenv(name); }
#else
static const char* tune_env(const char*) { return nullptr; }
#endif


static int env_int(const char* name, int dflt) {
  const char* e = tune_env(name);
  return e ? atoi(e) : dflt;
}

// ---------------------------------------------------------------- image-tile conv blocks
// (tk_conv_img.hip) whole-image tiles with the input patch + halo staged in LDS and the weights
// streamed through one LDS ring shared by the workgroup's waves.
// Bytes of the chunked weight image appended to the packed weight of a KHxKW > 1 conv ([rows]
// [cin_pad / 32][KH*KW][32]; 0 when the layout does not apply).
int64_t conv_img_chunked_bytes(int rows_pad, int cin_pad, int taps);
// Writes that image from the OIHW weight (int8, or uint8 stored xor 0x80).
int conv_img_pack(const tk_tensor* weight, int8_t* dst, int rows_pad, int cin_pad, hipStream_t s);
// tk_block_attrs.algo values (tk_conv2d_block_algos): 0 the library's choice, 1 im2col tiles
// (gemm_i8_kernel), 2 image tiles with the planner's plan, 3 / 4 persistent im2col tiles with
// cross-tile prefetch and a 2- / 3-slot ring (conv_pf_kernel), 16 + i image-tile plan i.
// 5: the small-batch dense tile kernel (tk_dense.hip) for dense blocks run as 1x1 conv blocks.
constexpr int kAlgoIm2col = 1, kAlgoImg = 2, kAlgoPf2 = 3, kAlgoPf3 = 4, kAlgoDense = 5, kAlgoImg0 = 16;
// Runs the conv block on the image-tile kernel when its plan applies (returns 1 and sets *rc;
// algo 0: the cheapest plan by the planner's estimate), else returns 0 (im2col path).
// `chunked`: the chunked weight image (NULL for 1x1 convs, whose packed weight has that layout).
int conv_img_try(const ConvGeom& g, const tk_conv2d_attrs* a, const GemmArgs& ga, const int8_t* chunked, void* scratch,
                 int algo, hipStream_t s, int* rc);
// scratch a 3x3 block's split-K image-tile plans need (their partial records), 0 if none apply
int64_t conv_img_split_scratch_bytes(const ConvGeom& g);
// The image-tile plans as algo values (16 + i), cheapest estimate first; returns how many exist.
int conv_img_algos(const ConvGeom& g, const tk_conv2d_attrs* a, const GemmArgs& ga, bool have_chunked,
                   int32_t* algos, int max_algos);

// ---------------------------------------------------------------- persistent im2col conv blocks
// (tk_conv_pf.hip) whether the launch arguments (conv2d_run's, before the tile grid) suit the
// persistent kernel, and its launch (ring: 2 or 3 slots).
bool conv_pf_applies(const ConvGeom& g, const GemmArgs& ga);
int conv_pf_run(const ConvGeom& g, GemmArgs ga, int ring, hipStream_t s);

// ---------------------------------------------------------------- small-batch dense blocks
// (tk_dense.hip) [B, K] x [U, K]^T on 32 x 32 tiles with K split over the four waves, one launch.
bool conv_dense_applies(const ConvGeom& g, const GemmArgs& ga);
// scratch: conv_dense_scratch_bytes(g) bytes for a K-sliced run (NULL: one launch, no slices)
int conv_dense_run(const ConvGeom& g, const GemmArgs& ga, void* scratch, hipStream_t s);
int64_t conv_dense_scratch_bytes(const ConvGeom& g);

}  // namespace tk
