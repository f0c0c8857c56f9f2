/*
 * tachikoma.h — C ABI of the MI355X (gfx950) integer inference-and-trace engine.
 *
 * Drop-in boundary for the reference's per-op CPU execution path
 * (CortexFoundation/tachikoma, a TVM 0.11.dev0 fork).  Every entry point is
 * plain C: raw pointers, sizes and POD structs, no C++ or torch types.
 *
 * Conventions (mirroring the reference's packed-function convention,
 * include/tvm/runtime/c_backend_api.h:49-51 and graph_executor.cc:486-493):
 *   - tensors are passed as `const tk_tensor*` (layout-identical to DLPack's
 *     DLTensor, include/tvm/runtime/c_runtime_api.h:174-208); inputs first,
 *     outputs after;
 *   - tensors are BORROWED: the caller owns device memory, nothing is retained
 *     past the call;
 *   - kernels are enqueued asynchronously on the given stream (`void*` =
 *     hipStream_t) and never synchronise; one stream per host thread makes
 *     concurrent calls safe;
 *   - return 0 on success or a negative tk_status; `tk_last_error()` returns a
 *     thread-local message (the analogue of TVMAPISetLastError).
 *
 * Integer semantics are the reference's pinned CPU semantics (target llvm, no
 * -mcpu): qnn conv/dense = Σ(a−zp_a)(w−zp_w) in int32,
 * requantize = RequantizeLowerInt + q_multiply_shift (UPWARD default).
 */
#ifndef TACHIKOMA_H_
#define TACHIKOMA_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* every declaration below is part of the exported ABI (the library builds with
 * -fvisibility=hidden) */
#pragma GCC visibility push(default)

#define TK_ABI_VERSION 1

/* ---------------------------------------------------------------- status */
typedef enum {
  TK_OK = 0,
  TK_ERR_INVALID_ARG = -1,
  TK_ERR_UNSUPPORTED = -2,
  TK_ERR_SHAPE = -3,
  TK_ERR_DTYPE = -4,
  TK_ERR_HIP = -5,
  TK_ERR_IO = -6,
  TK_ERR_FORMAT = -7,
} tk_status;

/* Thread-local message for the last failing call on this thread. */
const char* tk_last_error(void);
/* Library/ABI version (TK_ABI_VERSION) and the offload arch it was built for. */
int tk_abi_version(void);
const char* tk_build_arch(void);
/* Hex digest of the sources the library was compiled from (tachikoma_amd/build.py hashes
 * csrc/ and include/ and passes it as -DTK_SOURCE_HASH); the Python loader refuses a
 * library whose digest differs from the tree it is imported from. */
const char* tk_build_info(void);

/* ---------------------------------------------------------------- tensors */
/* Layout-identical to DLPack DLDevice / DLDataType / DLTensor. */
typedef struct { int32_t device_type; int32_t device_id; } tk_device;
typedef struct { uint8_t code; uint8_t bits; uint16_t lanes; } tk_dtype;
typedef struct {
  void* data;
  tk_device device;
  int32_t ndim;
  tk_dtype dtype;
  int64_t* shape;
  int64_t* strides; /* must be NULL (compact row-major) */
  uint64_t byte_offset;
} tk_tensor;

enum { TK_DL_INT = 0, TK_DL_UINT = 1, TK_DL_FLOAT = 2 };
enum { TK_DEV_CPU = 1, TK_DEV_ROCM = 10 };

/* ---------------------------------------------------------------- fixed point
 * Host ports of the reference's compile-time constant folding.            */

/* GetFixedPointMultiplierShift (src/relay/qnn/utils.cc:33-57). */
int tk_fixed_point_multiplier_shift(double multiplier, int32_t* significand, int32_t* shift);

enum { TK_ROUND_UPWARD = 0, TK_ROUND_TONEAREST = 1 };

/* Requantize modes chosen by tk_requantize_prepare
 * (RequantizeLowerInt, src/relay/qnn/op/requantize.cc:195-273). */
enum {
  TK_RQ_IDENTITY = 0,           /* per-tensor, input_scale == output_scale: FPM skipped (:226) */
  TK_RQ_TENSOR_POW2 = 1,        /* per-tensor UPWARD, m == 1<<30: int32 shift path (intrin_rule.cc:223-237) */
  TK_RQ_TENSOR_UPWARD = 2,      /* per-tensor UPWARD general (intrin_rule.cc:166-195) */
  TK_RQ_TENSOR_TONEAREST = 3,   /* FixedPointMultiplyToNearest (utils.cc:59-109) */
  TK_RQ_AXIS_UPWARD = 4,        /* q_multiply_shift_per_axis (intrin_rule.cc:252-267) */
  TK_RQ_AXIS_TONEAREST = 5,     /* FixedPointMultiplyPerChannel TONEAREST (utils.cc:137-216) */
};

/* Fold float32 scales into fixed-point constants exactly as the reference's
 * canonicalisation does.  `input_scales` has n_scales entries; n_scales == 0
 * means a rank-0 (per-tensor) scale held in input_scales[0].  On return
 * multipliers[i]/shifts[i] (capacity max(1, n_scales)) and *mode are set. */
int tk_requantize_prepare(const float* input_scales, int n_scales, float output_scale, int rounding,
                          int32_t* multipliers, int32_t* shifts, int* mode);

/* ---------------------------------------------------------------- op attrs */

/* qnn.requantize (src/relay/qnn/op/requantize.cc:195-273). */
typedef struct {
  int32_t mode;                 /* TK_RQ_* from tk_requantize_prepare */
  int32_t axis;                 /* channel axis for per-axis constants / zero points */
  int32_t multiplier;           /* per-tensor modes */
  int32_t shift;
  const int32_t* multipliers;   /* device, per-axis modes (len = shape[axis]) */
  const int32_t* shifts;        /* device, per-axis modes */
  int32_t input_zero_point;     /* used when input_zero_points == NULL */
  const int32_t* input_zero_points; /* device, optional per-axis */
  int32_t output_zero_point;
} tk_requantize_attrs;

/* qnn.conv2d, NCHW data / OIHW weight → int32 NCHW. */
typedef struct {
  int32_t strides[2];
  int32_t padding[4];           /* top, left, bottom, right */
  int32_t dilation[2];
  int32_t groups;
  int32_t input_zero_point;
  int32_t kernel_zero_point;    /* used when kernel_zero_points == NULL */
  const int32_t* kernel_zero_points; /* device, optional per-output-channel */
} tk_conv2d_attrs;

/* qnn.dense [M,K] x [N,K]^T → int32 [M,N]. */
typedef struct {
  int32_t input_zero_point;
  int32_t kernel_zero_point;
  const int32_t* kernel_zero_points; /* device, optional per-unit */
} tk_dense_attrs;

/* qnn.add with per-tensor parameters (src/relay/qnn/op/add.cc:40-96). The two
 * requantize-to-int32 plans come from tk_requantize_prepare (mode IDENTITY
 * with equal zero points = plain upcast, op_common.h:186-200). */
typedef struct {
  tk_requantize_attrs lhs;      /* lhs → output params, int32 result */
  tk_requantize_attrs rhs;
  int32_t output_zero_point;
  int32_t lhs_upcast;           /* 1: RequantizeOrUpcast took the Cast branch */
  int32_t rhs_upcast;
} tk_qnn_add_attrs;

/* A fused layer "block": qnn.conv2d|qnn.dense → nn.bias_add → qnn.requantize
 * [→ qnn.add(·, residual)] [→ clip].  One kernel computes the contraction and writes EVERY
 * op output of the chain from registers (each stays a separate trace record), so the int32
 * intermediates are never re-read from HBM.  Requantize/bias must run along the channel
 * axis (NCHW axis 1 / dense units).
 * outs = {conv int32, bias_add int32, requantize 8-bit, [add 8-bit], [clip 8-bit]}: with
 * has_add the clip (if any) applies to the add (the ResNet bottleneck tail). */
typedef struct {
  tk_conv2d_attrs conv;         /* conv blocks */
  tk_dense_attrs dense;         /* dense blocks */
  tk_requantize_attrs requantize;
  int32_t has_clip;
  int64_t clip_min, clip_max;
  int32_t has_add;              /* MFMA conv blocks only */
  int32_t block_is_rhs;         /* 1: the requantize output is qnn.add's rhs operand */
  const tk_tensor* residual;    /* the other qnn.add operand (same shape and dtype, NCHW) */
  tk_qnn_add_attrs add;
  int32_t algo;                 /* MFMA conv blocks: the kernel (tk_conv2d_block_algos): 0 = the
                                   library's choice, 1 = im2col tiles, 3 / 4 = persistent im2col
                                   tiles with cross-tile prefetch (2- / 3-slot ring), 16 + i =
                                   image-tile plan i.
                                   Every algo gives bit-identical records; only time differs. */
} tk_block_attrs;

/* The kernels an MFMA conv block can run on, as tk_block_attrs.algo values: 5 (dense tiles, for
 * [B, K] x [U, K]^T heads with a zero weight zero point), 1 (im2col tiles, always), then 16 + i for
 * each image-tile plan that applies (plain plans, then split-K plans), in the planner's
 * estimated-time order, then 3 and 4 where the persistent im2col kernel applies (planes of more
 * than 64 pixels, pixel count a multiple of 4, UPWARD requantize, no kernel zero point).  Writes at
 * most max_algos entries; returns how many exist (0: not an MFMA conv, the block has a single
 * kernel) or a negative tk_status.  The reference has one CPU kernel per op (its TOPI schedules are
 * chosen at compile time); this is the MI355X find step's search space. */
int tk_conv2d_block_algos(const tk_tensor* data, const tk_tensor* weight, const tk_block_attrs* attrs,
                          int32_t* algos, int max_algos);
/* A one-line description of one of those kernels (tile shape, stage width, ring, split) into buf
 * (NUL-terminated, truncated to len): for reports of what the find step picked.  TK_ERR_INVALID_ARG
 * for an algo the block does not list. */
int tk_conv2d_block_algo_info(const tk_tensor* data, const tk_tensor* weight, const tk_block_attrs* attrs, int algo,
                              char* buf, int len);

/* A fused residual join: qnn.add [→ clip].  One kernel writes both records and,
 * optionally, the int8 shadow (tk_conv2d_make_shadow layout) of the last output for the next MFMA conv. */
typedef struct {
  tk_qnn_add_attrs add;
  int32_t has_clip;
  int64_t clip_min, clip_max;
} tk_add_block_attrs;

typedef struct {
  int32_t pool_size[2];
  int32_t strides[2];
  int32_t padding[4];
  int32_t dilation[2];
  int32_t count_include_pad;
} tk_pool2d_attrs;

/* ---------------------------------------------------------------- per-op entry points
 * Each replaces one canonicalised reference op on the CPU graph executor
 * (graph_executor.cc:524-572 → LLVM TOPI kernel).                          */

/* Packed-weight workspace for the MFMA implicit-GEMM conv: [Cout][KH][KW][Cin_pad]
 * int8 (uint8 weights are stored xor 0x80) plus int32 per-channel sums. */
int64_t tk_conv2d_packed_weight_bytes(const tk_tensor* weight, int groups);
int tk_conv2d_pack_weight(const tk_tensor* weight, int groups, void* packed, int32_t* weight_sums,
                          void* stream);
/* The int8 "shadow" an MFMA conv reads its activations from: channel-blocked
 * [ceil(C/16)][N·H·W][16] (16 channels of one pixel per 16-byte chunk; a channel group's
 * pixels are contiguous), padded channels 0, uint8 data stored xor 0x80. */
int64_t tk_conv2d_shadow_bytes(const tk_tensor* data);
int tk_conv2d_make_shadow(const tk_tensor* data, void* shadow, void* stream);
/* Device scratch of a prepared conv (tk_qnn_conv2d_prepared: block = 0; tk_qnn_conv2d_block:
 * block = 1): per-pixel patch sums when the kernel zero point is non-zero, plus split-K
 * partial tiles for layers whose tile grid cannot fill the GPU, or (3x3 blocks) up to four
 * partial records of a split-K image-tile plan (tk_conv2d_block_algos).  0 = no scratch needed. */
int64_t tk_conv2d_scratch_bytes(const tk_tensor* data, const tk_tensor* weight, const tk_conv2d_attrs* attrs,
                                int block);
/* qnn.conv2d on a prepared shadow + packed weight (what the executor runs).
 * `scratch`: tk_conv2d_scratch_bytes(..., 0) bytes (may be NULL when that is 0). */
int tk_qnn_conv2d_prepared(const tk_tensor* data, const void* shadow, const tk_tensor* weight,
                           const void* packed, const int32_t* weight_sums, tk_tensor* out,
                           const tk_conv2d_attrs* attrs, void* scratch, void* stream);
/* One-shot qnn.conv2d (src/relay/qnn/op/convolution.cc:708-811; x86 legalization
 * python/tvm/relay/qnn/op/legalizations.py:177-232): prepares into `workspace`
 * (tk_qnn_conv2d_workspace_bytes) then runs. */
int64_t tk_qnn_conv2d_workspace_bytes(const tk_tensor* data, const tk_tensor* weight,
                                      const tk_conv2d_attrs* attrs);
int tk_qnn_conv2d(const tk_tensor* data, const tk_tensor* weight, tk_tensor* out,
                  const tk_conv2d_attrs* attrs, void* workspace, void* stream);

/* Fused conv block: outs = {conv int32, bias_add int32, requantize int8/uint8, clip (if has_clip)}.
 * `scratch`: tk_conv2d_scratch_bytes(..., 1) bytes.  `shadow_out` (optional): the int8 shadow
 * (tk_conv2d_make_shadow layout) of the block's last output, for a following MFMA conv. */
int tk_qnn_conv2d_block(const tk_tensor* data, const void* shadow, const tk_tensor* weight, const void* packed,
                        const int32_t* weight_sums, const tk_tensor* bias, tk_tensor* const* outs, int n_outs,
                        const tk_block_attrs* attrs, void* scratch, void* shadow_out, void* stream);

/* qnn.dense (src/relay/qnn/op/dense.cc:87-206). */
int64_t tk_qnn_dense_workspace_bytes(const tk_tensor* data, const tk_tensor* weight);
int tk_qnn_dense(const tk_tensor* data, const tk_tensor* weight, tk_tensor* out,
                 const tk_dense_attrs* attrs, void* workspace, void* stream);
/* Fused dense block (outs as for tk_qnn_conv2d_block). */
int tk_qnn_dense_block(const tk_tensor* data, const tk_tensor* weight, const tk_tensor* bias, tk_tensor* const* outs,
                       int n_outs, const tk_block_attrs* attrs, void* workspace, void* stream);

int tk_requantize(const tk_tensor* data, tk_tensor* out, const tk_requantize_attrs* attrs, void* stream);
int tk_qnn_add(const tk_tensor* lhs, const tk_tensor* rhs, tk_tensor* out, const tk_qnn_add_attrs* attrs,
               void* stream);
/* nn.bias_add / add with a broadcast vector along `axis` (int32 wraps). */
/* Fused qnn.add [→ clip] on 8-bit tensors (add.cc:40-96 + clip, python/tvm/topi/math.py:615-640).
 * outs = {add, [clip]}.  shadow_out (optional): int8 shadow (tk_conv2d_make_shadow layout) of the
 * last output (uint8 stored xor 0x80, padded channels written as 0); needs 4-D NCHW operands. */
int tk_qnn_add_block(const tk_tensor* lhs, const tk_tensor* rhs, tk_tensor* const* outs, int n_outs,
                     const tk_add_block_attrs* attrs, void* shadow_out, void* stream);

int tk_bias_add(const tk_tensor* data, const tk_tensor* bias, tk_tensor* out, int axis, void* stream);
/* clip: max(min(x, a_max), a_min) with bounds already cast to the dtype. */
int tk_clip(const tk_tensor* data, tk_tensor* out, int64_t a_min, int64_t a_max, void* stream);
/* integer cast (truncating narrow / sign- or zero-extending widen). */
int tk_cast(const tk_tensor* data, tk_tensor* out, void* stream);
int tk_max_pool2d(const tk_tensor* data, tk_tensor* out, const tk_pool2d_attrs* attrs, void* stream);
/* nn.max_pool2d of an 8-bit NCHW tensor read from its conv shadow (tk_conv2d_make_shadow
 * layout): writes the NCHW record and, when `out_shadow` is not NULL, the output's shadow. */
int tk_max_pool2d_shadow(const tk_tensor* data, const void* data_shadow, tk_tensor* out,
                         const tk_pool2d_attrs* attrs, void* out_shadow, void* stream);
int tk_avg_pool2d(const tk_tensor* data, tk_tensor* out, const tk_pool2d_attrs* attrs, void* stream);
int tk_global_avg_pool2d(const tk_tensor* data, tk_tensor* out, void* stream);
/* batch_flatten / reshape: byte copy (kept as a node so it is traced). */
int tk_copy(const tk_tensor* data, tk_tensor* out, void* stream);
/* nn.pad, constant mode (src/relay/op/nn/pad.cc, python/tvm/topi/nn/pad.py:24-82): up to 6-D, any
 * 1/2/4/8-byte dtype; out[i] = data[i - before] inside the data's range, else the pad value
 * (already cast to the dtype: value_i for integer tensors, value_f for float32). */
typedef struct {
  int64_t before[6], after[6];
  int64_t value_i;
  double value_f;
} tk_pad_attrs;
int tk_pad(const tk_tensor* data, tk_tensor* out, const tk_pad_attrs* attrs, void* stream);

/* tachikoma BYOC composite post-ops: the float32 tail of a tachikoma.qnn.conv2d /
 * tachikoma.qnn.dense composite after LegalizeQnnOpForTachikoma
 * (python/tvm/relay/op/contrib/tachikoma.py:1122-1306), executed by the reference's JSON
 * runtime as oneDNN post-ops (src/runtime/contrib/tachikoma/tachikoma_json_runtime.cc:142-185).
 * On the int32 contraction `acc` (zero zero points), per element of channel c along `axis`,
 * in float32, each operation rounded separately and in this order:
 *   t = (float(acc) + bias[c]) * o_scl[n_scales == 1 ? 0 : c]      output scales
 *   t = min(max(t, clip_lo), clip_hi) * act_scl                       eltwise clip, scaled
 *   t = sum_scl * float(sum_src) + t          (only when sum_src)     sum post-op
 *   t = t + dst_zp                                                    linear eltwise
 *   out = saturate(round_half_even(t))                                8-bit destination
 * bias and o_scl are float32 device arrays.  Replaces the composite's Run
 * (tachikoma_json_runtime.cc:93-106) for the post-op part; the contraction is tk_qnn_conv2d /
 * tk_qnn_dense with zero zero points. */
typedef struct {
  int32_t axis;
  int32_t n_scales;             /* 1: per-tensor output scale, else one per channel */
  float clip_lo, clip_hi, act_scl, sum_scl, dst_zp;
  const float* bias;            /* [channels] */
  const float* o_scl;           /* [n_scales] */
} tk_postops_attrs;
int tk_tachikoma_postops(const tk_tensor* acc, const tk_tensor* sum_src, tk_tensor* out,
                         const tk_postops_attrs* attrs, void* stream);

/* ---------------------------------------------------------------- relay.quantize-realized graphs
 * The ops `relay.quantize.quantize` leaves beside the int8 contractions (SURVEY.md §8(f) row 4;
 * src/relay/quantize/realize.cc:66-160 MulAndDiv / QuantizeRealize, realize.cc:300-345
 * UnifyDTypeScale): the int32 add / left_shift / right_shift / fixed_point_multiply chain that
 * moves activations between scales, the float32 input quantize (multiply, round, clip) and
 * the float32 layers left unquantized.  Realized int8 nn.conv2d / nn.dense run through
 * tk_qnn_conv2d / tk_qnn_dense with zero zero points; float casts go through tk_cast, float
 * per-channel adds through tk_bias_add, float pools through tk_max_pool2d /
 * tk_global_avg_pool2d.  Float contractions accumulate in a fixed order (conv: c, r, s;
 * dense: k; pool: row-major), one rounding per multiply and add. */
enum {
  TK_EW_ADD = 0,                  /* x + rhs (int: wraps) */
  TK_EW_MULTIPLY = 1,             /* x * rhs (int: wraps) */
  TK_EW_LEFT_SHIFT = 2,           /* int: x << rhs */
  TK_EW_RIGHT_SHIFT = 3,          /* int: x >> rhs (arithmetic) */
  TK_EW_ROUND = 4,                /* float: llvm.round (halves away from zero) */
  TK_EW_CLIP = 5,                 /* float: min(max(x, lo), hi) */
  TK_EW_RELU = 6,                 /* max(x, 0) */
  TK_EW_FIXED_POINT_MULTIPLY = 7, /* int: q_multiply_shift(x, multiplier, 31, shift), int32 result */
};
typedef struct {
  int32_t op;                   /* TK_EW_* */
  int32_t rhs_kind;             /* 0: unary, 1: scalar (scalar_f / scalar_i), 2: tensor of x's shape,
                                   3: one value per channel (axis 1) of x, add / multiply; for an int32
                                   fixed_point_multiply: int32[2C], the multipliers then the shifts
                                   (fixed_point_multiply_per_axis, no power-of-two special case) */
  double scalar_f;              /* float32 tensors */
  int64_t scalar_i;             /* integer tensors */
  double lo, hi;                /* TK_EW_CLIP */
  int32_t multiplier, shift;    /* TK_EW_FIXED_POINT_MULTIPLY */
} tk_ewise_attrs;
/* Elementwise op of a float32 / int8 / int16 / int32 / int64 tensor (topi broadcast ops with a scalar or
 * same-shape rhs; relay.round; relay.fixed_point_multiply, topi/math.py:644-673). */
int tk_ewise(const tk_tensor* x, const tk_tensor* rhs, tk_tensor* out, const tk_ewise_attrs* attrs, void* stream);
/* float32 nn.conv2d NCHW/OIHW (the conv the quantizer skips, skip_conv_layers) and nn.dense. */
int tk_conv2d_f32(const tk_tensor* data, const tk_tensor* weight, tk_tensor* out, const tk_conv2d_attrs* attrs,
                  void* stream);
int tk_dense_f32(const tk_tensor* data, const tk_tensor* weight, tk_tensor* out, void* stream);
/* relay.quantize kl_divergence calibration, host only (src/relay/quantize/calibrate.cc:35-146
 * MinimizeKL, called by kl_divergence.py:_find_scale_by_kl): hist = num_bins int32 counts over
 * float32 edges[num_bins + 1] symmetric about 0; writes the threshold whose 8-bit quantisation
 * (num_quantized_bins buckets) minimises the KL divergence. */
int tk_find_scale_by_kl(const int32_t* hist, const float* edges, int num_bins, int num_quantized_bins,
                        float* threshold);

/* ---------------------------------------------------------------- pre-quantized QNN graphs
 * The QNN ops a frontend-produced quantized graph carries besides conv / dense / requantize /
 * add: the float32 input quantize, the float32 head dequantize, and the
 * quantized concatenate / mul / subtract.  Each follows its reference canonicalization exactly;
 * float32 steps are single IEEE operations in the reference's order (no contraction, correctly
 * rounded division). */

/* Scale / zero point of qnn.quantize (output params) and qnn.dequantize (input params):
 * per-tensor (`scales` / `zero_points` NULL) or one float32 scale / int32 zero point per index
 * of `axis` (device arrays; ExpandBiasToMatchAxis). */
typedef struct {
  int32_t axis;
  float scale;
  const float* scales;
  int32_t zero_point;
  const int32_t* zero_points;
} tk_qparams_attrs;
/* qnn.quantize (src/relay/qnn/op/quantize.cc:113-149, QuantizeLower): float32 data →
 * int8 / uint8 / int16 / int32: out = cast(clip(round(x / scale) + float(zp), qmin, qmax)),
 * round = llvm.round (halves away from zero), every step float32. */
int tk_qnn_quantize(const tk_tensor* data, tk_tensor* out, const tk_qparams_attrs* attrs, void* stream);
/* qnn.dequantize (src/relay/qnn/op/dequantize.cc:96-129, DequantizeLower): int8 / uint8 / int16 /
 * int32 data → float32: out = float(int32(x) - zp) * scale (int32 subtract wraps). */
int tk_qnn_dequantize(const tk_tensor* data, tk_tensor* out, const tk_qparams_attrs* attrs, void* stream);

/* qnn.add / qnn.subtract / qnn.mul with numpy broadcasting (up to 6-D, BroadcastRel) and per-tensor
 * or per-axis parameters (QnnBroadcastRel, src/relay/qnn/op/op_common.h:231-320):
 *   add       (add.cc:40-96):       o = RQ(a) + RQ(b) - zp_c
 *   subtract  (subtract.cc:40-94):  o = RQ(a) - RQ(b) + zp_c
 *     RQ = RequantizeOrUpcast (op_common.h:193-207): requantize to int32 at the output params, or
 *     a plain upcast when scale and zero point equal the output's (`*_upcast`); `lhs.axis` /
 *     `rhs.axis` index the operand's own dimensions for per-axis plans;
 *   mul       (mul.cc:43-159):      o = RQ_out((int32(a) - zp_a) * (int32(b) - zp_b)) where the
 *     zero points are lhs.input_zero_point(s) / rhs.input_zero_point(s) (per lhs.axis / rhs.axis)
 *     and RQ_out (`out`) requantizes the int32 product from scale s_a*s_b, zero point 0 (per-axis
 *     along out.axis, an axis of lhs) — every int32 step wraps;
 * then clip to the output dtype (the input dtype) and cast. */
enum { TK_QB_ADD = 0, TK_QB_SUBTRACT = 1, TK_QB_MUL = 2 };
typedef struct {
  int32_t op;                   /* TK_QB_* */
  tk_requantize_attrs lhs, rhs;
  int32_t lhs_upcast, rhs_upcast;
  tk_requantize_attrs out;      /* TK_QB_MUL only */
  int32_t output_zero_point;    /* add / subtract */
} tk_qnn_binary_attrs;
int tk_qnn_binary(const tk_tensor* lhs, const tk_tensor* rhs, tk_tensor* out, const tk_qnn_binary_attrs* attrs,
                  void* stream);

/* qnn.concatenate (src/relay/qnn/op/concatenate.cc:153-221): input i is requantized to the output
 * params with out dtype = its own dtype (per-tensor, `requant[i]`) unless its scale and zero point
 * equal the output's, then all are concatenated along `axis`. */
#define TK_CONCAT_MAX 8
typedef struct {
  int32_t axis;
  int32_t n;
  int32_t requant[TK_CONCAT_MAX];
  tk_requantize_attrs rq[TK_CONCAT_MAX];
} tk_concat_attrs;
int tk_qnn_concatenate(const tk_tensor* const* inputs, int n, tk_tensor* out, const tk_concat_attrs* attrs,
                       void* stream);

/* transpose / layout_transform of a compact tensor (up to 6-D, 1/2/4/8-byte elements):
 * out.shape[k] = data.shape[perm[k]].  The NHWC / HWIO / OHWI / HWOI qnn.conv2d layouts run the
 * NCHW / OIHW kernels between two of these (convolution.cc:718-722 accepts them). */
typedef struct {
  int32_t ndim;
  int32_t perm[6];
} tk_transpose_attrs;
int tk_transpose(const tk_tensor* data, tk_tensor* out, const tk_transpose_attrs* attrs, void* stream);

/* qnn.leaky_relu (src/relay/qnn/op/leaky_relu.cc:85-140, QnnLeakyReluCanonicalize), int8 / uint8:
 *   q   = RequantizeOrUpcast(int32(x)) to the output params (`rq`, per-tensor; `upcast` = plain cast)
 *   out = int32(x) < input_zero_point ? FPM(q, alpha) + FPM(output_zero_point, 1 - alpha) : q
 * clipped and cast to the input dtype (ConvertDtype).  FPM = fixed_point_multiply =
 * tir.q_multiply_shift (intrin_rule.cc:197-250, the power-of-two branch included) with
 * GetFixedPointMultiplierShift(alpha) / (1 - alpha) from tk_fixed_point_multiplier_shift. */
typedef struct {
  tk_requantize_attrs rq;
  int32_t upcast;
  int32_t input_zero_point;
  int32_t output_zero_point;
  int32_t alpha_multiplier, alpha_shift;
  int32_t zp_multiplier, zp_shift;
} tk_leaky_relu_attrs;
int tk_qnn_leaky_relu(const tk_tensor* data, tk_tensor* out, const tk_leaky_relu_attrs* attrs, void* stream);

/* The qnn unary ops (qnn.sqrt / rsqrt / exp / erf / sigmoid / hardswish / tanh / log / abs,
 * src/relay/qnn/op/unary_elementwise_op.cc:31-56) legalize to a table lookup
 * (python/tvm/relay/qnn/op/legalizations.py:54-86, canonicalizations.py:32-160):
 * out = table[reinterpret<uint8>(x)], the 256-entry table built when the graph is built.
 * int8 / uint8 data, same-dtype output; `table` is a device array of 256 bytes. */
int tk_qnn_lookup(const tk_tensor* data, tk_tensor* out, const void* table, void* stream);

/* qnn.batch_matmul (src/relay/qnn/op/batch_matmul.cc:162-228): x [B, M, K] int8/uint8, y [B', N, K]
 * (transpose_b; B == B' or one of them 1) -> int32 [max(B, B'), M, N] = sum_k (x - zx)(y - zy)
 * modulo 2^32 (the four-term canonical form).  Runs the qnn.dense kernel per batch entry with
 * the zero points of `attrs` (input = x, kernel = y); workspace from
 * tk_qnn_batch_matmul_workspace_bytes. */
int64_t tk_qnn_batch_matmul_workspace_bytes(const tk_tensor* x, const tk_tensor* y);
int tk_qnn_batch_matmul(const tk_tensor* x, const tk_tensor* y, tk_tensor* out, const tk_dense_attrs* attrs,
                        void* workspace, void* stream);

/* qnn.conv2d_transpose (legalizations.py:97-130: int16 operand shifts, then nn.conv2d_transpose,
 * python/tvm/topi/nn/conv2d_transpose.py:79-140): NCHW int8/uint8 data, IOHW weight
 * (C, O / groups, KH, KW) -> int32 NCHW (N, O, (H-1)*sh + KH - pt - pb + oph, ...):
 *   out[n, o, y, x] = sum over c of o's group, r, s with y + pt - r = sh * iy, x + pl - s = sw * ix
 *                     of int16(d - zd) * int16(w[c, o % (O/groups), r, s] - zw)      (int32, wraps)
 * kernel_zero_points: optional device array of O/groups entries (bias_add on the weight's axis 1). */
typedef struct {
  int32_t strides[2];
  int32_t padding[4];           /* top, left, bottom, right */
  int32_t output_padding[2];
  int32_t groups;
  int32_t input_zero_point;
  int32_t kernel_zero_point;
  const int32_t* kernel_zero_points;
} tk_conv2d_transpose_attrs;
int tk_qnn_conv2d_transpose(const tk_tensor* data, const tk_tensor* weight, tk_tensor* out,
                            const tk_conv2d_transpose_attrs* attrs, void* stream);

/* qnn.simulated_quantize / qnn.simulated_dequantize (src/relay/qnn/op/simulated_quantize.cc:36-78,
 * simulated_dequantize.cc:36-76; compute python/tvm/topi/nn/qnn.py:40-190): float32 -> float32 of
 * the same shape.  The dtype arrives as an int32 device scalar (SQNN codes: 1 int8, 2 uint8,
 * 3 int32; any other value -- 0 "disable" -- passes the data through), so a graph may pick it at
 * run time.  Element index i along `axis` uses scales[i % n_scales] and zero_points[i % n_zero_points]
 * (tir.indexmod).  Per element, in float32 (the int32 zero point and integer bounds cast to float32):
 *   quantize:   max(min(round(x / scale) + zp, qmax), qmin)     round = llvm.round (half away)
 *   dequantize: (x - zp) * scale */
typedef struct {
  int32_t axis;                 /* -1 = last */
  int32_t n_scales, n_zero_points;
  const int32_t* dtype_code;    /* device, one int32 */
  const float* scales;          /* device, n_scales */
  const int32_t* zero_points;   /* device, n_zero_points */
} tk_simq_attrs;
int tk_qnn_simulated_quantize(const tk_tensor* data, tk_tensor* out, const tk_simq_attrs* attrs, void* stream);
int tk_qnn_simulated_dequantize(const tk_tensor* data, tk_tensor* out, const tk_simq_attrs* attrs, void* stream);

/* qnn.requantize with compute_dtype "float32" / "float64": RequantizeLowerFP<Bits>
 * (src/relay/qnn/op/requantize.cc:293-373, dispatch :392-403), chosen by
 * requantize_config(compute_dtype=...) or the op's own attribute (requantize_config.h:53-72).  As
 * the MRT llvm target without -mcpu runs it (no SSE4.1: the Upward / Tonearest forms of :127-173),
 * per element, every step one IEEE operation in the compute type, no contraction:
 *   t = F(x) - F(zp_in);  t = M * t (per-tensor, skipped when `scaled` == 0, i.e. the scales are
 *   structurally equal, :313-318) or t * M[c] (per-axis, always);  t = t + F(zp_out);
 *   UPWARD:    b = t + 0.5; f = F(I(b)); t = (b == f || b >= 0) ? f : f - 1
 *   TONEAREST: s = t < 0 ? -1 : 1; b = (t + 0.5 * s) * s; t = F(I(b)) * s     (t kept if not finite)
 *   q = int32(t), clipped to the output dtype unless it is int32.
 * F = float / double, I = int32 / int64 (Cast(.., Int(Bits))), M = the double multiplier
 * double(s_in) / double(s_out) converted to F.  Float -> int casts follow x86-64's cvtt* (what the
 * reference's LLVM code runs): truncation, and INT_MIN of the target width for NaN or out-of-range
 * values. */
typedef struct {
  int32_t bits;                 /* 32 (float32) or 64 (float64) */
  int32_t rounding;             /* TK_ROUND_* */
  int32_t axis;                 /* channel axis of per-axis multipliers / zero points */
  int32_t scaled;               /* per-tensor: 1 = multiply by `multiplier`, 0 = equal scales */
  double multiplier;            /* per-tensor double(s_in) / double(s_out) */
  const double* multipliers;    /* device, per-axis (len = shape[axis]); NULL = per-tensor */
  int32_t input_zero_point;     /* used when input_zero_points == NULL */
  const int32_t* input_zero_points; /* device, optional per-axis */
  int32_t output_zero_point;
} tk_requantize_fp_attrs;
int tk_requantize_fp(const tk_tensor* data, tk_tensor* out, const tk_requantize_fp_attrs* attrs, void* stream);

/* qnn.add / qnn.subtract / qnn.mul built under a float compute_dtype: tk_qnn_binary with every
 * inner Requantize (RequantizeOrUpcast's, op_common.h:193-207, and mul's, mul.cc:60-63) in the
 * RequantizeLowerFP form above, int32 output (no clip inside the requantize). */
typedef struct {
  int32_t op;                   /* TK_QB_* */
  tk_requantize_fp_attrs lhs, rhs;
  int32_t lhs_upcast, rhs_upcast;
  tk_requantize_fp_attrs out;   /* TK_QB_MUL only */
  int32_t output_zero_point;    /* add / subtract */
} tk_qnn_binary_fp_attrs;
int tk_qnn_binary_fp(const tk_tensor* lhs, const tk_tensor* rhs, tk_tensor* out, const tk_qnn_binary_fp_attrs* attrs,
                     void* stream);

/* ---------------------------------------------------------------- executor
 * Native run loop replacing GraphExecutor::Run (graph_executor.cc:61-66) and
 * the debug executor's per-node copy-out (graph_executor_debug.cc:249-284).
 * A module holds a flat list of nodes whose tensors are borrowed from the
 * caller for the module's lifetime (the caller keeps them alive).          */

enum {
  TK_NODE_CONV2D = 1,      /* in: data, weight; ext: shadow, packed, weight_sums, scratch */
  TK_NODE_DENSE = 2,       /* in: data, weight; ext: workspace */
  TK_NODE_REQUANTIZE = 3,
  TK_NODE_BIAS_ADD = 4,
  TK_NODE_CLIP = 5,
  TK_NODE_CAST = 6,
  TK_NODE_QNN_ADD = 7,
  TK_NODE_MAX_POOL2D = 8,   /* ext[0]: input shadow (optional), ext[4]: output shadow (optional) */
  TK_NODE_AVG_POOL2D = 9,
  TK_NODE_GLOBAL_AVG_POOL2D = 10,
  TK_NODE_COPY = 11,       /* batch_flatten / reshape */
  TK_NODE_SHADOW = 12,     /* NCHW→NHWC int8 shadow for a conv input (not traced) */
  TK_NODE_CONV_BLOCK = 13, /* in: data, weight, bias, [residual]; outs: 3-5; ext: shadow, packed, weight_sums, scratch, shadow_out */
  TK_NODE_DENSE_BLOCK = 14,/* in: data, weight, bias; outs: 3-4; ext: workspace */
  TK_NODE_ADD_BLOCK = 15,  /* in: lhs, rhs; outs: 1-2 (add, clip); ext[4]: shadow_out */
  TK_NODE_POSTOPS = 16,    /* tachikoma composite post-ops: in: acc int32, [sum_src]; out: dst */
  TK_NODE_EWISE = 17,      /* in: x, [rhs tensor]; attrs.ewise */
  TK_NODE_CONV2D_F32 = 18, /* in: data, weight (float32); attrs.conv2d */
  TK_NODE_DENSE_F32 = 19,  /* in: data, weight (float32) */
  TK_NODE_PAD = 20,        /* in: data; attrs.pad */
  TK_NODE_QUANTIZE = 21,   /* in: data (float32); attrs.qparams */
  TK_NODE_DEQUANTIZE = 22, /* in: data; out float32; attrs.qparams */
  TK_NODE_QNN_BINARY = 23, /* in: lhs, rhs; attrs.qnn_binary */
  TK_NODE_CONCAT = 24,     /* in: 1..TK_MAX_NODE_INPUTS tensors; attrs.concat */
  TK_NODE_TRANSPOSE = 25,  /* in: data; attrs.transpose (layout changes around NHWC convs) */
  TK_NODE_LEAKY_RELU = 26, /* in: data; attrs.leaky_relu */
  TK_NODE_LOOKUP = 27,     /* in: data; ext[0]: the 256-byte device table (qnn unary ops) */
  TK_NODE_BATCH_MATMUL = 28, /* in: x, y; attrs.dense (zero points); ext[0]: workspace */
  TK_NODE_CONV2D_TRANSPOSE = 29, /* in: data (NCHW), weight (IOHW); attrs.conv2d_transpose */
  TK_NODE_SIM_QUANTIZE = 30,   /* in: data (float32); attrs.simq */
  TK_NODE_SIM_DEQUANTIZE = 31, /* in: data (float32); attrs.simq */
  TK_NODE_REQUANTIZE_FP = 32,  /* in: data; attrs.requantize_fp (float compute_dtype) */
  TK_NODE_QNN_BINARY_FP = 33,  /* in: lhs, rhs; attrs.qnn_binary_fp (float compute_dtype) */
};

#define TK_MAX_NODE_INPUTS 8
#define TK_MAX_NODE_OUTPUTS 6

typedef struct {
  int32_t kind;                 /* TK_NODE_* */
  int32_t n_inputs;
  const tk_tensor* inputs[TK_MAX_NODE_INPUTS];
  int32_t n_outputs;            /* traced outputs (0 for SHADOW) */
  tk_tensor* outputs[TK_MAX_NODE_OUTPUTS];
  void* ext[5];                 /* kind-specific device pointers (see enum) */
  union {
    tk_conv2d_attrs conv2d;
    tk_dense_attrs dense;
    tk_requantize_attrs requantize;
    tk_qnn_add_attrs qnn_add;
    tk_pool2d_attrs pool2d;
    tk_block_attrs block;
    tk_add_block_attrs add_block;
    tk_postops_attrs postops;
    tk_ewise_attrs ewise;
    tk_pad_attrs pad;
    tk_qparams_attrs qparams;
    tk_qnn_binary_attrs qnn_binary;
    tk_concat_attrs concat;
    tk_transpose_attrs transpose;
    tk_leaky_relu_attrs leaky_relu;
    tk_conv2d_transpose_attrs conv2d_transpose;
    tk_simq_attrs simq;
    tk_requantize_fp_attrs requantize_fp;
    tk_qnn_binary_fp_attrs qnn_binary_fp;
    struct { int64_t a_min, a_max; } clip;
    struct { int32_t axis; } bias_add;
  } attrs;
} tk_node;

typedef struct tk_module tk_module;

int tk_module_create(const tk_node* nodes, int n_nodes, tk_module** out);
int tk_module_destroy(tk_module* mod);
int tk_module_num_nodes(const tk_module* mod);
/* Runs every node in order on `stream`.  If `capture_stream` and `host_dst`
 * are non-NULL, output k of node i is copied device→host into
 * host_dst[i * TK_MAX_NODE_OUTPUTS + k] (NULL entries are skipped) on
 * capture_stream, the copies gated by an event recorded after node i, so they
 * overlap the following nodes.  After the last copy an event is recorded on
 * capture_stream; every later tk_module_run* call first makes its stream wait on
 * it, so a run never overwrites buffers the previous traced run is still copying
 * (the call returns as soon as the work is enqueued, like GraphExecutor::Run on an
 * asynchronous device). */
int tk_module_run(tk_module* mod, void* stream, void* capture_stream, void* const* host_dst);
/* tk_module_run as one HIP graph: the first call captures the node loop (and the copies, forked
 * onto capture_stream and joined back) into a graph and instantiates it; later calls with the
 * same streams and host destinations replay it with a single launch on `stream`, so a run costs
 * one host API call instead of one per kernel and copy (the host side of a traced step no longer
 * depends on how fast the host issues ~300 calls).  Anything already queued on capture_stream
 * runs first, and capture_stream waits for the launch, so the copies are complete for anything
 * queued on it afterwards (as with tk_module_run).  Up to four graphs (streams / destinations)
 * are kept; tk_module_tune drops them; profiling mode runs tk_module_run. */
int tk_module_run_graph(tk_module* mod, void* stream, void* capture_stream, void* const* host_dst);
/* How tk_module_run_graph copies records to host memory:
 *   0 (default) packed: the node loop is cut into one graph per chunk of the trace image
 *     (tk_module_set_trace_chunks, 8 by default; a chunk ends at the node after which every record
 *     below it is written) plus a tail graph; each chunk graph ends with a kernel that gathers the
 *     chunk's records into a device mirror of the image range the records span (header bytes
 *     included, loaded once from the host image).  After launching a chunk graph the call records a
 *     host-side event on `stream` and issues the chunk's hipMemcpyAsync on capture_stream gated on
 *     it (torch's bundled HIP 7.0 refuses external event-record nodes in stream capture), so a run
 *     costs chunks + 1 graph launches.  Two mirrors alternate, so a run's kernels overlap the
 *     previous run's copies.  Device memory: each packed plan holds two mirrors the size of the whole
 *     span (ResNet-50 at 64 samples: 2 x 7.45 GB), and up to two plans (two host images: the file
 *     sink) are cached, i.e. up to 4 x span.  Whole-chunk copies run at 57.0 GB/s against 56.0 for
 *     per-record copies and 54.0-54.6 for graph memcpy nodes (profiles/r04c_copyprobe.jsonl).  Record
 *     buffers must be 16-byte aligned and readable in whole 16-byte chunks; host destinations must
 *     not overlap.
 *   2..4 one memcpy node per record in that many parallel chains (1 chain: pass 5);
 *   1 one copy kernel per node (kernel nodes writing pinned memory with 16-byte stores). */
int tk_module_set_graph_copies(tk_module* mod, int copy_kernels);
/* Chunks of the packed capture (1..256). */
int tk_module_set_trace_chunks(tk_module* mod, int chunks);
/* Copy trace of packed traced runs (the in-process counterpart of a memory-copy trace, e.g.
 * rocprofv3 --memory-copy-trace): with tracing on, each packed run records a timing event on the
 * compute stream before its first launch and two on the capture stream around every chunk copy.
 * tk_module_copy_trace then (after waiting for the last run's copies) writes, per chunk c,
 * out[3c .. 3c+2] = {bytes, copy start ms, copy end ms} relative to that first event, and returns
 * the chunk count (out may hold fewer: max_chunks). */
int tk_module_set_copy_trace(tk_module* mod, int enable);
int tk_module_copy_trace(tk_module* mod, double* out, int max_chunks);
/* Makes `stream` wait for the copies of the last traced run: call before writing any
 * tensor the module reads (GraphModule.set_input / load_params,
 * graph_executor.cc:158-166 SetInput) on a stream of your own. */
int tk_module_wait_capture(tk_module* mod, void* stream);
/* Runs nodes [begin, end) only (per-op record-and-run, Trace.calibrate analogue). */
int tk_module_run_range(tk_module* mod, int begin, int end, void* stream);
/* Runs once with a timing event after every node and returns per-node device time in
 * milliseconds (GraphExecutorDebug::RunIndividual analogue, graph_executor_debug.cc:70-116). */
int tk_module_run_profiled(tk_module* mod, void* stream, float* node_ms);
/* Profiling mode: subsequent tk_module_run calls (traced or not) also record a timing
 * event after every node on the compute stream; tk_module_node_times reads the last run. */
int tk_module_set_profiling(tk_module* mod, int enable);
int tk_module_node_times(tk_module* mod, float* node_ms);
/* Find step (MIOpen-style, replacing the reference's compile-time schedule choice): for every
 * MFMA conv-block node, times its first max_candidates kernels (tk_conv2d_block_algos; one
 * warm-up + `reps` back-to-back launches each, HIP events on `stream`) and keeps the fastest in
 * the node (block.algo).  Residual-join nodes (block.has_add) time each launch alone after a
 * 512 MiB cache-evicting fill, since their residual operand arrives from HBM in a network run.
 * Nodes with equal shapes and attributes share one measurement.
 * Overwrites node outputs (run afterwards); synchronises `stream`.  Optional reports, n_nodes x
 * (max_candidates + 1) each: algo_out[i][0] = the chosen algo (-1: node not tuned), [i][1 + c]
 * = candidate c (-1 past the last); us_out likewise in microseconds per launch. */
int tk_module_tune(tk_module* mod, void* stream, int max_candidates, int reps, int32_t* algo_out, float* us_out);
/* Sets conv-block node `node` to run kernel `algo` (0 = the library's choice, else one of
 * tk_conv2d_block_algos for that node): replays a saved find-step table, so that a profile and a
 * timed run use the same kernels.  TK_ERR_INVALID_ARG for other nodes or algos. */
int tk_module_set_node_algo(tk_module* mod, int node, int algo);

/* ---------------------------------------------------------------- trace format
 * NDArray-list blob (src/runtime/file_utils.cc:184-236, include/tvm/runtime/ndarray.h:447-494):
 *   u64 0xF7E58D4F05049CB7, u64 0, u64 n, n×(u64 len, bytes), u64 n,
 *   n × { u64 0xDD5E40F096B4A13F, u64 0, i32 dev_type=1, i32 dev_id=0, i32 ndim,
 *         u8 code, u8 bits, u16 lanes, i64 shape[ndim], i64 nbytes, bytes }.
 * The writer lays out a blob so that array payloads can be DMA'd straight into
 * their final positions.                                                   */

typedef struct {
  const char* name;
  int32_t ndim;
  const int64_t* shape;
  tk_dtype dtype;
} tk_array_meta;

/* Total blob size; data_offsets[i] receives the byte offset of array i's payload. */
int64_t tk_ndlist_layout(const tk_array_meta* arrays, int n, int64_t* data_offsets);
/* Writes every header/name byte of the blob into `blob` (payload bytes untouched). */
int tk_ndlist_write_headers(const tk_array_meta* arrays, int n, void* blob, int64_t blob_size);
/* Parses a blob: fills up to `cap` entries.  Names are NOT NUL-terminated: `name` points
 * at the name bytes inside the blob and their length is the u64 stored just before them
 * (((const uint64_t*)name)[-1], unaligned).  Shapes are written to shapes_storage. */
int tk_ndlist_parse(const void* blob, int64_t blob_size, int cap, tk_array_meta* arrays,
                    int64_t* data_offsets, int64_t* shapes_storage, int shapes_cap, int* n_out);

/* Trace container: "TKTRACE\0" | u64 version | u64 json_len | u64 params_off | u64 params_size |
 * u64 records_off | u64 records_size | json | pad | params blob | pad | records blob. */
#define TK_TRACE_MAGIC 0x0045434152544B54ULL /* "TKTRACE\0" little-endian */
#define TK_TRACE_VERSION 1
#define TK_TRACE_ALIGN 4096
typedef struct {
  uint64_t magic, version, json_len, params_off, params_size, records_off, records_size;
} tk_trace_header;

/* Sizes a trace image and fills the fixed header + json + blob headers into `image`
 * (if non-NULL).  param/record payload offsets (absolute, within the image) are returned. */
int64_t tk_trace_layout(const char* json, const tk_array_meta* params, int n_params,
                        const tk_array_meta* records, int n_records, int64_t* param_offsets,
                        int64_t* record_offsets);
int tk_trace_write_headers(const char* json, const tk_array_meta* params, int n_params,
                           const tk_array_meta* records, int n_records, void* image, int64_t image_size);
/* Writes `size` bytes of `image` to `path` (O_TRUNC): the file is sized once; a 4 KiB-aligned
 * image of 64 MiB or more goes out with O_DIRECT in 64 MiB pieces from 4 threads (the < 4 KiB
 * tail buffered), otherwise (or where the filesystem refuses direct I/O) buffered pwrites of
 * 256 MiB pieces from up to 8 threads. */
int tk_write_file(const char* path, const void* image, int64_t size);

/* ---------------------------------------------------------------- digest
 * Order-aware 64-bit digest computed on the device: Σ_i mix64(w_i ^ i·0x9E3779B97F4A7C15)
 * mod 2^64 over little-endian 8-byte words w_i (tail zero-padded), mix64 = the
 * splitmix64 finaliser.  Used by digest-only trace mode and the RCCL digest
 * all-gather.  Result written to *out_device. */
int tk_digest_bytes(const void* data, int64_t nbytes, uint64_t* out_device, void* stream);

#pragma GCC visibility pop

#ifdef __cplusplus
}
#endif
#endif /* TACHIKOMA_H_ */
