/*
 * C restatement of the reference's integer conv/dense (TEST INFRASTRUCTURE ONLY).
 *
 * Same semantics as oracle/qnn_ref.py (which is pinned to the reference's KATs):
 * the x86 "no fast int8" legalization (python/tvm/relay/qnn/op/legalizations.py:177-232,
 * 445-458) turns qnn.conv2d/qnn.dense into nn.conv2d/nn.dense on int16 operands with
 * the zero points subtracted, accumulated in int32 (wrap-around: built with -fwrapv).
 * Padded taps are zeros after the shift.  OpenMP-parallel: this is the CPU baseline
 * ("port") that bench.py times on the GPU box's host cores, and the bit-exactness
 * checker for full-size traces.  Never linked into the product.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static inline int32_t load_i(const void* p, int is_u8, int64_t i) {
  return is_u8 ? (int32_t)((const uint8_t*)p)[i] : (int32_t)((const int8_t*)p)[i];
}

int oracle_num_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* qnn.conv2d NCHW/OIHW → int32 NCHW.  zw_vec (per output channel) overrides zw when non-NULL. */
int oracle_qnn_conv2d(const void* x, int x_u8, const void* w, int w_u8, int32_t* out, int N, int C, int H, int W,
                      int O, int KH, int KW, int sh, int sw, int pt, int pl, int pb, int pr, int dh, int dw,
                      int groups, int32_t za, int32_t zw, const int32_t* zw_vec, int threads) {
  int OH = (H + pt + pb - dh * (KH - 1) - 1) / sh + 1;
  int OW = (W + pl + pr - dw * (KW - 1) - 1) / sw + 1;
  int cg = C / groups, og = O / groups;
  /* int16-shifted input plane, padded with zeros (the shift happens before padding) */
  int HP = H + pt + pb, WP = W + pl + pr;
  int16_t* xs = (int16_t*)malloc(sizeof(int16_t) * (size_t)N * C * HP * WP);
  if (!xs) return -1;
#pragma omp parallel for num_threads(threads) schedule(static)
  for (int64_t nc = 0; nc < (int64_t)N * C; ++nc) {
    int16_t* dst = xs + nc * HP * WP;
    memset(dst, 0, sizeof(int16_t) * HP * WP);
    for (int h = 0; h < H; ++h)
      for (int ww = 0; ww < W; ++ww)
        dst[(h + pt) * WP + (ww + pl)] = (int16_t)(load_i(x, x_u8, (nc * H + h) * W + ww) - za);
  }
#pragma omp parallel for collapse(2) num_threads(threads) schedule(dynamic, 1)
  for (int n = 0; n < N; ++n) {
    for (int o = 0; o < O; ++o) {
      int g = o / og;
      int32_t zwo = zw_vec ? zw_vec[o] : zw;
      uint32_t* acc = (uint32_t*)calloc((size_t)OH * OW, sizeof(uint32_t));
      for (int c = 0; c < cg; ++c) {
        const int16_t* plane = xs + ((int64_t)n * C + g * cg + c) * HP * WP;
        for (int kh = 0; kh < KH; ++kh) {
          for (int kw = 0; kw < KW; ++kw) {
            int32_t wv = load_i(w, w_u8, (((int64_t)o * cg + c) * KH + kh) * KW + kw) - zwo;
            int16_t w16 = (int16_t)wv;
            for (int oh = 0; oh < OH; ++oh) {
              const int16_t* row = plane + (oh * sh + kh * dh) * WP + kw * dw;
              uint32_t* arow = acc + oh * OW;
              if (sw == 1) {
                for (int ow = 0; ow < OW; ++ow) arow[ow] += (uint32_t)((int32_t)row[ow] * (int32_t)w16);
              } else {
                for (int ow = 0; ow < OW; ++ow) arow[ow] += (uint32_t)((int32_t)row[ow * sw] * (int32_t)w16);
              }
            }
          }
        }
      }
      int32_t* dst = out + ((int64_t)n * O + o) * OH * OW;
      for (int i = 0; i < OH * OW; ++i) dst[i] = (int32_t)acc[i];
      free(acc);
    }
  }
  free(xs);
  return 0;
}

/* qnn.dense [M,K] x [N,K]^T → int32 [M,N]. */
int oracle_qnn_dense(const void* x, int x_u8, const void* w, int w_u8, int32_t* out, int M, int K, int Nn,
                     int32_t za, int32_t zw, const int32_t* zw_vec, int threads) {
  int16_t* xs = (int16_t*)malloc(sizeof(int16_t) * (size_t)M * K);
  int16_t* ws = (int16_t*)malloc(sizeof(int16_t) * (size_t)Nn * K);
  if (!xs || !ws) {
    free(xs);
    free(ws);
    return -1;
  }
  for (int64_t i = 0; i < (int64_t)M * K; ++i) xs[i] = (int16_t)(load_i(x, x_u8, i) - za);
  for (int n = 0; n < Nn; ++n) {
    int32_t zwn = zw_vec ? zw_vec[n] : zw;
    for (int k = 0; k < K; ++k) ws[(int64_t)n * K + k] = (int16_t)(load_i(w, w_u8, (int64_t)n * K + k) - zwn);
  }
#pragma omp parallel for collapse(2) num_threads(threads) schedule(static)
  for (int m = 0; m < M; ++m) {
    for (int n = 0; n < Nn; ++n) {
      uint32_t acc = 0;
      const int16_t* a = xs + (int64_t)m * K;
      const int16_t* b = ws + (int64_t)n * K;
      for (int k = 0; k < K; ++k) acc += (uint32_t)((int32_t)a[k] * (int32_t)b[k]);
      out[(int64_t)m * Nn + n] = (int32_t)acc;
    }
  }
  free(xs);
  free(ws);
  return 0;
}
