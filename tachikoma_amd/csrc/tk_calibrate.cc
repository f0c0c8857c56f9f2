// Host-side calibration for relay.quantize's kl_divergence mode: the threshold that minimises
// the KL divergence between a layer's activation histogram and its 8-bit quantisation
// (src/relay/quantize/calibrate.cc:35-146, MinimizeKL, reached through
// python/tvm/relay/quantize/kl_divergence.py:_find_scale_by_kl).
//
// For each candidate window [zero - i, zero + i] (i from num_quantized_bins/2 to num_bins/2),
// p = the window's histogram with both tails folded into its end bins, q = the window merged
// into num_quantized_bins buckets and spread back over p's non-empty bins; both are smoothed
// (every zero bin gets eps, taken proportionally from the non-zero bins) and the divergence
// sum p log(p/q) of the normalised distributions is recorded; the threshold is the window's
// upper edge with the smallest divergence (first on ties).  Arithmetic is float32 in the same
// order as the reference so the selected threshold is the same.
#include <cmath>
#include <limits>
#include <vector>

#include "tk_common.h"

namespace {

// eps to each zero bin, eps * n_zero / n_nonzero taken from each non-zero bin; empty result if
// the distribution is all zeros or the correction would exceed 1.
std::vector<float> smooth(const std::vector<float>& p, float eps = 0.0001f) {
  size_t zeros = 0;
  for (float v : p) zeros += (v == 0.f);
  const size_t nonzeros = p.size() - zeros;
  if (nonzeros == 0) return {};
  const float eps1 = eps * static_cast<float>(zeros) / static_cast<float>(nonzeros);
  if (eps1 >= 1.0f) return {};
  std::vector<float> out(p);
  for (size_t i = 0; i < p.size(); ++i) {
    const bool z = p[i] == 0.f;
    out[i] += eps * static_cast<float>(z) - eps1 * static_cast<float>(!z);
  }
  return out;
}

float divergence(std::vector<float>& p, std::vector<float>& q) {
  float ps = 0.f, qs = 0.f;
  for (float v : p) ps += v;
  for (float v : q) qs += v;
  float d = 0.f;
  for (size_t i = 0; i < p.size(); ++i) {
    p[i] /= ps;
    q[i] /= qs;
    if (p[i] != 0.f && q[i] != 0.f) d += p[i] * std::log(p[i] / q[i]);
  }
  return d;
}

}  // namespace

extern "C" int tk_find_scale_by_kl(const int32_t* hist, const float* edges, int num_bins, int num_quantized_bins,
                                   float* threshold) {
  if (!hist || !edges || !threshold || num_bins < 3 || num_quantized_bins < 2 || num_quantized_bins > num_bins) {
    tk::set_error("tk_find_scale_by_kl: bad arguments");
    return TK_ERR_INVALID_ARG;
  }
  const int zero = num_bins / 2, half_q = num_quantized_bins / 2;
  const int n_cand = zero + 1 - half_q;
  if (n_cand <= 0) {
    tk::set_error("tk_find_scale_by_kl: num_quantized_bins too large for num_bins");
    return TK_ERR_INVALID_ARG;
  }
  std::vector<float> thr(n_cand, 0.f), div(n_cand, 0.f);
  std::vector<float> merged(num_quantized_bins, 0.f);
  for (int i = half_q; i <= zero; ++i) {
    const int lo = zero - i, hi = zero + i + 1;  // window [lo, hi) of the histogram
    thr[i - half_q] = edges[hi];
    const int len = hi - lo;
    std::vector<int> win(len, 0);
    std::vector<float> p(len, 0.f);
    for (int j = 0; j < num_bins; ++j) {
      if (j <= lo) {
        p[0] += static_cast<float>(hist[j]);
      } else if (j >= hi) {
        p[len - 1] += static_cast<float>(hist[j]);
      } else {
        win[j - lo] = hist[j];
        p[j - lo] = static_cast<float>(hist[j]);
      }
    }
    const int per = len / num_quantized_bins;  // window bins per quantised bucket
    for (int j = 0; j < num_quantized_bins; ++j) {
      int s = 0;
      for (int k = j * per; k < (j + 1) * per; ++k) s += win[k];
      merged[j] = static_cast<float>(s);
    }
    {
      int s = 0;
      for (int k = num_quantized_bins * per; k < len; ++k) s += win[k];
      merged[num_quantized_bins - 1] += static_cast<float>(s);
    }
    std::vector<float> q(len, 0.f);
    for (int j = 0; j < num_quantized_bins; ++j) {
      const int a = j * per, b = (j == num_quantized_bins - 1) ? len : (j + 1) * per;
      int nz = 0;
      for (int k = a; k < b; ++k) nz += (win[k] != 0);
      if (nz)
        for (int k = a; k < b; ++k)
          if (p[k] != 0.f) q[k] = merged[j] / static_cast<float>(nz);
    }
    p = smooth(p);
    q = smooth(q);
    div[i - half_q] = q.empty() ? std::numeric_limits<float>::infinity() : divergence(p, q);
  }
  int best = 0;
  for (int k = 1; k < n_cand; ++k)
    if (div[k] < div[best]) best = k;
  *threshold = thr[best];
  return TK_OK;
}
