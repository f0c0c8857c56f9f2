// Store-pattern probe for the fused block epilogue: a TR-channel x TC-pixel tile per
// workgroup writes int32 conv + int32 bias_add + int8 requantize + int8 clip records
// (NCHW) and optionally an int8 shadow (NHWC or channel-blocked [C/16][P][16]), with
// no arithmetic.  Shows what each write pattern alone reaches on HBM.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef int v4i __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s\n", hipGetErrorString(e)); exit(1);} } while (0)

// MASK: 1 conv, 2 bias, 4 rq, 8 clip, 16 shadow NHWC, 32 shadow blocked; SEQ: records one after another; NT: nontemporal
template <int TR, int TC, int MASK, bool SEQ, bool NT>
__global__ __launch_bounds__(256) void block_store(int* c32, int* b32, unsigned char* rq, unsigned char* cl,
                                                   unsigned char* sh, int N, int C, int HW, int cpad) {
  const int P = N * HW;
  const int tiles_p = P / TC;
  const int tp = blockIdx.x % tiles_p, tc = blockIdx.x / tiles_p;
  const int tid = threadIdx.x;
  constexpr int LPR = TC / 4;            // lanes per row
  constexpr int RPI = 256 / LPR;         // rows per iteration
  const int c4 = (tid % LPR) * 4;
  const int p = tp * TC + c4;
  const int img = p / HW, pix = p - img * HW;
  const long cbase = (long)img * C * HW + pix;
  auto st4 = [&](int* d, v4i v) { if (NT) __builtin_nontemporal_store(v, reinterpret_cast<v4i*>(d)); else *reinterpret_cast<v4i*>(d) = v; };
  auto st1 = [&](unsigned char* d, unsigned v) { if (NT) __builtin_nontemporal_store(v, reinterpret_cast<unsigned*>(d)); else *reinterpret_cast<unsigned*>(d) = v; };
  if (!SEQ) {
    for (int k = 0; k < TR / RPI; ++k) {
      const int ch = tc * TR + tid / LPR + RPI * k;
      const long off = cbase + (long)ch * HW;
      v4i v = v4i{ch, p, k, 7};
      if (MASK & 1) st4(c32 + off, v);
      if (MASK & 2) st4(b32 + off, v);
      if (MASK & 4) st1(rq + off, (unsigned)(ch * 7 + p));
      if (MASK & 8) st1(cl + off, (unsigned)(ch * 5 + p));
    }
  } else {
#define LOOP(COND, STMT) if (COND) for (int k = 0; k < TR / RPI; ++k) { const int ch = tc * TR + tid / LPR + RPI * k; const long off = cbase + (long)ch * HW; STMT; }
    LOOP(MASK & 1, st4(c32 + off, (v4i{ch, p, k, 7})));
    LOOP(MASK & 2, st4(b32 + off, (v4i{ch, p, k, 7})));
    LOOP(MASK & 4, st1(rq + off, (unsigned)(ch * 7 + p)));
    LOOP(MASK & 8, st1(cl + off, (unsigned)(ch * 5 + p)));
  }
  if (MASK & 16) {
    for (int it = tid; it < TR / 16 * TC; it += 256) {
      const int lc = it % TC, grp = it / TC;
      const long pp = (long)tp * TC + lc;
      *reinterpret_cast<v4i*>(sh + pp * cpad + tc * TR + grp * 16) = v4i{lc, grp, 1, 2};
    }
  }
  if (MASK & 32) {
    for (int it = tid; it < TR / 16 * TC; it += 256) {
      const int lc = it % TC, grp = it / TC;
      const long pp = (long)tp * TC + lc;
      const long g16 = (long)(tc * TR / 16 + grp);
      *reinterpret_cast<v4i*>(sh + (g16 * P + pp) * 16) = v4i{lc, grp, 1, 2};
    }
  }
}

template <int TR, int TC, int MASK, bool SEQ, bool NT>
void run(const char* name, int* c32, int* b32, unsigned char* rq, unsigned char* cl, unsigned char* sh, int N, int C,
         int HW) {
  int blocks = (N * HW / TC) * (C / TR);
  double bytes = 0, el = (double)N * C * HW;
  if (MASK & 1) bytes += 4 * el;
  if (MASK & 2) bytes += 4 * el;
  if (MASK & 4) bytes += el;
  if (MASK & 8) bytes += el;
  if (MASK & 48) bytes += el;
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  block_store<TR, TC, MASK, SEQ, NT><<<blocks, 256>>>(c32, b32, rq, cl, sh, N, C, HW, C);
  CK(hipEventRecord(a));
  for (int i = 0; i < 10; ++i) block_store<TR, TC, MASK, SEQ, NT><<<blocks, 256>>>(c32, b32, rq, cl, sh, N, C, HW, C);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  printf("%-44s %8.1f us  %6.0f GB/s\n", name, ms / 10 * 1e3, bytes / (ms / 10) / 1e6);
}

int main() {
  int N = 64, C = 256, HW = 3136;
  long n = (long)N * C * HW;
  // one arena; the four records at controlled relative offsets (skew = extra bytes between records)
  char* arena;
  const long slack = 64L << 20;
  CK(hipMalloc(&arena, n * 4 * 2 + n * 3 + 4 * slack));
  long skews[] = {0, 256, 4096, 65536, 1 << 20, 3 * 4096 + 256};
  for (long sk : skews) {
    auto align = [](long v) { return (v + (2L << 20) - 1) / (2L << 20) * (2L << 20); };
    long o0 = 0, o1 = align(o0 + n * 4) + sk, o2 = align(o1 + n * 4) + 2 * sk, o3 = align(o2 + n) + 3 * sk,
         o4 = align(o3 + n) + 4 * sk;
    int* c32 = (int*)(arena + o0); int* b32 = (int*)(arena + o1);
    unsigned char* rq = (unsigned char*)(arena + o2); unsigned char* cl = (unsigned char*)(arena + o3);
    unsigned char* sh = (unsigned char*)(arena + o4);
    char name[64];
    printf("-- skew %ld\n", sk);
    snprintf(name, 64, "4 rec interleaved");
    run<64, 128, 15, false, false>(name, c32, b32, rq, cl, sh, N, C, HW);
    snprintf(name, 64, "4 rec NT");
    run<64, 128, 15, false, true>(name, c32, b32, rq, cl, sh, N, C, HW);
    snprintf(name, 64, "conv+bias");
    run<64, 128, 3, false, false>(name, c32, b32, rq, cl, sh, N, C, HW);
    snprintf(name, 64, "4 rec + blocked shadow NT");
    run<64, 128, 47, false, true>(name, c32, b32, rq, cl, sh, N, C, HW);
  }
  return 0;
}
