// Store-pattern probe for the conv-block epilogue on small planes (14x14, 28x28, 7x7 at batch 64):
// the four records of a block (int32 conv, int32 bias_add, int8 requantize, int8 clip; NCHW) written
// with no arithmetic by
//   span:  64-channel x 128-pixel tiles over the flattened N*HW pixel axis (a tile's columns cross
//          image boundaries; channel rows of HW*4 bytes are not 128-byte multiples), 4 columns per
//          lane, rows (tid>>5)+8k -- the layout of gemm_i8_kernel's 4-column epilogue;
//   image: R-channel x one-image tiles: the tile's R*HW elements of each record are one contiguous
//          NCHW run, written as 4-element groups with consecutive lanes on consecutive groups.
// Output buffers rotate over `sets` copies (fresh lines per call, as in the network).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
typedef int v4i __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s\n", hipGetErrorString(e)); exit(1);} } while (0)

// TC-column tiles; ALIGN: tiles never cross an image (ceil(HW / TC) tiles per image, the last one ragged)
template <int TC, bool ALIGN>
__global__ __launch_bounds__(256) void span_store(int* c32, int* b32, unsigned* rq, unsigned* cl, int N, int C, int HW) {
  constexpr int LPR = TC / 4, RPI = 256 / LPR;  // lanes per channel row, rows per pass
  const int P = N * HW;
  const int tpi = (HW + TC - 1) / TC;
  const int tiles_p = ALIGN ? N * tpi : (P + TC - 1) / TC;
  const int tp = blockIdx.x % tiles_p, tc = blockIdx.x / tiles_p;
  const int tid = threadIdx.x;
  int img, pix, p;
  if (ALIGN) {
    img = tp / tpi;
    pix = (tp - img * tpi) * TC + (tid % LPR) * 4;
    if (pix >= HW) return;
    p = img * HW + pix;
  } else {
    p = tp * TC + (tid % LPR) * 4;
    if (p >= P) return;
    img = p / HW;
    pix = p - img * HW;
  }
  const long cbase = (long)img * C * HW + pix;
  for (int k = 0; k < 64 / RPI; ++k) {
    const int ch = tc * 64 + tid / LPR + RPI * k;
    const long off = cbase + (long)ch * HW;
    const v4i v = v4i{ch, p, k, 7};
    *reinterpret_cast<v4i*>(c32 + off) = v;
    *reinterpret_cast<v4i*>(b32 + off) = v;
    rq[off >> 2] = (unsigned)(ch * 7 + p);
    cl[off >> 2] = (unsigned)(ch * 5 + p);
  }
}

template <int R>
__global__ __launch_bounds__(256) void image_store(int* c32, int* b32, unsigned* rq, unsigned* cl, int N, int C, int HW) {
  const int ctiles = C / R;
  const int img = blockIdx.x / ctiles, tc = blockIdx.x - img * ctiles;
  const long base = ((long)img * C + (long)tc * R) * HW;  // element offset of the run
  const int groups = R * HW / 4;
  for (int g = threadIdx.x; g < groups; g += 256) {
    const long off = base + 4 * g;
    const v4i v = v4i{g, img, tc, 7};
    *reinterpret_cast<v4i*>(c32 + off) = v;
    *reinterpret_cast<v4i*>(b32 + off) = v;
    rq[off >> 2] = (unsigned)(g * 7);
    cl[off >> 2] = (unsigned)(g * 5);
  }
}

// walk: R channels x one image per workgroup, written as ceil(HW / TC) sub-tiles of TC pixels in turn
// (a persistent workgroup walking the N tiles of its image); per sub-tile the R channel segments
template <int R, int TC>
__global__ __launch_bounds__(256) void walk_store(int* c32, int* b32, unsigned* rq, unsigned* cl, int N, int C, int HW) {
  constexpr int LPR = TC / 4, RPI = 256 / LPR;
  const int ctiles = C / R;
  const int img = blockIdx.x / ctiles, tc = blockIdx.x - img * ctiles;
  const int tid = threadIdx.x;
  for (int p0 = 0; p0 < HW; p0 += TC) {
    const int pix = p0 + (tid % LPR) * 4;
    if (pix < HW) {
      for (int k = 0; k < R / RPI; ++k) {
        const int ch = tc * R + tid / LPR + RPI * k;
        const long off = ((long)img * C + ch) * HW + pix;
        const v4i v = v4i{ch, pix, k, 7};
        *reinterpret_cast<v4i*>(c32 + off) = v;
        *reinterpret_cast<v4i*>(b32 + off) = v;
        rq[off >> 2] = (unsigned)(ch * 7 + pix);
        cl[off >> 2] = (unsigned)(ch * 5 + pix);
      }
    }
  }
}

int main() {
  const int N = 64;
  struct Case { int C, HW; };
  const Case cases[] = {{1024, 196}, {512, 784}, {128, 784}, {256, 3136}, {64, 3136}};
  const int sets = 6;
  for (const Case& cs : cases) {
    const long n = (long)N * cs.C * cs.HW;
    std::vector<char*> bufs(sets);
    for (int s = 0; s < sets; ++s) CK(hipMalloc(&bufs[s], n * 10 + 4096));
    auto timeit = [&](const char* name, auto launch) {
      for (int s = 0; s < sets; ++s) launch(bufs[s]);
      CK(hipDeviceSynchronize());
      hipEvent_t a, b;
      CK(hipEventCreate(&a));
      CK(hipEventCreate(&b));
      const int iters = 24;
      CK(hipEventRecord(a));
      for (int i = 0; i < iters; ++i) launch(bufs[i % sets]);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      const double us = ms / iters * 1e3;
      printf("C=%5d HW=%5d %-22s %8.1f us %7.0f GB/s\n", cs.C, cs.HW, name, us, n * 10.0 / us / 1e3);
    };
    auto ptrs = [&](char* base, int*& c32, int*& b32, unsigned*& rq, unsigned*& cl) {
      c32 = (int*)base;
      b32 = (int*)(base + n * 4);
      rq = (unsigned*)(base + n * 8);
      cl = (unsigned*)(base + n * 9);
    };
    timeit("span 64x128", [&](char* base) {
      int *c32, *b32; unsigned *rq, *cl;
      ptrs(base, c32, b32, rq, cl);
      const int blocks = ((N * cs.HW + 127) / 128) * (cs.C / 64);
      span_store<128, false><<<blocks, 256>>>(c32, b32, rq, cl, N, cs.C, cs.HW);
    });
    timeit("span 64x256", [&](char* base) {
      int *c32, *b32; unsigned *rq, *cl;
      ptrs(base, c32, b32, rq, cl);
      const int blocks = ((N * cs.HW + 255) / 256) * (cs.C / 64);
      span_store<256, false><<<blocks, 256>>>(c32, b32, rq, cl, N, cs.C, cs.HW);
    });
    timeit("aligned 64x128", [&](char* base) {
      int *c32, *b32; unsigned *rq, *cl;
      ptrs(base, c32, b32, rq, cl);
      const int blocks = N * ((cs.HW + 127) / 128) * (cs.C / 64);
      span_store<128, true><<<blocks, 256>>>(c32, b32, rq, cl, N, cs.C, cs.HW);
    });
    timeit("aligned 64x256", [&](char* base) {
      int *c32, *b32; unsigned *rq, *cl;
      ptrs(base, c32, b32, rq, cl);
      const int blocks = N * ((cs.HW + 255) / 256) * (cs.C / 64);
      span_store<256, true><<<blocks, 256>>>(c32, b32, rq, cl, N, cs.C, cs.HW);
    });
    timeit("image R=64", [&](char* base) {
      int *c32, *b32; unsigned *rq, *cl;
      ptrs(base, c32, b32, rq, cl);
      image_store<64><<<N * (cs.C / 64), 256>>>(c32, b32, rq, cl, N, cs.C, cs.HW);
    });
    timeit("image R=32", [&](char* base) {
      int *c32, *b32; unsigned *rq, *cl;
      ptrs(base, c32, b32, rq, cl);
      image_store<32><<<N * (cs.C / 32), 256>>>(c32, b32, rq, cl, N, cs.C, cs.HW);
    });
    timeit("image R=16", [&](char* base) {
      int *c32, *b32; unsigned *rq, *cl;
      ptrs(base, c32, b32, rq, cl);
      image_store<16><<<N * (cs.C / 16), 256>>>(c32, b32, rq, cl, N, cs.C, cs.HW);
    });
    timeit("walk R=64 TC=128", [&](char* base) {
      int *c32, *b32; unsigned *rq, *cl;
      ptrs(base, c32, b32, rq, cl);
      walk_store<64, 128><<<N * (cs.C / 64), 256>>>(c32, b32, rq, cl, N, cs.C, cs.HW);
    });
    timeit("walk R=64 TC=256", [&](char* base) {
      int *c32, *b32; unsigned *rq, *cl;
      ptrs(base, c32, b32, rq, cl);
      walk_store<64, 256><<<N * (cs.C / 64), 256>>>(c32, b32, rq, cl, N, cs.C, cs.HW);
    });
    timeit("walk R=16 TC=256", [&](char* base) {
      int *c32, *b32; unsigned *rq, *cl;
      ptrs(base, c32, b32, rq, cl);
      walk_store<16, 256><<<N * (cs.C / 16), 256>>>(c32, b32, rq, cl, N, cs.C, cs.HW);
    });
    for (char* p : bufs) CK(hipFree(p));
  }
  return 0;
}
