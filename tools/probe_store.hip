// Write-pattern probe: NCHW int32 tile stores (channels x pixels per block) vs linear stores.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef int v4i __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s\n", hipGetErrorString(e)); exit(1);} } while (0)

// block writes a [TR channels][TC pixels] tile of out[N][C][HW]; thread -> 4 consecutive pixels
template <int TR, int TC>
__global__ __launch_bounds__(256) void tile_store(int* out, int N, int C, int HW) {
  int P = N * HW;
  int tiles_p = (P + TC - 1) / TC;
  int tp = blockIdx.x % tiles_p, tc = blockIdx.x / tiles_p;
  for (int item = threadIdx.x; item < TR * TC / 4; item += 256) {
    int r = item / (TC / 4), c4 = (item % (TC / 4)) * 4;
    int ch = tc * TR + r, p = tp * TC + c4;
    if (ch >= C || p >= P) continue;
    int img = p / HW, pix = p - img * HW;
    long off = ((long)img * C + ch) * HW + pix;
    *reinterpret_cast<v4i*>(out + off) = v4i{ch, p, 1, 2};
  }
}
__global__ void linear_store(int* out, long n) {
  long i = (blockIdx.x * 256L + threadIdx.x) * 4, stride = gridDim.x * 256L * 4;
  for (; i < n; i += stride) *reinterpret_cast<v4i*>(out + i) = v4i{1, 2, 3, 4};
}
template <int TR, int TC> float run(int* out, int N, int C, int HW) {
  int P = N * HW;
  int blocks = ((P + TC - 1) / TC) * ((C + TR - 1) / TR);
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  tile_store<TR, TC><<<blocks, 256>>>(out, N, C, HW);
  CK(hipEventRecord(a));
  for (int i = 0; i < 10; ++i) tile_store<TR, TC><<<blocks, 256>>>(out, N, C, HW);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms / 10;
}
int main() {
  int N = 64, C = 256, HW = 3136;
  long n = (long)N * C * HW;
  int* out; CK(hipMalloc(&out, n * 4));
  double bytes = n * 4.0;
  printf("tile 128x128: %.0f GB/s\n", bytes / run<128, 128>(out, N, C, HW) / 1e6);
  printf("tile 64x256 : %.0f GB/s\n", bytes / run<64, 256>(out, N, C, HW) / 1e6);
  printf("tile 32x512 : %.0f GB/s\n", bytes / run<32, 512>(out, N, C, HW) / 1e6);
  printf("tile 16x1024: %.0f GB/s\n", bytes / run<16, 1024>(out, N, C, HW) / 1e6);
  printf("tile 256x64 : %.0f GB/s\n", bytes / run<256, 64>(out, N, C, HW) / 1e6);
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  linear_store<<<4096, 256>>>(out, n);
  CK(hipEventRecord(a));
  for (int i = 0; i < 10; ++i) linear_store<<<4096, 256>>>(out, n);
  CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  printf("linear      : %.0f GB/s\n", bytes / (ms / 10) / 1e6);
  // 7x7 planes (HW=49): tile widths straddle images
  N = 64; C = 2048; HW = 49; n = (long)N * C * HW; bytes = n * 4.0;
  printf("7x7 tile 128x128: %.0f GB/s\n", bytes / run<128, 128>(out, N, C, HW) / 1e6);
  return 0;
}
