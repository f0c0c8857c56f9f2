// Hardware probe for the tachikoma-mi355x design (not product code).
// 1) verifies the int8 MFMA operand/accumulator lane maps with exact integer data,
// 2) measures the int8 MFMA issue rate across all CUs,
// 3) measures pinned D2H bandwidth (SDMA copy vs. kernel stores into mapped host memory),
// 4) measures device-to-device streaming bandwidth.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <chrono>
#include <cstring>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

// hypothesis: A[i][k] at lane i + 32*(k/16), byte k%16; B[k][j] at lane j + 32*(k/16)
__global__ void mfma32_probe(const int8_t* A, const int8_t* B, int* D) {
  int l = threadIdx.x;
  int8_t a[16], b[16];
  for (int j = 0; j < 16; ++j) {
    int k = 16 * (l >> 5) + j;
    a[j] = A[(l & 31) * 32 + k];
    b[j] = B[k * 32 + (l & 31)];
  }
  v4i av, bv;
  __builtin_memcpy(&av, a, 16);
  __builtin_memcpy(&bv, b, 16);
  v16i acc = {0};
  acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, acc, 0, 0, 0);
  for (int r = 0; r < 16; ++r) {
    int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
    int col = l & 31;
    D[row * 32 + col] = acc[r];
  }
}

__global__ void mfma16_probe(const int8_t* A, const int8_t* B, int* D) {
  int l = threadIdx.x;
  int8_t a[16], b[16];
  for (int j = 0; j < 16; ++j) {
    int k = 16 * (l >> 4) + j;
    a[j] = A[(l & 15) * 64 + k];
    b[j] = B[k * 16 + (l & 15)];
  }
  v4i av, bv;
  __builtin_memcpy(&av, a, 16);
  __builtin_memcpy(&bv, b, 16);
  v4i acc = {0};
  acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) {
    int row = 4 * (l >> 4) + r;
    int col = l & 15;
    D[row * 16 + col] = acc[r];
  }
}

// A-only permutation check: does A's lane/byte -> k map equal B's? Use A = one-hot rows.
__global__ void mfma_rate(int iters, int* sink, int seed) {
  v4i a = {seed, seed + 1, seed + 2, seed + 3};
  v4i b = {seed * 3, seed + 5, seed + 7, seed + 9};
  v16i c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0};
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, a, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, a, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, b, c3, 0, 0, 0);
  }
  int s = 0;
  for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
  if (s == 0x12345678) sink[threadIdx.x] = s;
}

__global__ void mfma16_rate(int iters, int* sink, int seed) {
  v4i a = {seed, seed + 1, seed + 2, seed + 3};
  v4i b = {seed * 3, seed + 5, seed + 7, seed + 9};
  v4i c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0};
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(b, a, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, a, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(b, b, c3, 0, 0, 0);
  }
  int s = 0;
  for (int r = 0; r < 4; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
  if (s == 0x12345678) sink[threadIdx.x] = s;
}

__global__ void copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) dst[i] = src[i];
}

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  int dev = 0;
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, dev));
  printf("device %s CUs=%d clock=%d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);

  // ---- 1) layout probes
  {
    std::vector<int8_t> A(32 * 32), B(32 * 32);
    srand(1);
    for (auto& x : A) x = (int8_t)(rand() % 255 - 127);
    for (auto& x : B) x = (int8_t)(rand() % 255 - 127);
    std::vector<int> ref(32 * 32, 0), got(32 * 32);
    for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) {
      int s = 0; for (int k = 0; k < 32; ++k) s += A[i * 32 + k] * B[k * 32 + j]; ref[i * 32 + j] = s; }
    int8_t *dA, *dB; int* dD;
    CK(hipMalloc(&dA, 1024)); CK(hipMalloc(&dB, 1024)); CK(hipMalloc(&dD, 4096 * 4));
    CK(hipMemcpy(dA, A.data(), 1024, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), 1024, hipMemcpyHostToDevice));
    mfma32_probe<<<1, 64>>>(dA, dB, dD);
    CK(hipMemcpy(got.data(), dD, 4096, hipMemcpyDeviceToHost));
    int bad = 0; for (int i = 0; i < 1024; ++i) bad += got[i] != ref[i];
    printf("mfma_i32_32x32x32_i8 layout hypothesis: %s (%d mismatches)\n", bad ? "FAIL" : "OK", bad);

    std::vector<int8_t> A2(16 * 64), B2(64 * 16);
    for (auto& x : A2) x = (int8_t)(rand() % 255 - 127);
    for (auto& x : B2) x = (int8_t)(rand() % 255 - 127);
    std::vector<int> ref2(256), got2(256);
    for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) {
      int s = 0; for (int k = 0; k < 64; ++k) s += A2[i * 64 + k] * B2[k * 16 + j]; ref2[i * 16 + j] = s; }
    CK(hipMemcpy(dA, A2.data(), 1024, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B2.data(), 1024, hipMemcpyHostToDevice));
    mfma16_probe<<<1, 64>>>(dA, dB, dD);
    CK(hipMemcpy(got2.data(), dD, 1024, hipMemcpyDeviceToHost));
    bad = 0; for (int i = 0; i < 256; ++i) bad += got2[i] != ref2[i];
    printf("mfma_i32_16x16x64_i8 layout hypothesis: %s (%d mismatches)\n", bad ? "FAIL" : "OK", bad);
  }

  // ---- 2) MFMA rate
  {
    int* sink; CK(hipMalloc(&sink, 4096));
    int iters = 20000;
    for (int variant = 0; variant < 2; ++variant) {
      for (int wpb : {4, 8}) {
        int blocks = p.multiProcessorCount * 2;
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        if (variant == 0) mfma_rate<<<blocks, 64 * wpb>>>(100, sink, 1); else mfma16_rate<<<blocks, 64 * wpb>>>(100, sink, 1);
        CK(hipEventRecord(e0));
        if (variant == 0) mfma_rate<<<blocks, 64 * wpb>>>(iters, sink, 1); else mfma16_rate<<<blocks, 64 * wpb>>>(iters, sink, 1);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        double macs_per = variant == 0 ? 32.0 * 32 * 32 : 16.0 * 16 * 64;
        double ops = 2.0 * macs_per * 4 * iters * (double)blocks * wpb;
        printf("%s waves/block=%d blocks=%d: %.1f TOPS (%.3f ms)\n", variant == 0 ? "mfma_i32_32x32x32_i8" : "mfma_i32_16x16x64_i8", wpb, blocks, ops / ms / 1e9, ms);
      }
    }
  }

  // ---- 3) D2H bandwidth
  {
    size_t bytes = (size_t)2 << 30;
    char* d; CK(hipMalloc(&d, bytes));
    CK(hipMemset(d, 1, bytes));
    char* h; CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
    memset(h, 0, bytes);
    for (int nstreams : {1, 2, 4, 8}) {
      std::vector<hipStream_t> s(nstreams);
      for (auto& x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
      size_t chunk = bytes / nstreams;
      CK(hipDeviceSynchronize());
      for (int rep = 0; rep < 2; ++rep) {
        double t0 = now();
        for (int i = 0; i < nstreams; ++i) CK(hipMemcpyAsync(h + i * chunk, d + i * chunk, chunk, hipMemcpyDeviceToHost, s[i]));
        for (auto& x : s) CK(hipStreamSynchronize(x));
        double t1 = now();
        if (rep == 1) printf("D2H hipMemcpyAsync %d streams: %.1f GB/s\n", nstreams, bytes / (t1 - t0) / 1e9);
      }
      for (auto& x : s) CK(hipStreamDestroy(x));
    }
    // many medium chunks on 1 stream (per-op records are 0.1-100 MB)
    {
      hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      for (size_t chunk : {(size_t)1 << 20, (size_t)8 << 20, (size_t)64 << 20}) {
        double t0 = now();
        for (size_t off = 0; off < bytes; off += chunk) CK(hipMemcpyAsync(h + off, d + off, chunk, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        double t1 = now();
        printf("D2H 1 stream chunk=%zu MB: %.1f GB/s\n", chunk >> 20, bytes / (t1 - t0) / 1e9);
      }
      CK(hipStreamDestroy(s));
    }
    // kernel stores into mapped pinned host memory
    {
      char* hm; CK(hipHostMalloc(&hm, bytes, hipHostMallocMapped));
      void* hd; CK(hipHostGetDevicePointer(&hd, hm, 0));
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipDeviceSynchronize());
        double t0 = now();
        copy_kernel<<<p.multiProcessorCount * 4, 256>>>((const uint4*)d, (uint4*)hd, bytes / 16);
        CK(hipDeviceSynchronize());
        double t1 = now();
        if (rep == 1) printf("D2H kernel stores to mapped host: %.1f GB/s\n", bytes / (t1 - t0) / 1e9);
      }
      CK(hipHostFree(hm));
    }
    // H2D for reference
    {
      double t0 = now();
      CK(hipMemcpy(d, h, bytes, hipMemcpyHostToDevice));
      double t1 = now();
      printf("H2D hipMemcpy: %.1f GB/s\n", bytes / (t1 - t0) / 1e9);
    }
    // ---- 4) D2D copy kernel
    {
      char* d2; CK(hipMalloc(&d2, bytes));
      for (int rep = 0; rep < 3; ++rep) {
        hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
        CK(hipEventRecord(e0));
        copy_kernel<<<p.multiProcessorCount * 8, 256>>>((const uint4*)d, (uint4*)d2, bytes / 16);
        CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        if (rep == 2) printf("D2D copy kernel: %.1f GB/s (read+write)\n", 2.0 * bytes / ms / 1e6);
      }
    }
    CK(hipHostFree(h));
  }
  printf("probe done\n");
  return 0;
}
