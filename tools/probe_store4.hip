// Store-only probe, part 4: does the record-store rate of whole-image runs (probe_store3's "image
// R=32" pattern: each workgroup writes R channels x one image of four records, 16-byte int32 and
// 4-byte int8 stores, contiguous across lanes) depend on how many workgroups a CU holds?  The
// conv-block kernels hold 1-4 (LDS); the probe holds 8.  Occupancy is forced with dynamic LDS.
// Also: plain vs nontemporal stores.
// hipcc --offload-arch=gfx950 -O3 -o /tmp/probe_store4 tools/probe_store4.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>
typedef int v4i __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <int R, bool NT>
__global__ __launch_bounds__(256) void image_store(int* c32, int* b32, unsigned* rq, unsigned* cl, int C, int HW) {
  extern __shared__ int lds_pad[];  // only to limit workgroups per CU
  const int ctiles = C / R;
  const int img = blockIdx.x / ctiles, tc = blockIdx.x - img * ctiles;
  const long base = ((long)img * C + (long)tc * R) * HW;
  const int groups = R * HW / 4;
  if (threadIdx.x == 1023) lds_pad[0] = 0;  // keep the allocation
  for (int g = threadIdx.x; g < groups; g += 256) {
    const long off = base + 4 * g;
    const v4i v = v4i{g, img, tc, 7};
    if (NT) {
      __builtin_nontemporal_store(v, reinterpret_cast<v4i*>(c32 + off));
      __builtin_nontemporal_store(v, reinterpret_cast<v4i*>(b32 + off));
      __builtin_nontemporal_store((unsigned)(g * 7), rq + (off >> 2));
      __builtin_nontemporal_store((unsigned)(g * 5), cl + (off >> 2));
    } else {
      *reinterpret_cast<v4i*>(c32 + off) = v;
      *reinterpret_cast<v4i*>(b32 + off) = v;
      rq[off >> 2] = (unsigned)(g * 7);
      cl[off >> 2] = (unsigned)(g * 5);
    }
  }
}

int main() {
  const int N = 64;
  struct Case { int C, HW; };
  const Case cases[] = {{512, 784}, {1024, 196}, {256, 3136}};
  const int sets = 4;
  const int lds_kb[] = {0, 36, 76, 150};
  for (const Case& cs : cases) {
    const long n = (long)N * cs.C * cs.HW;
    std::vector<char*> bufs(sets);
    for (int s = 0; s < sets; ++s) CK(hipMalloc(&bufs[s], n * 10 + 4096));
    for (int nt = 0; nt < 2; ++nt)
      for (int kb : lds_kb) {
        auto kern = nt ? image_store<32, true> : image_store<32, false>;
        if (kb * 1024 > 64 * 1024)
          CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern), hipFuncAttributeMaxDynamicSharedMemorySize,
                                 kb * 1024));
        auto launch = [&](char* base) {
          int* c32 = (int*)base;
          int* b32 = (int*)(base + n * 4);
          unsigned* rq = (unsigned*)(base + n * 8);
          unsigned* cl = (unsigned*)(base + n * 9);
          hipLaunchKernelGGL(kern, dim3(N * (cs.C / 32)), dim3(256), kb * 1024, 0, c32, b32, rq, cl, cs.C, cs.HW);
        };
        for (int s = 0; s < sets; ++s) launch(bufs[s]);
        CK(hipDeviceSynchronize());
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        const int iters = 16;
        CK(hipEventRecord(a));
        for (int i = 0; i < iters; ++i) launch(bufs[i % sets]);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        const double us = ms / iters * 1e3;
        printf("C=%5d HW=%5d image R=32 %s LDS %3d KB  %8.1f us %7.0f GB/s\n", cs.C, cs.HW, nt ? "NT   " : "plain", kb, us,
               n * 10.0 / us / 1e3);
        fflush(stdout);
      }
    for (char* p : bufs) CK(hipFree(p));
  }
  return 0;
}
