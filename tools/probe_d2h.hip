// Device->host ceiling probe: what moves trace bytes over PCIe fastest?
//   sdma1:  one hipMemcpyAsync of the whole buffer (the bench's 1 GiB probe)
//   sdmaS:  the buffer split into S equal copies on S streams, issued together
//   kern G: a copy kernel of G workgroups reading HBM and writing the host-mapped pinned buffer
//           with 16-byte nontemporal vector stores (zero-copy; no SDMA engine involved)
// Each variant runs `reps` times; the best and the median GB/s are printed as one JSON line.
// usage: probe_d2h [MiB=1024] [reps=5] [host buffer kind=mapped] [copy kernels=1]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
typedef int v4i __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ __launch_bounds__(256) void copy_kernel(const v4i* __restrict__ src, v4i* dst, long n16) {
  const long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) {
    v4i v = __builtin_nontemporal_load(src + i);
    __builtin_nontemporal_store(v, dst + i);
  }
}

static void report(const char* name, std::vector<float>& ms, double bytes) {
  std::sort(ms.begin(), ms.end());
  const double best = bytes / (ms.front() * 1e-3) / 1e9, med = bytes / (ms[ms.size() / 2] * 1e-3) / 1e9;
  printf("{\"variant\": \"%s\", \"bytes\": %.0f, \"best_GBps\": %.2f, \"median_GBps\": %.2f}\n", name, bytes, best, med);
  fflush(stdout);
}

int main(int argc, char** argv) {
  const size_t nbytes = (argc > 1 ? atol(argv[1]) : 1024) << 20;  // MiB
  const int reps = argc > 2 ? atoi(argv[2]) : 5;
  void *src, *dst, *dst_dev;
  CK(hipMalloc(&src, nbytes));
  CK(hipMemset(src, 1, nbytes));
  // host buffer kind (argv[3]): mapped (default, what torch's pin_memory gives), noncoherent,
  // coherent, writecombined, register (malloc + hipHostRegister)
  const char* kind = argc > 3 ? argv[3] : "mapped";
  if (!strcmp(kind, "register")) {
    dst = aligned_alloc(4096, nbytes);
    CK(hipHostRegister(dst, nbytes, hipHostRegisterMapped));
  } else {
    unsigned fl = hipHostMallocMapped;
    if (!strcmp(kind, "noncoherent")) fl |= hipHostMallocNonCoherent;
    if (!strcmp(kind, "coherent")) fl |= hipHostMallocCoherent;
    if (!strcmp(kind, "writecombined")) fl |= hipHostMallocWriteCombined;
    CK(hipHostMalloc(&dst, nbytes, fl));
  }
  printf("{\"host_buffer\": \"%s\"}\n", kind);
  memset(dst, 0, nbytes);  // first touch
  CK(hipHostGetDevicePointer(&dst_dev, dst, 0));
  hipStream_t st[8];
  for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1, done[8];
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto& ev : done) CK(hipEventCreate(&ev));

  for (int S : {1, 2, 4, 8}) {
    std::vector<float> ms;
    const size_t part = nbytes / S;
    for (int r = 0; r < reps + 1; ++r) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, st[0]));
      for (int s = 1; s < S; ++s) CK(hipStreamWaitEvent(st[s], e0, 0));
      for (int s = 0; s < S; ++s) {
        CK(hipMemcpyAsync((char*)dst + s * part, (char*)src + s * part, part, hipMemcpyDeviceToHost, st[s]));
        CK(hipEventRecord(done[s], st[s]));
      }
      for (int s = 1; s < S; ++s) CK(hipStreamWaitEvent(st[0], done[s], 0));
      CK(hipEventRecord(e1, st[0]));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      if (r) ms.push_back(t);  // first rep warms the queues
    }
    char name[32];
    snprintf(name, sizeof name, "sdma_streams%d", S);
    report(name, ms, (double)part * S);
  }
  // chunked like a trace step: 64 MiB copies back to back on one stream
  {
    std::vector<float> ms;
    const size_t chunk = 64ull << 20;
    for (int r = 0; r < reps + 1; ++r) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, st[0]));
      for (size_t off = 0; off < nbytes; off += chunk)
        CK(hipMemcpyAsync((char*)dst + off, (char*)src + off, std::min(chunk, nbytes - off), hipMemcpyDeviceToHost, st[0]));
      CK(hipEventRecord(e1, st[0]));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      if (r) ms.push_back(t);
    }
    report("sdma_chunks64MiB", ms, (double)nbytes);
  }
  const long n16 = nbytes / 16;
  const bool kernels = argc > 4 ? atoi(argv[4]) != 0 : true;
  for (int G : {16, 32, 64, 128, 256, 1024}) {
    if (!kernels) break;
    std::vector<float> ms;
    for (int r = 0; r < reps + 1; ++r) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, st[0]));
      copy_kernel<<<G, 256, 0, st[0]>>>((const v4i*)src, (v4i*)dst_dev, n16);
      CK(hipGetLastError());
      CK(hipEventRecord(e1, st[0]));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      if (r) ms.push_back(t);
    }
    char name[32];
    snprintf(name, sizeof name, "kernel_wg%d", G);
    report(name, ms, (double)nbytes);
  }
  // correctness of the kernel path: the host sees the device bytes
  long bad = 0;
  for (size_t i = 0; i < nbytes; i += 4099) bad += ((unsigned char*)dst)[i] != 1;
  printf("{\"check\": \"kernel copy host bytes\", \"bad\": %ld}\n", bad);
  CK(hipFree(src));
  if (!strcmp(kind, "register")) {
    CK(hipHostUnregister(dst));
    free(dst);
  } else {
    CK(hipHostFree(dst));
  }
  return 0;
}
