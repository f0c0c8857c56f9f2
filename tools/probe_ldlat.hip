// Load latency under a record-store stream: does a dependent load wait behind the stores that
// the same CU has issued?  (The conv-block kernels' K loop and epilogue stores "add up" on
// 28x28 planes, profiles/r03pq_store_side.txt; if a CU's vector-memory queue serialises loads
// behind its stores, the next tile's loads must be issued before the current tile's stores.)
// Each workgroup: wave 3 walks a dependent pointer chain (one lane, random hops in a 32 MB
// region) and records the time per hop; waves 0-2 meanwhile either idle (mode 0) or write
// probe_store4's whole-image record pattern (mode 1).  Mode 2: the chains run in their own
// workgroups (even blockIdx), the stores in others (odd): with blockIdx going round-robin over the
// 8 XCDs, on other XCDs.  Mode 3: one workgroup per CU (LDS), chains and stores on the same XCDs
// but never on the same CU.
// hipcc --offload-arch=gfx950 -O3 -o tools/_probe_ldlat tools/probe_ldlat.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <random>
#include <vector>
typedef int v4i __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__device__ void store_chunk(int* c32, int* b32, unsigned* rq, unsigned* cl, long base, int groups, int t0, int nt) {
  for (int g = t0; g < groups; g += nt) {
    const long off = base + 4 * g;
    const v4i v = v4i{g, (int)base, 3, 7};
    __builtin_nontemporal_store(v, reinterpret_cast<v4i*>(c32 + off));
    __builtin_nontemporal_store(v, reinterpret_cast<v4i*>(b32 + off));
    __builtin_nontemporal_store((unsigned)(g * 7), rq + (off >> 2));
    __builtin_nontemporal_store((unsigned)(g * 5), cl + (off >> 2));
  }
}

__global__ __launch_bounds__(256) void probe(int* c32, int* b32, unsigned* rq, unsigned* cl, const unsigned* chain,
                                             unsigned long long* out, int units, int HW, int mode, int hops,
                                             int per_wg) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  extern __shared__ int lds_pad[];  // mode 3: one workgroup per CU
  if (threadIdx.x == 1023) lds_pad[0] = 0;
  // mode 3: workgroups go round-robin over the 8 XCDs, so (blockIdx / 8) even = chains and odd =
  // stores puts both on every XCD (same L2) but, one workgroup per CU, never on the same CU
  const bool split = mode == 2 || mode == 3;
  const bool chain_wg = mode == 2 ? (blockIdx.x & 1) == 0 : ((blockIdx.x >> 3) & 1) == 0;
  const bool chaser = split ? chain_wg : wave == 3;
  const bool storer = mode == 1 ? wave < 3 : split ? !chain_wg : false;
  if (chaser && (!split || wave == 0)) {
    unsigned idx = (blockIdx.x * 7919u) & ((32u << 20) / 4 - 1);
    const unsigned long long t0 = wall_clock64();
    for (int h = 0; h < hops; ++h) idx = __builtin_nontemporal_load(chain + (idx ^ (unsigned)(lane & 15)));
    const unsigned long long t1 = wall_clock64();
    if (lane == 0) out[blockIdx.x] = ((t1 - t0) << 24) | (idx & 0xFFFFFF);
  } else if (storer) {
    // per_wg units of R=32 channels x one image each
    const int nt = mode == 1 ? 192 : 256;
    for (int u = 0; u < per_wg; ++u) {
      const long unit = ((long)blockIdx.x * per_wg + u) % units;
      store_chunk(c32, b32, rq, cl, unit * 32 * HW, 32 * HW / 4, threadIdx.x, nt);
    }
  }
}

int main() {
  const int C = 512, HW = 784, N = 64;
  const long n = (long)N * C * HW;
  const int units = N * C / 32;
  char* buf;
  CK(hipMalloc(&buf, n * 10 + 4096));
  const unsigned words = (32u << 20) / 4;
  std::vector<unsigned> h(words);
  // one random cycle over 64-byte-spaced slots
  const unsigned slots = words / 16;
  std::vector<unsigned> perm(slots);
  for (unsigned i = 0; i < slots; ++i) perm[i] = i;
  std::mt19937 rng(7);
  std::shuffle(perm.begin(), perm.end(), rng);
  for (unsigned i = 0; i < slots; ++i)
    for (unsigned k = 0; k < 16; ++k) h[perm[i] * 16 + k] = perm[(i + 1) % slots] * 16;
  unsigned* chain;
  CK(hipMalloc(&chain, words * 4));
  CK(hipMemcpy(chain, h.data(), words * 4, hipMemcpyHostToDevice));
  unsigned long long* out;
  CK(hipMalloc(&out, 4096 * 8));
  const int hops = 100;
  struct Cfg { int mode, grid, per_wg; const char* what; };
  const Cfg cfgs[] = {{0, 256, 0, "chain alone, 256 WGs          "},
                      {1, 256, 16, "chain + same-WG stores (3 waves)"},
                      {2, 512, 16, "chain WGs beside store WGs      "},
                      {0, 1024, 0, "chain alone, 1024 WGs         "},
                      {1, 1024, 4, "chain + same-WG stores, 1024 WGs"},
                      {3, 256, 32, "chain CUs beside store CUs, same XCDs"},
                      {1, 256, 16, "chain + same-WG stores, 1 WG per CU"}};
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(probe), hipFuncAttributeMaxDynamicSharedMemorySize, 120 * 1024));
  for (const Cfg& c : cfgs)
    for (int rep = 0; rep < 3; ++rep) {
      int* c32 = (int*)buf;
      int* b32 = (int*)(buf + n * 4);
      unsigned* rq = (unsigned*)(buf + n * 8);
      unsigned* cl = (unsigned*)(buf + n * 9);
      hipEvent_t a, b;
      CK(hipEventCreate(&a));
      CK(hipEventCreate(&b));
      CK(hipEventRecord(a));
      const bool one = &c >= &cfgs[5];
      hipLaunchKernelGGL(probe, dim3(c.grid), dim3(256), one ? 120 * 1024 : 0, 0, c32, b32, rq, cl, chain, out, units, HW, c.mode, hops,
                         c.per_wg);
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      std::vector<unsigned long long> o(c.grid);
      CK(hipMemcpy(o.data(), out, c.grid * 8, hipMemcpyDeviceToHost));
      double sum = 0, mx = 0;
      int cnt = 0;
      for (int i = 0; i < c.grid; ++i) {
        if ((c.mode == 2 && (i & 1)) || (c.mode == 3 && ((i >> 3) & 1))) continue;
        const double ns = (double)(o[i] >> 24) * 10.0 / hops;  // wall clock 100 MHz
        sum += ns;
        mx = ns > mx ? ns : mx;
        ++cnt;
      }
      const double stored = c.mode == 0 ? 0.0 : (double)(c.mode >= 2 ? c.grid / 2 : c.grid) * c.per_wg * 32 * HW * 10;
      printf("%s rep %d: %7.1f us kernel, %6.0f ns/hop mean %6.0f max, %5.0f GB/s stored\n", c.what, rep, ms * 1e3,
             sum / cnt, mx, stored / (ms * 1e6));
      fflush(stdout);
    }
  return 0;
}
