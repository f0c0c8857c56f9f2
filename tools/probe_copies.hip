// The traced step's copy pattern, isolated: where does graph mode lose D2H rate?
// Reads the record sizes of one step (one per line, bytes, in trace order) and moves them from
// separate device buffers (one per record, like the module's) into one pinned host image laid out
// like the trace file (records back to back with a 64-byte header gap), as
//   host1      one hipMemcpyAsync per record, one stream, issued from the host (per-copy events:
//              mean copy rate vs gaps between copies)
//   graphC     the same copies as memcpy nodes of one HIP graph in C parallel chains (1, 4)
//   packK      the records packed on the device into a mirror of the image (one kernel per chunk),
//              then K contiguous chunk copies, host-issued and as a graph
//   image1     one copy of the whole image (the ceiling)
// usage: probe_copies <sizes.txt> [reps=3]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#define CK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(err_), __LINE__); exit(1);} } while (0)

struct Rec {
  const unsigned char* src;
  long dst;  // offset in the image
  long n;
};

// dst chunk of 16 bytes per thread; each record's bytes land at image offset rec.dst (any alignment)
__global__ __launch_bounds__(256) void pack_kernel(const Rec* recs, int nrec, const long* first_blk,
                                                    unsigned char* img) {
  int lo = 0, hi = nrec - 1;
  const long b = blockIdx.x;
  while (lo < hi) {  // last record whose first block <= b
    int mid = (lo + hi + 1) / 2;
    if (first_blk[mid] <= b) lo = mid; else hi = mid - 1;
  }
  const Rec r = recs[lo];
  const long i = (b - first_blk[lo]) * 256 + threadIdx.x;  // byte group of 16 within the record
  const long start = i * 16;
  if (start >= r.n) return;
  const long n = r.n - start < 16 ? r.n - start : 16;
  for (long k = 0; k < n; ++k) img[r.dst + start + k] = r.src[start + k];
}

static double gbps(double bytes, float ms) { return bytes / (ms * 1e-3) / 1e9; }

int main(int argc, char** argv) {
  if (argc < 2) {
    printf("usage: probe_copies sizes.txt [reps]\n");
    return 2;
  }
  const int reps = argc > 2 ? atoi(argv[2]) : 3;
  std::vector<long> sizes;
  {
    FILE* f = fopen(argv[1], "r");
    if (!f) { printf("cannot open %s\n", argv[1]); return 2; }
    long v;
    while (fscanf(f, "%ld", &v) == 1) sizes.push_back(v);
    fclose(f);
  }
  const int n = (int)sizes.size();
  std::vector<unsigned char*> dev(n);
  std::vector<long> off(n);
  long total = 64, payload = 0;
  for (int i = 0; i < n; ++i) {
    CK(hipMalloc(&dev[i], std::max(16l, sizes[i])));
    CK(hipMemset(dev[i], i & 0xff, std::max(16l, sizes[i])));
    off[i] = total;
    total += sizes[i] + 64;
    payload += sizes[i];
  }
  printf("{\"records\": %d, \"payload_bytes\": %ld, \"image_bytes\": %ld}\n", n, payload, total);
  unsigned char* img;
  CK(hipHostMalloc((void**)&img, total, hipHostMallocMapped));
  memset(img, 0, total);
  unsigned char* mirror;
  CK(hipMalloc(&mirror, total));
  CK(hipMemset(mirror, 0, total));
  hipStream_t s, cs[4];
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  for (auto& c : cs) CK(hipStreamCreateWithFlags(&c, hipStreamNonBlocking));
  hipEvent_t e0, e1, fork, join[4];
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
  for (auto& j : join) CK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
  std::vector<hipEvent_t> ce(2 * n);
  for (auto& e : ce) CK(hipEventCreate(&e));

  // ---- host1 with per-copy events
  for (int r = 0; r <= reps; ++r) {
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < n; ++i) {
      CK(hipEventRecord(ce[2 * i], s));
      CK(hipMemcpyAsync(img + off[i], dev[i], sizes[i], hipMemcpyDeviceToHost, s));
      CK(hipEventRecord(ce[2 * i + 1], s));
    }
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float all, busy = 0, gap = 0, t;
    CK(hipEventElapsedTime(&all, e0, e1));
    for (int i = 0; i < n; ++i) {
      CK(hipEventElapsedTime(&t, ce[2 * i], ce[2 * i + 1]));
      busy += t;
      if (i) {
        CK(hipEventElapsedTime(&t, ce[2 * i - 1], ce[2 * i]));
        gap += t;
      }
    }
    if (r) printf("{\"variant\": \"host1_events\", \"GBps\": %.2f, \"copy_ms\": %.2f, \"gap_ms\": %.2f, \"copy_GBps\": %.2f}\n",
                  gbps(payload, all), busy, gap, gbps(payload, busy));
  }
  // ---- host1 plain
  for (int r = 0; r <= reps; ++r) {
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < n; ++i) CK(hipMemcpyAsync(img + off[i], dev[i], sizes[i], hipMemcpyDeviceToHost, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float t;
    CK(hipEventElapsedTime(&t, e0, e1));
    if (r) printf("{\"variant\": \"host1\", \"GBps\": %.2f}\n", gbps(payload, t));
  }
  // ---- graphs of per-record memcpy nodes in C chains
  for (int C : {1, 4}) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    CK(hipEventRecord(fork, s));
    for (int c = 0; c < C; ++c) CK(hipStreamWaitEvent(cs[c], fork, 0));
    for (int i = 0; i < n; ++i) CK(hipMemcpyAsync(img + off[i], dev[i], sizes[i], hipMemcpyDeviceToHost, cs[i % C]));
    for (int c = 0; c < C; ++c) {
      CK(hipEventRecord(join[c], cs[c]));
      CK(hipStreamWaitEvent(s, join[c], 0));
    }
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int r = 0; r <= reps; ++r) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, s));
      CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      if (r) printf("{\"variant\": \"graph_chains%d\", \"GBps\": %.2f}\n", C, gbps(payload, t));
    }
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  // ---- pack + chunked copies
  std::vector<Rec> recs(n);
  std::vector<long> first(n);
  long blocks = 0;
  for (int i = 0; i < n; ++i) {
    recs[i] = {dev[i], off[i], sizes[i]};
    first[i] = blocks;
    blocks += (sizes[i] + 4095) / 4096;
  }
  Rec* drecs;
  long* dfirst;
  CK(hipMalloc(&drecs, n * sizeof(Rec)));
  CK(hipMalloc(&dfirst, n * sizeof(long)));
  CK(hipMemcpy(drecs, recs.data(), n * sizeof(Rec), hipMemcpyHostToDevice));
  CK(hipMemcpy(dfirst, first.data(), n * sizeof(long), hipMemcpyHostToDevice));
  {
    float best = 1e9;
    for (int r = 0; r <= reps; ++r) {
      CK(hipEventRecord(e0, s));
      hipLaunchKernelGGL(pack_kernel, dim3((unsigned)blocks), dim3(256), 0, s, drecs, n, dfirst, mirror);
      CK(hipGetLastError());
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      if (r) best = std::min(best, t);
    }
    printf("{\"variant\": \"pack_bytewise\", \"ms\": %.3f, \"rw_GBps\": %.1f}\n", best, gbps(2.0 * payload, best));
  }
  for (int K : {1, 8, 32, 128}) {
    const long chunk = (total + K - 1) / K;
    for (int r = 0; r <= reps; ++r) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, s));
      for (long o = 0; o < total; o += chunk)
        CK(hipMemcpyAsync(img + o, mirror + o, std::min(chunk, total - o), hipMemcpyDeviceToHost, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      if (r) printf("{\"variant\": \"image_chunks%d_host\", \"GBps\": %.2f}\n", K, gbps(total, t));
    }
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (long o = 0; o < total; o += chunk)
      CK(hipMemcpyAsync(img + o, mirror + o, std::min(chunk, total - o), hipMemcpyDeviceToHost, s));
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int r = 0; r <= reps; ++r) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, s));
      CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      if (r) printf("{\"variant\": \"image_chunks%d_graph\", \"GBps\": %.2f}\n", K, gbps(total, t));
    }
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
  }
  // ---- per-record copies again, now that the link is warm (the first variants of a fresh process
  // can run at half rate, profiles/r03d2h_probe_host_buffer_kinds.jsonl)
  for (int r = 0; r <= reps; ++r) {
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < n; ++i) CK(hipMemcpyAsync(img + off[i], dev[i], sizes[i], hipMemcpyDeviceToHost, s));
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float t;
    CK(hipEventElapsedTime(&t, e0, e1));
    if (r) printf("{\"variant\": \"host1_warm\", \"GBps\": %.2f}\n", gbps(payload, t));
  }
  // ---- hipMemcpyBatchAsync: all records in G batches (one call each)
  for (int G : {1, 8, 32}) {
    std::vector<void*> dsts(n), srcs(n);
    std::vector<size_t> szs(n);
    for (int i = 0; i < n; ++i) dsts[i] = img + off[i], srcs[i] = dev[i], szs[i] = sizes[i];
    bool ok = true;
    for (int r = 0; r <= reps && ok; ++r) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, s));
      const int per = (n + G - 1) / G;
      for (int b = 0; b < n && ok; b += per) {
        size_t fail = 0;
        hipError_t e = hipMemcpyBatchAsync(dsts.data() + b, srcs.data() + b, szs.data() + b,
                                           (size_t)std::min(per, n - b), nullptr, nullptr, 0, &fail, s);
        if (e != hipSuccess) {
          printf("{\"variant\": \"batch%d\", \"error\": \"%s\", \"fail_index\": %zu}\n", G, hipGetErrorString(e), fail);
          (void)hipGetLastError();
          ok = false;
        }
      }
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      if (r && ok) printf("{\"variant\": \"batch%d\", \"GBps\": %.2f}\n", G, gbps(payload, t));
    }
  }
  // check: the packed image matches the per-record copies
  long bad = 0;
  std::vector<unsigned char> h(64);
  for (int i = 0; i < n; ++i) {
    unsigned char want = (unsigned char)(i & 0xff);
    if (img[off[i]] != want || img[off[i] + sizes[i] - 1] != want) ++bad;
  }
  printf("{\"check\": \"image bytes\", \"bad_records\": %ld}\n", bad);
  // ---- graph of kernels with external event-record nodes, copies issued from the host after
  // waits on those events (a graph launch followed by host-issued copies gated mid-graph)
  {
    const int K = 8;
    const long chunk = (total + K - 1) / K;
    hipEvent_t kev[K];
    for (auto& e : kev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < K; ++k) {
      const long o = k * chunk, len = std::min(chunk, total - o);
      CK(hipMemsetAsync(mirror + o, 0x40 + k, len, s));  // stands in for the chunk's kernels
      CK(hipEventRecordWithFlags(kev[k], s, hipEventRecordExternal));
    }
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    long bad = 0;
    for (int r = 0; r <= reps; ++r) {
      CK(hipDeviceSynchronize());
      memset(img, 0, total);
      CK(hipEventRecord(e0, s));
      CK(hipGraphLaunch(ge, s));
      for (int k = 0; k < K; ++k) {
        const long o = k * chunk, len = std::min(chunk, total - o);
        CK(hipStreamWaitEvent(cs[0], kev[k], 0));
        CK(hipMemcpyAsync(img + o, mirror + o, len, hipMemcpyDeviceToHost, cs[0]));
      }
      CK(hipEventRecord(e1, cs[0]));
      CK(hipEventSynchronize(e1));
      float t;
      CK(hipEventElapsedTime(&t, e0, e1));
      for (int k = 0; k < K; ++k) {
        const long o = k * chunk, len = std::min(chunk, total - o);
        for (long q = o; q < o + len; q += len / 7 + 1) bad += img[q] != (unsigned char)(0x40 + k);
        bad += img[o + len - 1] != (unsigned char)(0x40 + k);
      }
      if (r) printf("{\"variant\": \"graph_events_host_copies%d\", \"GBps\": %.2f, \"bad\": %ld}\n", K, gbps(total, t), bad);
    }
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    for (auto& e : kev) CK(hipEventDestroy(e));
  }
  fflush(stdout);
  for (auto p : dev) CK(hipFree(p));
  CK(hipFree(mirror));
  CK(hipFree(drecs));
  CK(hipFree(dfirst));
  CK(hipHostFree(img));
  return 0;
}
