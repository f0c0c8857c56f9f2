/* Host DRAM bandwidth of one NUMA node: the ceiling the trace images of the
 * GPUs on that node share.  T threads bound to the node's CPUs stream over their own buffers
 * (first-touched by the bound thread, so the pages sit on that node):
 *   write  16-byte non-temporal stores (what a D2H DMA into a pinned image does to DRAM)
 *   read   16-byte loads summed (what a file writer reading the image does)
 * for `secs` seconds each; prints one JSON line per pass.
 * usage: probe_hostmem <node> <threads> [secs=3] [MiB per thread=512] */
#define _GNU_SOURCE
#include <emmintrin.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static int node_cpus[4096], n_node_cpus;
static size_t per_thread;
static double secs;
static volatile int phase;  /* 0 idle, 1 write, 2 read, 3 exit */

typedef struct {
  int id;
  char* buf;
  double bytes;
  double sink;
} worker_t;

static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

static void* run(void* arg) {
  worker_t* w = (worker_t*)arg;
  cpu_set_t set;
  CPU_ZERO(&set);
  CPU_SET(node_cpus[w->id % n_node_cpus], &set);
  sched_setaffinity(0, sizeof set, &set);
  w->buf = aligned_alloc(4096, per_thread);
  memset(w->buf, 1, per_thread); /* first touch on this node */
  const size_t n16 = per_thread / 16;
  for (int p = 1; p <= 2; ++p) {
    while (phase < p) sched_yield();
    double t0 = now(), bytes = 0;
    __m128i v = _mm_set1_epi32(w->id);
    __m128i acc = _mm_setzero_si128();
    while (now() - t0 < secs) {
      __m128i* q = (__m128i*)w->buf;
      if (p == 1) {
        for (size_t i = 0; i < n16; ++i) _mm_stream_si128(q + i, v);
        _mm_sfence();
      } else {
        for (size_t i = 0; i < n16; ++i) acc = _mm_add_epi64(acc, _mm_load_si128(q + i));
      }
      bytes += (double)per_thread;
    }
    w->bytes = bytes / (now() - t0);
    w->sink += (double)_mm_cvtsi128_si64(acc);
    while (phase == p) sched_yield();
  }
  free(w->buf);
  return NULL;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: probe_hostmem <node> <threads> [secs] [MiB per thread]\n");
    return 2;
  }
  const int node = atoi(argv[1]), nt = atoi(argv[2]);
  secs = argc > 3 ? atof(argv[3]) : 3.0;
  per_thread = (size_t)(argc > 4 ? atol(argv[4]) : 512) << 20;
  char path[128];
  snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
  FILE* f = fopen(path, "r");
  if (!f) {
    fprintf(stderr, "no node %d\n", node);
    return 2;
  }
  char list[65536];
  if (!fgets(list, sizeof list, f)) list[0] = 0;
  fclose(f);
  cpu_set_t allowed;
  sched_getaffinity(0, sizeof allowed, &allowed);
  for (char* tok = strtok(list, ",\n"); tok; tok = strtok(NULL, ",\n")) {
    int a, b;
    if (sscanf(tok, "%d-%d", &a, &b) != 2) b = a = atoi(tok);
    for (int c = a; c <= b && n_node_cpus < 4096; ++c)
      if (CPU_ISSET(c, &allowed)) node_cpus[n_node_cpus++] = c;
  }
  if (!n_node_cpus) {
    fprintf(stderr, "node %d: none of its CPUs is in this process's affinity\n", node);
    return 2;
  }
  pthread_t th[512];
  worker_t ws[512];
  const int n = nt < 512 ? nt : 512;
  for (int i = 0; i < n; ++i) {
    memset(&ws[i], 0, sizeof ws[i]);
    ws[i].id = i;
    pthread_create(&th[i], NULL, run, &ws[i]);
  }
  struct timespec d = {0, 300 * 1000 * 1000};
  nanosleep(&d, NULL); /* let every thread first-touch its buffer */
  for (int p = 1; p <= 2; ++p) {
    phase = p;
    const double t0 = now();
    while (now() - t0 < secs + 0.5) nanosleep(&d, NULL);
    double gbps = 0;
    for (int i = 0; i < n; ++i) gbps += ws[i].bytes;
    printf("{\"node\": %d, \"threads\": %d, \"node_cpus_usable\": %d, \"pass\": \"%s\", \"GBps\": %.1f}\n", node, n,
           n_node_cpus, p == 1 ? "nt_write" : "read", gbps / 1e9);
    fflush(stdout);
  }
  phase = 3;
  for (int i = 0; i < n; ++i) pthread_join(th[i], NULL);
  return 0;
}
