// Trace-binary serialisation (host only).
//
// The tensor payload encoding is the reference's NDArray-list blob, written by
// SaveParams / SaveDLTensor (src/runtime/file_utils.cc:210-236,
// include/tvm/runtime/ndarray.h:447-494) and read by LoadParams (:184-206) and
// the dependency-free CRT reader (src/runtime/crt/graph_executor/graph_executor.c:781-860,
// src/runtime/crt/common/ndarray.c:72-131).  The layout is computed up front so
// device→host copies can land directly at each array's final payload offset.
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/tachikoma.h"

namespace tk {
void set_error(const std::string& msg);
}

namespace {

constexpr uint64_t kListMagic = 0xF7E58D4F05049CB7ULL;   // kTVMNDArrayListMagic (file_utils.h:107)
constexpr uint64_t kArrayMagic = 0xDD5E40F096B4A13FULL;  // kTVMNDArrayMagic (ndarray.h:447)

int64_t payload_bytes(const tk_array_meta& a) {
  int64_t n = 1;
  for (int i = 0; i < a.ndim; ++i) n *= a.shape[i];
  return n * ((a.dtype.bits + 7) / 8) * (a.dtype.lanes ? a.dtype.lanes : 1);
}

// header bytes of one array record: magic, reserved, device(8), ndim(4), dtype(4), shape, nbytes
int64_t array_header_bytes(const tk_array_meta& a) { return 8 + 8 + 8 + 4 + 4 + 8 * (int64_t)a.ndim + 8; }

struct Writer {
  uint8_t* p;
  int64_t off = 0, cap;
  bool ok = true;
  void bytes(const void* src, int64_t n) {
    if (off + n > cap) {
      ok = false;
      return;
    }
    if (p) std::memcpy(p + off, src, (size_t)n);
    off += n;
  }
  template <typename T> void pod(T v) { bytes(&v, sizeof(T)); }
};

int64_t align_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

}  // namespace

extern "C" {

int64_t tk_ndlist_layout(const tk_array_meta* arrays, int n, int64_t* data_offsets) {
  if (n < 0 || (n > 0 && !arrays)) {
    tk::set_error("tk_ndlist_layout: invalid argument");
    return TK_ERR_INVALID_ARG;
  }
  int64_t off = 8 + 8 + 8;  // magic, reserved, n_names
  for (int i = 0; i < n; ++i) off += 8 + (int64_t)std::strlen(arrays[i].name ? arrays[i].name : "");
  off += 8;  // n_arrays
  for (int i = 0; i < n; ++i) {
    off += array_header_bytes(arrays[i]);
    if (data_offsets) data_offsets[i] = off;
    off += payload_bytes(arrays[i]);
  }
  return off;
}

int tk_ndlist_write_headers(const tk_array_meta* arrays, int n, void* blob, int64_t blob_size) {
  if (!blob || n < 0 || (n > 0 && !arrays)) {
    tk::set_error("tk_ndlist_write_headers: invalid argument");
    return TK_ERR_INVALID_ARG;
  }
  Writer w{static_cast<uint8_t*>(blob), 0, blob_size};
  w.pod<uint64_t>(kListMagic);
  w.pod<uint64_t>(0);
  w.pod<uint64_t>((uint64_t)n);
  for (int i = 0; i < n; ++i) {
    const char* nm = arrays[i].name ? arrays[i].name : "";
    uint64_t len = std::strlen(nm);
    w.pod<uint64_t>(len);
    w.bytes(nm, (int64_t)len);
  }
  w.pod<uint64_t>((uint64_t)n);
  for (int i = 0; i < n; ++i) {
    const tk_array_meta& a = arrays[i];
    w.pod<uint64_t>(kArrayMagic);
    w.pod<uint64_t>(0);
    w.pod<int32_t>(TK_DEV_CPU);  // SaveDLTensor always records kDLCPU, device 0
    w.pod<int32_t>(0);
    w.pod<int32_t>(a.ndim);
    w.pod<tk_dtype>(a.dtype);
    for (int k = 0; k < a.ndim; ++k) w.pod<int64_t>(a.shape[k]);
    int64_t nb = payload_bytes(a);
    w.pod<int64_t>(nb);
    w.off += nb;  // payload is filled by the caller (device copy or memcpy)
  }
  if (!w.ok || w.off > blob_size) {
    tk::set_error("tk_ndlist_write_headers: blob too small");
    return TK_ERR_INVALID_ARG;
  }
  return TK_OK;
}

int tk_ndlist_parse(const void* blob, int64_t blob_size, int cap, tk_array_meta* arrays, int64_t* data_offsets,
                    int64_t* shapes_storage, int shapes_cap, int* n_out) {
  const uint8_t* p = static_cast<const uint8_t*>(blob);
  int64_t off = 0;
  auto rd = [&](void* dst, int64_t n) -> bool {
    if (off + n > blob_size) return false;
    std::memcpy(dst, p + off, (size_t)n);
    off += n;
    return true;
  };
  uint64_t magic = 0, reserved = 0, nn = 0;
  if (!blob || !n_out || !rd(&magic, 8) || magic != kListMagic || !rd(&reserved, 8) || !rd(&nn, 8)) {
    tk::set_error("tk_ndlist_parse: not an NDArray-list blob");
    return TK_ERR_FORMAT;
  }
  *n_out = (int)nn;
  // names: pointers cannot be NUL-terminated in place, so names are returned as offsets via
  // data_offsets when arrays == NULL; with arrays, name points at the length-prefixed bytes.
  std::vector<std::pair<int64_t, uint64_t>> names;
  for (uint64_t i = 0; i < nn; ++i) {
    uint64_t len = 0;
    if (!rd(&len, 8) || off + (int64_t)len > blob_size) {
      tk::set_error("tk_ndlist_parse: truncated names");
      return TK_ERR_FORMAT;
    }
    names.emplace_back(off, len);
    off += (int64_t)len;
  }
  uint64_t na = 0;
  if (!rd(&na, 8) || na != nn) {
    tk::set_error("tk_ndlist_parse: name/array count mismatch");
    return TK_ERR_FORMAT;
  }
  int shp = 0;
  for (uint64_t i = 0; i < na; ++i) {
    uint64_t am = 0, res = 0;
    int32_t dev_type = 0, dev_id = 0, ndim = 0;
    tk_dtype dt{};
    if (!rd(&am, 8) || am != kArrayMagic || !rd(&res, 8) || !rd(&dev_type, 4) || !rd(&dev_id, 4) || !rd(&ndim, 4) ||
        !rd(&dt, 4) || ndim < 0) {
      tk::set_error("tk_ndlist_parse: bad array header");
      return TK_ERR_FORMAT;
    }
    int64_t* shape = nullptr;
    if (shapes_storage && shp + ndim <= shapes_cap) shape = shapes_storage + shp;
    for (int k = 0; k < ndim; ++k) {
      int64_t d = 0;
      if (!rd(&d, 8)) {
        tk::set_error("tk_ndlist_parse: truncated shape");
        return TK_ERR_FORMAT;
      }
      if (shape) shape[k] = d;
    }
    shp += ndim;
    int64_t nb = 0;
    if (!rd(&nb, 8) || off + nb > blob_size) {
      tk::set_error("tk_ndlist_parse: truncated payload");
      return TK_ERR_FORMAT;
    }
    if ((int)i < cap) {
      if (arrays) {
        arrays[i].name = reinterpret_cast<const char*>(p + names[i].first);
        arrays[i].ndim = ndim;
        arrays[i].shape = shape;
        arrays[i].dtype = dt;
      }
      if (data_offsets) data_offsets[i] = off;
    }
    off += nb;
  }
  return TK_OK;
}

static int64_t trace_offsets(const char* json, const tk_array_meta* params, int n_params,
                             const tk_array_meta* records, int n_records, int64_t* params_off, int64_t* params_size,
                             int64_t* records_off, int64_t* records_size, int64_t* param_offsets,
                             int64_t* record_offsets) {
  int64_t jl = json ? (int64_t)std::strlen(json) : 0;
  int64_t head = (int64_t)sizeof(tk_trace_header) + jl;
  *params_off = align_up(head, TK_TRACE_ALIGN);
  *params_size = tk_ndlist_layout(params, n_params, param_offsets);
  if (*params_size < 0) return *params_size;
  *records_off = align_up(*params_off + *params_size, TK_TRACE_ALIGN);
  *records_size = tk_ndlist_layout(records, n_records, record_offsets);
  if (*records_size < 0) return *records_size;
  if (param_offsets)
    for (int i = 0; i < n_params; ++i) param_offsets[i] += *params_off;
  if (record_offsets)
    for (int i = 0; i < n_records; ++i) record_offsets[i] += *records_off;
  return *records_off + *records_size;
}

int64_t tk_trace_layout(const char* json, const tk_array_meta* params, int n_params, const tk_array_meta* records,
                        int n_records, int64_t* param_offsets, int64_t* record_offsets) {
  int64_t po, ps, ro, rs;
  return trace_offsets(json, params, n_params, records, n_records, &po, &ps, &ro, &rs, param_offsets, record_offsets);
}

int tk_trace_write_headers(const char* json, const tk_array_meta* params, int n_params, const tk_array_meta* records,
                           int n_records, void* image, int64_t image_size) {
  if (!image) {
    tk::set_error("tk_trace_write_headers: null image");
    return TK_ERR_INVALID_ARG;
  }
  int64_t po, ps, ro, rs;
  int64_t total = trace_offsets(json, params, n_params, records, n_records, &po, &ps, &ro, &rs, nullptr, nullptr);
  if (total < 0) return (int)total;
  if (total > image_size) {
    tk::set_error("tk_trace_write_headers: image too small");
    return TK_ERR_INVALID_ARG;
  }
  uint8_t* p = static_cast<uint8_t*>(image);
  tk_trace_header h{};
  h.magic = TK_TRACE_MAGIC;
  h.version = TK_TRACE_VERSION;
  h.json_len = json ? std::strlen(json) : 0;
  h.params_off = (uint64_t)po;
  h.params_size = (uint64_t)ps;
  h.records_off = (uint64_t)ro;
  h.records_size = (uint64_t)rs;
  std::memcpy(p, &h, sizeof(h));
  if (h.json_len) std::memcpy(p + sizeof(h), json, h.json_len);
  int64_t pad0 = (int64_t)sizeof(h) + (int64_t)h.json_len;
  std::memset(p + pad0, 0, (size_t)(po - pad0));
  int rc = tk_ndlist_write_headers(params, n_params, p + po, ps);
  if (rc) return rc;
  std::memset(p + po + ps, 0, (size_t)(ro - po - ps));
  return tk_ndlist_write_headers(records, n_records, p + ro, rs);
}

// Writes [p, p + size) at file offset `base` of fd with `threads` workers, each taking every
// threads-th `chunk`-byte piece (pwrite; chunk-aligned offsets, so O_DIRECT stays aligned).
static int write_range(int fd, const uint8_t* p, int64_t base, int64_t size, int64_t chunk, int threads) {
  std::atomic<int> err{0};
  const int64_t pieces = (size + chunk - 1) / chunk;
  auto worker = [&](int t) {
    for (int64_t k = t; k < pieces && !err.load(); k += threads) {
      int64_t done = k * chunk;
      const int64_t hi = std::min<int64_t>(size, done + chunk);
      while (done < hi && !err.load()) {
        ssize_t w = ::pwrite(fd, p + done, (size_t)(hi - done), (off_t)(base + done));
        if (w < 0) {
          if (errno == EINTR) continue;
          err.store(errno);
          return;
        }
        done += w;
      }
    }
  };
  const int n = (int)std::max<int64_t>(1, std::min<int64_t>(threads, pieces));
  std::vector<std::thread> pool;
  for (int t = 1; t < n; ++t) pool.emplace_back(worker, t);
  worker(0);
  for (auto& th : pool) th.join();
  return err.load();
}

// A shard image is GBs, produced into pinned memory at the PCIe rate: it is written with O_DIRECT
// (no page-cache copy on the writer's cores, no dirty-page writeback storm later) in 256 MiB
// pieces by 2 threads -- every piece 4 KiB aligned in memory, on disk and in length -- and the
// unaligned tail (< 4 KiB) through the page cache.  Written while the next step's D2H copies land
// in the other image, 2 x 256 MiB wrote 14.1 GB/s against 10.1 for 4 x 64 MiB (the round-3 shape)
// on the same box (profiles/r04j_file_sink_writer_sweep.txt); alone both write ~14.5-15.  Filesystems without O_DIRECT (tmpfs) and
// unaligned images take buffered pwrites of 256 MiB pieces from up to 8 threads.
int tk_write_file(const char* path, const void* image, int64_t size) {
  if (!path || (!image && size) || size < 0) {
    tk::set_error("tk_write_file: invalid argument");
    return TK_ERR_INVALID_ARG;
  }
  const uint8_t* p = static_cast<const uint8_t*>(image);
  // the writer's shape can be overridden for sink experiments: TK_WRITE_THREADS (direct writers,
  // default 2), TK_WRITE_PIECE_MB (direct piece, default 256), TK_WRITE_BUFFERED=1 (no O_DIRECT)
  auto env = [](const char* k, int64_t d) {
    const char* v = std::getenv(k);
    return v && *v ? (int64_t)std::atoll(v) : d;
  };
  const int direct_threads = (int)std::max<int64_t>(1, std::min<int64_t>(64, env("TK_WRITE_THREADS", 2)));
  const int64_t kDirectChunk = std::max<int64_t>(1, env("TK_WRITE_PIECE_MB", 256)) << 20;
  constexpr int64_t kAlign = 4096, kBufChunk = (int64_t)256 << 20;
  const int64_t aligned = size / kAlign * kAlign;
  int e = 0;
  int fd = -1;
  bool direct = false;
  if (!env("TK_WRITE_BUFFERED", 0) && aligned >= kDirectChunk && ((uintptr_t)p % kAlign) == 0) {
    fd = ::open(path, O_WRONLY | O_CREAT | O_TRUNC | O_DIRECT, 0644);
    direct = fd >= 0;
  }
  if (fd < 0) fd = ::open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) {
    tk::set_error(std::string("tk_write_file: open failed: ") + std::strerror(errno));
    return TK_ERR_IO;
  }
  if (size > 0 && ::ftruncate(fd, (off_t)size) != 0) e = errno;
  if (!e && direct) {
    e = write_range(fd, p, 0, aligned, kDirectChunk, direct_threads);
    if (e == EINVAL) {  // the filesystem refused direct I/O after all: everything buffered
      ::close(fd);
      direct = false;
      fd = ::open(path, O_WRONLY, 0644);
      e = fd < 0 ? errno : 0;
    }
  }
  if (!e && direct && aligned < size) {
    const int fd2 = ::open(path, O_WRONLY, 0644);
    if (fd2 < 0) {
      e = errno;
    } else {
      e = write_range(fd2, p + aligned, aligned, size - aligned, kBufChunk, 1);
      if (::close(fd2) != 0 && !e) e = errno;
    }
  }
  if (!e && !direct) e = write_range(fd, p, 0, size, kBufChunk, 8);
  if (fd >= 0 && ::close(fd) != 0 && !e) {
    tk::set_error(std::string("tk_write_file: close failed: ") + std::strerror(errno));
    return TK_ERR_IO;
  }
  if (e) {
    tk::set_error(std::string("tk_write_file: write failed: ") + std::strerror(e));
    return TK_ERR_IO;
  }
  return TK_OK;
}

}  // extern "C"
