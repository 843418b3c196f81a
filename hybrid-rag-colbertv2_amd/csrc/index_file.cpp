// index_file.cpp — the native on-disk index: one flat file per
// corpus (or per shard), read straight into HBM by any contiguous doc range.
//
// The reference persists its index with torch.save({'embeddings', 'corpus'},
// indexes/colbert/index.pt) and torch.load(map_location=device) (LRC:743-746,
// 751); that stays supported in Python (retriever.py).  At 1M docs x 32 KiB a
// pickle is neither shardable nor streamable, so the native format is:
//
//   [0, 4096)          header (cbv2_file_header below, little-endian)
//   doclens_off        int32 [n]
//   tokens_off         [n][ld][d] bf16 (2 B) or e4m3 (1 B)         4 KiB-aligned
//   scales_off         [n][ld][2] E8M0 bytes (MXFP8 only)            4 KiB-aligned
//
// ld = 128 token slots per doc, or 256 / 512 / 1024 for long documents (the
// layouts the kernels scan).
//
// A rank loads docs [begin, end) of the file: three contiguous byte ranges.
// Reads go through two pinned staging buffers: a reader thread fills one with
// pread (O_DIRECT for the 4 KiB-aligned token range, so a cold load is not
// throttled by the page cache) while the other is copied to HBM by
// hipMemcpyAsync on the caller's stream.  Writes mirror it (D2H + pwrite).
// The _host variants take host pointers and never touch the GPU (tests, tools).
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <thread>

#include "colbert_mi355x.h"

extern "C" int cbv2_set_error(int code, const char* msg);

namespace {
constexpr char kMagic[8] = {'C', 'B', 'V', '2', 'I', 'D', 'X', '1'};
constexpr uint64_t kAlign = 4096;
constexpr size_t kStage = 64ull << 20;  // bytes per staging buffer

struct cbv2_file_header {
  char magic[8];
  uint32_t version;    // 1
  int32_t dtype;       // CBV2_DTYPE_BF16 or CBV2_DTYPE_MXFP8
  int64_t n;           // docs in the file
  int32_t ld, d;       // token slots per doc (128, or 256 / 512 / 1024), 128
  int64_t id_base;     // global id of the file's doc 0
  uint64_t doclens_off, tokens_off, scales_off;  // scales_off 0 for bf16
  uint64_t file_bytes;
  uint8_t reserved[4096 - 8 - 4 - 4 - 8 - 8 - 8 - 8 * 4];
};
static_assert(sizeof(cbv2_file_header) == 4096, "header is one page");

int err(int code, const char* fmt, ...) {
  char buf[384];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  return cbv2_set_error(code, buf);
}

uint64_t up(uint64_t x) { return (x + kAlign - 1) & ~(kAlign - 1); }
size_t tok_bytes(int32_t dtype) { return dtype == CBV2_DTYPE_MXFP8 ? 1 : 2; }
// bytes of one doc's tokens / scales
size_t doc_bytes(const cbv2_file_header& h) { return (size_t)h.ld * 128 * tok_bytes(h.dtype); }
size_t scale_bytes(const cbv2_file_header& h) { return h.scales_off ? (size_t)h.ld * 2 : 0; }

int layout(int32_t dtype, int64_t n, int32_t ld, int64_t id_base, cbv2_file_header& h) {
  if (dtype != CBV2_DTYPE_BF16 && dtype != CBV2_DTYPE_MXFP8) return err(CBV2_EINVAL, "dtype %d not storable", dtype);
  if (n < 0 || id_base < 0) return err(CBV2_EINVAL, "bad n / id_base");
  if (ld != 128 && ld != 256 && ld != 512 && ld != 1024)
    return err(CBV2_EINVAL, "ld %d not storable (128, 256, 512 or 1024)", ld);
  memset(&h, 0, sizeof(h));
  memcpy(h.magic, kMagic, 8);
  h.version = 1;
  h.dtype = dtype;
  h.n = n;
  h.ld = ld;
  h.d = 128;
  h.id_base = id_base;
  h.doclens_off = kAlign;
  h.tokens_off = up(h.doclens_off + 4ull * n);
  const uint64_t tok_end = h.tokens_off + (uint64_t)n * doc_bytes(h);
  h.scales_off = dtype == CBV2_DTYPE_MXFP8 ? up(tok_end) : 0;
  h.file_bytes = dtype == CBV2_DTYPE_MXFP8 ? h.scales_off + (uint64_t)n * scale_bytes(h) : tok_end;
  return CBV2_OK;
}

int read_header(int fd, const char* path, cbv2_file_header& h) {
  if (pread(fd, &h, sizeof(h), 0) != (ssize_t)sizeof(h)) return err(CBV2_EINVAL, "%s: short header", path);
  if (memcmp(h.magic, kMagic, 8) != 0 || h.version != 1) return err(CBV2_EINVAL, "%s: not a cbv2 index file", path);
  cbv2_file_header want;
  if (layout(h.dtype, h.n, h.ld, h.id_base, want) != CBV2_OK || want.tokens_off != h.tokens_off ||
      want.scales_off != h.scales_off || h.d != 128)
    return err(CBV2_EINVAL, "%s: inconsistent header", path);
  struct stat st;
  if (fstat(fd, &st) != 0 || (uint64_t)st.st_size < h.file_bytes) return err(CBV2_EINVAL, "%s: truncated", path);
  return CBV2_OK;
}

int pread_full(int fd, void* dst, size_t bytes, uint64_t off) {
  uint8_t* p = (uint8_t*)dst;
  while (bytes) {
    const ssize_t r = pread(fd, p, bytes, (off_t)off);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return -1;
    p += r;
    off += (uint64_t)r;
    bytes -= (size_t)r;
  }
  return 0;
}

int pwrite_full(int fd, const void* src, size_t bytes, uint64_t off) {
  const uint8_t* p = (const uint8_t*)src;
  while (bytes) {
    const ssize_t r = pwrite(fd, p, bytes, (off_t)off);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return -1;
    p += r;
    off += (uint64_t)r;
    bytes -= (size_t)r;
  }
  return 0;
}

struct Fd {
  int fd = -1;
  ~Fd() {
    if (fd >= 0) close(fd);
  }
};

// Stream one byte range of the file into device memory through two pinned
// buffers: the reader thread preads chunk i+1 while chunk i is copied H2D.
int range_to_device(const char* path, int fd_buffered, int fd_direct, uint64_t off, size_t bytes, uint8_t* dst,
                    uint8_t* stage[2], hipStream_t st) {
  if (bytes == 0) return CBV2_OK;
  const size_t nchunks = (bytes + kStage - 1) / kStage;
  hipEvent_t done[2];
  if (hipEventCreateWithFlags(&done[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&done[1], hipEventDisableTiming) != hipSuccess)
    return err(CBV2_EHIP, "hipEventCreate failed");
  int rc = CBV2_OK;
  bool pending[2] = {false, false};
  int read_rc = 0;
  auto read_chunk = [&](size_t i, int b) {
    const size_t len = (i + 1 == nchunks) ? bytes - i * kStage : kStage;
    const uint64_t o = off + i * kStage;
    // O_DIRECT needs offset, length and buffer aligned to the block size
    if (fd_direct >= 0 && (o % kAlign) == 0 && (len % kAlign) == 0 && pread_full(fd_direct, stage[b], len, o) == 0)
      return;
    read_rc |= pread_full(fd_buffered, stage[b], len, o);  // unaligned, or O_DIRECT refused by the filesystem
  };
  std::thread reader;
  for (size_t i = 0; i < nchunks && rc == CBV2_OK; ++i) {
    const int b = (int)(i & 1);
    if (i == 0) read_chunk(0, 0);
    if (reader.joinable()) reader.join();
    if (read_rc) {
      rc = err(CBV2_EINVAL, "%s: read failed at chunk %zu", path, i);
      break;
    }
    // prefetch chunk i+1 into the other buffer once its previous copy is done
    if (i + 1 < nchunks) {
      if (pending[b ^ 1] && hipEventSynchronize(done[b ^ 1]) != hipSuccess) {
        rc = err(CBV2_EHIP, "hipEventSynchronize failed");
        break;
      }
      pending[b ^ 1] = false;
      reader = std::thread(read_chunk, i + 1, b ^ 1);
    }
    const size_t len = (i + 1 == nchunks) ? bytes - i * kStage : kStage;
    if (hipMemcpyAsync(dst + i * kStage, stage[b], len, hipMemcpyHostToDevice, st) != hipSuccess ||
        hipEventRecord(done[b], st) != hipSuccess) {
      rc = err(CBV2_EHIP, "hipMemcpyAsync H2D failed");
      break;
    }
    pending[b] = true;
  }
  if (reader.joinable()) reader.join();
  if (rc == CBV2_OK && read_rc) rc = err(CBV2_EINVAL, "%s: read failed", path);
  for (int b = 0; b < 2; ++b)
    if (pending[b]) (void)hipEventSynchronize(done[b]);
  (void)hipEventDestroy(done[0]);
  (void)hipEventDestroy(done[1]);
  return rc;
}

// Device -> file for one range: copy chunk i+1 D2H while chunk i is written.
int range_from_device(const char* path, int fd, uint64_t off, size_t bytes, const uint8_t* src, uint8_t* stage[2],
                      hipStream_t st) {
  if (bytes == 0) return CBV2_OK;
  const size_t nchunks = (bytes + kStage - 1) / kStage;
  hipEvent_t done[2];
  if (hipEventCreateWithFlags(&done[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&done[1], hipEventDisableTiming) != hipSuccess)
    return err(CBV2_EHIP, "hipEventCreate failed");
  int rc = CBV2_OK;
  auto copy = [&](size_t i) -> int {
    const size_t len = (i + 1 == nchunks) ? bytes - i * kStage : kStage;
    if (hipMemcpyAsync(stage[i & 1], src + i * kStage, len, hipMemcpyDeviceToHost, st) != hipSuccess ||
        hipEventRecord(done[i & 1], st) != hipSuccess)
      return err(CBV2_EHIP, "hipMemcpyAsync D2H failed");
    return CBV2_OK;
  };
  rc = copy(0);
  for (size_t i = 0; i < nchunks && rc == CBV2_OK; ++i) {
    if (hipEventSynchronize(done[i & 1]) != hipSuccess) {
      rc = err(CBV2_EHIP, "hipEventSynchronize failed");
      break;
    }
    if (i + 1 < nchunks && (rc = copy(i + 1)) != CBV2_OK) break;
    const size_t len = (i + 1 == nchunks) ? bytes - i * kStage : kStage;
    if (pwrite_full(fd, stage[i & 1], len, off + i * kStage)) rc = err(CBV2_EINVAL, "%s: write failed", path);
  }
  (void)hipStreamSynchronize(st);
  (void)hipEventDestroy(done[0]);
  (void)hipEventDestroy(done[1]);
  return rc;
}

struct Pinned {
  uint8_t* p[2] = {nullptr, nullptr};
  int alloc() {
    for (int b = 0; b < 2; ++b)
      if (hipHostMalloc((void**)&p[b], kStage, hipHostMallocDefault) != hipSuccess)
        return err(CBV2_EHIP, "hipHostMalloc(%zu) failed", kStage);
    return CBV2_OK;
  }
  ~Pinned() {
    for (int b = 0; b < 2; ++b)
      if (p[b]) (void)hipHostFree(p[b]);
  }
};

int check_range(const cbv2_file_header& h, int64_t begin, int64_t end) {
  if (begin < 0 || end < begin || end > h.n)
    return err(CBV2_EINVAL, "doc range [%lld, %lld) outside [0, %lld)", (long long)begin, (long long)end,
               (long long)h.n);
  return CBV2_OK;
}
}  // namespace

extern "C" {

int cbv2_index_file_info(const char* path, int32_t* dtype, int64_t* n, int64_t* id_base) {
  return cbv2_index_file_info_ld(path, dtype, n, id_base, nullptr);
}

int cbv2_index_file_info_ld(const char* path, int32_t* dtype, int64_t* n, int64_t* id_base, int32_t* ld) {
  if (!path) return err(CBV2_EINVAL, "null path");
  Fd f;
  f.fd = open(path, O_RDONLY);
  if (f.fd < 0) return err(CBV2_EINVAL, "%s: cannot open (%s)", path, strerror(errno));
  cbv2_file_header h;
  if (int rc = read_header(f.fd, path, h)) return rc;
  if (dtype) *dtype = h.dtype;
  if (n) *n = h.n;
  if (id_base) *id_base = h.id_base;
  if (ld) *ld = h.ld;
  return CBV2_OK;
}

int cbv2_index_file_write_host(const char* path, int32_t dtype, int64_t n, const void* tokens, const void* scales,
                               const int32_t* doclens, int64_t id_base) {
  return cbv2_index_file_write_host_ld(path, dtype, n, 128, tokens, scales, doclens, id_base);
}

int cbv2_index_file_write_host_ld(const char* path, int32_t dtype, int64_t n, int32_t ld, const void* tokens,
                                  const void* scales, const int32_t* doclens, int64_t id_base) {
  cbv2_file_header h;
  if (int rc = layout(dtype, n, ld, id_base, h)) return rc;
  if (!path || (n > 0 && (!tokens || !doclens || (dtype == CBV2_DTYPE_MXFP8 && !scales))))
    return err(CBV2_EINVAL, "null pointer");
  Fd f;
  f.fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (f.fd < 0) return err(CBV2_EINVAL, "%s: cannot create (%s)", path, strerror(errno));
  if (pwrite_full(f.fd, &h, sizeof(h), 0) || (n && pwrite_full(f.fd, doclens, 4ull * n, h.doclens_off)) ||
      (n && pwrite_full(f.fd, tokens, (size_t)n * doc_bytes(h), h.tokens_off)) ||
      (n && h.scales_off && pwrite_full(f.fd, scales, (size_t)n * scale_bytes(h), h.scales_off)) ||
      ftruncate(f.fd, (off_t)h.file_bytes) != 0)
    return err(CBV2_EINVAL, "%s: write failed (%s)", path, strerror(errno));
  return CBV2_OK;
}

int cbv2_index_file_read_host(const char* path, int64_t begin, int64_t end, void* tokens, void* scales,
                              int32_t* doclens) {
  if (!path) return err(CBV2_EINVAL, "null path");
  Fd f;
  f.fd = open(path, O_RDONLY);
  if (f.fd < 0) return err(CBV2_EINVAL, "%s: cannot open (%s)", path, strerror(errno));
  cbv2_file_header h;
  if (int rc = read_header(f.fd, path, h)) return rc;
  if (int rc = check_range(h, begin, end)) return rc;
  const int64_t m = end - begin;
  if (m == 0) return CBV2_OK;
  if (!tokens || !doclens || (h.scales_off && !scales)) return err(CBV2_EINVAL, "null output");
  const size_t per = doc_bytes(h), sper = scale_bytes(h);
  if (pread_full(f.fd, doclens, 4ull * m, h.doclens_off + 4ull * begin) ||
      pread_full(f.fd, tokens, per * m, h.tokens_off + per * begin) ||
      (h.scales_off && pread_full(f.fd, scales, sper * m, h.scales_off + sper * begin)))
    return err(CBV2_EINVAL, "%s: read failed", path);
  return CBV2_OK;
}

int cbv2_index_file_write(const char* path, int32_t dtype, int64_t n, const void* tokens, const void* scales,
                          const int32_t* doclens, int64_t id_base, void* stream) {
  return cbv2_index_file_write_ld(path, dtype, n, 128, tokens, scales, doclens, id_base, stream);
}

int cbv2_index_file_write_ld(const char* path, int32_t dtype, int64_t n, int32_t ld, const void* tokens,
                             const void* scales, const int32_t* doclens, int64_t id_base, void* stream) {
  cbv2_file_header h;
  if (int rc = layout(dtype, n, ld, id_base, h)) return rc;
  if (!path || (n > 0 && (!tokens || !doclens || (dtype == CBV2_DTYPE_MXFP8 && !scales))))
    return err(CBV2_EINVAL, "null pointer");
  Fd f;
  f.fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (f.fd < 0) return err(CBV2_EINVAL, "%s: cannot create (%s)", path, strerror(errno));
  if (pwrite_full(f.fd, &h, sizeof(h), 0)) return err(CBV2_EINVAL, "%s: write failed", path);
  Pinned pin;
  if (int rc = pin.alloc()) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (int rc = range_from_device(path, f.fd, h.doclens_off, 4ull * n, (const uint8_t*)doclens, pin.p, st)) return rc;
  if (int rc = range_from_device(path, f.fd, h.tokens_off, (size_t)n * doc_bytes(h), (const uint8_t*)tokens, pin.p,
                                 st))
    return rc;
  if (h.scales_off)
    if (int rc = range_from_device(path, f.fd, h.scales_off, (size_t)n * scale_bytes(h), (const uint8_t*)scales,
                                   pin.p, st))
      return rc;
  if (ftruncate(f.fd, (off_t)h.file_bytes) != 0) return err(CBV2_EINVAL, "%s: truncate failed", path);
  return CBV2_OK;
}

int cbv2_index_file_read(const char* path, int64_t begin, int64_t end, void* tokens, void* scales, int32_t* doclens,
                         void* stream) {
  if (!path) return err(CBV2_EINVAL, "null path");
  Fd f, fdir;
  f.fd = open(path, O_RDONLY);
  if (f.fd < 0) return err(CBV2_EINVAL, "%s: cannot open (%s)", path, strerror(errno));
  fdir.fd = open(path, O_RDONLY | O_DIRECT);  // optional: falls back to buffered reads
  cbv2_file_header h;
  if (int rc = read_header(f.fd, path, h)) return rc;
  if (int rc = check_range(h, begin, end)) return rc;
  const int64_t m = end - begin;
  if (m == 0) return CBV2_OK;
  if (!tokens || !doclens || (h.scales_off && !scales)) return err(CBV2_EINVAL, "null output");
  Pinned pin;
  if (int rc = pin.alloc()) return rc;
  hipStream_t st = (hipStream_t)stream;
  const size_t per = doc_bytes(h), sper = scale_bytes(h);
  if (int rc = range_to_device(path, f.fd, -1, h.doclens_off + 4ull * begin, 4ull * m, (uint8_t*)doclens, pin.p, st))
    return rc;
  if (int rc = range_to_device(path, f.fd, fdir.fd, h.tokens_off + per * begin, per * m, (uint8_t*)tokens, pin.p, st))
    return rc;
  if (h.scales_off)
    if (int rc = range_to_device(path, f.fd, -1, h.scales_off + sper * begin, sper * m, (uint8_t*)scales, pin.p,
                                 st))
      return rc;
  return CBV2_OK;
}

// ---------------------------------------------------------------------------
// Streaming writer (bounded-memory ingest): the header is written last, by
// close(), once every doc of the declared count has been appended, so a file
// whose ingest stopped early never reads as valid.
// ---------------------------------------------------------------------------
struct cbv2_index_writer {
  cbv2_file_header h;
  int fd = -1;
  int64_t written = 0;
  Pinned pin;
  bool pinned = false;
  char path[1024];
};

int cbv2_index_writer_open(const char* path, int32_t dtype, int64_t n, int64_t id_base, cbv2_index_writer** out) {
  return cbv2_index_writer_open_ld(path, dtype, n, 128, id_base, out);
}

int cbv2_index_writer_open_ld(const char* path, int32_t dtype, int64_t n, int32_t ld, int64_t id_base,
                              cbv2_index_writer** out) {
  if (!out) return err(CBV2_EINVAL, "null output handle pointer");
  *out = nullptr;
  if (!path || strlen(path) >= 1024) return err(CBV2_EINVAL, "bad path");
  auto* w = new cbv2_index_writer;
  if (int rc = layout(dtype, n, ld, id_base, w->h)) {
    delete w;
    return rc;
  }
  snprintf(w->path, sizeof(w->path), "%s", path);
  w->fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (w->fd < 0) {
    const int e = errno;
    delete w;
    return err(CBV2_EINVAL, "%s: cannot create (%s)", path, strerror(e));
  }
  cbv2_file_header blank;
  memset(&blank, 0, sizeof(blank));  // not a valid header until close()
  if (pwrite_full(w->fd, &blank, sizeof(blank), 0) || ftruncate(w->fd, (off_t)w->h.file_bytes) != 0) {
    close(w->fd);
    delete w;
    return err(CBV2_EINVAL, "%s: cannot size the file", path);
  }
  *out = w;
  return CBV2_OK;
}

int cbv2_index_writer_append(cbv2_index_writer* w, int64_t count, const void* tokens, const void* scales,
                             const int32_t* doclens, int32_t on_device, void* stream) {
  if (!w || w->fd < 0) return err(CBV2_EINVAL, "null or closed writer");
  if (count < 0 || w->written + count > w->h.n)
    return err(CBV2_EINVAL, "append of %lld docs past the declared %lld (written %lld)", (long long)count,
               (long long)w->h.n, (long long)w->written);
  if (count == 0) return CBV2_OK;
  const bool fp8 = w->h.scales_off != 0;
  if (!tokens || !doclens || (fp8 && !scales)) return err(CBV2_EINVAL, "null pointer");
  const size_t per = doc_bytes(w->h), sper = scale_bytes(w->h);
  const uint64_t d0 = (uint64_t)w->written;
  if (on_device) {
    if (!w->pinned) {
      if (int rc = w->pin.alloc()) return rc;
      w->pinned = true;
    }
    hipStream_t st = (hipStream_t)stream;
    if (int rc = range_from_device(w->path, w->fd, w->h.doclens_off + 4 * d0, 4ull * count, (const uint8_t*)doclens,
                                   w->pin.p, st))
      return rc;
    if (int rc = range_from_device(w->path, w->fd, w->h.tokens_off + per * d0, per * count, (const uint8_t*)tokens,
                                   w->pin.p, st))
      return rc;
    if (fp8)
      if (int rc = range_from_device(w->path, w->fd, w->h.scales_off + sper * d0, sper * count,
                                     (const uint8_t*)scales, w->pin.p, st))
        return rc;
  } else if (pwrite_full(w->fd, doclens, 4ull * count, w->h.doclens_off + 4 * d0) ||
             pwrite_full(w->fd, tokens, per * count, w->h.tokens_off + per * d0) ||
             (fp8 && pwrite_full(w->fd, scales, sper * count, w->h.scales_off + sper * d0))) {
    return err(CBV2_EINVAL, "%s: write failed (%s)", w->path, strerror(errno));
  }
  w->written += count;
  return CBV2_OK;
}

int64_t cbv2_index_writer_count(const cbv2_index_writer* w) { return w ? w->written : -1; }

int cbv2_index_writer_close(cbv2_index_writer* w) {
  if (!w) return CBV2_OK;
  int rc = CBV2_OK;
  if (w->fd >= 0) {
    if (w->written != w->h.n)
      rc = err(CBV2_EINVAL, "%s: closed after %lld of %lld docs (partial file removed)", w->path,
               (long long)w->written, (long long)w->h.n);
    else if (pwrite_full(w->fd, &w->h, sizeof(w->h), 0) || fsync(w->fd) != 0)
      rc = err(CBV2_EINVAL, "%s: header write failed (file removed)", w->path);
    close(w->fd);
    if (rc != CBV2_OK) unlink(w->path);  // never leave a full-size file without a valid header behind
  }
  delete w;
  return rc;
}

}  // extern "C"
