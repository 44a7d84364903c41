// dq_ingest.cpp -- host-resident Arrow batches into HBM for dq_scan, without a JVM.
//
// Reference seam: AnalysisRunner.runScanningAnalyzers hands Spark's DataFrame to data.agg(...)
// (analyzers/runners/AnalysisRunner.scala:279-326); a drop-in shim receives the columns as Arrow record
// batches (Spark's ArrowColumnVector / toArrow export, pyarrow, arrow-rs all speak the Arrow C Data
// Interface).  dq_arrow_import maps one exported ArrowArray / ArrowSchema to the host buffers of a
// dq column; dq_upload moves a chunk of such columns into device memory through pinned staging
// buffers, double- (n-) buffered so the copy of chunk k + 1 overlaps the scan of chunk k:
//
//     host Arrow buffers --(CPU threads, memcpy)--> pinned slot s --(DMA, copy stream)--> device slot s
//     scan stream: waits for the slot's copy (dq_upload_fence), scans, then frees the slot (dq_upload_release)
//
// The CPU copy into pinned memory is what lets the DMA engine stream at full PCIe rate from pageable
// Arrow memory; a slot is reused only after the scan that read it has passed its release event.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/dqscan.h"
#include "dq_internal.h"

using dq::set_error;

namespace {

constexpr int64_t kAlign = 256;  // every buffer of a slot starts 256-byte aligned (values need 16)

int64_t align_up(int64_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

int32_t type_of_format(const char* f) {
  if (!f) return 0;
  if (std::strcmp(f, "g") == 0) return DQ_TYPE_F64;
  if (std::strcmp(f, "l") == 0) return DQ_TYPE_I64;
  if (std::strcmp(f, "i") == 0) return DQ_TYPE_I32;
  if (std::strcmp(f, "u") == 0) return DQ_TYPE_UTF8;
  if (std::strcmp(f, "U") == 0) return DQ_TYPE_LARGE_UTF8;
  if (std::strcmp(f, "f") == 0) return DQ_TYPE_F32;
  if (std::strcmp(f, "s") == 0) return DQ_TYPE_I16;
  if (std::strcmp(f, "c") == 0) return DQ_TYPE_I8;
  if (std::strcmp(f, "b") == 0) return DQ_TYPE_BOOL;
  if (std::strcmp(f, "tdD") == 0) return DQ_TYPE_DATE32;
  // timestamp[us, tz]: Spark's TimestampType is UTC microseconds whatever the session zone (other units are not
  // TimestampType values: a producer converts them)
  if (std::strncmp(f, "tsu:", 4) == 0) return DQ_TYPE_TIMESTAMP;
  // decimal128 "d:precision,scale[,128]" (Spark's DecimalType(p, s); no negative scales, no 256-bit width)
  if (f[0] == 'd' && f[1] == ':') {
    int p = -1, sc = -1, w = 128, n = 0;
    const int k = std::sscanf(f + 2, "%d,%d%n", &p, &sc, &n);
    if (k != 2) return 0;
    const char* rest = f + 2 + n;
    if (*rest == ',') {
      if (std::sscanf(rest + 1, "%d", &w) != 1) return 0;
    } else if (*rest != '\0') {
      return 0;
    }
    if (w != 128 || p < 1 || p > dq::kDecMaxPrecision || sc < 0 || sc > p) return 0;
    return DQ_DECIMAL128(p, sc);
  }
  return 0;
}

// bytes per value of a fixed-width type (BOOL: bit-packed, 0)
int64_t value_width(int32_t type) {
  switch (type) {
    case DQ_TYPE_F64: case DQ_TYPE_I64: case DQ_TYPE_TIMESTAMP: return 8;
    case DQ_TYPE_I32: case DQ_TYPE_F32: case DQ_TYPE_DATE32: return 4;
    case DQ_TYPE_I16: return 2;
    case DQ_TYPE_I8: return 1;
    default: return dq::is_decimal(type) ? 16 : 0;
  }
}

// parallel copy of a list of pieces over up to `threads` CPU threads.  A piece is a memcpy, or -- for an
// Arrow slice -- a rebase of its string offsets (minus the slice's first offset) or a shift of its
// validity bitmap (the slice's row 0 at bit `shift` of the first source byte).
struct Piece {
  char* dst;
  const char* src;
  int64_t bytes;           // destination bytes
  int kind = 0;            // 0 memcpy, 1 int32 offsets - base, 2 int64 offsets - base, 3 bitmap >> shift
  int64_t base = 0;        // kinds 1, 2
  int shift = 0;           // kind 3 (1..7)
  int64_t src_bytes = 0;   // kind 3: readable source bytes
};

void copy_part(const Piece& p, int64_t a, int64_t b) {  // destination bytes [a, b) of piece p
  switch (p.kind) {
    case 0: std::memcpy(p.dst + a, p.src + a, (size_t)(b - a)); break;
    case 1: {
      const int32_t base = (int32_t)p.base;
      for (int64_t i = a / 4; i < b / 4; ++i) {
        int32_t v;
        std::memcpy(&v, p.src + 4 * i, 4);
        v -= base;
        std::memcpy(p.dst + 4 * i, &v, 4);
      }
      break;
    }
    case 2:
      for (int64_t i = a / 8; i < b / 8; ++i) {
        int64_t v;
        std::memcpy(&v, p.src + 8 * i, 8);
        v -= p.base;
        std::memcpy(p.dst + 8 * i, &v, 8);
      }
      break;
    default: {
      const uint8_t* src = reinterpret_cast<const uint8_t*>(p.src);
      for (int64_t i = a; i < b; ++i) {
        const uint32_t lo = src[i], hi = i + 1 < p.src_bytes ? src[i + 1] : 0u;
        p.dst[i] = (char)(uint8_t)((lo >> p.shift) | (hi << (8 - p.shift)));
      }
    }
  }
}

void parallel_copy(const std::vector<Piece>& pieces, int threads) {
  int64_t total = 0;
  for (const Piece& p : pieces) total += p.bytes;
  constexpr int64_t kGrain = 8 << 20;
  const int n = (int)std::max<int64_t>(1, std::min<int64_t>(threads, total / kGrain));
  if (n <= 1) {
    for (const Piece& p : pieces)
      if (p.bytes) copy_part(p, 0, p.bytes);
    return;
  }
  // split the concatenated byte range [0, total) into n contiguous shares; inside a piece the share
  // boundaries are rounded down to 8 bytes (whole offsets), the same way on both sides of a boundary
  auto work = [&](int t) {
    const int64_t lo = total * t / n, hi = total * (t + 1) / n;
    int64_t at = 0;
    for (const Piece& p : pieces) {
      if (at + p.bytes > lo && at < hi) {
        const int64_t a = lo <= at ? 0 : ((lo - at) & ~int64_t(7));
        const int64_t b = hi >= at + p.bytes ? p.bytes : ((hi - at) & ~int64_t(7));
        if (a < b) copy_part(p, a, b);
      }
      at += p.bytes;
      if (at >= hi) break;
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < n; ++t) pool.emplace_back(work, t);
  work(0);
  for (std::thread& th : pool) th.join();
}

}  // namespace

struct dq_uploader {
  int device = 0;
  int threads = 8;
  int64_t slot_bytes = 0;
  std::vector<char*> pinned, dev;
  std::vector<hipEvent_t> copied, released;
  std::vector<bool> used;
  hipStream_t copy = nullptr;
  int64_t next = 0;  // chunks uploaded
  double host_ms = 0.0;
  int64_t bytes = 0;
};

extern "C" {

dq_status dq_arrow_import(const struct ArrowSchema* schema, const struct ArrowArray* array, dq_host_column* out) {
  if (!schema || !array || !out) return set_error(DQ_E_INVALID, "dq_arrow_import: bad argument");
  if (!schema->release || !array->release) return set_error(DQ_E_INVALID, "dq_arrow_import: released Arrow structure");
  const int32_t type = type_of_format(schema->format);
  if (!type)
    return set_error(DQ_E_UNSUPPORTED, "Arrow format '%s' is not a GPU column type (g, f, l, i, s, c, b, tdD, tsu:, d:p,s, u, U)",
                     schema->format ? schema->format : "(null)");
  if (schema->n_children != 0 || array->n_children != 0 || schema->dictionary || array->dictionary)
    return set_error(DQ_E_UNSUPPORTED, "nested / dictionary-encoded Arrow arrays are not GPU columns");
  const bool str = type == DQ_TYPE_UTF8 || type == DQ_TYPE_LARGE_UTF8;
  if (array->n_buffers != (str ? 3 : 2) || !array->buffers)
    return set_error(DQ_E_INVALID, "Arrow array of format '%s' with %lld buffers", schema->format,
                     (long long)array->n_buffers);
  const int64_t n = array->length, off = array->offset;
  if (n < 0 || off < 0) return set_error(DQ_E_INVALID, "Arrow array with negative length / offset");
  dq_host_column c{};
  c.type = type;
  c.n_rows = n;
  if (n == 0) {  // producers may export NULL buffers for an empty array: touch none
    *out = c;
    return DQ_OK;
  }
  const uint8_t* validity = static_cast<const uint8_t*>(array->buffers[0]);
  if (array->null_count == 0) validity = nullptr;  // buffers[0] may be NULL then
  if (array->null_count != 0 && !validity && array->null_count != -1)
    return set_error(DQ_E_INVALID, "Arrow array with %lld nulls and no validity buffer", (long long)array->null_count);
  if (!array->buffers[1]) return set_error(DQ_E_INVALID, "Arrow array of format '%s' without its %s buffer",
                                           schema->format, str ? "offsets" : "values");
  c.nullable = validity ? 1 : 0;
  // a slice (RecordBatch.slice, to_batches(max_chunksize)): row 0 is bit off % 8 of byte off / 8; dq_upload
  // shifts the bitmap into place while it copies (a boolean array's value bits too)
  const bool bits = type == DQ_TYPE_BOOL;
  c.validity = validity ? validity + off / 8 : nullptr;
  c.validity_bytes = validity ? (n + 7) / 8 : 0;
  c.validity_bit = validity || bits ? (int32_t)(off & 7) : 0;
  if (bits) {
    c.values = static_cast<const char*>(array->buffers[1]) + off / 8;
    c.value_bytes = (n + 7) / 8;
    c.offsets = nullptr;
    c.offset_bytes = 0;
  } else if (!str) {
    const int64_t w = value_width(type);
    c.values = static_cast<const char*>(array->buffers[1]) + off * w;
    c.value_bytes = n * w;
    c.offsets = nullptr;
    c.offset_bytes = 0;
  } else {
    const int64_t w = type == DQ_TYPE_UTF8 ? 4 : 8;
    const char* offs = static_cast<const char*>(array->buffers[1]) + off * w;
    int64_t o0, o1;
    if (w == 4) {
      o0 = reinterpret_cast<const int32_t*>(offs)[0];
      o1 = reinterpret_cast<const int32_t*>(offs)[n];
    } else {
      o0 = reinterpret_cast<const int64_t*>(offs)[0];
      o1 = reinterpret_cast<const int64_t*>(offs)[n];
    }
    if (o0 < 0 || o1 < o0) return set_error(DQ_E_INVALID, "Arrow string offsets %lld..%lld", (long long)o0, (long long)o1);
    if (o1 > o0 && !array->buffers[2]) return set_error(DQ_E_INVALID, "Arrow string array without its data buffer");
    // a slice's offsets start at o0: dq_upload copies the bytes from o0 and writes offsets - o0
    c.offsets = offs;
    c.offset_bytes = (n + 1) * w;
    c.offset_base = o0;
    c.values = o1 > o0 ? static_cast<const char*>(array->buffers[2]) + o0 : nullptr;
    c.value_bytes = o1 - o0;
  }
  *out = c;
  return DQ_OK;
}

dq_status dq_uploader_create(int32_t device, int32_t n_slots, int64_t slot_bytes, int32_t host_threads,
                             dq_uploader** out) {
  if (!out || n_slots < 1 || n_slots > 8 || slot_bytes <= 0) return set_error(DQ_E_INVALID, "dq_uploader_create: bad argument");
  dq_uploader* u = new dq_uploader();
  u->device = device;
  u->threads = host_threads > 0 ? host_threads : (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  u->slot_bytes = align_up(slot_bytes);
  auto fail = [&](hipError_t e, const char* what) {
    dq_uploader_destroy(u);
    return set_error(e == hipErrorOutOfMemory ? DQ_E_OOM : DQ_E_HIP, "%s failed: %s", what, hipGetErrorString(e));
  };
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return fail(e, "hipSetDevice");
  if ((e = hipStreamCreateWithFlags(&u->copy, hipStreamNonBlocking)) != hipSuccess) return fail(e, "hipStreamCreate");
  for (int s = 0; s < n_slots; ++s) {
    char* h = nullptr;
    char* d = nullptr;
    hipEvent_t a = nullptr, b = nullptr;
    if ((e = hipHostMalloc(reinterpret_cast<void**>(&h), (size_t)u->slot_bytes, hipHostMallocDefault)) != hipSuccess)
      return fail(e, "hipHostMalloc");
    u->pinned.push_back(h);
    if ((e = hipMalloc(reinterpret_cast<void**>(&d), (size_t)u->slot_bytes)) != hipSuccess) return fail(e, "hipMalloc");
    u->dev.push_back(d);
    if ((e = hipEventCreateWithFlags(&a, hipEventDisableTiming)) != hipSuccess) return fail(e, "hipEventCreate");
    u->copied.push_back(a);
    if ((e = hipEventCreateWithFlags(&b, hipEventDisableTiming)) != hipSuccess) return fail(e, "hipEventCreate");
    u->released.push_back(b);
    u->used.push_back(false);
  }
  *out = u;
  return DQ_OK;
}

dq_status dq_upload(dq_uploader* u, const dq_host_column* cols, int32_t n_cols, dq_column_view* dev_views) {
  if (!u || (n_cols > 0 && (!cols || !dev_views)) || n_cols < 0) return set_error(DQ_E_INVALID, "dq_upload: bad argument");
  const int s = (int)(u->next % (int64_t)u->pinned.size());
  // layout of the slot
  std::vector<Piece> pieces;
  int64_t at = 0;
  std::vector<int64_t> pos(3 * (size_t)n_cols, -1);
  for (int32_t c = 0; c < n_cols; ++c) {
    const dq_host_column& h = cols[c];
    if (h.validity_bit < 0 || h.validity_bit > 7 || h.offset_base < 0)
      return set_error(DQ_E_INVALID, "dq_upload: column %d: bad slice rebase", c);
    const void* src[3] = {h.values, h.validity, h.offsets};
    const int64_t len[3] = {h.value_bytes, h.validity_bytes, h.offset_bytes};
    for (int k = 0; k < 3; ++k) {
      if (!src[k] || len[k] <= 0) continue;
      pos[3 * (size_t)c + k] = at;
      at = align_up(at + len[k]);
    }
  }
  if (at > u->slot_bytes)
    return set_error(DQ_E_INVALID, "dq_upload: chunk needs %lld bytes, slot holds %lld", (long long)at,
                     (long long)u->slot_bytes);
  hipError_t e = hipSetDevice(u->device);
  if (e != hipSuccess) return set_error(DQ_E_HIP, "hipSetDevice failed: %s", hipGetErrorString(e));
  // the slot's previous DMA must have drained the pinned buffer before the CPU overwrites it
  if (u->used[(size_t)s] && (e = hipEventSynchronize(u->copied[(size_t)s])) != hipSuccess)
    return set_error(DQ_E_HIP, "hipEventSynchronize failed: %s", hipGetErrorString(e));
  for (int32_t c = 0; c < n_cols; ++c) {
    const dq_host_column& h = cols[c];
    const void* src[3] = {h.values, h.validity, h.offsets};
    const int64_t len[3] = {h.value_bytes, h.validity_bytes, h.offset_bytes};
    for (int k = 0; k < 3; ++k) {
      if (pos[3 * (size_t)c + k] < 0) continue;
      Piece p{u->pinned[(size_t)s] + pos[3 * (size_t)c + k], static_cast<const char*>(src[k]), len[k]};
      if ((k == 1 || (k == 0 && h.type == DQ_TYPE_BOOL)) && h.validity_bit) {  // bitmaps of a slice
        p.kind = 3;
        p.shift = h.validity_bit;
        p.src_bytes = (h.validity_bit + h.n_rows + 7) / 8;
      }
      if (k == 2 && h.offset_base) {
        p.kind = h.type == DQ_TYPE_UTF8 ? 1 : 2;
        p.base = h.offset_base;
      }
      pieces.push_back(p);
    }
  }
  parallel_copy(pieces, u->threads);
  // the scan that last read the device slot must have passed its release before the DMA overwrites it
  if (u->used[(size_t)s] && (e = hipStreamWaitEvent(u->copy, u->released[(size_t)s], 0)) != hipSuccess)
    return set_error(DQ_E_HIP, "hipStreamWaitEvent failed: %s", hipGetErrorString(e));
  if (at > 0 && (e = hipMemcpyAsync(u->dev[(size_t)s], u->pinned[(size_t)s], (size_t)at, hipMemcpyHostToDevice, u->copy)) !=
                    hipSuccess)
    return set_error(DQ_E_HIP, "hipMemcpyAsync failed: %s", hipGetErrorString(e));
  if ((e = hipEventRecord(u->copied[(size_t)s], u->copy)) != hipSuccess)
    return set_error(DQ_E_HIP, "hipEventRecord failed: %s", hipGetErrorString(e));
  for (int32_t c = 0; c < n_cols; ++c) {
    char* base = u->dev[(size_t)s];
    const int64_t* p = &pos[3 * (size_t)c];
    dev_views[c].values = p[0] >= 0 ? base + p[0] : nullptr;
    dev_views[c].validity = p[1] >= 0 ? reinterpret_cast<const uint8_t*>(base + p[1]) : nullptr;
    dev_views[c].offsets = p[2] >= 0 ? base + p[2] : nullptr;
    dev_views[c].reserved = 0;
  }
  u->used[(size_t)s] = true;
  u->bytes += at;
  ++u->next;
  return DQ_OK;
}

dq_status dq_upload_fence(dq_uploader* u, void* hip_stream) {
  if (!u || u->next == 0) return set_error(DQ_E_INVALID, "dq_upload_fence: nothing uploaded");
  const size_t s = (size_t)((u->next - 1) % (int64_t)u->pinned.size());
  const hipError_t e = hipStreamWaitEvent(static_cast<hipStream_t>(hip_stream), u->copied[s], 0);
  return e == hipSuccess ? DQ_OK : set_error(DQ_E_HIP, "hipStreamWaitEvent failed: %s", hipGetErrorString(e));
}

dq_status dq_upload_release(dq_uploader* u, void* hip_stream) {
  if (!u || u->next == 0) return set_error(DQ_E_INVALID, "dq_upload_release: nothing uploaded");
  const size_t s = (size_t)((u->next - 1) % (int64_t)u->pinned.size());
  const hipError_t e = hipEventRecord(u->released[s], static_cast<hipStream_t>(hip_stream));
  return e == hipSuccess ? DQ_OK : set_error(DQ_E_HIP, "hipEventRecord failed: %s", hipGetErrorString(e));
}

dq_status dq_upload_sync(dq_uploader* u) {
  if (!u) return set_error(DQ_E_INVALID, "dq_upload_sync: bad argument");
  const hipError_t e = hipStreamSynchronize(u->copy);
  return e == hipSuccess ? DQ_OK : set_error(DQ_E_HIP, "hipStreamSynchronize failed: %s", hipGetErrorString(e));
}

void dq_uploader_destroy(dq_uploader* u) {
  if (!u) return;
  (void)hipSetDevice(u->device);
  if (u->copy) (void)hipStreamSynchronize(u->copy);
  for (char* h : u->pinned) (void)hipHostFree(h);
  for (char* d : u->dev) (void)hipFree(d);
  for (hipEvent_t e : u->copied) (void)hipEventDestroy(e);
  for (hipEvent_t e : u->released) (void)hipEventDestroy(e);
  if (u->copy) (void)hipStreamDestroy(u->copy);
  delete u;
}

}  // extern "C"
