// rsk_bitset.hip -- RBitSet on the GPU: a Redis string addressed as bits.
//
// Replaces the commands RedissonBitSet (src/main/java/org/redisson/RedissonBitSet.java)
// sends: SETBIT / GETBIT (:70-80, :196-209), BITCOUNT (:240-243), STRLEN
// (size(), BitsSizeReplayConvertor.java:21-27), BITOP AND/OR/XOR/NOT
// (:125-145, :216-268), GET / SET (:88-91, :211-214), DEL (clear()), and the
// Lua length() (:175-189).
//
// Layout: the string's bytes in HBM, bit i in byte i>>3 under mask
// 0x80 >> (i&7) (bitops.c, MSB-first) -- the same layout as the Bloom filter.
// The string has a logical length (STRLEN); SETBIT beyond it grows the
// string with zero bytes to (offset>>3)+1 whatever the value, as Redis does.
#include <algorithm>
#include <cstring>
#include <vector>

#include "rsk_internal.h"

struct rsk_bitset {
  rsk_ctx* ctx = nullptr;
  uint8_t* d = nullptr;    // device bytes, capacity `cap` (zero beyond len)
  uint64_t len = 0;        // STRLEN
  uint64_t cap = 0;
  // A view of a Bloom filter's bit string (rsk_bloom_bitset): in Redis the
  // filter's bits ARE the string key `name` (RedissonBloomFilter SETBITs it,
  // RedissonBitSet reads it), so getBitSet(filterName) sees them.  d is the
  // filter's buffer (not owned); the string can hold at most the filter's
  // ceil(size/8) bytes.  STRLEN is Redis's: the highest byte any SETBIT
  // touched + 1 -- a Bloom add only sets bits, so for its part that is the
  // last non-zero byte + 1; `floor` carries what writes through the view
  // (clears, SET, BITOP) fixed beyond that.
  rsk_bloom* alias = nullptr;
  uint64_t floor = 0;
  // the filter's write / SET generations this view's len reflects (rsk_bloom::wgen, rgen)
  uint64_t seen = 0, rseen = 0;
};

namespace {

using rsk::RskError;

template <class F>
int guarded(F&& fn) {
  try {
    fn();
    rsk::set_error("");
    return RSK_OK;
  } catch (const RskError& e) {
    rsk::set_error(e.msg);
    return e.code;
  } catch (const std::exception& e) {
    rsk::set_error(e.what());
    return RSK_ERR_DEVICE;
  }
}

void need(bool cond, const char* msg) {
  if (!cond) throw RskError{RSK_ERR_INVALID_ARG, msg};
}

struct Lock {
  std::lock_guard<std::recursive_mutex> g;
  explicit Lock(rsk_ctx* c) : g(c->mu) { RSK_HIP(hipSetDevice(c->device)); }
};

// Redis limits a string to 512 MB: offsets up to 2^32 - 1 bits.
constexpr uint64_t MAX_BIT_OFFSET = (1ull << 32) - 1;

uint32_t grid_of(rsk_ctx* c, uint64_t n);
__global__ void length_kernel(const uint4* __restrict__ d, uint64_t len, unsigned long long* __restrict__ out);

// Highest set bit + 1 of bytes [0, len) (0 when none); the buffer is padded
// to 16 bytes and zero past len.  Under the context lock.
uint64_t length_bits(rsk_ctx* c, const uint8_t* d, uint64_t len) {
  if (len == 0) return 0;
  rsk::ProfScope ps(c, "bitset_length");
  auto* dl = reinterpret_cast<unsigned long long*>(c->d_small + 320);
  RSK_HIP(hipMemsetAsync(dl, 0, 8, c->stream));
  hipLaunchKernelGGL(length_kernel, dim3(grid_of(c, (len + 15) / 16)), dim3(256), 0, c->stream,
                     reinterpret_cast<const uint4*>(d), len, dl);
  RSK_CHECK_LAUNCH("bitset_length");
  RSK_HIP(hipMemcpyAsync(c->h_small + 320, dl, 8, hipMemcpyDeviceToHost, c->stream));
  RSK_HIP(hipStreamSynchronize(c->stream));
  uint64_t v;
  std::memcpy(&v, c->h_small + 320, 8);
  return v;
}

// A view's STRLEN as it stands now (Bloom adds may have grown it since the
// last call): refreshes b->d / cap / len.  Plain strings are left alone.
// The scan runs only when the filter was written since this view last looked
// (a GETBIT / GET through the view does not rescan a 1.2 GB filter).
void sync_view(rsk_bitset* b) {
  if (!b->alias) return;
  rsk_bloom* f = b->alias;
  b->d = reinterpret_cast<uint8_t*>(f->d_bits);
  b->cap = f->nwords * 4;
  if (b->rseen != f->rgen) {  // the string was SET (rsk_bloom_import_bits, a SET / DEL / BITOP through a view)
    b->floor = f->set_len;
    b->rseen = f->rgen;
    b->seen = 0;
  }
  if (b->seen == f->wgen) return;
  const uint64_t bits = length_bits(b->ctx, b->d, f->nbytes);
  const uint64_t used = bits ? ((bits - 1) >> 3) + 1 : 0;
  b->len = std::max(b->floor, used);
  b->seen = f->wgen;
}

// After a write through view b (its len already maintained by grow): other
// views of the filter rescan; set: the write replaced the whole string
// (STRLEN = b->len for every view).
void view_written(rsk_bitset* b, bool set = false) {
  if (!b->alias) return;
  rsk_bloom* f = b->alias;
  ++f->wgen;
  b->seen = f->wgen;
  if (set) {
    ++f->rgen;
    f->set_len = b->len;
    b->rseen = f->rgen;
  }
}

// Grow the string to `newlen` bytes (zero filled), keeping 16-byte padding.
void grow(rsk_bitset* b, uint64_t newlen) {
  if (b->alias) {  // the filter's buffer is the string: it cannot move or grow past the filter
    need(newlen <= b->alias->nbytes, "ERR the string of a GPU Bloom filter cannot grow past the filter's size");
    b->floor = std::max(b->floor, newlen);
    b->len = std::max(b->len, newlen);
    return;
  }
  if (newlen <= b->len) return;
  rsk_ctx* c = b->ctx;
  if (newlen > b->cap) {
    uint64_t cap = std::max<uint64_t>(newlen + 16, b->cap * 2);
    cap = (cap + 15) & ~uint64_t(15);
    uint8_t* nd = nullptr;
    RSK_HIP(hipMalloc(&nd, cap));
    RSK_HIP(hipMemsetAsync(nd, 0, cap, c->stream));
    if (b->d && b->len) RSK_HIP(hipMemcpyAsync(nd, b->d, b->len, hipMemcpyDeviceToDevice, c->stream));
    if (b->d) {
      RSK_HIP(hipStreamSynchronize(c->stream));
      RSK_HIP(hipFree(b->d));
    }
    b->d = nd;
    b->cap = cap;
  }
  b->len = newlen;  // bytes past the old length are already zero
}

__device__ __forceinline__ uint8_t bmask(uint64_t off) { return (uint8_t)(0x80u >> (off & 7)); }

// SETBIT for a list of offsets (value v); byte-level atomicOr/And on the
// containing u32 word (bits of one word may be set by different lanes).
__global__ void setbits_kernel(uint8_t* __restrict__ d, const uint64_t* __restrict__ offs, uint64_t n, int v) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t off = offs[i];
    const uint64_t byte = off >> 3;
    uint32_t* w = reinterpret_cast<uint32_t*>(d + (byte & ~uint64_t(3)));
    const uint32_t m = (uint32_t)bmask(off) << (8 * (byte & 3));
    if (v) atomicOr(w, m);
    else atomicAnd(w, ~m);
  }
}

__global__ void getbits_kernel(const uint8_t* __restrict__ d, uint64_t len, const uint64_t* __restrict__ offs,
                               uint64_t n, uint8_t* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t off = offs[i];
    const uint64_t byte = off >> 3;
    out[i] = byte < len ? (uint8_t)((d[byte] & bmask(off)) != 0) : 0;
  }
}

// Bits [from, to) := v, byte-wise: partial first/last bytes by mask.
__global__ void range_kernel(uint8_t* __restrict__ d, uint64_t from, uint64_t to, int v) {
  const uint64_t b0 = from >> 3, b1 = (to - 1) >> 3;
  for (uint64_t b = b0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b <= b1;
       b += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t lo = from > b * 8 ? from : b * 8, hi = to < b * 8 + 8 ? to : b * 8 + 8;
    uint8_t m = 0;
    for (uint64_t i = lo; i < hi; ++i) m |= bmask(i);
    d[b] = v ? (uint8_t)(d[b] | m) : (uint8_t)(d[b] & ~m);
  }
}

// BITOP: out = op over srcs (bytes past a source's length read as 0), in
// 16-byte chunks.  Every string buffer is zero past its length and padded to
// 16 bytes, so a chunk that starts inside a source is read whole and a chunk
// past its end reads as zero; only NOT needs the output's tail masked.
struct SrcList {
  const uint8_t* p[16];
  uint64_t len[16];
  uint32_t k;
};

RSK_DEV uint4 op16(uint4 a, uint4 b, int op) {
  if (op == RSK_BITOP_AND) return make_uint4(a.x & b.x, a.y & b.y, a.z & b.z, a.w & b.w);
  if (op == RSK_BITOP_OR) return make_uint4(a.x | b.x, a.y | b.y, a.z | b.z, a.w | b.w);
  return make_uint4(a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w);
}

__global__ void bitop_kernel(uint4* __restrict__ out, uint64_t n, SrcList s, int op) {
  const uint64_t n16 = (n + 15) >> 4;
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n16; c += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t b = c << 4;
    uint4 acc = b < s.len[0] ? reinterpret_cast<const uint4*>(s.p[0])[c] : make_uint4(0, 0, 0, 0);
    if (op == RSK_BITOP_NOT) {
      uint32_t w[4] = {~acc.x, ~acc.y, ~acc.z, ~acc.w};
      if (b + 16 > n) {  // bytes at or past n stay zero
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int64_t keep = (int64_t)n - (int64_t)(b + 4 * q);  // bytes of word q below n
          w[q] = keep >= 4 ? w[q] : keep <= 0 ? 0u : (w[q] & ((1u << (8 * keep)) - 1));
        }
      }
      acc = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
      for (uint32_t j = 1; j < s.k; ++j) {
        const uint4 x = b < s.len[j] ? reinterpret_cast<const uint4*>(s.p[j])[c] : make_uint4(0, 0, 0, 0);
        acc = op16(acc, x, op);
      }
    }
    out[c] = acc;
  }
}

// Highest set bit index + 1 (0 if none), 16 bytes per lane: the last nonzero
// byte b of the chunk holds MSB-first bit 8b + 7 - ctz(byte).
__global__ void length_kernel(const uint4* __restrict__ d, uint64_t len, unsigned long long* __restrict__ out) {
  unsigned long long best = 0;
  const uint64_t n16 = (len + 15) >> 4;
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < n16; c += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = d[c];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (w[q]) {
        const uint32_t byte = 3 - (__builtin_clz(w[q]) >> 3);  // highest nonzero byte of the LE word
        const uint32_t bv = (w[q] >> (8 * byte)) & 0xFFu;
        best = (c << 7) + 8ull * (4 * q + byte) + 8 - __builtin_ctz(bv);
      }
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    const unsigned long long o = __shfl_down(best, off, 64);
    best = o > best ? o : best;
  }
  if ((threadIdx.x & 63) == 0 && best) atomicMax(out, best);
}

uint32_t grid_of(rsk_ctx* c, uint64_t n) {
  uint64_t g = (n + 255) / 256;
  uint64_t cap = (uint64_t)c->num_cus * 8;
  return (uint32_t)std::max<uint64_t>(1, std::min(g, cap));
}

const uint64_t* device_offsets(rsk_ctx* c, const uint64_t* offs, uint64_t n, uint32_t location, uint64_t* max_out) {
  uint64_t mx = 0;
  if (location == RSK_MEM_HOST) {
    for (uint64_t i = 0; i < n; ++i) mx = std::max(mx, offs[i]);
    uint64_t* d = reinterpret_cast<uint64_t*>(c->work(n * 8 + 256));
    RSK_HIP(hipMemcpyAsync(d, offs, n * 8, hipMemcpyHostToDevice, c->stream));
    *max_out = mx;
    return d;
  }
  need(location == RSK_MEM_DEVICE, "bad location");
  // device offsets: read them back once to size the string (SETBIT growth)
  std::vector<uint64_t> h(n);
  RSK_HIP(hipMemcpyAsync(h.data(), offs, n * 8, hipMemcpyDeviceToHost, c->stream));
  RSK_HIP(hipStreamSynchronize(c->stream));
  for (uint64_t v : h) mx = std::max(mx, v);
  *max_out = mx;
  return offs;
}

}  // namespace

extern "C" {

int rsk_bitset_create(rsk_ctx* c, rsk_bitset** out) {
  return guarded([&] {
    need(c && out, "NULL argument");
    auto* b = new rsk_bitset();
    b->ctx = c;
    *out = b;
  });
}

int rsk_bitset_destroy(rsk_bitset* b) {
  if (!b) return RSK_OK;
  int rc = guarded([&] {
    Lock l(b->ctx);
    RSK_HIP(hipStreamSynchronize(b->ctx->stream));
    if (b->d && !b->alias) RSK_HIP(hipFree(b->d));
  });
  delete b;
  return rc;
}

// The bit string of Bloom filter f as an RBitSet (see rsk_bitset.alias).
int rsk_bloom_bitset(rsk_bloom* f, rsk_bitset** out) {
  return guarded([&] {
    need(f && out, "NULL argument");
    Lock l(f->ctx);
    auto* b = new rsk_bitset();
    b->ctx = f->ctx;
    b->alias = f;
    sync_view(b);
    *out = b;
  });
}

int rsk_bitset_strlen(rsk_bitset* b, uint64_t* out) {
  return guarded([&] {
    need(b && out, "NULL argument");
    if (b->alias) {
      Lock l(b->ctx);
      sync_view(b);
    }
    *out = b->len;
  });
}

int rsk_bitset_setbits(rsk_bitset* b, const uint64_t* offs, uint64_t n, int value, uint32_t location) {
  return guarded([&] {
    need(b && (offs || n == 0), "NULL argument");
    need(value == 0 || value == 1, "bit value must be 0 or 1");
    if (n == 0) return;
    rsk_ctx* c = b->ctx;
    Lock l(c);
    sync_view(b);
    uint64_t mx = 0;
    const uint64_t* d_offs = device_offsets(c, offs, n, location, &mx);
    need(mx <= MAX_BIT_OFFSET, "ERR bit offset is not an integer or out of range");
    if (b->alias && value == 0) b->floor = std::max(b->floor, b->len);  // cleared bits keep the length
    grow(b, (mx >> 3) + 1);
    rsk::ProfScope ps(c, "bitset_setbits");
    hipLaunchKernelGGL(setbits_kernel, dim3(grid_of(c, n)), dim3(256), 0, c->stream, b->d, d_offs, n, value);
    RSK_CHECK_LAUNCH("bitset_setbits");
    RSK_HIP(hipStreamSynchronize(c->stream));
    view_written(b);
  });
}

int rsk_bitset_getbits(rsk_bitset* b, const uint64_t* offs, uint64_t n, uint32_t location, uint8_t* out) {
  return guarded([&] {
    need(b && out && (offs || n == 0), "NULL argument");
    if (n == 0) return;
    rsk_ctx* c = b->ctx;
    Lock l(c);
    sync_view(b);
    uint64_t mx = 0;
    const uint64_t* d_offs = device_offsets(c, offs, n, location, &mx);
    need(mx <= MAX_BIT_OFFSET, "ERR bit offset is not an integer or out of range");
    if (b->len == 0) {  // absent key: every GETBIT replies 0
      if (location == RSK_MEM_HOST) std::memset(out, 0, n);
      else RSK_HIP(hipMemsetAsync(out, 0, n, c->stream));
      RSK_HIP(hipStreamSynchronize(c->stream));
      return;
    }
    uint8_t* d_out = location == RSK_MEM_DEVICE ? out : c->work(n * 8 + 256 + n) + ((n * 8 + 255) & ~255ull);
    hipLaunchKernelGGL(getbits_kernel, dim3(grid_of(c, n)), dim3(256), 0, c->stream, b->d, b->len, d_offs, n, d_out);
    RSK_CHECK_LAUNCH("bitset_getbits");
    if (location == RSK_MEM_HOST) RSK_HIP(hipMemcpyAsync(out, d_out, n, hipMemcpyDeviceToHost, c->stream));
    RSK_HIP(hipStreamSynchronize(c->stream));
  });
}

int rsk_bitset_set_range(rsk_bitset* b, uint64_t from, uint64_t to, int value) {
  return guarded([&] {
    need(b != nullptr, "NULL argument");
    need(value == 0 || value == 1, "bit value must be 0 or 1");
    if (to <= from) return;  // the reference's loop issues no SETBIT
    need(to - 1 <= MAX_BIT_OFFSET, "ERR bit offset is not an integer or out of range");
    rsk_ctx* c = b->ctx;
    Lock l(c);
    sync_view(b);
    if (b->alias && value == 0) b->floor = std::max(b->floor, b->len);
    grow(b, ((to - 1) >> 3) + 1);
    // Whole bytes by a memset; the partial first / last byte by the mask kernel.
    const uint64_t full_lo = (from + 7) >> 3, full_hi = to >> 3;  // bytes [full_lo, full_hi) are covered whole
    if (full_hi > full_lo) {
      RSK_HIP(hipMemsetAsync(b->d + full_lo, value ? 0xFF : 0x00, full_hi - full_lo, c->stream));
      if (from < full_lo * 8)
        hipLaunchKernelGGL(range_kernel, dim3(1), dim3(64), 0, c->stream, b->d, from, full_lo * 8, value);
      if (full_hi * 8 < to)
        hipLaunchKernelGGL(range_kernel, dim3(1), dim3(64), 0, c->stream, b->d, full_hi * 8, to, value);
    } else {
      hipLaunchKernelGGL(range_kernel, dim3(1), dim3(64), 0, c->stream, b->d, from, to, value);
    }
    RSK_CHECK_LAUNCH("bitset_range");
    RSK_HIP(hipStreamSynchronize(c->stream));
    view_written(b);
  });
}

int rsk_bitset_bitcount(rsk_bitset* b, uint64_t* out) {
  return guarded([&] {
    need(b && out, "NULL argument");
    rsk_ctx* c = b->ctx;
    Lock l(c);
    sync_view(b);
    if (b->len == 0) {
      *out = 0;
      return;
    }
    uint64_t* d = reinterpret_cast<uint64_t*>(c->d_small + 256);
    // bytes past len are zero and the buffer is padded to 16 bytes
    rsk::bloom_bitcount_launch(c, reinterpret_cast<const uint32_t*>(b->d), ((b->len + 15) / 16) * 4, d);
    RSK_HIP(hipMemcpyAsync(c->h_small + 256, d, 8, hipMemcpyDeviceToHost, c->stream));
    RSK_HIP(hipStreamSynchronize(c->stream));
    std::memcpy(out, c->h_small + 256, 8);
  });
}

int rsk_bitset_length(rsk_bitset* b, uint64_t* out) {
  return guarded([&] {
    need(b && out, "NULL argument");
    rsk_ctx* c = b->ctx;
    Lock l(c);
    sync_view(b);
    *out = length_bits(c, b->d, b->len);
  });
}

int rsk_bitset_bitop(int op, rsk_bitset* dst, rsk_bitset* const* srcs, uint32_t k) {
  return guarded([&] {
    need(dst && srcs && k >= 1 && k <= 16, "BITOP takes 1..16 source keys");
    need(op >= RSK_BITOP_AND && op <= RSK_BITOP_NOT, "bad BITOP operation");
    need(op != RSK_BITOP_NOT || k == 1, "BITOP NOT must be called with a single source key.");
    rsk_ctx* c = dst->ctx;
    Lock l(c);
    sync_view(dst);
    SrcList s{};
    s.k = k;
    uint64_t maxlen = 0;
    for (uint32_t j = 0; j < k; ++j) {
      need(srcs[j] && srcs[j]->ctx == c, "sources must share the context");
      sync_view(srcs[j]);
      s.p[j] = srcs[j]->d;
      s.len[j] = srcs[j]->len;
      maxlen = std::max(maxlen, srcs[j]->len);
    }
    if (maxlen == 0) {  // every source empty: Redis deletes the destination
      dst->len = 0;
      dst->floor = 0;
      if (dst->d) RSK_HIP(hipMemsetAsync(dst->d, 0, dst->cap, c->stream));
      RSK_HIP(hipStreamSynchronize(c->stream));
      view_written(dst, true);
      return;
    }
    if (dst->alias)
      need(maxlen <= dst->alias->nbytes, "ERR the string of a GPU Bloom filter cannot grow past the filter's size");
    // Compute into a fresh buffer (dst may be one of the sources), then swap.
    const uint64_t cap = (maxlen + 16 + 15) & ~uint64_t(15);
    uint8_t* nd = nullptr;
    RSK_HIP(hipMalloc(&nd, cap));
    RSK_HIP(hipMemsetAsync(nd, 0, cap, c->stream));
    hipLaunchKernelGGL(bitop_kernel, dim3(grid_of(c, (maxlen + 15) / 16)), dim3(256), 0, c->stream,
                       reinterpret_cast<uint4*>(nd), maxlen, s, op);
    RSK_CHECK_LAUNCH("bitset_bitop");
    if (dst->alias) {  // written into the filter's own buffer (zero past the result)
      RSK_HIP(hipMemsetAsync(dst->d, 0, dst->cap, c->stream));
      RSK_HIP(hipMemcpyAsync(dst->d, nd, maxlen, hipMemcpyDeviceToDevice, c->stream));
      RSK_HIP(hipStreamSynchronize(c->stream));
      RSK_HIP(hipFree(nd));
      dst->floor = dst->len = maxlen;
      view_written(dst, true);
      return;
    }
    RSK_HIP(hipStreamSynchronize(c->stream));
    if (dst->d) RSK_HIP(hipFree(dst->d));
    dst->d = nd;
    dst->cap = cap;
    dst->len = maxlen;
  });
}

int rsk_bitset_get_bytes(rsk_bitset* b, uint8_t* buf, size_t cap, size_t* len) {
  return guarded([&] {
    need(b && len, "NULL argument");
    Lock l(b->ctx);
    sync_view(b);
    need(cap >= b->len && (buf || b->len == 0), "buffer smaller than STRLEN");
    if (b->len) {
      RSK_HIP(hipMemcpyAsync(buf, b->d, b->len, hipMemcpyDeviceToHost, b->ctx->stream));
      RSK_HIP(hipStreamSynchronize(b->ctx->stream));
    }
    *len = b->len;
  });
}

int rsk_bitset_set_bytes(rsk_bitset* b, const uint8_t* buf, size_t len) {
  return guarded([&] {
    need(b && (buf || len == 0), "NULL argument");
    rsk_ctx* c = b->ctx;
    Lock l(c);
    sync_view(b);
    if (b->alias)
      need(len <= b->alias->nbytes, "ERR the string of a GPU Bloom filter cannot grow past the filter's size");
    if (b->d) RSK_HIP(hipMemsetAsync(b->d, 0, b->cap, c->stream));
    b->len = 0;
    b->floor = 0;
    grow(b, len);
    if (len) RSK_HIP(hipMemcpyAsync(b->d, buf, len, hipMemcpyHostToDevice, c->stream));
    RSK_HIP(hipStreamSynchronize(c->stream));
    view_written(b, true);
  });
}

int rsk_bitset_clear(rsk_bitset* b) {
  return guarded([&] {
    need(b != nullptr, "NULL argument");
    Lock l(b->ctx);
    sync_view(b);
    if (b->d) RSK_HIP(hipMemsetAsync(b->d, 0, b->cap, b->ctx->stream));
    RSK_HIP(hipStreamSynchronize(b->ctx->stream));
    b->len = 0;
    b->floor = 0;
    view_written(b, true);
  });
}

}  // extern "C"
