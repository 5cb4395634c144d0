// rsk_diag.hip -- memory-system microbenchmarks that give the sketch kernels
// their measured roofline denominators on the box they run on:
//   mode 0: streaming read (16 B/lane nontemporal loads)  -> GB/s
//   mode 1: random 4 B gathers over the buffer            -> gathers/s
//   mode 2: random 4 B atomicOr over the buffer           -> atomics/s
//   mode 3: streaming copy (read + write halves)          -> GB/s (read+write)
//   mode 4: streaming write (16 B/lane plain stores)       -> GB/s
//   mode 5: streaming write (16 B/lane nontemporal stores) -> GB/s
//   mode 6: scattered 256 B / 512 B / 1 KiB segment reads  -> GB/s (FETCH_SIZE calibration)
//   mode 7: streaming copy, loads and stores in different waves -> GB/s (read+write)
//   mode 8: streaming read, 4 B/lane (the grouped pass's id loads) -> GB/s (FETCH_SIZE calibration)
//   mode 9: scattered 128 B / 256 B segment reads, one dword per lane (the
//           fine-bin pass's medium segments)                    -> GB/s (FETCH_SIZE calibration)
// Indices come from splitmix64(i), as uniform as the Bloom probe stream.
// Also: the route overrides of a context (rsk_diag_set_route) and the timed
// launches of the kernels' tuning variants (rsk_diag_kernels.hip).
#include <cstring>

#include "rsk_diag_internal.h"

namespace rsk {

__global__ __launch_bounds__(256) void diag_stream_read(const uint4* __restrict__ p, uint64_t n16,
                                                        uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    uint4 v = ld_nt16(p + i);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;  // keeps the loads alive
}

// FETCH_SIZE calibration for segment reads (the Bloom apply passes): groups
// of L lanes each load one 16 L-byte segment (one uint4 per lane), segments
// visited in a scattered order (index times an odd constant, mod a power of
// two), every byte of the buffer read exactly once.
template <int L>
__global__ __launch_bounds__(256) void diag_segment_read(const uint4* __restrict__ p, uint64_t nseg_log,
                                                         uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  const uint64_t nseg = 1ull << nseg_log, mask = nseg - 1;
  const uint64_t g0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / L, lane = threadIdx.x % L;
  const uint64_t gs = (uint64_t)gridDim.x * blockDim.x / L;
  for (uint64_t g = g0; g < nseg; g += gs) {
    const uint64_t s = (g * 0x9E3779B97F4A7C15ull) & mask;
    const uint4 v = ld_nt16(p + s * L + lane);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;
}

// Modes 8 / 9: the same with 4-byte loads (a dword per lane; L lanes per
// segment in mode 9, L = 0 for a plain stream).
template <int L>
__global__ __launch_bounds__(256) void diag_read4(const uint32_t* __restrict__ p, uint64_t n4, uint64_t nseg_log,
                                                  uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  if (L == 0) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x)
      acc ^= p[i];
  } else {
    const uint64_t nseg = 1ull << nseg_log, mask = nseg - 1;
    const uint64_t g0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / (L ? L : 1), lane = threadIdx.x % (L ? L : 1);
    const uint64_t gs = (uint64_t)gridDim.x * blockDim.x / (L ? L : 1);
    for (uint64_t g = g0; g < nseg; g += gs) {
      const uint64_t s = (g * 0x9E3779B97F4A7C15ull) & mask;
      acc ^= p[s * L + lane];
    }
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void diag_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, uint64_t n16) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = ld_nt16(src + i);
}

// Copy with the loads and the stores in different waves (mode 7): gfx9's
// vmcnt counts a wave's loads and stores in issue order, so a wave that
// copies waits for its stores each time it waits for its next loads.  Waves
// 0-3 load 16 KiB chunks (the next one in flight) into a double-buffered LDS
// stage, waves 4-7 store them; one barrier per chunk.
__global__ __launch_bounds__(512) void diag_copy_split(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                       uint64_t n16) {
  constexpr uint32_t CH = 256 * 4;  // uint4 per chunk (16 KiB)
  __shared__ uint4 buf[2][CH];
  const bool loader = threadIdx.x < 256;
  const uint32_t t = threadIdx.x & 255;
  const uint64_t nch = n16 / CH;
  uint4 v[4];
  uint64_t c = blockIdx.x;
  if (loader && c < nch)
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ld_nt16(src + c * CH + t + u * 256);
  for (uint32_t j = 0; c < nch; ++j, c += gridDim.x) {
    if (loader) {
#pragma unroll
      for (int u = 0; u < 4; ++u) buf[j & 1][t + u * 256] = v[u];
      const uint64_t cn = c + gridDim.x;
      if (cn < nch)
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = ld_nt16(src + cn * CH + t + u * 256);
    }
    lds_barrier();
    if (!loader)
#pragma unroll
      for (int u = 0; u < 4; ++u) dst[c * CH + t + u * 256] = buf[j & 1][t + u * 256];
  }
}

template <bool NT>
__global__ __launch_bounds__(256) void diag_stream_write(uint4* __restrict__ p, uint64_t n16) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t v = (uint32_t)i;
    if (NT) {
      u32x4 x = {v, v, v, v};
      __builtin_nontemporal_store(x, reinterpret_cast<u32x4*>(p + i));
    } else {
      p[i] = make_uint4(v, v, v, v);
    }
  }
}

__global__ __launch_bounds__(256) void diag_gather(const uint32_t* __restrict__ w, uint64_t nwords, uint64_t nops,
                                                   uint32_t* __restrict__ sink) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nops; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t r = splitmix64(i);
    acc ^= w[__umul64hi(r, nwords)];
  }
  if (acc == 0x9E3779B9u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void diag_atomic_or(uint32_t* __restrict__ w, uint64_t nwords, uint64_t nops) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nops; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t r = splitmix64(i);
    atomicOr(&w[__umul64hi(r, nwords)], 1u << (r & 31));
  }
}

}  // namespace rsk

namespace rsk {
namespace diag {
static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }

// Device time of whatever `launch` enqueues on the context stream.
template <class F>
double timed(rsk_ctx* c, F&& launch) {
  hipEvent_t a, b;
  RSK_HIP(hipEventCreate(&a));
  RSK_HIP(hipEventCreate(&b));
  RSK_HIP(hipEventRecord(a, c->stream));
  launch();
  RSK_HIP(hipEventRecord(b, c->stream));
  RSK_HIP(hipEventSynchronize(b));
  float f = 0;
  RSK_HIP(hipEventElapsedTime(&f, a, b));
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  return f;
}
}  // namespace diag
}  // namespace rsk

using namespace rsk;

extern "C" {

const char* rsk_diag_last_error(void) { return diag::g_err.c_str(); }

int rsk_diag_set_route(rsk_ctx* c, const char* name, int64_t value) {
  return diag::guarded([&] {
    diag::need(c && name, "NULL argument");
    diag::Lock l(c);
    const std::string k(name);
    Tuning& t = c->tune;
    if (k == "bloom_stream") t.bloom_stream = (int)value;
    else if (k == "bloom_part") t.bloom_part = (int)value;
    else if (k == "bloom_chunk") t.bloom_chunk = (uint64_t)value;
    else if (k == "sa_tiny") t.sa_tiny = (int)value;
    else if (k == "sa_kc") t.sa_kc = (int)value;
    else if (k == "sa_v") t.sa_v = (int)value;
    else if (k == "sa_dbg") t.sa_dbg = (int)value;
    else if (k == "sa_hash") t.sa_hash = (int)value;
    else if (k == "gpart_dbg") t.gpart_dbg = (int)value;
    else if (k == "sa_full") t.sa_full = (int)value;
    else if (k == "sa_parts") t.sa_parts = (uint32_t)value;
    else if (k == "reply") t.reply = (int)value;
    else if (k == "reply_chunk") t.reply_chunk = (uint64_t)value;
    else if (k == "reply_u") t.reply_u = (int)value;
    else if (k == "reply_v") t.reply_v = (int)value;
    else if (k == "reply_dbg") t.reply_dbg = (int)value;
    else if (k == "reply_s") t.reply_s = (int)value;
    else if (k == "reply_bal") t.reply_bal = (int)value;
    else if (k == "gpart") t.gpart = (int)value;
    else if (k == "gpart_tm") t.gpart_tm = (int)value;
    else if (k == "gpart_poison") t.gpart_poison = (int)value;
    else if (k == "gpart_tile") t.gpart_tile = (int)value;
    else if (k == "route_vranks") t.route_vranks = (int)value;
    else if (k == "route_vrank") t.route_vrank = (int)value;
    else if (k == "route_heavy") t.route_heavy = (int)value;
    else if (k == "gapply_st") t.gapply_st = (int)value;
    else if (k == "gpart_rt") t.gpart_rt = (int)value;
    else if (k == "io_trace") t.io_trace = (int)value;
    else if (k == "io_piece") t.io_piece = (int)value;
    else if (k == "io_drain") t.io_drain = (int)value;
    else if (k == "copy_nt") t.copy_nt = (int)value;
    else if (k == "io_pin") t.io_pin = (int)value;
    else if (k == "io_engine") t.io_engine = (int)value;
    else if (k == "reset") t = Tuning{};
    else throw RskError{RSK_ERR_INVALID_ARG, "unknown route: " + k};
  });
}

int rsk_diag_copy_engine(rsk_ctx* c, int to_host, int* engine, float* rates) {
  return diag::guarded([&] {
    diag::need(c && engine && rates, "NULL argument");
    diag::Lock l(c);
    *engine = to_host ? c->d2h_engine : c->h2d_engine;
    for (int e = 0; e < 8; ++e) rates[e] = to_host ? c->d2h_rate[e] : c->h2d_rate[e];
  });
}

int rsk_diag_reply_stats(rsk_ctx* c, uint64_t* pending_groups, uint64_t* fallbacks) {
  return diag::guarded([&] {
    diag::need(c && pending_groups && fallbacks, "NULL argument");
    diag::Lock l(c);
    *pending_groups = c->rp_pending_groups;
    *fallbacks = c->rp_fallbacks;
  });
}

int rsk_diag_mark_dead(rsk_ctx* c) {
  return diag::guarded([&] {
    diag::need(c != nullptr, "NULL argument");
    std::lock_guard<std::recursive_mutex> g(c->mu);
    c->dead = true;
  });
}

int rsk_diag_hll_variant(rsk_ctx* c, int variant, const void* dev_keys16, uint64_t n, double* ms) {
  return diag::guarded([&] {
    diag::need(c && dev_keys16 && ms && n, "bad arguments");
    diag::Lock l(c);
    *ms = diag::timed(c, [&] { hll_variant_launch(c, variant, reinterpret_cast<const uint4*>(dev_keys16), n); });
  });
}

int rsk_diag_bloom_contains_variant(rsk_ctx* c, int variant, rsk_bloom* bf, const void* dev_keys16, uint64_t n,
                                    uint8_t* dev_out, double* ms) {
  return diag::guarded([&] {
    diag::need(c && bf && dev_keys16 && dev_out && ms && n, "bad arguments");
    diag::Lock l(c);
    *ms = diag::timed(c, [&] {
      bloom_contains_variant_launch(c, bf, reinterpret_cast<const uint4*>(dev_keys16), n, dev_out, variant);
    });
  });
}

int rsk_diag_membench(rsk_ctx* c, int mode, void* buf, uint64_t bytes, uint64_t nops, double* ms) {
  return diag::guarded([&] {
    diag::need(c && buf && ms && bytes >= 64 && mode >= 0 && mode <= 9, "bad arguments");
    // mode 6: segment reads of nops bytes (256, 512 or 1024) over the largest
    // power-of-two number of segments that fits (mode 9: 128 or 256 B)
    diag::need(mode != 6 || nops == 256 || nops == 512 || nops == 1024, "segment bytes must be 256, 512 or 1024");
    diag::need(mode != 9 || nops == 128 || nops == 256, "segment bytes must be 128 or 256");
    uint64_t nseg_log = 0;
    if (mode == 6 || mode == 9)
      while ((2ull << nseg_log) * nops <= bytes) ++nseg_log;
    diag::Lock l(c);
    uint32_t* sink = reinterpret_cast<uint32_t*>(c->d_small + 512);
    const uint32_t grid = (uint32_t)c->num_cus * 8;
    *ms = diag::timed(c, [&] {
      switch (mode) {
        case 0:
          hipLaunchKernelGGL(diag_stream_read, dim3(grid), dim3(256), 0, c->stream, reinterpret_cast<const uint4*>(buf),
                             bytes / 16, sink);
          break;
        case 1:
          hipLaunchKernelGGL(diag_gather, dim3(grid), dim3(256), 0, c->stream, reinterpret_cast<const uint32_t*>(buf),
                             bytes / 4, nops, sink);
          break;
        case 2:
          hipLaunchKernelGGL(diag_atomic_or, dim3(grid), dim3(256), 0, c->stream, reinterpret_cast<uint32_t*>(buf),
                             bytes / 4, nops);
          break;
        case 4:
          hipLaunchKernelGGL(diag_stream_write<false>, dim3(grid), dim3(256), 0, c->stream, reinterpret_cast<uint4*>(buf),
                             bytes / 16);
          break;
        case 5:
          hipLaunchKernelGGL(diag_stream_write<true>, dim3(grid), dim3(256), 0, c->stream, reinterpret_cast<uint4*>(buf),
                             bytes / 16);
          break;
        case 7: {  // split copy: buffer halves, as mode 3
          const uint64_t half = bytes / 32;
          hipLaunchKernelGGL(diag_copy_split, dim3((uint32_t)c->num_cus * 4), dim3(512), 0, c->stream,
                             reinterpret_cast<const uint4*>(buf), reinterpret_cast<uint4*>(buf) + half, half);
          break;
        }
        case 6: {
          const uint4* p = reinterpret_cast<const uint4*>(buf);
          if (nops == 256)
            hipLaunchKernelGGL(diag_segment_read<16>, dim3(grid), dim3(256), 0, c->stream, p, nseg_log, sink);
          else if (nops == 512)
            hipLaunchKernelGGL(diag_segment_read<32>, dim3(grid), dim3(256), 0, c->stream, p, nseg_log, sink);
          else
            hipLaunchKernelGGL(diag_segment_read<64>, dim3(grid), dim3(256), 0, c->stream, p, nseg_log, sink);
          break;
        }
        case 8:
          hipLaunchKernelGGL(diag_read4<0>, dim3(grid), dim3(256), 0, c->stream, reinterpret_cast<const uint32_t*>(buf),
                             bytes / 4, 0ull, sink);
          break;
        case 9:
          if (nops == 128)
            hipLaunchKernelGGL(diag_read4<32>, dim3(grid), dim3(256), 0, c->stream,
                               reinterpret_cast<const uint32_t*>(buf), bytes / 4, nseg_log, sink);
          else
            hipLaunchKernelGGL(diag_read4<64>, dim3(grid), dim3(256), 0, c->stream,
                               reinterpret_cast<const uint32_t*>(buf), bytes / 4, nseg_log, sink);
          break;
        default: {
          const uint64_t half = bytes / 32;  // uint4 elements per half
          hipLaunchKernelGGL(diag_copy, dim3(grid), dim3(256), 0, c->stream, reinterpret_cast<const uint4*>(buf),
                             reinterpret_cast<uint4*>(buf) + half, half);
          break;
        }
      }
      RSK_CHECK_LAUNCH("diag");
    });
  });
}

int rsk_diag_bloom_contains_probes(rsk_ctx* c, rsk_bloom* bf, const void* dev_keys16, uint64_t n, uint8_t* dev_out,
                                   uint64_t* probes) {
  return diag::guarded([&] {
    diag::need(c && bf && dev_keys16 && dev_out && probes && n, "bad arguments");
    diag::Lock l(c);
    auto* d = reinterpret_cast<unsigned long long*>(c->d_small + 384);
    RSK_HIP(hipMemsetAsync(d, 0, 8, c->stream));
    bloom_contains_probe_count_launch(c, bf, reinterpret_cast<const uint4*>(dev_keys16), n, dev_out, d);
    RSK_HIP(hipMemcpyAsync(c->h_small + 384, d, 8, hipMemcpyDeviceToHost, c->stream));
    RSK_HIP(hipStreamSynchronize(c->stream));
    std::memcpy(probes, c->h_small + 384, 8);
  });
}

int rsk_diag_hll_var_variant(rsk_ctx* c, int variant, const void* dev_data, const uint64_t* dev_offsets, uint64_t n,
                             double* ms) {
  return diag::guarded([&] {
    diag::need(c && dev_data && dev_offsets && ms && n, "bad arguments");
    diag::Lock l(c);
    *ms = diag::timed(c, [&] {
      hll_var_variant_launch(c, variant, reinterpret_cast<const uint8_t*>(dev_data), dev_offsets, n);
    });
  });
}

}  // extern "C"
