// rsk_api.hip -- the C ABI of librsketch.so (include/rsketch.h).
//
// Host-side state machine of the Redis commands the reference issues for
// this path (key existence, the HLL cardinality cache, Bloom sizing with
// Java double semantics), plus staging of host key batches and error
// mapping.  All arithmetic on keys runs in the HIP kernels of rsk_hll.hip /
// rsk_bloom.hip; nothing here hashes a key.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <thread>
#include <vector>
#include <unordered_map>

#include <pthread.h>
#if !defined(__HIP_DEVICE_COMPILE__)
#include <emmintrin.h>
#endif

#include "rsk_internal.h"

using rsk::DevKeys;
using rsk::RskError;

namespace rsk {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }

template <class F>
static int guarded(F&& fn) {
  try {
    fn();
    g_last_error.clear();
    return RSK_OK;
  } catch (const RskError& e) {
    g_last_error = e.msg;
    return e.code;
  } catch (const std::bad_alloc&) {
    g_last_error = "host allocation failed";
    return RSK_ERR_OUT_OF_MEMORY;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return RSK_ERR_DEVICE;
  }
}

[[noreturn]] static void fail(int code, const std::string& msg) { throw RskError{code, msg}; }

// The address the copy engines use for a registered host range (0: the runtime has none).
static uintptr_t reg_dptr(void* p) {
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return reinterpret_cast<uintptr_t>(d);
}

void prof_begin(rsk_ctx* c, const char*, hipEvent_t* a, hipEvent_t* b) {
  if (!c->prof.on) return;
  for (hipEvent_t* e : {a, b}) {
    if (!c->prof.free_events.empty()) {
      *e = c->prof.free_events.back();
      c->prof.free_events.pop_back();
    } else if (hipEventCreate(e) != hipSuccess) {
      *e = nullptr;
    }
  }
  if (*a) (void)hipEventRecord(*a, c->stream);
}

void prof_end(rsk_ctx* c, const char* name, hipEvent_t a, hipEvent_t b) {
  if (!c->prof.on || !a || !b) return;
  (void)hipEventRecord(b, c->stream);
  c->prof.pending.push_back({name, a, b});
}

static void prof_fold(rsk_ctx* c) {
  for (auto& p : c->prof.pending) {
    float ms = 0;
    if (hipEventSynchronize(p.b) == hipSuccess && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
      auto& e = c->prof.totals[p.name];
      e.ms += ms;
      e.launches += 1;
    }
    c->prof.free_events.push_back(p.a);
    c->prof.free_events.push_back(p.b);
  }
  c->prof.pending.clear();
}

}  // namespace rsk

uint8_t* rsk_ctx::work(uint64_t bytes) {
  if (bytes > work_bytes) {
    if (d_work) {
      RSK_HIP(hipStreamSynchronize(stream));
      RSK_HIP(hipFree(d_work));
      d_work = nullptr;
      work_bytes = 0;
    }
    uint64_t sz = std::max<uint64_t>(bytes, 64ull << 20);
    RSK_HIP(hipMalloc(&d_work, sz));
    work_bytes = sz;
  }
  return d_work;
}

static uint8_t* grow_dev(hipStream_t stream, uint8_t*& p, uint64_t& have, uint64_t bytes) {
  if (bytes > have) {
    if (p) {
      RSK_HIP(hipStreamSynchronize(stream));
      RSK_HIP(hipFree(p));
      p = nullptr;
      have = 0;
    }
    const uint64_t sz = std::max<uint64_t>(bytes, 16ull << 20);
    RSK_HIP(hipMalloc(&p, sz));
    have = sz;
  }
  return p;
}

uint8_t* rsk_ctx::xbuf(uint64_t bytes) { return grow_dev(stream, d_xbuf, xbuf_bytes, bytes); }
uint8_t* rsk_ctx::sbuf(uint64_t bytes) { return grow_dev(stream, d_sbuf, sbuf_bytes, bytes); }
uint8_t* rsk_ctx::hrows(uint64_t bytes) { return grow_dev(stream, d_hrows, hrows_bytes, bytes); }
uint8_t* rsk_ctx::cslow(uint64_t bytes) { return grow_dev(stream, d_cslow, cslow_bytes, bytes); }

uint8_t* rsk_ctx::pinned(uint64_t bytes) {
  // every call that fills this buffer waits for its DMA before returning
  if (bytes > h_batch_bytes) {
    if (h_batch) {
      RSK_HIP(hipStreamSynchronize(stream));
      RSK_HIP(hipHostFree(h_batch));
      h_batch = nullptr;
      h_batch_bytes = 0;
    }
    const uint64_t sz = std::max<uint64_t>(bytes, 4ull << 20);
    RSK_HIP(hipHostMalloc(&h_batch, sz, hipHostMallocDefault));
    h_batch_bytes = sz;
  }
  return h_batch;
}

namespace {

using namespace rsk;

struct CtxLock {
  std::lock_guard<std::recursive_mutex> g;
  explicit CtxLock(rsk_ctx* c) : g(c->mu) {
    if (c->dead) fail(RSK_ERR_DEVICE, "the context's device work failed earlier; shut it down");
    hipError_t e = hipSetDevice(c->device);
    if (e != hipSuccess) fail(RSK_ERR_DEVICE, std::string("hipSetDevice: ") + hipGetErrorString(e));
  }
};

void need(bool cond, const char* msg) {
  if (!cond) fail(RSK_ERR_INVALID_ARG, msg);
}

// Device output scratch that is distinct from ctx->work (used inside
// algorithms).  Kept per context, grown on demand.
uint8_t* out_scratch(rsk_ctx* c, uint64_t bytes) {
  if (bytes > c->out_bytes) {
    if (c->d_out) {
      RSK_HIP(hipStreamSynchronize(c->stream));
      RSK_HIP(hipFree(c->d_out));
      c->d_out = nullptr;
      c->out_bytes = 0;
    }
    uint64_t sz = std::max<uint64_t>(bytes, 16ull << 20);
    RSK_HIP(hipMalloc(&c->d_out, sz));
    c->out_bytes = sz;
  }
  return c->d_out;
}

void ensure_stage(rsk_ctx* c) {
  if (!c->d_stage) RSK_HIP(hipMalloc(&c->d_stage, c->stage_bytes + c->stage_bytes / 4));
}

// A pointer a kernel will dereference must be one the GPU can reach (device,
// managed or registered/pinned host memory); a pageable host pointer passed
// as RSK_MEM_DEVICE is rejected here instead of faulting the device.
// Device memory must belong to the context's GPU (no peer access is enabled).
void need_gpu_ptr(const rsk_ctx* c, const void* p, const char* msg) {
  if (!p) return;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    fail(RSK_ERR_INVALID_ARG, msg);
  }
  if (a.type == hipMemoryTypeUnregistered) fail(RSK_ERR_INVALID_ARG, msg);
  if (a.type == hipMemoryTypeDevice && c && a.device != c->device)
    fail(RSK_ERR_INVALID_ARG, std::string(msg) + " (device memory of another GPU)");
}

void check_keys(const rsk_ctx* c, const rsk_keys* k) {
  need(k != nullptr, "keys is NULL");
  need(k->location == RSK_MEM_HOST || k->location == RSK_MEM_DEVICE, "keys.location must be RSK_MEM_HOST or RSK_MEM_DEVICE");
  need(k->n == 0 || k->data != nullptr || (k->offsets == nullptr && k->fixed_len == 0), "keys.data is NULL");
  if (k->location == RSK_MEM_DEVICE && k->n > 0) {
    need_gpu_ptr(c, k->data, "keys.data is not GPU-accessible memory (location RSK_MEM_DEVICE)");
    need_gpu_ptr(c, k->offsets, "keys.offsets is not GPU-accessible memory (location RSK_MEM_DEVICE)");
  }
}

// Per-key outputs follow the keys' location.
void check_out(const rsk_ctx* c, const rsk_keys* k, const void* out) {
  if (k->location == RSK_MEM_DEVICE && k->n > 0)
    need_gpu_ptr(c, out, "output is not GPU-accessible memory (keys are RSK_MEM_DEVICE)");
}

// Host batches go through two pinned host stages: host threads fill one
// (par_copy) while the DMA of the other runs, so the pageable user buffer is
// read at memcpy speed and the link carries pinned transfers.  Each stage has
// its own device twin, so chunk i+1's DMA may queue behind chunk i's kernels
// without a host wait.  rsk_options.stage_threads (default 8) sets the copy threads.
// The copy threads persist (one pool per process, grown on demand, one job
// at a time): a staged copy is cut into ~8 pieces per call, and starting and
// joining the threads per piece cost more than a 32 MiB piece's memcpy.
// Host copies of the staged paths with streaming (non-temporal) 16-byte stores:
// the destination is not read back soon (a user buffer filled from a stage, or
// a stage the DMA reads next), and ordinary stores would first read every line
// they write (read-for-ownership) -- a quarter of the host DRAM traffic of a
// staged copy (DMA write + copy read + write + that read).
void host_copy(uint8_t* dst, const uint8_t* src, uint64_t n, bool nt) {
#if !defined(__HIP_DEVICE_COMPILE__)
  if (nt && n >= 4096) {
    uint64_t h = (16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15;
    std::memcpy(dst, src, h);
    dst += h;
    src += h;
    n -= h;
    const uint64_t m = n & ~uint64_t(63);
    for (uint64_t i = 0; i < m; i += 64) {
      const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i));
      const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 16));
      const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 32));
      const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 48));
      _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), a);
      _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 16), b);
      _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 32), c);
      _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 48), d);
    }
    std::memcpy(dst + m, src + m, n - m);
    _mm_sfence();  // the streamed lines are globally visible before the copy counts as done
    return;
  }
#endif
  std::memcpy(dst, src, n);
}

class CopyPool {
 public:
  static CopyPool& get() {
    // never destroyed (its threads may be waiting at exit); a forked child, which has none of
    // the threads, starts a fresh pool
    static std::once_flag once;
    std::call_once(once, [] {
      inst_ = new CopyPool();
      pthread_atfork(nullptr, nullptr, [] { inst_ = new CopyPool(); });
    });
    return *inst_;
  }
  // slices 1 .. nt-1 on the workers, slice 0 on the caller
  void run(uint8_t* dst, const uint8_t* src, uint64_t n, uint64_t piece, unsigned nt, bool stream_st) {
    std::lock_guard<std::mutex> job(job_mu_);
    {
      std::unique_lock<std::mutex> lk(mu_);
      while (workers_ + 1 < nt) {
        const unsigned t = workers_++;
        const uint64_t g0 = gen_;  // the generation before this job: the new worker takes part in it
        std::thread([this, t, g0] { loop(t, g0); }).detach();
      }
      dst_ = dst;
      src_ = src;
      n_ = n;
      piece_ = piece;
      nt_ = nt;
      stream_st_ = stream_st;
      pending_ = nt - 1;
      ++gen_;
    }
    cv_.notify_all();
    host_copy(dst, src, std::min<uint64_t>(n, piece), stream_st);
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return pending_ == 0; });
  }

 private:
  void loop(unsigned t, uint64_t seen) {
    while (true) {
      uint8_t* dst;
      const uint8_t* src;
      uint64_t lo, hi;
      bool st;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (t + 1 >= nt_) continue;  // not part of this job
        dst = dst_;
        src = src_;
        st = stream_st_;
        lo = std::min<uint64_t>(n_, (uint64_t)(t + 1) * piece_);
        hi = std::min<uint64_t>(n_, lo + piece_);
      }
      if (hi > lo) host_copy(dst + lo, src + lo, hi - lo, st);
      std::lock_guard<std::mutex> lk(mu_);
      if (--pending_ == 0) done_cv_.notify_all();
    }
  }
  static inline CopyPool* inst_ = nullptr;
  std::mutex job_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  unsigned workers_ = 0, nt_ = 0, pending_ = 0;
  bool stream_st_ = true;
  uint64_t gen_ = 0, n_ = 0, piece_ = 0;
  uint8_t* dst_ = nullptr;
  const uint8_t* src_ = nullptr;
};

// stream_st: streaming stores (host_copy); off only for A/B (route copy_nt = -1)
void par_copy(uint8_t* dst, const uint8_t* src, uint64_t n, unsigned threads, bool stream_st = true) {
  const uint64_t min_piece = 2ull << 20;
  const unsigned nt = (unsigned)std::min<uint64_t>(threads, n / min_piece);
  if (nt <= 1) {
    if (n) host_copy(dst, src, n, stream_st);
    return;
  }
  const uint64_t piece = ((n + nt - 1) / nt + 4095) & ~uint64_t(4095);
  CopyPool::get().run(dst, src, n, piece, nt, stream_st);
}

// f(lo, hi) over [0, n) on up to `threads` threads (slices of at least 64Ki
// items): the batched import's per-string header pass.
template <class F>
void par_for(uint64_t n, unsigned threads, F&& f) {
  const unsigned nt = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(threads, n >> 16));
  if (nt <= 1) {
    f(uint64_t(0), n);
    return;
  }
  const uint64_t per = (n + nt - 1) / nt;
  std::vector<std::thread> th;
  th.reserve(nt - 1);
  for (unsigned t = 1; t < nt; ++t) th.emplace_back([&, t] { f(std::min(n, t * per), std::min(n, (t + 1) * per)); });
  f(uint64_t(0), std::min(n, per));
  for (auto& x : th) x.join();
}

// Allocates the pinned stages once per context; on failure the context
// copies from the pageable source instead (pin_off).
void ensure_pinned(rsk_ctx* c) {
  if (c->pin_off || c->h_pin[0]) return;
  const uint64_t bytes = c->stage_bytes + c->stage_bytes / 4;
  bool ok = hipHostMalloc(&c->h_pin[0], bytes, hipHostMallocDefault) == hipSuccess &&
            hipHostMalloc(&c->h_pin[1], bytes, hipHostMallocDefault) == hipSuccess &&
            hipMalloc(&c->d_pin[1], bytes) == hipSuccess &&
            hipEventCreateWithFlags(&c->pin_ev[0], hipEventDisableTiming) == hipSuccess &&
            hipEventCreateWithFlags(&c->pin_ev[1], hipEventDisableTiming) == hipSuccess;
  for (int r = 0; r < 8 && ok; ++r) ok = hipEventCreateWithFlags(&c->ring_ev[r], hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    (void)hipGetLastError();
    for (int b = 0; b < 2; ++b) {
      if (c->h_pin[b]) (void)hipHostFree(c->h_pin[b]);
      if (c->d_pin[b]) (void)hipFree(c->d_pin[b]);
      if (c->pin_ev[b]) (void)hipEventDestroy(c->pin_ev[b]);
      c->h_pin[b] = c->d_pin[b] = nullptr;
      c->pin_ev[b] = nullptr;
    }
    for (auto& e : c->ring_ev) {
      if (e) (void)hipEventDestroy(e);
      e = nullptr;
    }
    c->pin_off = true;
  }
}

// Bulk copies between device memory and a pageable host buffer through the
// two pinned stages: host threads copy one stage while the DMA of the other
// runs (the export / import of a pool's Redis strings: GBs at a time), in
// about 8 pieces per call (at least 8 MiB each), so the first copy and the
// last DMA, which nothing overlaps, stay short.
uint64_t staged_piece(const rsk_ctx* c, uint64_t bytes) {
  return std::min<uint64_t>(c->stage_bytes, std::max<uint64_t>(8ull << 20, ((bytes / 8) + 4095) & ~uint64_t(4095)));
}
// A stage may still feed a DMA an earlier h2d_staged queued (it returns with
// its copies in flight): both stages' last events are waited for first.
void pinned_idle(rsk_ctx* c) {
  for (int b = 0; b < 2; ++b) RSK_HIP(hipEventSynchronize(c->pin_ev[b]));
}
// The SDMA engines of the batched export's device->host copies and the batched import's
// host->device ones (rsk_ctx::d2h_engine / h2d_engine).  The engine the runtime picks is not
// the fastest on every box: round 6 measured one engine at 26-30 GB/s both ways and its
// neighbours at 57 on some boxes (profiles/r06_sdma_engines.jsonl), so each of the first 8
// engines the runtime reports free moves a 4 MiB warm-up and then 32 MiB between a device
// scratch and a pinned stage in each direction, once per context (~15 ms), and the fastest per
// direction is kept.  Anything the runtime refuses: HIP's copies (-1).
static hsa_status_t first_cpu_agent(hsa_agent_t a, void* out) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
    *static_cast<hsa_agent_t*>(out) = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

// one copy of `bytes` on engine e, signal g (1 while in flight): device->host, or host->device
static bool engine_copy(rsk_ctx* c, int e, hsa_signal_t g, void* to, const void* from, uint64_t bytes,
                        bool to_host = true) {
  hsa_signal_store_relaxed(g, 1);
  return hsa_amd_memory_async_copy_on_engine(to, to_host ? c->cpu_agent : c->gpu_agent, from,
                                             to_host ? c->gpu_agent : c->cpu_agent, bytes, 0, nullptr, g,
                                             (hsa_amd_sdma_engine_id_t)(1u << e), false) == HSA_STATUS_SUCCESS;
}
static hsa_signal_value_t engine_wait(hsa_signal_t g) {
  hsa_signal_value_t v;
  while ((v = hsa_signal_wait_scacquire(g, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE)) >= 1) {
  }
  return v;
}

void measure_copy_engines(rsk_ctx* c) {
  c->d2h_engine = c->h2d_engine = -1;
  if (hsa_init() != HSA_STATUS_SUCCESS) return;  // (the runtime HIP runs on: a reference, never shut down)
  const uint64_t B = c->stage_bytes + c->stage_bytes / 4;
  const uint64_t warm = std::min<uint64_t>(4ull << 20, B), big = std::min<uint64_t>(32ull << 20, B);
  uint8_t* d = nullptr;
  if (hipMalloc(&d, big) != hipSuccess) {
    (void)hipGetLastError();
    return;
  }
  hsa_amd_pointer_info_t info{};
  info.size = sizeof(info);
  hsa_agent_t cpu{};
  bool ok = hsa_amd_pointer_info(d, &info, nullptr, nullptr, nullptr) == HSA_STATUS_SUCCESS &&
            info.type == HSA_EXT_POINTER_TYPE_HSA && hsa_iterate_agents(first_cpu_agent, &cpu) == HSA_STATUS_INFO_BREAK;
  for (int j = 0; j < 8 && ok; ++j)
    if (!c->eng_sig[j].handle) ok = hsa_signal_create(0, 0, nullptr, &c->eng_sig[j]) == HSA_STATUS_SUCCESS;
  if (ok) {
    c->gpu_agent = info.agentOwner;
    c->cpu_agent = cpu;
    for (int dir = 0; dir < 2; ++dir) {  // 0: device -> host, 1: host -> device
      const bool to_host = dir == 0;
      uint32_t mask = 0;
      if ((to_host ? hsa_amd_memory_copy_engine_status(cpu, c->gpu_agent, &mask)
                   : hsa_amd_memory_copy_engine_status(c->gpu_agent, cpu, &mask)) != HSA_STATUS_SUCCESS)
        mask = 0xFF;
      float* rate = to_host ? c->d2h_rate : c->h2d_rate;
      int& pick = to_host ? c->d2h_engine : c->h2d_engine;
      float best = 0;
      void* to = to_host ? (void*)c->h_pin[0] : (void*)d;
      const void* from = to_host ? (const void*)d : (const void*)c->h_pin[0];
      for (int e = 0; e < 8; ++e) {
        if (!(mask >> e & 1)) continue;
        const hsa_signal_t g = c->eng_sig[0];
        if (!engine_copy(c, e, g, to, from, warm, to_host) || engine_wait(g) < 0) continue;
        const auto t0 = std::chrono::steady_clock::now();
        if (!engine_copy(c, e, g, to, from, big, to_host) || engine_wait(g) < 0) continue;
        const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        rate[e] = (float)(big / sec / 1e9);
        if (rate[e] > best) {
          best = rate[e];
          pick = e;
        }
      }
    }
  }
  (void)hipFree(d);
}

// The engine of this call's copies in one direction: route io_engine, else the measured
// fastest (-1: HIP's copies).
int copy_engine(rsk_ctx* c, bool to_host) {
  if (c->tune.io_engine < 0) return -1;
  ensure_pinned(c);
  if (c->pin_off) return -1;
  if (c->d2h_engine == -2) {
    pinned_idle(c);  // (the measurement uses a stage)
    measure_copy_engines(c);
  }
  if (!c->gpu_agent.handle) return -1;
  return c->tune.io_engine > 0 ? std::min(c->tune.io_engine - 1, 15) : to_host ? c->d2h_engine : c->h2d_engine;
}
int export_engine(rsk_ctx* c) { return copy_engine(c, true); }

// A large pageable host buffer (>= 256 MiB: a checkpoint's strings) pinned in place for one call
// (hipHostRegister, a few ms for 2 GB) so the call's copies go to / from it by DMA instead of
// through the pinned stages and a host copy, which is bound by the box's host memory (round 6:
// the C5 export 80-85 ms staged against 44-48 registered on such a box); unpinned when the call
// ends.  Not possible (pinned by someone else, too little lockable memory, route io_pin = -1):
// the staged copies.
struct CallPin {
  rsk_ctx* c = nullptr;
  void* p = nullptr;
  void pin(rsk_ctx* cc, const void* ptr, uint64_t bytes) {
    if (!ptr || bytes < (256ull << 20) || cc->tune.io_pin < 0 || cc->host_registered(ptr, bytes)) return;
    void* q = const_cast<void*>(ptr);  // (registering does not write the range)
    if (hipHostRegister(q, bytes, hipHostRegisterDefault) != hipSuccess) {
      (void)hipGetLastError();
      return;
    }
    c = cc;
    p = q;
    c->host_regs.push_back({reinterpret_cast<uintptr_t>(q), bytes, reg_dptr(q)});
  }
  ~CallPin() {
    if (!p) return;
    (void)hipStreamSynchronize(c->xin);  // no DMA may still use it
    (void)hipStreamSynchronize(c->xout);
    (void)hipStreamSynchronize(c->stream);
    auto& v = c->host_regs;
    for (size_t i = 0; i < v.size(); ++i)
      if (v[i].base == reinterpret_cast<uintptr_t>(p)) {
        v.erase(v.begin() + (long)i);
        break;
      }
    (void)hipHostUnregister(p);
  }
};

// Pageable (or registered) host -> device on SDMA engine `engine` through the two pinned stages:
// a ring of NS slots of S bytes, a host copy into each slot while the engine moves the previous
// one, each piece's completion a signal; a registered range is copied straight from (no slot).
// put() returns with the pieces issued (their host copies done); wait_upto(mark) waits for the
// pieces issued before mark -- the device work that reads them is launched after that.
class H2DStream {
 public:
  H2DStream(rsk_ctx* c, int engine, uint64_t piece) : c_(c), eng_(engine), S_(piece) {
    pinned_idle(c);  // (a stage may still feed an earlier HIP copy)
    const uint64_t B = c->stage_bytes + c->stage_bytes / 4;
    const uint32_t per = (uint32_t)std::min<uint64_t>(4, std::max<uint64_t>(1, B / S_));
    NS_ = 2 * (per >= 4 ? 4 : per >= 2 ? 2 : 1);
  }
  void put(uint8_t* dst, const uint8_t* src, uint64_t bytes) {
    const rsk_ctx::HostReg* reg = c_->host_reg(src, bytes);
    if (reg && !reg->dptr) reg = nullptr;
    for (uint64_t o = 0; o < bytes; o += S_) {
      const uint64_t m = std::min<uint64_t>(S_, bytes - o);
      if (issued_ - done_ == NS_) wait_upto(done_ + 1);  // the slot (and signal) this piece takes is free
      const uint32_t j = (uint32_t)(issued_ % NS_);
      const void* from;
      if (reg) {
        from = reinterpret_cast<const void*>(reg->dptr + (reinterpret_cast<uintptr_t>(src + o) - reg->base));
      } else {
        par_copy(slot(j), src + o, m, c_->stage_threads, c_->tune.copy_nt >= 0);
        from = slot(j);
      }
      if (!engine_copy(c_, eng_, c_->eng_sig[j], dst + o, from, m, false)) {
        hsa_signal_store_relaxed(c_->eng_sig[j], 0);  // (never issued)
        fail(RSK_ERR_DEVICE, "host->device copy on SDMA engine " + std::to_string(eng_) + " refused");
      }
      ++issued_;
    }
  }
  uint64_t issued() const { return issued_; }
  void wait_upto(uint64_t mark) {
    for (; done_ < mark; ++done_)
      if (engine_wait(c_->eng_sig[done_ % NS_]) < 0) {
        ++done_;
        fail(RSK_ERR_DEVICE, "host->device copy on an SDMA engine failed");
      }
  }
  ~H2DStream() {  // unwound by an error: no DMA may still read a stage or write the device
    for (; done_ < issued_; ++done_) (void)engine_wait(c_->eng_sig[done_ % NS_]);
  }

 private:
  uint8_t* slot(uint32_t j) const { return c_->h_pin[j & 1] + (uint64_t)(j >> 1) * S_; }
  rsk_ctx* c_;
  int eng_;
  uint64_t S_, issued_ = 0, done_ = 0;
  uint32_t NS_ = 2;
};

// Device -> pageable host through the two pinned stages, as a stream of
// pieces that may span several calls of put(): a ring of NS slots over the two
// stages (2, 4 or 8: as many pieces of S as they hold), the DMAs of up to
// NS - 1 pieces queued ahead of the host copy-out, so the copy engine never
// waits for the host between pieces -- nor between the chunks of a batched
// export, whose pieces go through one stream (drain() at the end).  The DMAs
// go on stream `s`, or with engine >= 0 straight to that SDMA engine (HSA
// copies, each piece's completion a signal; the host orders them after the
// device work that wrote their source, and order_after() orders the device
// work that overwrites it after them).  Pieces for a registered range go
// straight into it (on an engine: in ring pieces, with no copy-out).
class D2HStream {
 public:
  D2HStream(rsk_ctx* c, hipStream_t s, uint64_t piece, int engine = -1) : c_(c), s_(s) {
    ensure_pinned(c);
    if (c->pin_off) return;
    pinned_idle(c);  // a stage may still feed a DMA an earlier h2d_staged queued
    eng_ = engine;
    S_ = piece;
    const uint64_t B = c->stage_bytes + c->stage_bytes / 4;
    const uint32_t per = (uint32_t)std::min<uint64_t>(4, std::max<uint64_t>(1, B / S_));
    NS_ = 2 * (per >= 4 ? 4 : per >= 2 ? 2 : 1);
  }
  // bytes from device src to host dst, after event `after` (when not null)
  void put(uint8_t* dst, const uint8_t* src, uint64_t bytes, hipEvent_t after) {
    const rsk_ctx::HostReg* reg = c_->pin_off ? nullptr : c_->host_reg(dst, bytes);
    if (eng_ >= 0 && (!reg || reg->dptr)) {
      if (after) service_until(after);  // the source is written (copy-outs meanwhile)
      for (uint64_t o = 0; o < bytes; o += S_) {
        const uint64_t m = std::min<uint64_t>(S_, bytes - o);
        if (fifo_n_ == NS_ - 1) pop();
        const uint32_t j = (uint32_t)(issued_++ % NS_);
        void* to = reg ? reinterpret_cast<void*>(reg->dptr + (reinterpret_cast<uintptr_t>(dst + o) - reg->base)) : slot(j);
        fifo_[(head_ + fifo_n_++) % 8] = Piece{dst + o, m, j, reg != nullptr};
        if (!engine_copy(c_, eng_, c_->eng_sig[j], to, src + o, m)) {
          hsa_signal_store_relaxed(c_->eng_sig[j], 0);  // (never issued)
          fail(RSK_ERR_DEVICE, "device->host copy on SDMA engine " + std::to_string(eng_) + " refused");
        }
      }
      return;
    }
    if (after) RSK_HIP(hipStreamWaitEvent(s_, after, 0));
    if (c_->pin_off || reg) {  // (a registered range: DMA straight into it)
      if (bytes) RSK_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s_));
      return;
    }
    for (uint64_t o = 0; o < bytes; o += S_) {
      const uint64_t m = std::min<uint64_t>(S_, bytes - o);
      if (fifo_n_ == NS_ - 1) pop();  // the slot this piece takes was copied out by then
      const uint32_t j = (uint32_t)(issued_++ % NS_);
      RSK_HIP(hipMemcpyAsync(slot(j), src + o, m, hipMemcpyDeviceToHost, s_));
      RSK_HIP(hipEventRecord(c_->ring_ev[j], s_));
      fifo_[(head_ + fifo_n_++) % 8] = Piece{dst + o, m, j, false};
    }
  }
  // wait for event e, copying out the pieces whose DMA is done meanwhile (the ring keeps moving)
  void service_until(hipEvent_t e) {
    while (true) {
      const hipError_t q = hipEventQuery(e);
      if (q == hipSuccess) return;
      if (q != hipErrorNotReady) RSK_HIP(q);
      if (fifo_n_ && done(fifo_[head_].slot)) pop();
      else std::this_thread::yield();
    }
  }
  // pieces put so far (a mark for order_after)
  uint64_t issued() const { return issued_; }
  // the device work queued on stream s next may overwrite the sources of the pieces put before
  // `mark`: after event ev (recorded on this stream behind them) and, on an engine, once they are done
  void order_after(uint64_t mark, hipEvent_t ev, hipStream_t s) {
    RSK_HIP(hipStreamWaitEvent(s, ev, 0));
    if (eng_ >= 0)
      while (issued_ - fifo_n_ < mark) pop();
  }
  ~D2HStream() {  // unwound by an error: no DMA may still fill a stage the next call refills
    if (!fifo_n_) return;
    if (eng_ < 0) {
      (void)hipStreamSynchronize(s_);
      return;
    }
    for (uint32_t i = 0; i < fifo_n_; ++i) (void)engine_wait(c_->eng_sig[fifo_[(head_ + i) % 8].slot]);
    (void)hipStreamSynchronize(s_);
  }
  // every piece copied out, the stream synchronised
  void drain() {
    while (fifo_n_) pop();
    RSK_HIP(hipStreamSynchronize(s_));
  }

 private:
  struct Piece {
    uint8_t* dst;
    uint64_t bytes;
    uint32_t slot;
    bool direct;  // DMA'd into its destination: nothing to copy out
  };
  uint8_t* slot(uint32_t j) const { return c_->h_pin[j & 1] + (uint64_t)(j >> 1) * S_; }
  bool done(uint32_t j) const {
    return eng_ >= 0 ? hsa_signal_load_scacquire(c_->eng_sig[j]) < 1 : hipEventQuery(c_->ring_ev[j]) == hipSuccess;
  }
  void pop() {
    const Piece p = fifo_[head_];
    head_ = (head_ + 1) % 8;
    --fifo_n_;
    if (eng_ >= 0) {
      if (engine_wait(c_->eng_sig[p.slot]) < 0) fail(RSK_ERR_DEVICE, "device->host copy on an SDMA engine failed");
    } else {
      RSK_HIP(hipEventSynchronize(c_->ring_ev[p.slot]));
    }
    if (!p.direct) par_copy(p.dst, slot(p.slot), p.bytes, c_->stage_threads, c_->tune.copy_nt >= 0);
  }
  rsk_ctx* c_;
  hipStream_t s_;
  int eng_ = -1;
  uint64_t S_ = 0, issued_ = 0;
  uint32_t NS_ = 2, head_ = 0, fifo_n_ = 0;
  Piece fifo_[8] = {};
};

// The other way; returns with the copies queued on the stream (ordered
// before the caller's next launch).
// On stream s; consecutive calls keep the link busy (a stage is refilled as
// soon as the DMA that last read it is done, whichever call issued it).
void h2d_staged_on(rsk_ctx* c, hipStream_t s, uint8_t* dst, const uint8_t* src, uint64_t bytes) {
  ensure_pinned(c);
  if (c->pin_off || c->host_registered(src, bytes)) {  // (a registered range: DMA straight from it)
    if (bytes) RSK_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
    return;
  }
  const uint64_t S = staged_piece(c, bytes);
  for (uint64_t o = 0, k = 0; o < bytes; o += S, ++k) {
    const int slot = (int)(k & 1);
    const uint64_t n = std::min<uint64_t>(S, bytes - o);
    RSK_HIP(hipEventSynchronize(c->pin_ev[slot]));  // the DMA that last read this stage is done
    par_copy(c->h_pin[slot], src + o, n, c->stage_threads, c->tune.copy_nt >= 0);
    RSK_HIP(hipMemcpyAsync(dst + o, c->h_pin[slot], n, hipMemcpyHostToDevice, s));
    RSK_HIP(hipEventRecord(c->pin_ev[slot], s));
  }
}
void h2d_staged(rsk_ctx* c, uint8_t* dst, const uint8_t* src, uint64_t bytes) {
  h2d_staged_on(c, c->stream, dst, src, bytes);
}

// Calls fn(dev_keys, first_index, count) over the batch; host batches are
// copied through the staging buffers in whole-key chunks.  On return every
// chunk's work has completed.
// Leaves the context stream drained when a call exits by exception, so no
// queued copy still reads a pinned stage the next call refills (and no queued
// kernel consumes the next call's keys).
struct DrainOnThrow {
  rsk_ctx* c;
  ~DrainOnThrow() {
    if (std::uncaught_exceptions() > 0) (void)hipStreamSynchronize(c->stream);
  }
};

template <class F>
void for_each_chunk(rsk_ctx* c, const rsk_keys* k, F&& fn) {
  check_keys(c, k);
  DrainOnThrow drain{c};
  if (k->n == 0) return;
  if (k->location == RSK_MEM_DEVICE) {
    fn(DevKeys{reinterpret_cast<const uint8_t*>(k->data), k->offsets, k->n, k->fixed_len}, 0, k->n);
    return;
  }
  ensure_stage(c);
  ensure_pinned(c);
  const bool pinned = !c->pin_off;
  uint8_t* const dbuf[2] = {c->d_stage, pinned ? c->d_pin[1] : c->d_stage};
  const uint64_t off_cap = c->stage_bytes / 4 / 8 - 1;  // keys per chunk (offsets)
  const uint8_t* src = reinterpret_cast<const uint8_t*>(k->data);
  // One host->device copy of a chunk's bytes: through the free pinned stage,
  // or straight from the source when the context has none.
  auto h2d = [&](int slot, uint64_t at, const void* from, uint64_t bytes) {
    if (!bytes) return;
    if (pinned) {
      par_copy(c->h_pin[slot] + at, reinterpret_cast<const uint8_t*>(from), bytes, c->stage_threads);
      RSK_HIP(hipMemcpyAsync(dbuf[slot] + at, c->h_pin[slot] + at, bytes, hipMemcpyHostToDevice, c->stream));
    } else {
      RSK_HIP(hipMemcpyAsync(dbuf[slot] + at, from, bytes, hipMemcpyHostToDevice, c->stream));
    }
  };
  uint64_t first = 0;
  int slot = 0;
  bool recorded[2] = {false, false};  // earlier calls ended with a stream sync
  // A large batch (>= 64 MiB) goes up on the SDMA engine measured fastest (copy_engine): chunk
  // k's copies are issued, then chunk k - 1's work is launched once its copies are in (so the
  // engine moves chunk k while the host launches k - 1); pin_ev[slot], recorded behind a chunk's
  // work, frees its stage for chunk k + 2.
  const uint64_t total = k->offsets ? k->offsets[k->n] - k->offsets[0] + 8 * (k->n + 1) : k->n * k->fixed_len;
  const int eng = pinned && total >= (64ull << 20) ? copy_engine(c, false) : -1;
  if (eng >= 0) {
    RSK_HIP(hipStreamSynchronize(c->stream));  // (no earlier work may still use a device stage)
    struct Chunk {
      bool on = false;
      int slot = 0;
      uint64_t first = 0, m = 0, base = 0;
      bool copies[2] = {false, false};  // data, offsets: their signals are eng_sig[2 * slot + i]
    } pend;
    struct WaitCopies {  // unwound by an error: no engine copy may still write a stage
      rsk_ctx* c;
      Chunk* p;
      Chunk* q;
      ~WaitCopies() {
        for (Chunk* x : {p, q})
          for (int i = 0; i < 2; ++i)
            if (x->on && x->copies[i]) (void)engine_wait(c->eng_sig[2 * x->slot + i]);
      }
    };
    Chunk cur;
    WaitCopies wc{c, &pend, &cur};
    auto issue = [&](int sl, int i, uint64_t at, const void* from, uint64_t bytes) {
      if (!bytes) return;
      par_copy(c->h_pin[sl] + at, reinterpret_cast<const uint8_t*>(from), bytes, c->stage_threads);
      cur.copies[i] = true;
      if (!engine_copy(c, eng, c->eng_sig[2 * sl + i], dbuf[sl] + at, c->h_pin[sl] + at, bytes, false)) {
        cur.copies[i] = false;
        fail(RSK_ERR_DEVICE, "host->device copy on SDMA engine " + std::to_string(eng) + " refused");
      }
    };
    auto launch = [&](Chunk& ch) {  // its copies in, then its work on the context stream
      for (int i = 0; i < 2; ++i)
        if (ch.copies[i]) {
          ch.copies[i] = false;
          if (engine_wait(c->eng_sig[2 * ch.slot + i]) < 0) fail(RSK_ERR_DEVICE, "host->device copy on an SDMA engine failed");
        }
      uint8_t* d_data = dbuf[ch.slot];
      if (k->offsets == nullptr) {
        fn(DevKeys{d_data, nullptr, ch.m, k->fixed_len}, ch.first, ch.m);
      } else {
        fn(DevKeys{d_data - ch.base, reinterpret_cast<uint64_t*>(d_data + c->stage_bytes), ch.m, 0}, ch.first, ch.m);
      }
      RSK_HIP(hipEventRecord(c->pin_ev[ch.slot], c->stream));
      recorded[ch.slot] = true;
      ch.on = false;
    };
    while (first < k->n) {
      if (recorded[slot]) RSK_HIP(hipEventSynchronize(c->pin_ev[slot]));  // chunk k - 2's work is done with it
      cur = Chunk{};
      cur.on = true;
      cur.slot = slot;
      cur.first = first;
      if (k->offsets == nullptr) {
        uint64_t m = k->fixed_len ? c->stage_bytes / k->fixed_len : k->n;
        m = std::min<uint64_t>(m, k->n - first);
        need(m > 0, "key longer than the staging buffer");
        cur.m = m;
        issue(slot, 0, 0, src + first * k->fixed_len, m * k->fixed_len);
      } else {
        const uint64_t base = k->offsets[first];
        const uint64_t lim = std::min<uint64_t>(k->n - first, off_cap);
        const uint64_t* o = k->offsets + first;
        const uint64_t m = (uint64_t)(std::upper_bound(o + 1, o + lim + 1, base + c->stage_bytes) - (o + 1));
        need(m > 0, "key longer than the staging buffer");
        need(k->offsets[first + m] >= base, "offsets must be non-decreasing");
        cur.m = m;
        cur.base = base;
        issue(slot, 1, c->stage_bytes, k->offsets + first, (m + 1) * 8);
        issue(slot, 0, 0, src + base, k->offsets[first + m] - base);
      }
      if (pend.on) launch(pend);
      pend = cur;
      cur.on = false;
      first += pend.m;
      slot ^= 1;
    }
    if (pend.on) launch(pend);
    RSK_HIP(hipStreamSynchronize(c->stream));
    return;
  }
  while (first < k->n) {
    // The pinned stage is free once the DMA that last read it has finished.
    if (pinned && recorded[slot]) RSK_HIP(hipEventSynchronize(c->pin_ev[slot]));
    uint8_t* d_data = dbuf[slot];
    uint64_t* d_offs = reinterpret_cast<uint64_t*>(d_data + c->stage_bytes);
    uint64_t m;
    if (k->offsets == nullptr) {
      m = k->fixed_len ? c->stage_bytes / k->fixed_len : k->n;
      m = std::min<uint64_t>(m, k->n - first);
      need(m > 0, "key longer than the staging buffer");
      if (k->fixed_len) h2d(slot, 0, src + first * k->fixed_len, m * k->fixed_len);
      if (pinned) RSK_HIP(hipEventRecord(c->pin_ev[slot], c->stream));
      recorded[slot] = pinned;
      fn(DevKeys{d_data, nullptr, m, k->fixed_len}, first, m);
    } else {
      const uint64_t base = k->offsets[first];
      uint64_t lim = std::min<uint64_t>(k->n - first, off_cap);
      // largest m <= lim with offsets[first+m] - base <= stage_bytes
      const uint64_t* o = k->offsets + first;
      m = (uint64_t)(std::upper_bound(o + 1, o + lim + 1, base + c->stage_bytes) - (o + 1));
      need(m > 0, "key longer than the staging buffer");
      need(k->offsets[first + m] >= base, "offsets must be non-decreasing");
      h2d(slot, c->stage_bytes, k->offsets + first, (m + 1) * 8);
      h2d(slot, 0, src + base, k->offsets[first + m] - base);
      if (pinned) RSK_HIP(hipEventRecord(c->pin_ev[slot], c->stream));
      recorded[slot] = pinned;
      // Offsets stay absolute: shift the data pointer instead of rebasing.
      fn(DevKeys{d_data - base, d_offs, m, 0}, first, m);
    }
    // Without pinned stages the single device stage is reused by the next
    // chunk (and the pageable copy is host-synchronous anyway).
    if (!pinned) RSK_HIP(hipStreamSynchronize(c->stream));
    first += m;
    slot ^= 1;
  }
  RSK_HIP(hipStreamSynchronize(c->stream));
}

void check_hll(const rsk_hll* h, uint64_t id) {
  need(h != nullptr, "hll handle is NULL");
  need(id < h->n, "sketch id out of range");
  CtxLock l(h->ctx);                   // the pool's host state is the context's
  rsk::hll_materialize_ids(h, &id, 1);  // every caller reads or writes this row's registers
  rsk::hll_touch(h);        // conservatively: every caller may write them
}

// check_hll for a batch of ids of one pool: ranges checked in one pass, the
// pool materialised and touched once (10^5-pair countWith / mergeWith batches).
// writes: the caller may write registers (its precomputed PFCOUNTs are retired); read-only
// callers (count, countWith) keep them.
void check_hll_ids(const rsk_hll* h, const uint64_t* a, uint64_t na, const uint64_t* b = nullptr, uint64_t nb = 0,
                   bool writes = true) {
  need(h != nullptr, "hll handle is NULL");
  uint64_t bad = 0;
  for (uint64_t i = 0; i < na; ++i) bad |= a[i] >= h->n;
  for (uint64_t i = 0; i < nb; ++i) bad |= b[i] >= h->n;
  need(!bad, "sketch id out of range");
  CtxLock l(h->ctx);
  rsk::hll_materialize_ids(h, a, na);  // the rows these calls read or write (a partial lazy clear)
  if (nb) rsk::hll_materialize_ids(h, b, nb);
  if (writes) rsk::hll_touch(h);
}

uint8_t* regs_of(rsk_hll* h, uint64_t id) { return h->d_regs + id * (uint64_t)HLL_REGS; }

// Redis createHLLObject: registers zero, card bytes zero (cache valid = 0).
void create_if_missing(rsk_hll* h, uint64_t id, bool* created) {
  *created = !h->exists[id];
  h->exists[id] = 1;
}

// card[7] |= 0x80 (HLL_INVALIDATE_CACHE) for one sketch, on the stream.
__global__ void invalidate_kernel(uint64_t* card, const uint32_t* flag, int force) {
  if (force || (flag && *flag)) *card |= (1ull << 63);
}

__global__ void invalidate_list_kernel(uint64_t* card, const uint64_t* ids, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    atomicOr(reinterpret_cast<unsigned long long*>(card + ids[i]), 1ull << 63);
}

__global__ void invalidate_all_kernel(uint64_t* card, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    card[i] |= (1ull << 63);
}

void invalidate(rsk_hll* h, uint64_t id, const uint32_t* d_flag, bool force) {
  hipLaunchKernelGGL(invalidate_kernel, dim3(1), dim3(1), 0, h->ctx->stream, h->d_card + id, d_flag, force ? 1 : 0);
  RSK_CHECK_LAUNCH("invalidate");
}

// Redis sparse HLL payload (hyperloglog.c: ZERO 00xxxxxx run 1..64, XZERO
// 01xxxxxx yyyyyyyy run 1..16384, VAL 1vvvvvxx value 1..32 run 1..4), the
// canonical form: maximal runs, each cut into the longest opcodes.  Returns
// the payload length, 0 if a register exceeds 32 or cap is too small.
constexpr size_t HLL_SPARSE_MAX_BYTES = 3000;  // server.hll_sparse_max_bytes (whole string)
size_t encode_sparse(const uint8_t* raw, uint8_t* out, size_t cap) {
  size_t o = 0;
  for (int j = 0; j < HLL_REGS;) {
    const uint8_t v = raw[j];
    int run = 1;
    while (j + run < HLL_REGS && raw[j + run] == v) ++run;
    j += run;
    if (v > 32) return 0;
    while (run > 0) {
      if (v == 0 && run > 64) {
        const int l = run < 16384 ? run : 16384;
        if (o + 2 > cap) return 0;
        out[o++] = (uint8_t)(0x40 | ((l - 1) >> 8));
        out[o++] = (uint8_t)((l - 1) & 0xff);
        run -= l;
      } else if (v == 0) {
        if (o + 1 > cap) return 0;
        out[o++] = (uint8_t)(run - 1);
        run = 0;
      } else {
        const int l = run < 4 ? run : 4;
        if (o + 1 > cap) return 0;
        out[o++] = (uint8_t)(0x80 | ((v - 1) << 2) | (l - 1));
        run -= l;
      }
    }
  }
  return o;
}

// ------------------------------------------------ Java double semantics
int64_t java_d2l(double d) {
  if (std::isnan(d)) return 0;
  if (d >= 9223372036854775807.0) return INT64_MAX;
  if (d <= -9223372036854775808.0) return INT64_MIN;
  return (int64_t)d;
}
int32_t java_d2i(double d) {
  if (std::isnan(d)) return 0;
  if (d >= 2147483647.0) return INT32_MAX;
  if (d <= -2147483648.0) return INT32_MIN;
  return (int32_t)d;
}
int64_t java_round(double a) {
  if (a == 0x1.fffffffffffffp-2) return 0;
  return java_d2l(std::floor(a + 0.5));
}

// RedissonBloomFilter.optimalNumOfBits (:73-78).
int64_t optimal_bits(int64_t n, double p) {
  if (p == 0) p = 4.9e-324;  // Double.MIN_VALUE
  volatile double num = (double)(-n) * std::log(p);
  volatile double den = std::log(2.0) * std::log(2.0);
  return java_d2l(num / den);
}
// RedissonBloomFilter.optimalNumOfHashFunctions (:69-71).
int32_t optimal_k(int64_t n, int64_t m) {
  volatile double r = (double)m / (double)n;
  volatile double x = r * std::log(2.0);
  int32_t k = (int32_t)java_round(x);
  return k > 1 ? k : 1;
}

constexpr int64_t BLOOM_MAX_SIZE = 2147483647LL * 2;  // RedissonBloomFilter.java:52
constexpr int64_t BLOOM_EXT_MAX = 1LL << 44;          // 2 TiB of bits: beyond any single GPU

FastMod63 make_fastmod(uint64_t d) {
  FastMod63 f{};
  f.d = d;
  uint32_t l = 0;
  while (l < 64 && ((unsigned __int128)1 << l) < d) ++l;
  f.l = l;
  if (l == 0) {
    f.M = 0;
  } else {
    unsigned __int128 num = ((unsigned __int128)1 << (63 + l)) + d - 1;
    f.M = (uint64_t)(num / d);
  }
  f.r63 = d ? (uint64_t)((1ULL << 63) % d) : 0;
  return f;
}

// The submission number of the last asynchronous call issued so far.
uint64_t done_mark(rsk_ctx* c) {
  std::lock_guard<std::mutex> g(c->done_mu);
  return c->done_submitted;
}

// Waits until the completions of every call up to submission number `upto`
// have run (copy done, callback returned).  Callbacks may call back into the
// library (and take the context lock), so this must never run under the
// context lock: a thread holding it while waiting here would wait for a
// callback that waits for the lock.
void drain_done(rsk_ctx* c, uint64_t upto) {
  std::unique_lock<std::mutex> lk(c->done_mu);
  if (c->done_thr.get_id() == std::this_thread::get_id()) return;  // a callback calling in: do not wait for itself
  c->done_cv.wait(lk, [&] { return c->done_delivered >= upto; });
}

// Drains and joins the completion thread (the stream must be drained first,
// so no host function can queue another op).
void stop_done(rsk_ctx* c) {
  {
    std::lock_guard<std::mutex> g(c->done_mu);
    c->done_stop = true;
  }
  c->done_cv.notify_all();
  if (c->done_thr.joinable()) c->done_thr.join();
}

}  // namespace

namespace {
// Small host <-> device transfers by a kernel that reads or writes pinned host
// memory directly (mapped into the device's address space): queued on the
// context stream between kernels without going through a copy engine, so they
// never wait behind a bulk DMA queued on the copy streams (the batched export's
// per-chunk ids, flags, offsets and lengths).
__global__ __launch_bounds__(256) void xfer_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                   uint64_t n) {
  const uint64_t n4 = n / 4;
  const uint32_t* s4 = reinterpret_cast<const uint32_t*>(src);
  uint32_t* d4 = reinterpret_cast<uint32_t*>(dst);
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x)
    d4[i] = s4[i];
  const uint64_t t = 4 * n4 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) dst[t] = src[t];
}
void xfer(rsk_ctx* c, void* dst, const void* src, uint64_t n) {  // both 4-byte aligned
  if (!n) return;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>(512, (n / 4 + 255) / 256 + 1);
  hipLaunchKernelGGL(xfer_kernel, dim3(blocks), dim3(256), 0, c->stream, static_cast<const uint8_t*>(src),
                     static_cast<uint8_t*>(dst), n);
  RSK_CHECK_LAUNCH("xfer");
}

// Rows of a partial lazy clear, zeroed by id: one workgroup per row, 16-byte stores.
__global__ __launch_bounds__(256) void zero_rows_kernel(uint4* __restrict__ pool, const uint64_t* __restrict__ ids,
                                                        uint64_t n) {
  constexpr uint32_t ROW_U4 = rsk::HLL_REGS / 16;
  for (uint64_t r = blockIdx.x; r < n; r += gridDim.x) {
    uint4* dst = pool + ids[r] * ROW_U4;
    for (uint32_t q = threadIdx.x; q < ROW_U4; q += 256) dst[q] = make_uint4(0, 0, 0, 0);
  }
}

// Zero the given pending rows (ascending), clear their flags, and wait: runs
// of consecutive rows by memset when there are few, a row list otherwise (in a
// buffer of its own: the caller may hold the context's scratch).
void zero_pending_rows(const rsk_hll* h, const std::vector<uint64_t>& rows) {
  if (rows.empty()) return;
  rsk_ctx* c = h->ctx;
  rsk::ProfScope ps(c, "hll_clear");
  std::vector<std::pair<uint64_t, uint64_t>> runs;
  for (uint64_t id : rows) {
    if (!runs.empty() && runs.back().first + runs.back().second == id) ++runs.back().second;
    else runs.push_back({id, 1});
  }
  if (runs.size() <= 64) {
    for (const auto& r : runs)
      RSK_HIP(hipMemsetAsync(h->d_regs + r.first * (uint64_t)rsk::HLL_REGS, 0, r.second * (uint64_t)rsk::HLL_REGS,
                             c->stream));
    RSK_HIP(hipStreamSynchronize(c->stream));
  } else {
    uint64_t* d_ids = nullptr;
    RSK_HIP(hipMalloc(&d_ids, 8 * rows.size()));
    struct Free {
      uint64_t* p;
      ~Free() { (void)hipFree(p); }
    } fr{d_ids};
    RSK_HIP(hipMemcpyAsync(d_ids, rows.data(), 8 * rows.size(), hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(zero_rows_kernel, dim3((uint32_t)std::min<uint64_t>(rows.size(), 1u << 16)), dim3(256), 0,
                       c->stream, reinterpret_cast<uint4*>(h->d_regs), d_ids, (uint64_t)rows.size());
    RSK_CHECK_LAUNCH("zero_rows");
    RSK_HIP(hipStreamSynchronize(c->stream));
  }
  for (uint64_t id : rows) h->pend[id] = 0;
  h->pend_n -= rows.size();
  rsk::hll_touch(h);
}
}  // namespace

namespace rsk {
void hll_materialize(const rsk_hll* h) {
  if (h->pend_n) {
    CtxLock l(h->ctx);
    std::vector<uint64_t> rows;
    rows.reserve(h->pend_n);
    for (uint64_t g = 0; g < h->n; ++g)
      if (h->pend[g]) rows.push_back(g);
    zero_pending_rows(h, rows);
    return;
  }
  if (!h->pending_clear) return;
  CtxLock l(h->ctx);
  ProfScope ps(h->ctx, "hll_clear");
  RSK_HIP(hipMemsetAsync(h->d_regs, 0, h->n * (uint64_t)HLL_REGS, h->ctx->stream));
  h->pending_clear = false;
  hll_touch(h);
}

void hll_materialize_ids(const rsk_hll* h, const uint64_t* ids, uint64_t n) {
  if (h->pending_clear) return hll_materialize(h);
  if (!h->pend_n) return;
  CtxLock l(h->ctx);
  std::vector<uint64_t> rows;
  for (uint64_t i = 0; i < n; ++i)
    if (ids[i] < h->n && h->pend[ids[i]]) rows.push_back(ids[i]);
  std::sort(rows.begin(), rows.end());
  rows.erase(std::unique(rows.begin(), rows.end()), rows.end());
  zero_pending_rows(h, rows);
}

void hll_materialize_range(const rsk_hll* h, uint64_t first, uint64_t count) {
  if (h->pending_clear) return hll_materialize(h);
  if (!h->pend_n) return;
  CtxLock l(h->ctx);
  std::vector<uint64_t> rows;
  for (uint64_t g = first; g < first + count && g < h->n; ++g)
    if (h->pend[g]) rows.push_back(g);
  zero_pending_rows(h, rows);
}

void hll_pend_outside(const rsk_hll* h, uint64_t first, uint64_t count) {
  h->pend.assign(h->n, 1);
  std::fill(h->pend.begin() + first, h->pend.begin() + first + count, 0);
  h->pend_n = h->n - count;
}

void hll_unpend(const rsk_hll* h, const uint64_t* ids, uint64_t n) {
  if (!h->pend_n) return;
  for (uint64_t i = 0; i < n; ++i)
    if (h->pend[ids[i]]) {
      h->pend[ids[i]] = 0;
      --h->pend_n;
    }
}

void hll_touch(const rsk_hll* h) {
  h->zero = false;
  if (++h->pc_epoch == 0) {  // wrapped: clear every stamp so no stale one can match again
    RSK_HIP(hipMemsetAsync(h->d_pepoch, 0, 4 * h->n, h->ctx->stream));
    h->pc_epoch = 1;
  }
}
}  // namespace rsk

extern "C" {

int rsk_abi_version(void) { return RSK_ABI_VERSION; }
const char* rsk_last_error(void) { return rsk::g_last_error.c_str(); }

int rsk_init(const rsk_options* opts, rsk_ctx** out) {
  return guarded([&] {
    need(out != nullptr, "out is NULL");
    *out = nullptr;
    rsk_options o{};
    if (opts) o = *opts;
    if (o.redis_version == 0) o.redis_version = 320;
    need(o.redis_version == 320, "only Redis 3.2.0 semantics (redis_version = 320) are implemented");
    // Each stage holds stage_bytes of key bytes plus stage_bytes/4 of u64 offsets.
    need(o.staging_bytes == 0 || (o.staging_bytes >= (1ull << 20) && o.staging_bytes % 256 == 0),
         "staging_bytes must be 0 (default) or a multiple of 256 that is >= 1 MiB");
    need(o.stage_threads <= 64, "stage_threads must be in [0, 64]");
    need(o.reserved == 0, "rsk_options.reserved must be 0");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) fail(RSK_ERR_NO_DEVICE, "no HIP device visible");
    need(o.device >= 0 && o.device < ndev, "device ordinal out of range");
    hipDeviceProp_t prop;
    RSK_HIP(hipGetDeviceProperties(&prop, o.device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
      fail(RSK_ERR_NO_DEVICE, std::string("librsketch is built for gfx950 only; device is ") + prop.gcnArchName);
    auto* c = new rsk_ctx();
    std::unique_ptr<rsk_ctx> guard(c);
    c->device = o.device;
    c->num_cus = prop.multiProcessorCount;
    RSK_HIP(hipSetDevice(c->device));
    RSK_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    RSK_HIP(hipStreamCreateWithFlags(&c->xin, hipStreamNonBlocking));
    RSK_HIP(hipStreamCreateWithFlags(&c->xout, hipStreamNonBlocking));
    c->stage_bytes = o.staging_bytes ? o.staging_bytes : (256ull << 20);
    c->stage_threads = o.stage_threads ? o.stage_threads : 8;
    c->slab_count = std::min<uint32_t>(RSK_MAX_SLABS, 8u * (uint32_t)c->num_cus);
    RSK_HIP(hipMalloc(&c->d_slab, (uint64_t)c->slab_count * HLL_REGS));
    c->small_bytes = 1 << 20;
    RSK_HIP(hipMalloc(&c->d_small, c->small_bytes));
    RSK_HIP(hipHostMalloc(&c->h_small, c->small_bytes, hipHostMallocDefault));
    // Linear-counting table: m*log(m/ez), evaluated by the host libm exactly
    // as Redis's hllCount does (E = m*log(m/ez)).
    std::vector<double> lc(HLL_REGS + 1, 0.0);
    const double m = HLL_REGS;
    for (int ez = 1; ez <= HLL_REGS; ++ez) {
      volatile double q = m / ez;
      lc[ez] = m * std::log(q);
    }
    RSK_HIP(hipMalloc(&c->d_lc, lc.size() * sizeof(double)));
    RSK_HIP(hipMemcpy(c->d_lc, lc.data(), lc.size() * sizeof(double), hipMemcpyHostToDevice));
    *out = guard.release();
  });
}

int rsk_shutdown(rsk_ctx* c) {
  if (!c) return RSK_OK;
  int rc = guarded([&] {
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    if (c->xin) (void)hipStreamSynchronize(c->xin);
    if (c->xout) (void)hipStreamSynchronize(c->xout);
    stop_done(c);
    rsk::prof_fold(c);
    for (auto e : c->prof.free_events) (void)hipEventDestroy(e);
    (void)hipFree(c->d_stage);
    for (int b = 0; b < 2; ++b) {
      (void)hipHostFree(c->h_pin[b]);
      (void)hipFree(c->d_pin[b]);
      if (c->pin_ev[b]) (void)hipEventDestroy(c->pin_ev[b]);
    }
    for (hipEvent_t e : c->ring_ev)
      if (e) (void)hipEventDestroy(e);
    (void)hipFree(c->d_slab);
    (void)hipFree(c->d_small);
    (void)hipHostFree(c->h_small);
    if (c->h_io) (void)hipHostFree(c->h_io);
    if (c->h_batch) (void)hipHostFree(c->h_batch);
    (void)hipFree(c->d_work);
    (void)hipFree(c->d_out);
    (void)hipFree(c->d_xbuf);
    (void)hipFree(c->d_sbuf);
    (void)hipFree(c->d_hrows);
    (void)hipFree(c->d_cslow);
    (void)hipFree(c->d_lc);
    for (rsk::AsyncOp* op : c->async_all) {  // stream and completion queue drained: every op is idle
      if (op->h_buf) (void)hipHostFree(op->h_buf);
      if (op->h_res) (void)hipHostFree(op->h_res);
      if (op->d_buf) (void)hipFree(op->d_buf);
      if (op->ev_in) (void)hipEventDestroy(op->ev_in);
      if (op->ev_out) (void)hipEventDestroy(op->ev_out);
      delete op;
    }
    c->async_all.clear();
    c->async_free.clear();
    if (c->comm) (void)rsk_comm_destroy(c);
    for (const auto& r : c->host_regs) (void)hipHostUnregister(reinterpret_cast<void*>(r.base));
    c->host_regs.clear();
    for (hsa_signal_t& g : c->eng_sig)
      if (g.handle) (void)hsa_signal_destroy(g);
    (void)hipStreamDestroy(c->stream);
    if (c->xin) (void)hipStreamDestroy(c->xin);
    if (c->xout) (void)hipStreamDestroy(c->xout);
  });
  delete c;
  return rc;
}

void* rsk_ctx_stream(rsk_ctx* c) { return c ? (void*)c->stream : nullptr; }

int rsk_host_register(rsk_ctx* c, void* p, uint64_t bytes) {
  return guarded([&] {
    need(c && p && bytes, "NULL argument or empty range");
    CtxLock l(c);
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    for (const auto& r : c->host_regs)
      need(a + bytes <= r.base || a >= r.base + r.bytes, "range overlaps a registered one");
    RSK_HIP(hipHostRegister(p, bytes, hipHostRegisterDefault));
    c->host_regs.push_back({a, bytes, rsk::reg_dptr(p)});
  });
}

int rsk_host_unregister(rsk_ctx* c, void* p) {
  return guarded([&] {
    need(c && p, "NULL argument");
    CtxLock l(c);
    // no queued transfer may still use the range
    RSK_HIP(hipStreamSynchronize(c->stream));
    RSK_HIP(hipStreamSynchronize(c->xin));
    RSK_HIP(hipStreamSynchronize(c->xout));
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    auto it = std::find_if(c->host_regs.begin(), c->host_regs.end(), [&](const auto& r) { return r.base == a; });
    need(it != c->host_regs.end(), "not a registered range");
    c->host_regs.erase(it);
    RSK_HIP(hipHostUnregister(p));
  });
}

int rsk_trim(rsk_ctx* c) {
  return guarded([&] {
    need(c != nullptr, "ctx is NULL");
    CtxLock l(c);
    RSK_HIP(hipStreamSynchronize(c->stream));
    RSK_HIP(hipStreamSynchronize(c->xin));
    RSK_HIP(hipStreamSynchronize(c->xout));
    RSK_HIP(hipFree(c->d_work));
    RSK_HIP(hipFree(c->d_out));
    RSK_HIP(hipFree(c->d_xbuf));
    RSK_HIP(hipFree(c->d_sbuf));
    RSK_HIP(hipFree(c->d_hrows));
    RSK_HIP(hipFree(c->d_cslow));
    c->d_work = c->d_out = c->d_xbuf = c->d_sbuf = c->d_hrows = c->d_cslow = nullptr;
    c->work_bytes = c->out_bytes = c->xbuf_bytes = c->sbuf_bytes = c->hrows_bytes = c->cslow_bytes = 0;
    if (c->h_batch) RSK_HIP(hipHostFree(c->h_batch));
    c->h_batch = nullptr;
    c->h_batch_bytes = 0;
  });
}

int rsk_sync(rsk_ctx* c) {
  return guarded([&] {
    need(c != nullptr, "ctx is NULL");
    uint64_t upto;
    {
      CtxLock l(c);
      RSK_HIP(hipStreamSynchronize(c->stream));
      RSK_HIP(hipStreamSynchronize(c->xin));
      RSK_HIP(hipStreamSynchronize(c->xout));
      upto = done_mark(c);  // every call so far has reached the completion thread
    }
    // outside the lock: a callback still running may call into this context
    drain_done(c, upto);
    if (c->dead) fail(RSK_ERR_DEVICE, "the context's device work failed");
  });
}

int rsk_prof_enable(rsk_ctx* c, int on) {
  return guarded([&] {
    need(c != nullptr, "ctx is NULL");
    CtxLock l(c);
    c->prof.on = on != 0;
  });
}

int rsk_prof_reset(rsk_ctx* c) {
  return guarded([&] {
    need(c != nullptr, "ctx is NULL");
    CtxLock l(c);
    rsk::prof_fold(c);
    c->prof.totals.clear();
  });
}

int rsk_prof_read(rsk_ctx* c, const char* name, double* ms, uint64_t* launches) {
  return guarded([&] {
    need(c && name && ms && launches, "NULL argument");
    CtxLock l(c);
    rsk::prof_fold(c);
    auto it = c->prof.totals.find(name);
    *ms = it == c->prof.totals.end() ? 0.0 : it->second.ms;
    *launches = it == c->prof.totals.end() ? 0 : it->second.launches;
  });
}

// ------------------------------------------------------------------ HLL
int rsk_hll_create(rsk_ctx* c, uint64_t n, rsk_hll** out) {
  return guarded([&] {
    need(c && out, "NULL argument");
    need(n > 0, "n_sketches must be > 0");
    CtxLock l(c);
    *out = nullptr;
    auto* h = new rsk_hll();
    std::unique_ptr<rsk_hll> guard(h);
    h->ctx = c;
    h->n = n;
    h->exists.assign(n, 0);
    h->dense.assign(n, 0);
    RSK_HIP(hipMalloc(&h->d_regs, n * (uint64_t)HLL_REGS));
    RSK_HIP(hipMalloc(&h->d_card, n * 8));
    RSK_HIP(hipMalloc(&h->d_pcount, n * 8));
    RSK_HIP(hipMalloc(&h->d_pepoch, n * 4));
    RSK_HIP(hipMemsetAsync(h->d_pepoch, 0, n * 4, c->stream));
    RSK_HIP(hipMemsetAsync(h->d_regs, 0, n * (uint64_t)HLL_REGS, c->stream));
    RSK_HIP(hipMemsetAsync(h->d_card, 0, n * 8, c->stream));
    RSK_HIP(hipStreamSynchronize(c->stream));
    h->zero = true;
    *out = guard.release();
  });
}

int rsk_hll_destroy(rsk_hll* h) {
  if (!h) return RSK_OK;
  int rc = guarded([&] {
    CtxLock l(h->ctx);
    RSK_HIP(hipStreamSynchronize(h->ctx->stream));
    RSK_HIP(hipFree(h->d_regs));
    RSK_HIP(hipFree(h->d_card));
    RSK_HIP(hipFree(h->d_pcount));
    RSK_HIP(hipFree(h->d_pepoch));
  });
  delete h;
  return rc;
}

uint64_t rsk_hll_size(const rsk_hll* h) { return h ? h->n : 0; }

int rsk_hll_exists(rsk_hll* h, uint64_t id, int* out) {
  return guarded([&] {
    check_hll(h, id);
    need(out != nullptr, "out is NULL");
    *out = h->exists[id];
  });
}

int rsk_hll_delete(rsk_hll* h, uint64_t id) {
  return guarded([&] {
    check_hll(h, id);
    CtxLock l(h->ctx);
    hll_forget_import(h, id);
    RSK_HIP(hipMemsetAsync(regs_of(h, id), 0, HLL_REGS, h->ctx->stream));
    RSK_HIP(hipMemsetAsync(h->d_card + id, 0, 8, h->ctx->stream));
    h->exists[id] = 0;
    h->dense[id] = 0;
  });
}

int rsk_hll_clear(rsk_hll* h) {
  return guarded([&] {
    if (!h) throw RskError{RSK_ERR_INVALID_ARG, "NULL handle"};
    CtxLock l(h->ctx);
    hll_forget_imports(h);
    {
      ProfScope ps(h->ctx, "hll_clear");
      // registers: lazily (hll_materialize, or rewritten whole by the next grouped add)
      RSK_HIP(hipMemsetAsync(h->d_card, 0, h->n * 8, h->ctx->stream));
    }
    std::fill(h->exists.begin(), h->exists.end(), 0);
    std::fill(h->dense.begin(), h->dense.end(), 0);
    h->pending_clear = true;  // the whole pool: supersedes any partially pending rows
    h->pend.clear();
    h->pend_n = 0;
    h->zero = true;
  });
}

int rsk_hll_add(rsk_hll* h, uint64_t id, const rsk_keys* keys, uint8_t* changed_out) {
  return guarded([&] {
    check_hll(h, id);
    rsk_ctx* c = h->ctx;
    CtxLock l(c);
    check_keys(c, keys);  // before the key is created: a refused batch leaves it absent
    // An imported string stays the key's GET until a register changes (Redis
    // leaves the string alone after a PFADD that changes nothing).
    const bool had_import = h->imported.count(id) != 0;
    bool created;
    create_if_missing(h, id, &created);
    // The reduce kernel raises the flag to this call's epoch when a register
    // grows and invalidates the card cache itself: no memset, no extra launch.
    uint32_t* d_flag = reinterpret_cast<uint32_t*>(c->d_small);
    if (++c->epoch == 0) {  // wrapped: restart the epoch sequence from a clean flag
      RSK_HIP(hipMemsetAsync(d_flag, 0, 4, c->stream));
      c->epoch = 1;
    }
    const uint32_t epoch = c->epoch;
    bool any_chunk = false;
    for_each_chunk(c, keys, [&](const DevKeys& dk, uint64_t, uint64_t) {
      hll_add_launch(c, dk, regs_of(h, id), h->d_card + id, d_flag, epoch, created && !any_chunk);
      any_chunk = true;
    });
    if (!any_chunk && created) invalidate(h, id, nullptr, true);  // PFADD key (no elements) creates it
    if (changed_out || had_import) {
      RSK_HIP(hipMemcpyAsync(c->h_small, d_flag, 4, hipMemcpyDeviceToHost, c->stream));
      RSK_HIP(hipStreamSynchronize(c->stream));
      uint32_t f;
      std::memcpy(&f, c->h_small, 4);
      const bool changed = (f == epoch) || created;
      if (changed_out) *changed_out = (uint8_t)changed;
      if (changed) hll_forget_import(h, id);
    }
  });
}

int rsk_hll_add_each(rsk_hll* h, uint64_t id, const rsk_keys* keys, uint8_t* out) {
  return guarded([&] {
    check_hll(h, id);
    need(out != nullptr, "out is NULL");
    rsk_ctx* c = h->ctx;
    CtxLock l(c);
    bool created;
    check_keys(c, keys);
    check_out(c, keys, out);
    create_if_missing(h, id, &created);
    // Sub-chunks bounded for the 32-bit sort; replies compose sequentially.
    const uint64_t max_chunk = 1ull << 26;
    rsk_keys sub = *keys;
    uint64_t done = 0;
    while (done < keys->n) {
      uint64_t m = std::min<uint64_t>(max_chunk, keys->n - done);
      sub.n = m;
      if (keys->offsets) {
        sub.offsets = keys->offsets + done;
        sub.data = keys->data;
      } else {
        sub.offsets = nullptr;
        sub.data = reinterpret_cast<const uint8_t*>(keys->data) + done * keys->fixed_len;
      }
      for_each_chunk(c, &sub, [&](const DevKeys& dk, uint64_t first, uint64_t cnt) {
        uint8_t* d_out = keys->location == RSK_MEM_DEVICE ? out + done + first : out_scratch(c, cnt);
        hll_add_each_launch(c, dk, regs_of(h, id), d_out);
        if (keys->location == RSK_MEM_HOST) {
          RSK_HIP(hipMemcpyAsync(out + done + first, d_out, cnt, hipMemcpyDeviceToHost, c->stream));
          RSK_HIP(hipStreamSynchronize(c->stream));
        }
      });
      done += m;
    }
    // Any reply of 1 means a register grew: invalidate the cache.
    if (keys->n > 0) {
      if (keys->location == RSK_MEM_HOST) {
        bool any = created;
        for (uint64_t i = 0; i < keys->n && !any; ++i) any = out[i] != 0;
        if (any) invalidate(h, id, nullptr, true);
        if (any) hll_forget_import(h, id);  // a kept SET string survives PFADDs that change nothing (as rsk_hll_add)
        if (created) out[0] = 1;
      } else {
        // Device replies: cheap on-device OR via the flag word.
        invalidate(h, id, nullptr, true);  // conservative: a no-op PFADD keeps the old card bytes valid in Redis
        hll_forget_import(h, id);          // conservative too (device replies are not read back)
        if (created) RSK_HIP(hipMemsetAsync(out, 1, 1, c->stream));
      }
    } else if (created) {
      invalidate(h, id, nullptr, true);
    }
  });
}

}  // extern "C"

namespace {
// Grouped PFADD in pieces: the host marks the touched sketches (host group
// ids; device ids mark the whole pool), each chunk is launched, then every
// cache of the pool is invalidated.  A pending lazy clear is completed by the
// partitioned add's first launch (every row written); any other path zeroes
// the pool first.
void hll_mark_groups(rsk_hll* h, const uint32_t* groups, uint64_t n) {
  if (!groups) {
    std::fill(h->exists.begin(), h->exists.end(), 1);
    return;
  }
  for (uint64_t i = 0; i < n; ++i)
    if (groups[i] < h->n) h->exists[groups[i]] = 1;
}
// pool_zero: the pool was all zero when the call began (first chunk only).
void hll_add_grouped_chunk(rsk_hll* h, const DevKeys& dk, const uint32_t* d_groups, bool pool_zero) {
  rsk_ctx* c = h->ctx;
  const bool write_all = h->pending_clear && hll_grouped_partition_applies(c, dk, h->n);
  if (!write_all) hll_materialize(h);
  hll_touch(h);  // estimates of earlier chunks are stale once this one lands
  hll_add_grouped_launch(c, dk, d_groups, h->d_regs, h->n, pool_zero, write_all,
                         PCount{h->d_pcount, h->d_pepoch, h->pc_epoch});
  h->pending_clear = false;
}
void hll_add_grouped_finish(rsk_hll* h) {
  // Every pool member may have changed: invalidate all caches (card |= bit 63).
  hipLaunchKernelGGL(invalidate_all_kernel, dim3(256), dim3(256), 0, h->ctx->stream, h->d_card, h->n);
  RSK_CHECK_LAUNCH("invalidate_all");
}
// Device keys (any size) in one piece; host_groups (the caller's ids, when
// they are on the host) mark the sketches touched.
void hll_add_grouped_enqueue(rsk_hll* h, const DevKeys& dk, const uint32_t* d_groups, const uint32_t* host_groups) {
  hll_forget_imports(h);
  const bool pool_zero = h->zero;
  hll_touch(h);
  hll_add_grouped_chunk(h, dk, d_groups, pool_zero);
  hll_mark_groups(h, host_groups, dk.n);  // host bookkeeping after the launches: the device starts sooner
  hll_add_grouped_finish(h);
}
}  // namespace

extern "C" {

int rsk_hll_add_grouped(rsk_hll* h, const rsk_keys* keys, const uint32_t* groups) {
  return guarded([&] {
    need(h != nullptr, "hll handle is NULL");
    need(keys == nullptr || keys->n == 0 || groups != nullptr, "groups is NULL");
    rsk_ctx* c = h->ctx;
    CtxLock l(c);
    check_keys(c, keys);
    if (keys->n == 0) return;
    check_out(c, keys, groups);
    const bool host = keys->location == RSK_MEM_HOST;
    if (!host) {
      hll_add_grouped_enqueue(h, DevKeys{reinterpret_cast<const uint8_t*>(keys->data), keys->offsets, keys->n,
                                         keys->fixed_len},
                              groups, nullptr);
    } else {  // staged in chunks
      hll_forget_imports(h);
      const bool pool_zero = h->zero;
      hll_touch(h);
      hll_mark_groups(h, groups, keys->n);
      for_each_chunk(c, keys, [&](const DevKeys& dk, uint64_t first, uint64_t cnt) {
        auto* d_groups = reinterpret_cast<uint32_t*>(out_scratch(c, cnt * 4));
        RSK_HIP(hipMemcpyAsync(d_groups, groups + first, cnt * 4, hipMemcpyHostToDevice, c->stream));
        hll_add_grouped_chunk(h, dk, d_groups, pool_zero && first == 0);
      });
      hll_add_grouped_finish(h);
    }
    RSK_HIP(hipStreamSynchronize(c->stream));
  });
}

int rsk_hll_count(rsk_hll* h, const uint64_t* ids, uint64_t n, uint64_t* out) {
  return guarded([&] {
    need(h != nullptr && out != nullptr, "NULL argument");
    rsk_ctx* c = h->ctx;
    CtxLock l(c);
    if (ids) hll_materialize_ids(h, ids, n);
    else hll_materialize(h);
    if (n == 0) return;
    uint64_t* d_ids = nullptr;
    SmallIds small{};
    const bool by_value = ids && n <= 8;
    uint8_t* s = out_scratch(c, (ids ? n * 8 : 0) + n * 8 + 256);
    if (ids) {
      for (uint64_t i = 0; i < n; ++i) need(ids[i] < h->n, "sketch id out of range");
      if (by_value) {
        for (uint64_t i = 0; i < n; ++i) small.v[i] = ids[i];
        small.n = (uint32_t)n;
      } else {
        d_ids = reinterpret_cast<uint64_t*>(s);
        RSK_HIP(hipMemcpyAsync(d_ids, ids, n * 8, hipMemcpyHostToDevice, c->stream));
      }
    } else {
      need(n <= h->n, "n exceeds pool size");
    }
    uint64_t* d_out = reinterpret_cast<uint64_t*>(s + (ids ? ((n * 8 + 255) & ~255ull) : 0));
    hll_count_launch(c, h->d_regs, h->d_card, d_ids, small, n, d_out, PCount{h->d_pcount, h->d_pepoch, h->pc_epoch});
    if (n * 8 <= 4096) {  // small results come back through the pinned buffer
      RSK_HIP(hipMemcpyAsync(c->h_small + 4096, d_out, n * 8, hipMemcpyDeviceToHost, c->stream));
      RSK_HIP(hipStreamSynchronize(c->stream));
      std::memcpy(out, c->h_small + 4096, n * 8);
    } else {  // large ones (count of a whole pool: 8 MB at 10^6 sketches) through the
              // pinned per-call buffer: one full-speed DMA, then host threads copy out
      uint8_t* hb = c->pinned(n * 8);
      RSK_HIP(hipMemcpyAsync(hb, d_out, n * 8, hipMemcpyDeviceToHost, c->stream));
      RSK_HIP(hipStreamSynchronize(c->stream));
      par_copy(reinterpret_cast<uint8_t*>(out), hb, n * 8, c->stage_threads);
    }
  });
}

namespace {
// ptrs: n * arity member pointers, in pinned host memory (rsk_ctx::pinned)
// with n * 8 bytes after them for the results.
void union_impl(rsk_ctx* c, const uint8_t* const* ptrs, uint32_t arity, uint64_t n, uint64_t* out) {
  const uint64_t np = n * arity;
  uint8_t* s = out_scratch(c, np * 8 + n * 8 + 512);
  auto* d_ptrs = reinterpret_cast<const uint8_t**>(s);
  auto* d_out = reinterpret_cast<uint64_t*>(s + ((np * 8 + 255) & ~255ull));
  uint64_t* h_out = const_cast<uint64_t*>(reinterpret_cast<const uint64_t*>(ptrs + np));
  RSK_HIP(hipMemcpyAsync(d_ptrs, ptrs, np * 8, hipMemcpyHostToDevice, c->stream));
  hll_union_count_launch(c, d_ptrs, arity, n, d_out);
  RSK_HIP(hipMemcpyAsync(h_out, d_out, n * 8, hipMemcpyDeviceToHost, c->stream));
  RSK_HIP(hipStreamSynchronize(c->stream));
  std::memcpy(out, h_out, n * 8);
}
}  // namespace

namespace {
// rsk_hll_merge_batch(_async): PFMERGEs run in input order in Redis; a batch
// whose destinations are also sources of other pairs depends on that order.
// Level the pairs: a pair runs after the last writer of its source (RAW) and
// of its destination (WAW), and after the last reader of its destination
// (WAR).  Pairs of one level are independent and run as one launch.
// Per-sketch last writer / last reader levels live in one flat per-pool
// array, reset lazily by an epoch stamp (no hashing, no clearing).
uint64_t merge_batch_seg(uint64_t n) { return (8 * n + 255) & ~255ull; }
uint64_t merge_batch_host_bytes(uint64_t n) { return 3 * merge_batch_seg(n) + 4 * n + 256; }
uint64_t merge_batch_dev_bytes(uint64_t n) { return 3 * merge_batch_seg(n) + 512; }

void merge_batch_check(rsk_hll* h, const uint64_t* dst_ids, const uint64_t* src_ids, uint64_t n) {
  check_hll_ids(h, dst_ids, n, src_ids, n);
}

// hb: pinned host buffer of merge_batch_host_bytes(n); d: device scratch of
// merge_batch_dev_bytes(n) -- pointer arrays built in hb, one DMA, one merge
// launch per level, one cache invalidation for the batch.
void op_stage_in(AsyncOp* op, void* dst, const void* src, uint64_t bytes);  // (below)

void merge_batch_enqueue(rsk_hll* h, const uint64_t* dst_ids, const uint64_t* src_ids, uint64_t n, uint8_t* hb,
                         uint8_t* d, AsyncOp* op = nullptr) {
  rsk_ctx* c = h->ctx;
  for (uint64_t i = 0; i < n && !h->imported.empty(); ++i) hll_forget_import(h, dst_ids[i]);
  if (h->lv.size() != h->n) {
    h->lv.assign(h->n, rsk_hll::Level{0, 0, 0});
    h->lv_epoch = 0;
  }
  if (++h->lv_epoch == 0) {
    for (auto& e : h->lv) e.stamp = 0;
    h->lv_epoch = 1;
  }
  const uint32_t ep = h->lv_epoch;
  auto touch = [&](uint64_t id) -> rsk_hll::Level& {
    rsk_hll::Level& e = h->lv[id];
    if (e.stamp != ep) e = rsk_hll::Level{ep, 0, 0};
    return e;
  };
  // pinned: [dst pointers n][src pointers n][dst ids n][level n (u32)]
  const uint64_t seg = merge_batch_seg(n);
  auto* dps = reinterpret_cast<uint8_t**>(hb);
  auto* sps = reinterpret_cast<const uint8_t**>(hb + seg);
  auto* ids = reinterpret_cast<uint64_t*>(hb + 2 * seg);
  auto* level = reinterpret_cast<uint32_t*>(hb + 3 * seg);
  uint32_t max_level = 0;
  std::vector<uint8_t> src_exists(n);  // as of the pair's turn in input order
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t s_ = src_ids[i], dd = dst_ids[i];
    src_exists[i] = h->exists[s_];
    h->exists[dd] = 1;
    h->dense[dd] = 1;
    rsk_hll::Level& ls = touch(s_);
    rsk_hll::Level& ld = touch(dd);
    const uint32_t lv = std::max(std::max(ls.w, ld.w), ld.r) + 1;
    level[i] = lv;
    ld.w = lv;
    ls.r = std::max(ls.r, lv);
    max_level = std::max(max_level, lv);
  }
  std::vector<uint64_t> start(max_level + 2, 0);
  for (uint64_t i = 0; i < n; ++i) start[level[i] + 1]++;
  for (uint32_t l = 1; l <= max_level + 1; ++l) start[l] += start[l - 1];
  {
    std::vector<uint64_t> fill(start.begin(), start.end());
    for (uint64_t i = 0; i < n; ++i) {
      const uint64_t p = fill[level[i]]++;
      sps[p] = src_exists[i] ? regs_of(h, src_ids[i]) : nullptr;
      dps[p] = regs_of(h, dst_ids[i]);
    }
  }
  std::memcpy(ids, dst_ids, n * 8);
  auto* d_dst = reinterpret_cast<uint8_t**>(d);
  auto* d_src = reinterpret_cast<const uint8_t**>(d + seg);
  auto* d_ids = reinterpret_cast<uint64_t*>(d + 2 * seg);
  if (op) op_stage_in(op, d_dst, dps, 3 * seg);  // pointers and ids, one DMA (async call: on the input stream)
  else RSK_HIP(hipMemcpyAsync(d_dst, dps, 3 * seg, hipMemcpyHostToDevice, c->stream));
  for (uint32_t l = 1; l <= max_level; ++l)
    hll_merge_launch(c, d_dst + start[l], d_src + start[l], 1, start[l + 1] - start[l]);
  // PFMERGE invalidates every destination's cache (one launch for the batch).
  hipLaunchKernelGGL(invalidate_list_kernel, dim3((uint32_t)std::min<uint64_t>((n + 255) / 256, 1024)), dim3(256), 0,
                     c->stream, h->d_card, d_ids, n);
  RSK_CHECK_LAUNCH("invalidate_list");
}
}  // namespace

int rsk_hll_count_union(rsk_hll* const* hs, const uint64_t* ids, uint32_t k, uint64_t* out) {
  return guarded([&] {
    need(hs && ids && out && k >= 1, "bad arguments");
    rsk_ctx* c = hs[0]->ctx;
    CtxLock l(c);
    auto* ptrs = reinterpret_cast<const uint8_t**>(c->pinned(8ull * k + 8));
    for (uint32_t a = 0; a < k; ++a) {
      check_hll(hs[a], ids[a]);
      need(hs[a]->ctx == c, "all sketches must share one context");
      ptrs[a] = hs[a]->exists[ids[a]] ? regs_of(hs[a], ids[a]) : nullptr;
    }
    union_impl(c, ptrs, k, 1, out);
  });
}

int rsk_hll_count_union_batch(rsk_hll* h, const uint64_t* member_ids, uint32_t arity, uint64_t n, uint64_t* out) {
  return guarded([&] {
    need(h && member_ids && out && arity >= 1, "bad arguments");
    rsk_ctx* c = h->ctx;
    CtxLock l(c);
    if (n == 0) return;
    check_hll_ids(h, member_ids, n * arity, nullptr, 0, false);
    auto* ptrs = reinterpret_cast<const uint8_t**>(c->pinned(8ull * n * arity + 8ull * n));
    const uint8_t* e = h->exists.data();
    for (uint64_t i = 0; i < n * arity; ++i) {
      const uint64_t id = member_ids[i];
      ptrs[i] = e[id] ? regs_of(h, id) : nullptr;
    }
    union_impl(c, ptrs, arity, n, out);
  });
}

int rsk_hll_merge(rsk_hll* dst, uint64_t dst_id, rsk_hll* const* srcs, const uint64_t* src_ids, uint32_t k) {
  return guarded([&] {
    check_hll(dst, dst_id);
    need(k == 0 || (srcs && src_ids), "srcs is NULL");
    rsk_ctx* c = dst->ctx;
    CtxLock l(c);
    std::vector<const uint8_t*> sp(k);
    for (uint32_t a = 0; a < k; ++a) {
      check_hll(srcs[a], src_ids[a]);
      need(srcs[a]->ctx == c, "all sketches must share one context");
      sp[a] = srcs[a]->exists[src_ids[a]] ? regs_of(srcs[a], src_ids[a]) : nullptr;
    }
    bool created;
    hll_forget_import(dst, dst_id);
    create_if_missing(dst, dst_id, &created);
    dst->dense[dst_id] = 1;  // pfmergeCommand converts the destination to dense
    if (k) {
      uint8_t* s = out_scratch(c, 8 + k * 8 + 512);
      auto* d_dst = reinterpret_cast<uint8_t**>(s);
      auto* d_src = reinterpret_cast<const uint8_t**>(s + 256);
      uint8_t* dp = regs_of(dst, dst_id);
      RSK_HIP(hipMemcpyAsync(d_dst, &dp, 8, hipMemcpyHostToDevice, c->stream));
      RSK_HIP(hipMemcpyAsync(d_src, sp.data(), k * 8, hipMemcpyHostToDevice, c->stream));
      hll_merge_launch(c, d_dst, d_src, k, 1);
    }
    invalidate(dst, dst_id, nullptr, true);
    RSK_HIP(hipStreamSynchronize(c->stream));
  });
}

int rsk_hll_merge_batch(rsk_hll* h, const uint64_t* dst_ids, const uint64_t* src_ids, uint64_t n) {
  return guarded([&] {
    need(h && dst_ids && src_ids, "NULL argument");
    rsk_ctx* c = h->ctx;
    CtxLock l(c);
    if (n == 0) return;
    merge_batch_check(h, dst_ids, src_ids, n);
    merge_batch_enqueue(h, dst_ids, src_ids, n, c->pinned(merge_batch_host_bytes(n)),
                        out_scratch(c, merge_batch_dev_bytes(n)));
    RSK_HIP(hipStreamSynchronize(c->stream));
  });
}

int rsk_hll_merge_raw(rsk_hll* h, uint64_t id, const uint8_t* regs, uint32_t location) {
  return guarded([&] {
    check_hll(h, id);
    need(regs != nullptr, "regs is NULL");
    need(location == RSK_MEM_HOST || location == RSK_MEM_DEVICE, "bad location");
    rsk_ctx* c = h->ctx;
    CtxLock l(c);
    bool created;
    hll_forget_import(h, id);
    create_if_missing(h, id, &created);
    h->dense[id] = 1;
    const uint8_t* src = regs;
    if (location == RSK_MEM_HOST) {
      uint8_t* s = out_scratch(c, HLL_REGS);
      RSK_HIP(hipMemcpyAsync(s, regs, HLL_REGS, hipMemcpyHostToDevice, c->stream));
      src = s;
    }
    hll_max_into_launch(c, regs_of(h, id), src, nullptr);
    invalidate(h, id, nullptr, true);  // PFMERGE always invalidates
    RSK_HIP(hipStreamSynchronize(c->stream));
  });
}

int rsk_hll_get_registers(rsk_hll* h, uint64_t id, uint8_t* out, uint32_t location) {
  return guarded([&] {
    check_hll(h, id);
    need(out != nullptr, "out is NULL");
    CtxLock l(h->ctx);
    RSK_HIP(hipMemcpyAsync(out, regs_of(h, id), HLL_REGS,
                           location == RSK_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                           h->ctx->stream));
    RSK_HIP(hipStreamSynchronize(h->ctx->stream));
  });
}

void* rsk_hll_device_registers(rsk_hll* h) {  // the caller may read or write through it
  if (!h) return nullptr;
  try {
    rsk::hll_materialize(h);
    hll_forget_imports(h);
    hll_touch(h);
    RSK_HIP(hipStreamSynchronize(h->ctx->stream));
  } catch (const RskError&) {
    return nullptr;
  }
  return h->d_regs;
}

int rsk_hll_export_redis(rsk_hll* h, uint64_t id, uint8_t* buf, size_t cap, size_t* len) {
  return guarded([&] {
    check_hll(h, id);
    need(len != nullptr, "len is NULL");
    CtxLock l(h->ctx);
    if (!h->exists[id]) {  // GET of a missing key: nil
      *len = 0;
      return;
    }
    need(buf != nullptr && cap >= RSK_HLL_DENSE_BYTES, "buffer smaller than 12304 bytes");
    std::vector<uint8_t> raw(HLL_REGS);
    uint64_t card = 0;
    RSK_HIP(hipMemcpyAsync(raw.data(), regs_of(h, id), HLL_REGS, hipMemcpyDeviceToHost, h->ctx->stream));
    RSK_HIP(hipMemcpyAsync(&card, h->d_card + id, 8, hipMemcpyDeviceToHost, h->ctx->stream));
    RSK_HIP(hipStreamSynchronize(h->ctx->stream));
    const auto imp = h->imported.find(id);
    if (imp != h->imported.end()) {  // SET bytes, unwritten since: returned as they are
      const std::vector<uint8_t>& v = imp->second;
      need(cap >= v.size(), "buffer smaller than the stored string");
      std::memcpy(buf, v.data(), v.size());
      for (int b = 0; b < 8; ++b) buf[8 + b] = (uint8_t)(card >> (8 * b));  // PFCOUNT's cache, as Redis keeps it
      *len = v.size();
      return;
    }
    std::memset(buf, 0, RSK_HLL_DENSE_BYTES);
    std::memcpy(buf, "HYLL", 4);
    for (int b = 0; b < 8; ++b) buf[8 + b] = (uint8_t)(card >> (8 * b));
    if (!h->dense[id]) {
      const size_t n = encode_sparse(raw.data(), buf + 16, RSK_HLL_DENSE_BYTES - 16);
      if (n && 16 + n <= HLL_SPARSE_MAX_BYTES) {
        buf[4] = 1;  // HLL_SPARSE
        *len = 16 + n;
        return;
      }
      h->dense[id] = 1;  // promoted (hllSparseSet -> hllSparseToDense), for good
      std::memset(buf + 16, 0, RSK_HLL_DENSE_BYTES - 16);
    }
    buf[4] = 0;  // HLL_DENSE
    uint8_t* p = buf + 16;
    for (int j = 0; j < HLL_REGS; ++j) {  // HLL_DENSE_SET_REGISTER, 6 bits LSB-first
      uint32_t bitpos = (uint32_t)j * 6, byte = bitpos >> 3, fb = bitpos & 7;
      uint32_t v = raw[j] & 63;
      p[byte] |= (uint8_t)(v << fb);
      if (fb > 2) p[byte + 1] |= (uint8_t)(v >> (8 - fb));
    }
    *len = RSK_HLL_DENSE_BYTES;
  });
}

int rsk_hll_import_redis(rsk_hll* h, uint64_t id, const uint8_t* buf, size_t len) {
  return guarded([&] {
    check_hll(h, id);
    need(buf != nullptr || len == 0, "buf is NULL");
    // isHLLObjectOrReply: header, magic, encoding, exact dense length.
    if (len < 16 || std::memcmp(buf, "HYLL", 4) != 0 || buf[4] > 1 || (buf[4] == 0 && len != RSK_HLL_DENSE_BYTES))
      fail(RSK_ERR_WRONGTYPE, "WRONGTYPE Key is not a valid HyperLogLog string value.");
    std::vector<uint8_t> raw(HLL_REGS, 0);
    if (buf[4] == 0) {
      const uint8_t* p = buf + 16;
      for (int j = 0; j < HLL_REGS; ++j) {
        uint32_t bitpos = (uint32_t)j * 6, byte = bitpos >> 3, fb = bitpos & 7;
        uint32_t b0 = p[byte], b1 = byte + 1 < 12288 ? p[byte + 1] : 0;
        raw[j] = (uint8_t)(((b0 >> fb) | (b1 << (8 - fb))) & 63);
      }
    } else {
      // Sparse opcodes: ZERO 00xxxxxx, XZERO 01xxxxxx yyyyyyyy, VAL 1vvvvvxx.
      const uint8_t *p = buf + 16, *end = buf + len;
      uint64_t i = 0;
      bool overflow = false;
      while (p < end) {
        if ((*p & 0xc0) == 0) {
          i += (*p & 0x3f) + 1;
          p++;
        } else if ((*p & 0xc0) == 0x40) {
          if (p + 1 >= end) {
            overflow = true;
            break;
          }
          i += (((uint64_t)(*p & 0x3f) << 8) | p[1]) + 1;
          p += 2;
        } else {
          uint64_t run = (*p & 3) + 1;
          uint8_t v = (uint8_t)(((*p >> 2) & 0x1f) + 1);
          if (run + i > HLL_REGS) {
            overflow = true;
            break;
          }
          while (run--) {
            raw[i] = std::max(raw[i], v);
            ++i;
          }
          p++;
        }
      }
      if (overflow || i != HLL_REGS) fail(RSK_ERR_INVALID_HLL, "INVALIDOBJ Corrupted HLL object detected");
    }
    uint64_t card = 0;
    for (int b = 0; b < 8; ++b) card |= (uint64_t)buf[8 + b] << (8 * b);
    rsk_ctx* c = h->ctx;
    CtxLock l(c);
    RSK_HIP(hipMemcpyAsync(regs_of(h, id), raw.data(), HLL_REGS, hipMemcpyHostToDevice, c->stream));
    RSK_HIP(hipMemcpyAsync(h->d_card + id, &card, 8, hipMemcpyHostToDevice, c->stream));
    RSK_HIP(hipStreamSynchronize(c->stream));
    h->exists[id] = 1;
    h->dense[id] = buf[4] == 0;
    // GET must return the SET bytes until the key is written.  Export
    // re-encodes canonically (dense packing; sparse runs cut into the longest
    // opcodes), so a copy is kept only when that re-encoding would differ:
    // non-zero unused header bytes, or a sparse string Redis would hold in
    // another form (other run chunking, or longer than the sparse limit).
    bool canonical = buf[5] == 0 && buf[6] == 0 && buf[7] == 0;
    if (canonical && buf[4] == 1) {
      std::vector<uint8_t> enc(RSK_HLL_DENSE_BYTES);
      const size_t n = encode_sparse(raw.data(), enc.data(), enc.size());
      canonical = n != 0 && 16 + n <= HLL_SPARSE_MAX_BYTES && 16 + n == len && std::memcmp(enc.data(), buf + 16, n) == 0;
    }
    if (canonical) hll_forget_import(h, id);
    else h->imported[id].assign(buf, buf + len);
  });
}

// Batched GET / SET of the Redis strings (rsk_hll_io.hip): the checkpoint of
// a pool, one encode pass and one copy per 65536 keys (export), one upload and
// two kernels (import) instead of a synchronous round trip per key.
int rsk_hll_export_redis_batch(rsk_hll* h, const uint64_t* ids, uint64_t n, uint8_t* out, uint64_t cap,
                               uint64_t* offsets) {
  return guarded([&] {
    need(h != nullptr, "hll handle is NULL");
    need(offsets != nullptr && (ids != nullptr || n == 0), "NULL argument");
    need(n < (1ull << 31), "at most 2^31 - 1 keys per call");
    offsets[0] = 0;
    if (n == 0) return;
    const auto tE = std::chrono::steady_clock::now();
    uint64_t bad = 0;
    for (uint64_t i = 0; i < n; ++i) bad |= ids[i] >= h->n;
    need(!bad, "sketch id out of range");
    rsk_ctx* c = h->ctx;
    CtxLock l(c);
    rsk::hll_materialize(h);  // a pending lazy clear: GET reads zero registers (export writes none)
    // A large pageable output buffer is pinned in place for the call (CallPin) so the strings
    // go to it by DMA, not through the stages and a host copy.
    const auto tR = std::chrono::steady_clock::now();
    CallPin treg;
    treg.pin(c, out, cap);
    const auto tG = std::chrono::steady_clock::now();
    const int eng = export_engine(c);  // (before any of this call's work is queued)
    const auto tI0 = std::chrono::steady_clock::now();
    // keys the device encodes (present, not a kept SET string), in call order: counted, then
    // listed, in slices on the host threads (4.4 ms on one thread for the C5 pool's 10^6 keys)
    const bool any_imp = !h->imported.empty();
    auto on_device = [&](uint64_t id) { return h->exists[id] && !(any_imp && h->imported.count(id)); };
    std::unique_ptr<uint64_t[]> dev_i(new uint64_t[n]), dev_id(new uint64_t[n]);
    std::unique_ptr<uint8_t[]> want(new uint8_t[n]);
    uint64_t nd = 0;
    {
      const unsigned nt = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(std::max(1u, c->stage_threads), n >> 16));
      const uint64_t per = (n + nt - 1) / nt;
      std::vector<uint64_t> at(nt + 1, 0);
      auto slices = [&](auto&& f) {
        std::vector<std::thread> th;
        for (unsigned t = 1; t < nt; ++t) th.emplace_back([&, t] { f(t); });
        f(0u);
        for (auto& x : th) x.join();
      };
      slices([&](unsigned t) {
        uint64_t k = 0;
        for (uint64_t i = t * per, e = std::min(n, (t + 1) * per); i < e; ++i) k += on_device(ids[i]);
        at[t + 1] = k;
      });
      for (unsigned t = 0; t < nt; ++t) at[t + 1] += at[t];
      slices([&](unsigned t) {
        uint64_t k = at[t];
        for (uint64_t i = t * per, e = std::min(n, (t + 1) * per); i < e; ++i) {
          const uint64_t id = ids[i];
          if (!on_device(id)) continue;
          dev_i[k] = i;
          dev_id[k] = id;
          want[k++] = h->dense[id] ? 0 : 1;
        }
      });
      nd = at[nt];
    }
    const auto tI = std::chrono::steady_clock::now();
    auto al = [](uint64_t x) { return (x + 255) & ~uint64_t(255); };
    // Chunks of KC device keys: each encoded once into its slot (12304 bytes
    // apart), the lengths copied back, the offsets advanced to the chunk's last
    // key (kept SET strings and missing keys in between from the host), then
    // the chunk's strings packed into a stage and copied to `out` -- unless the
    // strings no longer fit in cap: then only the lengths go on, for
    // offsets[n], and the call fails.
    constexpr uint64_t KC = 1ull << 16;
    const uint64_t kc = std::min<uint64_t>(KC, std::max<uint64_t>(nd, 1));
    // chunk boundaries: the first chunk 16384 keys, so the copy-out starts after a short encode
    auto chunk_end = [&](uint64_t d0) { return std::min<uint64_t>(nd, d0 + (d0 == 0 ? std::min<uint64_t>(kc, 16384) : kc)); };
    uint8_t* w = c->work(al(8 * kc) * 2 + al(kc) + al(4 * kc) + 3 * al(kc * (uint64_t)RSK_HLL_DENSE_BYTES) + 256);
    uint64_t* d_ids = reinterpret_cast<uint64_t*>(w);
    uint64_t* d_pos = reinterpret_cast<uint64_t*>(w + al(8 * kc));
    uint8_t* d_want = w + 2 * al(8 * kc);
    uint32_t* d_len = reinterpret_cast<uint32_t*>(w + 2 * al(8 * kc) + al(kc));
    uint8_t* d_slots = w + 2 * al(8 * kc) + al(kc) + al(4 * kc);
    // two packed stages: chunk k + 1 packs into one while chunk k's strings leave the other
    uint8_t* d_stage[2] = {d_slots + al(kc * (uint64_t)RSK_HLL_DENSE_BYTES),
                           d_slots + 2 * al(kc * (uint64_t)RSK_HLL_DENSE_BYTES)};
    std::unique_ptr<uint32_t[]> len(new uint32_t[nd ? nd : 1]);  // (every chunk's lengths copied in before use)
    // the chunk's ids, flags, lengths and string offsets live in pinned memory, moved by small
    // kernels on the context stream (xfer): a pageable copy would hold the host until the stream
    // reaches it, and a DMA would queue behind the bulk copy-out on the copy engine
    if (!c->h_io) RSK_HIP(hipHostMalloc(&c->h_io, 21 * KC, hipHostMallocDefault));
    uint64_t* h_ids = reinterpret_cast<uint64_t*>(c->h_io);
    uint64_t* pos = h_ids + KC;
    uint32_t* h_len = reinterpret_cast<uint32_t*>(pos + KC);
    uint8_t* h_want = reinterpret_cast<uint8_t*>(h_len + KC);
    uint64_t o = 0, next_i = 0;  // offsets[0 .. next_i] are final
    bool fits = true;
    auto advance = [&](uint64_t upto, uint64_t d) {  // offsets of keys [next_i, upto); d: the next device key
      for (; next_i < upto; ++next_i) {
        const uint64_t id = ids[next_i];
        uint64_t L = 0;
        if (d < nd && dev_i[d] == next_i) {
          L = len[d++] & 0x7FFFFFFFu;
        } else if (h->exists[id]) {
          L = h->imported.find(id)->second.size();
        }
        o += L;
        offsets[next_i + 1] = o;
      }
      return d;
    };
    uint64_t dcur = 0;  // device keys whose offsets are final
    // packed: chunk k's strings are in their stage; out_done[s]: the copy-out of stage s was queued
    // (chunk k + 2 packs into it after that, on the device)
    hipEvent_t packed = nullptr, lens = nullptr, out_done[2] = {nullptr, nullptr};
    struct EvGuard {
      hipEvent_t* e[4];
      ~EvGuard() {
        for (hipEvent_t* p : e)
          if (*p) (void)hipEventDestroy(*p);
      }
    } eg{{&packed, &lens, &out_done[0], &out_done[1]}};
    auto encode = [&](uint64_t d0) {  // chunk d0's encode and its lengths, queued on the context stream
      const uint64_t m = chunk_end(d0) - d0;
      std::memcpy(h_ids, dev_id.get() + d0, 8 * m);  // (the previous chunk's copies are done: synchronised)
      std::memcpy(h_want, want.get() + d0, m);
      xfer(c, d_ids, h_ids, 8 * m);  // (kernels, not copies: a copy here would queue behind the bulk D2H)
      xfer(c, d_want, h_want, m);
      hll_export_launch(c, h->d_regs, h->d_card, d_ids, d_want, (uint32_t)m, d_len, d_slots);
      xfer(c, h_len, d_len, 4 * m);
      RSK_HIP(hipEventRecord(lens, c->stream));
    };
    const auto tQ = std::chrono::steady_clock::now();
    if (nd) {
      RSK_HIP(hipEventCreateWithFlags(&packed, hipEventDisableTiming));
      RSK_HIP(hipEventCreateWithFlags(&lens, hipEventDisableTiming));
      RSK_HIP(hipEventCreateWithFlags(&out_done[0], hipEventDisableTiming));
      RSK_HIP(hipEventCreateWithFlags(&out_done[1], hipEventDisableTiming));
      encode(0);
    }
    // chunk k's strings leave through the copy stream (c->xout) while chunk k + 1 encodes and
    // packs; the pieces of every chunk go through one D2H stream (16 MiB pieces, up to 7 in
    // flight), so the copy engine runs on across chunk boundaries
    D2HStream xo(c, c->xout, (c->tune.io_piece ? (uint64_t)c->tune.io_piece : 16ull) << 20, eng);  // (A/B: io_piece MiB)
    uint64_t left[2] = {0, 0};  // xo.issued() after each stage's last put
    const bool trace = c->tune.io_trace != 0;  // (route io_trace: phase times to stderr)
    double t_sync = 0, t_adv = 0, t_pack = 0, t_enc = 0, t_d2h = 0;
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    const auto t00 = now();
    for (uint64_t d0 = 0, d1, ck = 0; d0 < nd; d0 = d1, ++ck) {
      d1 = chunk_end(d0);
      const uint64_t m = d1 - d0;
      uint8_t* stage = d_stage[ck & 1];
      auto t0 = now();
      if (c->tune.io_drain) RSK_HIP(hipEventSynchronize(lens));  // (A/B: route io_drain)
      else xo.service_until(lens);  // chunk d0's lengths (and the previous pack) done; copy-outs meanwhile
      std::memcpy(len.get() + d0, h_len, 4 * m);
      auto t1 = now();
      t_sync += ms(t0, t1);
      dcur = advance(dev_i[d0 + m - 1] + 1, dcur);
      t0 = now();
      t_adv += ms(t1, t0);
      fits = fits && o <= cap && out != nullptr;
      uint64_t base = 0, end = 0;
      if (fits) {
        base = offsets[dev_i[d0]];
        end = offsets[dev_i[d0 + m - 1] + 1];
        for (uint64_t d = 0; d < m; ++d) pos[d] = offsets[dev_i[d0 + d]] - base;
        xfer(c, d_pos, pos, 8 * m);
        if (ck >= 2) xo.order_after(left[ck & 1], out_done[ck & 1], c->stream);  // chunk k - 2 left this stage
        hll_export_pack_launch(c, d_slots, d_len, d_pos, (uint32_t)m, stage);
        RSK_HIP(hipEventRecord(packed, c->stream));
      }
      t1 = now();
      t_pack += ms(t0, t1);
      if (d1 < nd) encode(d1);  // (after the pack on the same stream: the slots are free)
      t0 = now();
      t_enc += ms(t1, t0);
      if (fits) {
        xo.put(out + base, stage, end - base, packed);  // returns with up to 7 pieces in flight
        RSK_HIP(hipEventRecord(out_done[ck & 1], c->xout));
        left[ck & 1] = xo.issued();
        if (c->tune.io_drain) xo.drain();  // (A/B: each chunk's copy-out finished before the next chunk)
      }
      t_d2h += ms(t0, now());
    }
    {
      const auto t0 = now();
      xo.drain();
      t_d2h += ms(t0, now());
    }
    const auto t01 = now();
    advance(n, dcur);  // the keys after the last device key
    if (o > cap) fail(RSK_ERR_INVALID_ARG, "output buffer smaller than the strings (offsets[n] holds the bytes needed)");
    need(out != nullptr || o == 0, "out is NULL");
    // promoted for good (hllSparseSet -> hllSparseToDense), as the per-key GET
    par_for(nd, std::max(1u, c->stage_threads), [&](uint64_t lo, uint64_t hi) {
      for (uint64_t d = lo; d < hi; ++d)
        if (want[d] && !(len[d] >> 31)) h->dense[dev_id[d]] = 1;  // (a repeated id: the same byte, the same 1)
    });
    // kept SET strings: their bytes, card bytes as PFCOUNT last left them (rare: copied one by one)
    for (uint64_t i = 0; i < (any_imp ? n : 0); ++i) {
      const uint64_t id = ids[i];
      if (!h->exists[id]) continue;
      const auto imp = h->imported.find(id);
      if (imp == h->imported.end()) continue;
      uint64_t card = 0;
      RSK_HIP(hipMemcpy(&card, h->d_card + id, 8, hipMemcpyDeviceToHost));
      uint8_t* d = out + offsets[i];
      std::memcpy(d, imp->second.data(), imp->second.size());
      for (int b = 0; b < 8; ++b) d[8 + b] = (uint8_t)(card >> (8 * b));
    }
    if (trace)
      std::fprintf(stderr,
                   "export: %.2f ms: before the loop %.2f (checks %.2f, pin %.2f, engine %.2f, key list %.2f, "
                   "scratch %.2f, first encode %.2f), loop %.2f (sync %.2f advance %.2f pack %.2f encode %.2f "
                   "d2h %.2f, engine %d), after %.2f\n",
                   ms(tE, now()), ms(tE, t00), ms(tE, tR), ms(tR, tG), ms(tG, tI0), ms(tI0, tI), ms(tI, tQ), ms(tQ, t00),
                   ms(t00, t01), t_sync, t_adv, t_pack, t_enc, t_d2h, eng, ms(t01, now()));
  });
}

int rsk_hll_import_redis_batch(rsk_hll* h, const uint64_t* ids, uint64_t n, const uint8_t* data,
                               const uint64_t* offsets) {
  return guarded([&] {
    need(h != nullptr, "hll handle is NULL");
    need(n == 0 || (ids != nullptr && offsets != nullptr && data != nullptr), "NULL argument");
    need(n < (1ull << 31), "at most 2^31 - 1 keys per call");
    if (n == 0) return;
    const bool trace = h->ctx->tune.io_trace != 0;  // (route io_trace: phase times to stderr)
    auto now = [] { return std::chrono::steady_clock::now(); };
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    const auto tA = now();
    const unsigned nth = std::max(1u, h->ctx->stage_threads);
    std::atomic<uint64_t> bad_off{~0ull};
    par_for(n, nth, [&](uint64_t lo, uint64_t hi) {
      for (uint64_t i = lo; i < hi; ++i)
        if (offsets[i + 1] < offsets[i]) {
          bad_off.store(i);
          return;
        }
    });
    need(bad_off.load() == ~0ull, "offsets must be non-decreasing");
    rsk_ctx* c = h->ctx;
    // held from the pending-clear completion through the kernels: an rsk_hll_clear
    // from another thread in between would otherwise zero the imported rows later
    CtxLock l(c);
    check_hll_ids(h, ids, n);
    // isHLLObjectOrReply per string (as rsk_hll_import_redis), on the host: header, magic,
    // encoding, exact dense length; the sparse opcodes are checked on the device.  One pass
    // over the headers (threads), leaving per string: bit 0 sparse, bit 1 a non-zero unused
    // header byte (kept as SET), bit 7 not an HLL string / too long (the first one fails).
    // Then the SETs of one key in one call: the last wins (a pass from the end marks each id
    // once).  Both run on a helper thread while the strings go up (below); no string is
    // checked on the device before its header passed.
    std::vector<uint8_t> hf(n), apply(n, 0);
    std::atomic<uint64_t> first_bad{~0ull};
    bool hdr_oom = false;
    std::thread hdr([&] {
      try {
        par_for(n, nth, [&](uint64_t lo, uint64_t hi) {
          for (uint64_t i = lo; i < hi; ++i) {
            const uint8_t* s = data + offsets[i];
            const uint64_t len = offsets[i + 1] - offsets[i];
            uint8_t f = 0;
            if (len < 16 || std::memcmp(s, "HYLL", 4) != 0 || s[4] > 1 || (s[4] == 0 && len != RSK_HLL_DENSE_BYTES) ||
                len > (1ull << 31)) {
              f = 0x80;
              uint64_t cur = first_bad.load();
              while (i < cur && !first_bad.compare_exchange_weak(cur, i)) {
              }
            } else {
              f = (uint8_t)(s[4] | ((s[5] | s[6] | s[7]) ? 2 : 0));
            }
            hf[i] = f;
          }
        });
        std::vector<uint8_t> seen(h->n, 0);
        for (uint64_t i = n; i-- > 0;)
          if (!seen[ids[i]]) {
            seen[ids[i]] = 1;
            apply[i] = 1;
          }
      } catch (const std::bad_alloc&) {
        hdr_oom = true;
      }
    });
    struct Join {
      std::thread& t;
      ~Join() {
        if (t.joinable()) t.join();
      }
    } hj{hdr};
    auto headers = [&] {  // the helper's verdict (the first bad header fails the call)
      hdr.join();
      if (hdr_oom) fail(RSK_ERR_OUT_OF_MEMORY, "host memory for the import's bookkeeping");
      if (first_bad.load() != ~0ull) {
        const uint64_t i = first_bad.load(), len = offsets[i + 1] - offsets[i];
        const uint8_t* s = data + offsets[i];
        if (len >= 16 && std::memcmp(s, "HYLL", 4) == 0 && s[4] <= 1 && !(s[4] == 0 && len != RSK_HLL_DENSE_BYTES))
          need(false, "string too long");
        fail(RSK_ERR_WRONGTYPE, "WRONGTYPE Key is not a valid HyperLogLog string value. (string " + std::to_string(i) +
                                    ")");
      }
    };
    const uint64_t base = offsets[0], total = offsets[n] - base;
    auto al = [](uint64_t x) { return (x + 255) & ~uint64_t(255); };
    // Decode each chunk as soon as it is checked (overlapped with the next chunk's upload), with
    // the rows it replaces copied aside first and copied back if a later string fails its check
    // (all or nothing): when the copy (16 KiB + 8 B per string) fits in a quarter of the free
    // device memory; otherwise every string is decoded after the last check.
    const uint64_t base_bytes = al(8 * n) + al(8 * (n + 1)) + 2 * al(n) + 256 + al(total) + 256;
    const uint64_t bak_bytes = al(n * (uint64_t)HLL_REGS) + al(8 * n);
    bool early = false;
    {
      size_t fr = 0, tot = 0;
      if (hipMemGetInfo(&fr, &tot) == hipSuccess)
        early = (double)bak_bytes < 0.25 * (double)(fr + (c->work_bytes >= base_bytes ? c->work_bytes - base_bytes : 0));
      (void)hipGetLastError();
    }
    uint8_t* w = nullptr;
    if (early) {
      try {
        w = c->work(base_bytes + bak_bytes);
      } catch (const RskError& e) {
        if (e.code != RSK_ERR_OUT_OF_MEMORY) throw;
        (void)hipGetLastError();
        early = false;
      }
    }
    if (!early) w = c->work(base_bytes);
    uint8_t* d_bak = w + base_bytes;
    uint64_t* d_bak_card = reinterpret_cast<uint64_t*>(d_bak + al(n * (uint64_t)HLL_REGS));
    uint64_t* d_ids = reinterpret_cast<uint64_t*>(w);
    uint64_t* d_off = reinterpret_cast<uint64_t*>(w + al(8 * n));
    uint8_t* d_apply = w + al(8 * n) + al(8 * (n + 1));
    uint8_t* d_canon = d_apply + al(n);
    auto* d_err = reinterpret_cast<unsigned long long*>(d_canon + al(n));
    uint8_t* d_data = d_canon + al(n) + 256;
    CallPin in_pin;  // the strings DMA'd straight from the caller's buffer (>= 256 MiB)
    in_pin.pin(c, data + base, total);
    std::unique_ptr<uint64_t[]> off(new uint64_t[n + 1]);
    par_for(n + 1, nth, [&](uint64_t lo, uint64_t hi) {
      for (uint64_t i = lo; i < hi; ++i) off[i] = offsets[i] - base;
    });
    // On an SDMA engine (the fastest measured, copy_engine) the ids, offsets and strings go up as
    // engine copies through the pinned ring, and chunk q's check is launched once its pieces are
    // in, after chunk q + 1's first pieces are on their way (so the engine is not idle while the
    // host launches it); otherwise HIP's copies, the strings on the input copy stream.
    const int ein = copy_engine(c, false);
    std::unique_ptr<H2DStream> xi;
    if (ein >= 0) {
      RSK_HIP(hipStreamSynchronize(c->stream));  // the device work queued before (it may use this scratch) is done
      xi.reset(new H2DStream(c, ein, 16ull << 20));
      xi->put(reinterpret_cast<uint8_t*>(d_ids), reinterpret_cast<const uint8_t*>(ids), 8 * n);
      xi->put(reinterpret_cast<uint8_t*>(d_off), reinterpret_cast<const uint8_t*>(off.get()), 8 * (n + 1));
    } else {
      h2d_staged(c, reinterpret_cast<uint8_t*>(d_ids), reinterpret_cast<const uint8_t*>(ids), 8 * n);
      h2d_staged(c, reinterpret_cast<uint8_t*>(d_off), reinterpret_cast<const uint8_t*>(off.get()), 8 * (n + 1));
    }
    RSK_HIP(hipMemsetAsync(d_err, 0xFF, 8, c->stream));
    RSK_HIP(hipMemsetAsync(d_canon, 1, n, c->stream));
    // The strings in 8 chunks of about equal bytes, each checked on the device as soon as it is
    // there (the check of chunk q runs while chunk q + 1 crosses the link); the headers are in
    // by the end of the first chunk.  Early: each chunk then decoded behind its check (its rows
    // copied aside first); otherwise the decode waits for every check.
    // (the strings go up on the input copy stream, c->xin: a check kernel on the context
    // stream would otherwise hold the next chunk's copies behind it)
    constexpr uint64_t NCH = 8;
    uint64_t cut[NCH + 1];
    hipEvent_t up = nullptr;
    RSK_HIP(hipEventCreateWithFlags(&up, hipEventDisableTiming));
    struct EvFree {
      hipEvent_t e;
      ~EvFree() { (void)hipEventDestroy(e); }
    } uf{up};
    RSK_HIP(hipEventRecord(up, c->stream));  // ids / offsets staged first (same stages)
    RSK_HIP(hipStreamWaitEvent(c->xin, up, 0));
    cut[0] = 0;
    cut[NCH] = n;
    for (uint64_t q = 1; q < NCH; ++q)
      cut[q] = std::max<uint64_t>(cut[q - 1], (uint64_t)(std::lower_bound(offsets, offsets + n, base + q * (total / NCH)) -
                                                         offsets));
    const auto t0 = now();
    uint64_t checked = 0;  // chunks [0, checked) have their check queued
    bool hdr_ok = false;
    auto launch_chunk = [&](uint64_t qq) {  // chunk qq's check (and, early, its rows aside and its decode)
      const uint64_t a = cut[qq], b = cut[qq + 1];
      hll_import_launch(c, d_data, d_off + a, d_ids + a, nullptr, (uint32_t)(b - a), h->d_regs, h->d_card,
                        d_canon + a, d_err, (uint32_t)a);
      if (early) {
        hll_rows_bak_launch(c, false, h->d_regs, h->d_card, d_ids + a, d_apply + a, (uint32_t)(b - a),
                            d_bak + a * (uint64_t)HLL_REGS, d_bak_card + a, d_err);
        hll_import_launch(c, d_data, d_off + a, d_ids + a, d_apply + a, (uint32_t)(b - a), h->d_regs, h->d_card,
                          d_canon + a, d_err, (uint32_t)a);
      }
    };
    uint64_t in_mark[NCH] = {}, apply_mark = 0;  // xi->issued() after each chunk / after d_apply
    for (uint64_t q = 0; q < NCH; ++q) {
      const uint64_t i0 = cut[q], i1 = cut[q + 1];
      if (xi) {
        xi->put(d_data + off[i0], data + offsets[i0], off[i1] - off[i0]);
        in_mark[q] = xi->issued();
      } else {
        h2d_staged_on(c, c->xin, d_data + off[i0], data + offsets[i0], off[i1] - off[i0]);
        RSK_HIP(hipEventRecord(up, c->xin));
        RSK_HIP(hipStreamWaitEvent(c->stream, up, 0));  // chunk q's check after its strings
      }
      if (!hdr_ok) {
        headers();
        hdr_ok = true;
        if (early && xi) {
          xi->put(d_apply, apply.data(), n);  // (the dedup is in with the headers)
          apply_mark = xi->issued();
        } else if (early) {
          h2d_staged(c, d_apply, apply.data(), n);
        }
      }
      if (xi) {
        if (q == 0) continue;
        xi->wait_upto(std::max(in_mark[q - 1], apply_mark));  // chunk q - 1 (and the dedup flags) in
      }
      for (; checked < (xi ? q : q + 1); ++checked) launch_chunk(checked);
    }
    if (xi) {  // the last chunk
      xi->wait_upto(std::max(in_mark[NCH - 1], apply_mark));
      for (; checked < NCH; ++checked) launch_chunk(checked);
      xi.reset();  // (every piece is in: the stages are free for the HIP copies below)
    }
    const auto t1 = now();
    if (early) {  // a failed check anywhere: every replaced row back as it was
      hll_rows_bak_launch(c, true, h->d_regs, h->d_card, d_ids, d_apply, (uint32_t)n, d_bak, d_bak_card, d_err);
    } else {
      h2d_staged(c, d_apply, apply.data(), n);
      hll_import_launch(c, d_data, d_off, d_ids, d_apply, (uint32_t)n, h->d_regs, h->d_card, d_canon, d_err);
    }
    std::vector<uint8_t> canon(n);
    unsigned long long err = 0;
    RSK_HIP(hipMemcpyAsync(canon.data(), d_canon, n, hipMemcpyDeviceToHost, c->stream));
    RSK_HIP(hipMemcpyAsync(&err, d_err, 8, hipMemcpyDeviceToHost, c->stream));
    RSK_HIP(hipStreamSynchronize(c->stream));
    const auto t2 = now();
    if (err != ~0ull)
      fail(RSK_ERR_INVALID_HLL, "INVALIDOBJ Corrupted HLL object detected (string " + std::to_string(err) + ")");
    // host state per SET (the ids with apply[i] are distinct): exists / dense on threads; the
    // kept strings (a copy only where the canonical re-encoding would differ, as
    // rsk_hll_import_redis) and the forgotten ones in one serial pass over those only
    std::atomic<uint64_t> n_keep{0};
    par_for(n, nth, [&](uint64_t lo, uint64_t hi) {
      uint64_t k = 0;
      for (uint64_t i = lo; i < hi; ++i) {
        if (!apply[i]) continue;
        const uint64_t id = ids[i];
        const bool sparse = hf[i] & 1;
        h->exists[id] = 1;
        h->dense[id] = !sparse;
        bool canonical = !(hf[i] & 2);
        if (canonical && sparse) canonical = canon[i] && offsets[i + 1] - offsets[i] <= HLL_SPARSE_MAX_BYTES;
        canon[i] = canonical ? 1 : 0;  // (from here: 1 = re-encode, 0 = keep the SET string)
        k += !canonical;
      }
      n_keep += k;
    });
    if (n_keep.load() || !h->imported.empty()) {
      for (uint64_t i = 0; i < n; ++i) {
        if (!apply[i]) continue;
        const uint64_t id = ids[i];
        if (canon[i]) {
          hll_forget_import(h, id);
        } else {
          const uint8_t* s = data + offsets[i];
          h->imported[id].assign(s, s + (offsets[i + 1] - offsets[i]));
        }
      }
    }
    if (trace)
      std::fprintf(stderr, "import: metadata %.2f ms, strings up + checks %.2f, decode + sync %.2f, post %.2f\n",
                   ms(tA, t0), ms(t0, t1), ms(t1, t2), ms(t2, now()));
  });
}

// ---------------------------------------------------------------- Bloom
int rsk_bloom_params(int64_t n, double p, uint32_t mode, int64_t* size_out, int32_t* k_out) {
  return guarded([&] {
    need(size_out && k_out, "NULL argument");
    need(mode == RSK_BLOOM_COMPAT || mode == RSK_BLOOM_EXTENDED, "bad mode");
    int64_t size = optimal_bits(n, p);
    if (mode == RSK_BLOOM_COMPAT && size > BLOOM_MAX_SIZE)
      fail(RSK_ERR_INVALID_ARG, "Bloom filter can't be greater than " + std::to_string(BLOOM_MAX_SIZE) +
                                    ". But calculated size is " + std::to_string(size));
    if (size > BLOOM_EXT_MAX) fail(RSK_ERR_INVALID_ARG, "Bloom filter size " + std::to_string(size) + " exceeds device limit");
    *size_out = size;
    *k_out = optimal_k(n, size);
  });
}

int rsk_bloom_create(rsk_ctx* c, int64_t size, int32_t k, rsk_bloom** out) {
  return guarded([&] {
    need(c && out, "NULL argument");
    need(size > 0, "Bloom filter size must be > 0");
    need(size <= BLOOM_EXT_MAX, "Bloom filter size exceeds device limit");
    need(k >= 1 && k <= 4096, "hashIterations must be in [1, 4096]");
    CtxLock l(c);
    *out = nullptr;
    auto* b = new rsk_bloom();
    std::unique_ptr<rsk_bloom> guard(b);
    b->ctx = c;
    b->size = size;
    b->k = k;
    b->nbytes = ((uint64_t)size + 7) / 8;
    b->nwords = ((b->nbytes + 15) / 16) * 4;
    b->fm = make_fastmod((uint64_t)size);
    RSK_HIP(hipMalloc(&b->d_bits, b->nwords * 4));
    RSK_HIP(hipMemsetAsync(b->d_bits, 0, b->nwords * 4, c->stream));
    RSK_HIP(hipStreamSynchronize(c->stream));
    *out = guard.release();
  });
}

int rsk_bloom_init(rsk_ctx* c, int64_t n, double p, uint32_t mode, rsk_bloom** out, int64_t* size_out,
                   int32_t* k_out) {
  int64_t size = 0;
  int32_t k = 0;
  int rc = rsk_bloom_params(n, p, mode, &size, &k);
  if (rc != RSK_OK) return rc;
  if (size_out) *size_out = size;
  if (k_out) *k_out = k;
  return rsk_bloom_create(c, size, k, out);
}

int rsk_bloom_destroy(rsk_bloom* b) {
  if (!b) return RSK_OK;
  int rc = guarded([&] {
    CtxLock l(b->ctx);
    RSK_HIP(hipStreamSynchronize(b->ctx->stream));
    RSK_HIP(hipFree(b->d_bits));
  });
  delete b;
  return rc;
}

int rsk_bloom_info(const rsk_bloom* b, int64_t* size, int32_t* k) {
  return guarded([&] {
    need(b && size && k, "NULL argument");
    *size = b->size;
    *k = b->k;
  });
}

int rsk_bloom_add(rsk_bloom* b, const rsk_keys* keys, uint8_t* added_out) {
  return guarded([&] {
    need(b != nullptr, "bloom handle is NULL");
    rsk_ctx* c = b->ctx;
    CtxLock l(c);
    check_keys(c, keys);
    check_out(c, keys, added_out);
    ++b->wgen;
    if (!added_out) {
      for_each_chunk(c, keys, [&](const DevKeys& dk, uint64_t, uint64_t) { bloom_add_launch(c, b, dk); });
      return;
    }
    for_each_chunk(c, keys, [&](const DevKeys& dk, uint64_t first, uint64_t cnt) {
      uint8_t* d_out = keys->location == RSK_MEM_DEVICE ? added_out + first : out_scratch(c, cnt);
      bloom_add_replies_launch(c, b, dk, d_out);
      if (keys->location == RSK_MEM_HOST) {
        RSK_HIP(hipMemcpyAsync(added_out + first, d_out, cnt, hipMemcpyDeviceToHost, c->stream));
        RSK_HIP(hipStreamSynchronize(c->stream));
      }
    });
    RSK_HIP(hipStreamSynchronize(c->stream));
  });
}

int rsk_bloom_contains(rsk_bloom* b, const rsk_keys* keys, uint8_t* out) {
  return guarded([&] {
    need(b != nullptr && out != nullptr, "NULL argument");
    rsk_ctx* c = b->ctx;
    CtxLock l(c);
    check_keys(c, keys);
    check_out(c, keys, out);
    for_each_chunk(c, keys, [&](const DevKeys& dk, uint64_t first, uint64_t cnt) {
      if (keys->location == RSK_MEM_DEVICE) {
        bloom_contains_launch(c, b, dk, out + first);
      } else {
        uint8_t* d_out = out_scratch(c, cnt);
        bloom_contains_launch(c, b, dk, d_out);
        RSK_HIP(hipMemcpyAsync(out + first, d_out, cnt, hipMemcpyDeviceToHost, c->stream));
        RSK_HIP(hipStreamSynchronize(c->stream));
      }
    });
  });
}

int rsk_hash_to_base64(rsk_ctx* c, const rsk_keys* keys, char* out) {
  return guarded([&] {
    need(c != nullptr, "ctx is NULL");
    check_keys(c, keys);
    need(keys->n == 0 || out != nullptr, "out is NULL");
    check_out(c, keys, out);
    CtxLock l(c);
    for_each_chunk(c, keys, [&](const DevKeys& dk, uint64_t first, uint64_t cnt) {
      if (keys->location == RSK_MEM_DEVICE) {
        hash_b64_launch(c, dk, out + 22 * first);
      } else {
        char* d = reinterpret_cast<char*>(out_scratch(c, 22 * cnt));
        hash_b64_launch(c, dk, d);
        RSK_HIP(hipMemcpyAsync(out + 22 * first, d, 22 * cnt, hipMemcpyDeviceToHost, c->stream));
      }
    });
    RSK_HIP(hipStreamSynchronize(c->stream));
  });
}

int rsk_bloom_bitcount(rsk_bloom* b, uint64_t* out) {
  return guarded([&] {
    need(b && out, "NULL argument");
    rsk_ctx* c = b->ctx;
    CtxLock l(c);
    uint64_t* d = reinterpret_cast<uint64_t*>(c->d_small + 128);
    bloom_bitcount_launch(c, b->d_bits, b->nwords, d);
    RSK_HIP(hipMemcpyAsync(c->h_small + 128, d, 8, hipMemcpyDeviceToHost, c->stream));
    RSK_HIP(hipStreamSynchronize(c->stream));
    std::memcpy(out, c->h_small + 128, 8);
  });
}

int rsk_bloom_count(rsk_bloom* b, int32_t* out) {
  uint64_t bc = 0;
  int rc = rsk_bloom_bitcount(b, &bc);
  if (rc != RSK_OK) return rc;
  return guarded([&] {
    need(out != nullptr, "out is NULL");
    // (int) (-size / ((double) k) * Math.log(1 - bitcount / ((double) size)))
    volatile double a = (double)(-b->size) / (double)b->k;
    volatile double q = (double)bc / (double)b->size;
    volatile double lg = std::log(1 - q);
    *out = java_d2i(a * lg);
  });
}

int rsk_bloom_export_bits(rsk_bloom* b, uint8_t* buf, size_t cap, size_t* len) {
  return guarded([&] {
    need(b && len, "NULL argument");
    need(buf != nullptr && cap >= b->nbytes, "buffer smaller than ceil(size/8)");
    rsk_ctx* c = b->ctx;
    CtxLock l(c);
    if (b->nbytes < (64ull << 20)) {
      RSK_HIP(hipMemcpyAsync(buf, b->d_bits, b->nbytes, hipMemcpyDeviceToHost, c->stream));
      RSK_HIP(hipStreamSynchronize(c->stream));
    } else {
      // a large filter (C3: 1.2 GB) goes out as the batched HLL export's strings do: 16 MiB pieces
      // on the fastest SDMA engine through the pinned ring (or straight into a registered buffer)
      const int eng = export_engine(c);
      hipEvent_t written = nullptr;
      RSK_HIP(hipEventCreateWithFlags(&written, hipEventDisableTiming));
      struct EvGuard {
        hipEvent_t e;
        ~EvGuard() { (void)hipEventDestroy(e); }
      } eg{written};
      RSK_HIP(hipEventRecord(written, c->stream));
      D2HStream xo(c, c->xout, 16ull << 20, eng);
      xo.put(buf, reinterpret_cast<const uint8_t*>(b->d_bits), b->nbytes, written);
      xo.drain();
    }
    *len = b->nbytes;
  });
}

int rsk_bloom_import_bits(rsk_bloom* b, const uint8_t* buf, size_t len) {
  return guarded([&] {
    need(b != nullptr, "NULL argument");
    need(len <= b->nbytes, "bit string longer than the filter");
    need(buf != nullptr || len == 0, "buf is NULL");
    CtxLock l(b->ctx);
    rsk_ctx* c = b->ctx;
    RSK_HIP(hipMemsetAsync(b->d_bits, 0, b->nwords * 4, c->stream));
    const int ein = len >= (64ull << 20) ? copy_engine(c, false) : -1;
    if (ein >= 0) {  // a large string: on the measured SDMA engine through the pinned stages
      RSK_HIP(hipStreamSynchronize(c->stream));  // (the zeroing first)
      H2DStream xi(c, ein, 16ull << 20);
      xi.put(reinterpret_cast<uint8_t*>(b->d_bits), buf, len);
      xi.wait_upto(xi.issued());
    } else if (len >= (64ull << 20)) {
      h2d_staged(c, reinterpret_cast<uint8_t*>(b->d_bits), buf, len);
    } else if (len) {
      RSK_HIP(hipMemcpyAsync(b->d_bits, buf, len, hipMemcpyHostToDevice, c->stream));
    }
    RSK_HIP(hipStreamSynchronize(c->stream));
    ++b->wgen;  // SET of the whole string: its views take STRLEN = len
    ++b->rgen;
    b->set_len = len;
  });
}

int rsk_bloom_or_bits(rsk_bloom* b, const uint8_t* bits, size_t len, uint32_t location) {
  return guarded([&] {
    need(b != nullptr && (bits != nullptr || len == 0), "NULL argument");
    need(len <= b->nbytes, "bit string longer than the filter");
    rsk_ctx* c = b->ctx;
    CtxLock l(c);
    if (len == 0) return;
    ++b->wgen;
    const uint8_t* src = bits;
    if (location == RSK_MEM_HOST) {
      uint8_t* s = out_scratch(c, len);
      RSK_HIP(hipMemcpyAsync(s, bits, len, hipMemcpyHostToDevice, c->stream));
      src = s;
    }
    bloom_or_launch(c, b->d_bits, src, len);
    RSK_HIP(hipStreamSynchronize(c->stream));
  });
}

void* rsk_bloom_device_bits(rsk_bloom* b) {
  if (!b) return nullptr;
  std::lock_guard<std::recursive_mutex> g(b->ctx->mu);
  ++b->wgen;  // the caller may write through the pointer: views rescan their STRLEN
  return b->d_bits;
}

}  // extern "C"

// ------------------------------------------------------------ asynchronous
namespace {

enum AsyncKind { K_PRESET = 0, K_RES_U64 = 1, K_HLL_FLAG = 2, K_OUT_BYTES = 3 };
constexpr uint64_t ASYNC_STAGE_MAX = 256ull << 20;  // larger host batches run synchronously

// Runs on the context's completion thread after the stream passed the op.
// Derives the reply, copies per-key outputs to the caller, hands the op back
// to the pool, then calls the caller.  A device error recorded on the op's
// stream (its completion event reports it) is passed on as RSK_ERR_DEVICE.
void op_complete(AsyncOp* op) {
  uint64_t v = op->value;
  int status = RSK_OK;
  const hipError_t e = hipEventQuery(op->ev_out);
  if (e != hipSuccess && e != hipErrorNotReady) {
    (void)hipGetLastError();
    status = RSK_ERR_DEVICE;
    op->kind = K_PRESET;  // nothing valid to read back
    v = 0;
    op->c->dead = true;
  }
  switch (op->kind) {
    case K_RES_U64:
      v = op->h_res[0];
      break;
    case K_HLL_FLAG:
      v = ((uint32_t)op->h_res[0] == op->epoch || op->created) ? 1 : 0;
      break;
    case K_OUT_BYTES:  // large outputs (a pool's counts: 8 MB at 10^6 sketches) on host threads
      if (op->user_out && op->n_out) par_copy(op->user_out, op->h_out, op->n_out, op->c->stage_threads);
      break;
    default:
      break;
  }
  const rsk_done_fn cb = op->cb;
  void* user = op->user;
  rsk_ctx* c = op->c;
  {
    std::lock_guard<std::mutex> g(c->async_mu);
    c->async_free.push_back(op);
  }
  if (cb) cb(user, status, v);
}

// An op with >= host_bytes of pinned and >= dev_bytes of device buffer
// (called under the context lock; a pooled op is never in flight).
AsyncOp* op_get(rsk_ctx* c, uint64_t host_bytes, uint64_t dev_bytes) {
  AsyncOp* op = nullptr;
  {
    // Best fit: the smallest free op whose buffers already hold the call, else
    // the largest one (grown below).  Growing frees and reallocates pinned and
    // device memory, and hipFree waits for the device: taking ops LIFO made a
    // pipelined C5 step (add, count, countWith, mergeWith: four sizes) regrow
    // buffers every step, with the GPU idle behind each regrowth.
    std::lock_guard<std::mutex> g(c->async_mu);
    size_t best = c->async_free.size();
    for (size_t i = 0; i < c->async_free.size(); ++i) {
      const AsyncOp* o = c->async_free[i];
      const bool fits = o->h_bytes >= host_bytes && o->d_bytes >= dev_bytes;
      if (best == c->async_free.size()) {
        best = i;
        continue;
      }
      const AsyncOp* b = c->async_free[best];
      const bool bfits = b->h_bytes >= host_bytes && b->d_bytes >= dev_bytes;
      if (fits && (!bfits || o->h_bytes + o->d_bytes < b->h_bytes + b->d_bytes)) best = i;
      else if (!fits && !bfits && o->h_bytes + o->d_bytes > b->h_bytes + b->d_bytes) best = i;
    }
    if (best < c->async_free.size()) {
      op = c->async_free[best];
      c->async_free.erase(c->async_free.begin() + best);
    }
  }
  if (!op) {
    op = new AsyncOp();
    op->c = c;
    if (hipHostMalloc(&op->h_res, 64, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      delete op;
      throw RskError{RSK_ERR_OUT_OF_MEMORY, "pinned allocation for an asynchronous call failed"};
    }
    std::lock_guard<std::mutex> g(c->async_mu);
    c->async_all.push_back(op);
  }
  auto give_back = [&] {
    std::lock_guard<std::mutex> g(c->async_mu);
    c->async_free.push_back(op);
  };
  try {
    if (host_bytes > op->h_bytes) {
      if (op->h_buf) RSK_HIP(hipHostFree(op->h_buf));
      op->h_buf = nullptr;
      op->h_bytes = 0;
      const uint64_t sz = std::max<uint64_t>(host_bytes, 1ull << 20);
      RSK_HIP(hipHostMalloc(&op->h_buf, sz, hipHostMallocDefault));
      op->h_bytes = sz;
    }
    if (dev_bytes > op->d_bytes) {
      if (op->d_buf) RSK_HIP(hipFree(op->d_buf));
      op->d_buf = nullptr;
      op->d_bytes = 0;
      const uint64_t sz = std::max<uint64_t>(dev_bytes, 1ull << 20);
      RSK_HIP(hipMalloc(&op->d_buf, sz));
      op->d_bytes = sz;
    }
  } catch (...) {
    give_back();
    throw;
  }
  op->cb = nullptr;
  op->user = nullptr;
  op->kind = K_PRESET;
  op->value = 0;
  op->failed = false;
  op->user_out = op->h_out = nullptr;
  op->n_out = 0;
  op->created = false;
  op->epoch = 0;
  op->on_xfer = false;
  if (!op->ev_in) {
    if (hipEventCreateWithFlags(&op->ev_in, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&op->ev_out, hipEventDisableTiming) != hipSuccess) {
      (void)hipGetLastError();
      give_back();
      throw RskError{RSK_ERR_OUT_OF_MEMORY, "event creation for an asynchronous call failed"};
    }
  }
  return op;
}

void op_release(AsyncOp* op) {  // an op that was taken but will not be submitted (error paths)
  // its copies on the copy streams may still be in flight into its buffers
  (void)hipStreamSynchronize(op->c->xin);
  (void)hipStreamSynchronize(op->c->xout);
  std::lock_guard<std::mutex> g(op->c->async_mu);
  op->c->async_free.push_back(op);
}

// A sticky error on one of the context's streams (a faulted kernel or copy):
// the host functions queued behind it may never run.
bool streams_failed(rsk_ctx* c) {
  for (hipStream_t s : {c->stream, c->xin, c->xout}) {
    const hipError_t e = hipStreamQuery(s);
    if (e != hipSuccess && e != hipErrorNotReady) {
      (void)hipGetLastError();
      return true;
    }
  }
  return false;
}

void done_loop(rsk_ctx* c) {
  (void)hipSetDevice(c->device);
  std::unique_lock<std::mutex> lk(c->done_mu);
  // entries of ops the watchdog already failed (filed before it took them) are dropped
  auto ready = [c] {
    while (!c->done_arrived.empty() && c->done_arrived.begin()->first <= c->done_delivered)
      c->done_arrived.erase(c->done_arrived.begin());
    return !c->done_arrived.empty() && c->done_arrived.begin()->first == c->done_delivered + 1;
  };
  for (;;) {
    const bool woke = c->done_cv.wait_for(lk, std::chrono::milliseconds(500), [&] {
      return ready() || (c->done_stop && c->done_delivered == c->done_submitted);
    });
    if (!woke) {
      // Calls outstanding and nothing arrived for a while: if a stream holds a
      // device error, their host functions may never fire; fail them (in
      // order) rather than leave their callers waiting forever.
      if (c->done_pending.empty() || !streams_failed(c)) continue;
      c->dead = true;
      while (!c->done_pending.empty()) {
        auto it = c->done_pending.begin();
        AsyncOp* op = it->second;
        c->done_pending.erase(it);
        c->done_arrived.erase(op->seq);
        // marked while done_mu is held: a host function of this op firing while the
        // callback below runs (lock released) must not file it again (op_reached)
        op->failed = true;
        lk.unlock();
        if (op->cb) op->cb(op->user, RSK_ERR_DEVICE, 0);  // the op is not recycled: its copies may still be queued
        lk.lock();
        c->done_delivered = std::max(c->done_delivered, op->seq);
        c->done_cv.notify_all();
      }
      continue;
    }
    if (!ready()) return;  // stopping, every op delivered
    AsyncOp* op = c->done_arrived.begin()->second;
    c->done_arrived.erase(c->done_arrived.begin());
    c->done_pending.erase(op->seq);
    lk.unlock();
    op_complete(op);
    lk.lock();
    ++c->done_delivered;
    c->done_cv.notify_all();  // drain_done waiters
  }
}

// A stream's host function: file the op and return at once.
void op_reached(void* p) {
  auto* op = static_cast<AsyncOp*>(p);
  rsk_ctx* c = op->c;
  {
    std::lock_guard<std::mutex> g(c->done_mu);
    if (op->failed || op->seq <= c->done_delivered) return;  // already failed by the watchdog
    c->done_arrived.emplace(op->seq, op);
  }
  c->done_cv.notify_all();
}

// Inputs of an async call: host (pinned, inside op->h_buf) -> device on the
// input stream (so they are not queued behind an earlier call's read-back);
// the context stream waits for them before its next launch.
void op_stage_in(AsyncOp* op, void* dst, const void* src, uint64_t bytes) {
  rsk_ctx* c = op->c;
  RSK_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->xin));
  RSK_HIP(hipEventRecord(op->ev_in, c->xin));
  RSK_HIP(hipStreamWaitEvent(c->stream, op->ev_in, 0));
}

// Outputs of an async call (device memory owned by the op): read back on the
// output stream once the context stream's work so far is done; the call then
// completes on the output stream.
void op_read_back(AsyncOp* op, void* dst, const void* src, uint64_t bytes) {
  rsk_ctx* c = op->c;
  RSK_HIP(hipEventRecord(op->ev_out, c->stream));
  RSK_HIP(hipStreamWaitEvent(c->xout, op->ev_out, 0));
  RSK_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->xout));
  op->on_xfer = true;
}

void op_submit(AsyncOp* op, rsk_done_fn cb, void* user) {
  rsk_ctx* c = op->c;
  op->cb = cb;
  op->user = user;
  // every call completes on the output stream (after an event for the
  // context stream's part): a host function on the context stream would hold
  // the kernels queued behind it for the runtime's round trip (~40 us)
  if (!op->on_xfer) {
    RSK_HIP(hipEventRecord(op->ev_out, c->stream));
    RSK_HIP(hipStreamWaitEvent(c->xout, op->ev_out, 0));
  }
  {
    std::lock_guard<std::mutex> g(c->done_mu);
    if (!c->done_thr.joinable()) c->done_thr = std::thread(done_loop, c);
    op->seq = ++c->done_submitted;  // (callers hold the context lock: one submitter at a time)
    c->done_pending.emplace(op->seq, op);
  }
  const hipError_t e = hipLaunchHostFunc(c->xout, op_reached, op);
  if (e != hipSuccess) {  // never filed: take its number back
    {
      std::lock_guard<std::mutex> g(c->done_mu);
      c->done_pending.erase(op->seq);
      --c->done_submitted;
    }
    RSK_HIP(e);
  }
}

uint64_t al256(uint64_t x) { return (x + 255) & ~uint64_t(255); }

// Bytes of a host batch's keys (+ offsets) as one staged copy.
uint64_t host_key_bytes(const rsk_keys* k) {
  if (k->n == 0) return 0;
  if (!k->offsets) return k->n * k->fixed_len;
  need(k->offsets[k->n] >= k->offsets[0], "offsets must be non-decreasing");
  return al256(k->offsets[k->n] - k->offsets[0]) + 8 * (k->n + 1);
}

// Copies a host batch into op's pinned buffer at `at` (one memcpy by host
// threads) and enqueues one DMA to the op's device buffer; returns the device
// view of the keys.  Device batches are used in place.
DevKeys stage_keys(rsk_ctx* c, const rsk_keys* k, AsyncOp* op, uint64_t at) {
  if (k->location == RSK_MEM_DEVICE || k->n == 0)
    return DevKeys{reinterpret_cast<const uint8_t*>(k->data), k->offsets, k->n, k->fixed_len};
  const uint8_t* src = reinterpret_cast<const uint8_t*>(k->data);
  if (!k->offsets) {
    const uint64_t bytes = k->n * k->fixed_len;
    par_copy(op->h_buf + at, src, bytes, c->stage_threads);
    op_stage_in(op, op->d_buf + at, op->h_buf + at, bytes);
    return DevKeys{op->d_buf + at, nullptr, k->n, k->fixed_len};
  }
  for (uint64_t i = 0; i < k->n; ++i) need(k->offsets[i + 1] >= k->offsets[i], "offsets must be non-decreasing");
  const uint64_t base = k->offsets[0], data_bytes = al256(k->offsets[k->n] - base);
  par_copy(op->h_buf + at, src + base, k->offsets[k->n] - base, c->stage_threads);
  std::memcpy(op->h_buf + at + data_bytes, k->offsets, 8 * (k->n + 1));
  op_stage_in(op, op->d_buf + at, op->h_buf + at, data_bytes + 8 * (k->n + 1));
  // offsets stay absolute: shift the data pointer instead of rebasing
  return DevKeys{op->d_buf + at - base, reinterpret_cast<const uint64_t*>(op->d_buf + at + data_bytes), k->n, 0};
}

// The synchronous call, then the callback on the calling thread (host batches
// above ASYNC_STAGE_MAX: staging them whole would pin that much memory).
template <class F>
int run_now(rsk_ctx* c, F&& sync_call, rsk_done_fn cb, void* user, uint64_t value_if_void, bool value_from_call) {
  uint64_t v = value_if_void;
  const int rc = sync_call(&v);
  if (rc == RSK_OK && cb) {
    drain_done(c, done_mark(c));  // earlier calls' callbacks first
    cb(user, RSK_OK, value_from_call ? v : value_if_void);
  }
  return rc;
}

}  // namespace

extern "C" {

int rsk_hll_add_async(rsk_hll* h, uint64_t id, const rsk_keys* keys, rsk_done_fn cb, void* user) {
  if (keys && keys->location == RSK_MEM_HOST && keys->n && h && id < h->n) {
    uint64_t kb = 0;
    int rc = guarded([&] { kb = host_key_bytes(keys); });
    if (rc != RSK_OK) return rc;
    if (kb > ASYNC_STAGE_MAX)
      return run_now(h->ctx, [&](uint64_t* v) {
        uint8_t ch = 0;
        const int r = rsk_hll_add(h, id, keys, &ch);
        *v = ch;
        return r;
      }, cb, user, 0, true);
  }
  return guarded([&] {
    check_hll(h, id);
    rsk_ctx* c = h->ctx;
    CtxLock l(c);
    check_keys(c, keys);
    const uint64_t kb = keys->location == RSK_MEM_HOST ? host_key_bytes(keys) : 0;
    AsyncOp* op = op_get(c, kb, kb);
    bool created = false;
    try {
      create_if_missing(h, id, &created);
      const bool had_import = h->imported.count(id) != 0;
      uint32_t* d_flag = reinterpret_cast<uint32_t*>(c->d_small);
      if (++c->epoch == 0) {
        RSK_HIP(hipMemsetAsync(d_flag, 0, 4, c->stream));
        c->epoch = 1;
      }
      op->epoch = c->epoch;
      op->created = created;
      op->kind = K_HLL_FLAG;
      const DevKeys dk = stage_keys(c, keys, op, 0);
      if (dk.n) hll_add_launch(c, dk, regs_of(h, id), h->d_card + id, d_flag, op->epoch, created);
      else if (created) invalidate(h, id, nullptr, true);
      RSK_HIP(hipMemcpyAsync(op->h_res, d_flag, 4, hipMemcpyDeviceToHost, c->stream));
      if (had_import) {
        // A kept SET string survives a PFADD that changes nothing (as rsk_hll_add): the
        // decision needs the flag before any later call reads the key, so this (rare)
        // call waits for it here instead of in the completion.
        RSK_HIP(hipStreamSynchronize(c->stream));
        if ((uint32_t)op->h_res[0] == op->epoch || created) hll_forget_import(h, id);
      }
      op_submit(op, cb, user);
    } catch (...) {
      (void)hipStreamSynchronize(c->stream);
      op_release(op);
      throw;
    }
  });
}

int rsk_hll_count_async(rsk_hll* h, uint64_t id, rsk_done_fn cb, void* user) {
  return guarded([&] {
    check_hll(h, id);
    rsk_ctx* c = h->ctx;
    CtxLock l(c);
    AsyncOp* op = op_get(c, 0, 256);
    try {
      SmallIds small{};
      small.v[0] = id;
      small.n = 1;
      uint64_t* d_out = reinterpret_cast<uint64_t*>(op->d_buf);
      hll_count_launch(c, h->d_regs, h->d_card, nullptr, small, 1, d_out, PCount{h->d_pcount, h->d_pepoch, h->pc_epoch});
      RSK_HIP(hipMemcpyAsync(op->h_res, d_out, 8, hipMemcpyDeviceToHost, c->stream));
      op->kind = K_RES_U64;
      op_submit(op, cb, user);
    } catch (...) {
      (void)hipStreamSynchronize(c->stream);
      op_release(op);
      throw;
    }
  });
}

int rsk_hll_count_union_async(rsk_hll* const* hs, const uint64_t* ids, uint32_t k, rsk_done_fn cb, void* user) {
  return guarded([&] {
    need(hs && ids && k >= 1 && hs[0], "bad arguments");
    rsk_ctx* c = hs[0]->ctx;
    CtxLock l(c);
    for (uint32_t a = 0; a < k; ++a) {
      check_hll(hs[a], ids[a]);
      need(hs[a]->ctx == c, "all sketches must share one context");
    }
    const uint64_t pb = al256(8ull * k);
    AsyncOp* op = op_get(c, pb, pb + 256);
    try {
      auto* ptrs = reinterpret_cast<const uint8_t**>(op->h_buf);
      for (uint32_t a = 0; a < k; ++a) ptrs[a] = hs[a]->exists[ids[a]] ? regs_of(hs[a], ids[a]) : nullptr;
      auto* d_ptrs = reinterpret_cast<const uint8_t**>(op->d_buf);
      auto* d_out = reinterpret_cast<uint64_t*>(op->d_buf + pb);
      RSK_HIP(hipMemcpyAsync(d_ptrs, ptrs, 8ull * k, hipMemcpyHostToDevice, c->stream));
      hll_union_count_launch(c, d_ptrs, k, 1, d_out);
      RSK_HIP(hipMemcpyAsync(op->h_res, d_out, 8, hipMemcpyDeviceToHost, c->stream));
      op->kind = K_RES_U64;
      op_submit(op, cb, user);
    } catch (...) {
      (void)hipStreamSynchronize(c->stream);
      op_release(op);
      throw;
    }
  });
}

int rsk_hll_merge_async(rsk_hll* dst, uint64_t dst_id, rsk_hll* const* srcs, const uint64_t* src_ids, uint32_t k,
                        rsk_done_fn cb, void* user) {
  return guarded([&] {
    check_hll(dst, dst_id);
    need(k == 0 || (srcs && src_ids), "srcs is NULL");
    rsk_ctx* c = dst->ctx;
    CtxLock l(c);
    for (uint32_t a = 0; a < k; ++a) {
      check_hll(srcs[a], src_ids[a]);
      need(srcs[a]->ctx == c, "all sketches must share one context");
    }
    const uint64_t pb = al256(8ull * k + 8);
    AsyncOp* op = op_get(c, pb, pb);
    try {
      auto* ptrs = reinterpret_cast<const uint8_t**>(op->h_buf);
      ptrs[0] = regs_of(dst, dst_id);
      for (uint32_t a = 0; a < k; ++a) ptrs[1 + a] = srcs[a]->exists[src_ids[a]] ? regs_of(srcs[a], src_ids[a]) : nullptr;
      bool created;
      create_if_missing(dst, dst_id, &created);
      hll_forget_import(dst, dst_id);
      dst->dense[dst_id] = 1;  // pfmergeCommand converts the destination to dense
      if (k) {
        RSK_HIP(hipMemcpyAsync(op->d_buf, ptrs, 8ull * (k + 1), hipMemcpyHostToDevice, c->stream));
        hll_merge_launch(c, reinterpret_cast<uint8_t**>(op->d_buf), reinterpret_cast<const uint8_t**>(op->d_buf) + 1, k, 1);
      }
      invalidate(dst, dst_id, nullptr, true);
      op_submit(op, cb, user);
    } catch (...) {
      (void)hipStreamSynchronize(c->stream);
      op_release(op);
      throw;
    }
  });
}

int rsk_hll_merge_batch_async(rsk_hll* h, const uint64_t* dst_ids, const uint64_t* src_ids, uint64_t n, rsk_done_fn cb,
                              void* user) {
  return guarded([&] {
    need(h && (n == 0 || (dst_ids && src_ids)), "NULL argument");
    rsk_ctx* c = h->ctx;
    CtxLock l(c);
    merge_batch_check(h, dst_ids, src_ids, n);
    AsyncOp* op = op_get(c, n ? merge_batch_host_bytes(n) : 0, n ? merge_batch_dev_bytes(n) : 0);
    try {
      if (n) merge_batch_enqueue(h, dst_ids, src_ids, n, op->h_buf, op->d_buf, op);
      op_submit(op, cb, user);
    } catch (...) {
      (void)hipStreamSynchronize(c->stream);
      op_release(op);
      throw;
    }
  });
}

int rsk_hll_add_grouped_async(rsk_hll* h, const rsk_keys* keys, const uint32_t* groups, rsk_done_fn cb,
                              void* user) {
  if (h && keys && keys->location == RSK_MEM_HOST && keys->n) {
    uint64_t kb = 0;
    int rc = guarded([&] { kb = host_key_bytes(keys) + 4 * keys->n; });
    if (rc != RSK_OK) return rc;
    if (kb > ASYNC_STAGE_MAX) return run_now(h->ctx, [&](uint64_t*) { return rsk_hll_add_grouped(h, keys, groups); }, cb, user, 0, false);
  }
  return guarded([&] {
    need(h != nullptr, "hll handle is NULL");
    need(keys == nullptr || keys->n == 0 || groups != nullptr, "groups is NULL");
    rsk_ctx* c = h->ctx;
    CtxLock l(c);
    check_keys(c, keys);
    check_out(c, keys, groups);
    const bool host = keys->location == RSK_MEM_HOST;
    const uint64_t kb = host ? al256(host_key_bytes(keys)) : 0;
    const uint64_t gb = host ? al256(4 * keys->n) : 0;
    AsyncOp* op = op_get(c, kb + gb, kb + gb);
    try {
      if (keys->n) {
        const DevKeys dk = stage_keys(c, keys, op, 0);
        const uint32_t* d_groups = groups;
        if (host) {
          std::memcpy(op->h_buf + kb, groups, 4 * keys->n);
          op_stage_in(op, op->d_buf + kb, op->h_buf + kb, 4 * keys->n);
          d_groups = reinterpret_cast<const uint32_t*>(op->d_buf + kb);
        }
        hll_add_grouped_enqueue(h, dk, d_groups, host ? groups : nullptr);
      }
      op->value = keys->n;
      op_submit(op, cb, user);
    } catch (...) {
      (void)hipStreamSynchronize(c->stream);
      op_release(op);
      throw;
    }
  });
}

int rsk_hll_count_ids_async(rsk_hll* h, const uint64_t* ids, uint64_t n, uint64_t* out, rsk_done_fn cb, void* user) {
  return guarded([&] {
    need(h != nullptr && out != nullptr, "NULL argument");
    rsk_ctx* c = h->ctx;
    CtxLock l(c);
    if (ids) check_hll_ids(h, ids, n, nullptr, 0, false);
    else need(n <= h->n, "n exceeds pool size");
    const uint64_t ib = ids ? al256(8 * n) : 0, ob = al256(8 * n);
    AsyncOp* op = op_get(c, ib + ob, ib + ob);
    try {
      if (!ids) hll_materialize(h);  // (listed ids: check_hll_ids above)
      if (n) {
        uint64_t* d_ids = nullptr;
        if (ids) {
          std::memcpy(op->h_buf, ids, 8 * n);
          op_stage_in(op, op->d_buf, op->h_buf, 8 * n);
          d_ids = reinterpret_cast<uint64_t*>(op->d_buf);
        }
        auto* d_out = reinterpret_cast<uint64_t*>(op->d_buf + ib);
        hll_count_launch(c, h->d_regs, h->d_card, d_ids, SmallIds{}, n, d_out,
                         PCount{h->d_pcount, h->d_pepoch, h->pc_epoch});
        op_read_back(op, op->h_buf + ib, d_out, 8 * n);
        op->h_out = op->h_buf + ib;
        op->user_out = reinterpret_cast<uint8_t*>(out);
        op->n_out = 8 * n;
      }
      op->kind = K_OUT_BYTES;
      op->value = n;
      op_submit(op, cb, user);
    } catch (...) {
      (void)hipStreamSynchronize(c->stream);
      op_release(op);
      throw;
    }
  });
}

int rsk_hll_count_union_batch_async(rsk_hll* h, const uint64_t* member_ids, uint32_t arity, uint64_t n,
                                    uint64_t* out, rsk_done_fn cb, void* user) {
  return guarded([&] {
    need(h && member_ids && out && arity >= 1, "bad arguments");
    rsk_ctx* c = h->ctx;
    CtxLock l(c);
    check_hll_ids(h, member_ids, n * arity, nullptr, 0, false);
    const uint64_t pb = al256(8 * n * arity), ob = al256(8 * n);
    AsyncOp* op = op_get(c, pb + ob, pb + ob);
    try {
      if (n) {
        auto* ptrs = reinterpret_cast<const uint8_t**>(op->h_buf);
        const uint8_t* e = h->exists.data();
        for (uint64_t i = 0; i < n * arity; ++i) {  // members as they stand at this point of the call order
          const uint64_t id = member_ids[i];
          ptrs[i] = e[id] ? regs_of(h, id) : nullptr;
        }
        auto* d_ptrs = reinterpret_cast<const uint8_t**>(op->d_buf);
        auto* d_out = reinterpret_cast<uint64_t*>(op->d_buf + pb);
        op_stage_in(op, d_ptrs, ptrs, 8 * n * arity);
        hll_union_count_launch(c, d_ptrs, arity, n, d_out);
        op_read_back(op, op->h_buf + pb, d_out, 8 * n);
        op->h_out = op->h_buf + pb;
        op->user_out = reinterpret_cast<uint8_t*>(out);
        op->n_out = 8 * n;
      }
      op->kind = K_OUT_BYTES;
      op->value = n;
      op_submit(op, cb, user);
    } catch (...) {
      (void)hipStreamSynchronize(c->stream);
      op_release(op);
      throw;
    }
  });
}

}  // extern "C"

namespace {
// Shared body of the Bloom async calls: keys staged, `launch` enqueues the
// kernels writing per-key outputs to d_out, outputs read back for host keys.
template <class L>
int bloom_async(rsk_bloom* b, const rsk_keys* keys, uint8_t* out, bool out_required, rsk_done_fn cb, void* user,
                L&& launch, int (*sync_call)(rsk_bloom*, const rsk_keys*, uint8_t*)) {
  if (b && keys && keys->location == RSK_MEM_HOST && keys->n) {
    uint64_t kb = 0;
    int rc = guarded([&] { kb = host_key_bytes(keys) + keys->n; });
    if (rc != RSK_OK) return rc;
    if (kb > ASYNC_STAGE_MAX)
      return run_now(b->ctx, [&](uint64_t*) { return sync_call(b, keys, out); }, cb, user, keys->n, false);
  }
  return guarded([&] {
    need(b != nullptr, "bloom handle is NULL");
    need(!out_required || out != nullptr, "out is NULL");
    rsk_ctx* c = b->ctx;
    CtxLock l(c);
    check_keys(c, keys);
    check_out(c, keys, out);
    const bool host = keys->location == RSK_MEM_HOST;
    const uint64_t kb = host ? al256(host_key_bytes(keys)) : 0;
    const uint64_t ob = (host && out) ? keys->n : 0;
    if (!out_required) ++b->wgen;  // an add (contains writes no bit)
    AsyncOp* op = op_get(c, kb + ob, kb + ob);
    try {
      const DevKeys dk = stage_keys(c, keys, op, 0);
      uint8_t* d_out = out ? (host ? op->d_buf + kb : out) : nullptr;
      if (dk.n) launch(c, b, dk, d_out);
      if (host && out && keys->n) {
        op_read_back(op, op->h_buf + kb, d_out, keys->n);
        op->h_out = op->h_buf + kb;
        op->user_out = out;
        op->n_out = keys->n;
      }
      op->kind = K_OUT_BYTES;
      op->value = keys->n;
      op_submit(op, cb, user);
    } catch (...) {
      (void)hipStreamSynchronize(c->stream);
      op_release(op);
      throw;
    }
  });
}
}  // namespace

extern "C" {

int rsk_bloom_add_async(rsk_bloom* b, const rsk_keys* keys, uint8_t* added_out, rsk_done_fn cb, void* user) {
  return bloom_async(
      b, keys, added_out, false, cb, user,
      [](rsk_ctx* c, rsk_bloom* bf, const DevKeys& dk, uint8_t* d_out) {
        if (d_out) bloom_add_replies_launch(c, bf, dk, d_out);
        else bloom_add_launch(c, bf, dk);
      },
      rsk_bloom_add);
}

int rsk_bloom_contains_async(rsk_bloom* b, const rsk_keys* keys, uint8_t* out, rsk_done_fn cb, void* user) {
  return bloom_async(
      b, keys, out, true, cb, user,
      [](rsk_ctx* c, rsk_bloom* bf, const DevKeys& dk, uint8_t* d_out) { bloom_contains_launch(c, bf, dk, d_out); },
      rsk_bloom_contains);
}

}  // extern "C"
