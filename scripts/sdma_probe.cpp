// Host<->device copy rate per SDMA engine (GPU box only; measurement aid, not product).
//
// Round-6 probe for the checkpoint export's bimodal device->host rate (DESIGN.md §4
// round 6): a process either moves ~57 GB/s or ~30 GB/s over the host link on every
// hipMemcpyAsync, whatever the stream (profiles/r06_copy_streams.jsonl). This times
// hsa_amd_memory_async_copy_on_engine on each SDMA engine the runtime reports, plus the
// auto-assigned hsa_amd_memory_async_copy and hipMemcpyAsync, in one process.
//
// Build: hipcc --offload-arch=gfx950 -O2 scripts/sdma_probe.cpp -o scripts/sdma_probe -lhsa-runtime64
//        (and -shared -fPIC -DSDMA_PROBE_LIB -o scripts/libsdma_probe.so for an in-process call
//        from scripts/io_profile.py, IO_SDMA=1)
// Run:   scripts/sdma_probe [MiB] [memset_first=1] [engines=16]   (one JSON line per measurement)
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define HIPCK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)
#define HSACK(x) do { hsa_status_t s_ = (x); if (s_ != HSA_STATUS_SUCCESS) { \
  std::fprintf(stderr, "%s: hsa status 0x%x\n", #x, (unsigned)s_); std::exit(1); } } while (0)

static std::vector<hsa_agent_t> g_gpu, g_cpu;

static hsa_status_t agent_cb(hsa_agent_t a, void*) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU) g_gpu.push_back(a);
  if (t == HSA_DEVICE_TYPE_CPU) g_cpu.push_back(a);
  return HSA_STATUS_SUCCESS;
}

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// One timed HSA copy; engine 0 = auto-assigned (hsa_amd_memory_async_copy).
static double hsa_copy(void* dst, hsa_agent_t da, const void* src, hsa_agent_t sa, size_t n,
                       uint32_t engine, hsa_status_t* st) {
  hsa_signal_t sig;
  HSACK(hsa_signal_create(1, 0, nullptr, &sig));
  double t = now();
  *st = engine ? hsa_amd_memory_async_copy_on_engine(dst, da, src, sa, n, 0, nullptr, sig,
                                                     (hsa_amd_sdma_engine_id_t)engine, true)
               : hsa_amd_memory_async_copy(dst, da, src, sa, n, 0, nullptr, sig);
  if (*st != HSA_STATUS_SUCCESS) { hsa_signal_destroy(sig); return 0; }
  while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX,
                                   HSA_WAIT_STATE_ACTIVE) >= 1) {}
  double dt = now() - t;
  hsa_signal_destroy(sig);
  return n / dt / 1e9;
}

extern "C" int sdma_probe_run(size_t mib, int memset_first, int engines) {
  size_t n = mib << 20;
  HIPCK(hipSetDevice(0));
  void *dev = nullptr, *host = nullptr;
  HIPCK(hipMalloc(&dev, n));
  HIPCK(hipHostMalloc(&host, n, 0));
  if (memset_first) HIPCK(hipMemset(dev, 1, n));
  HIPCK(hipDeviceSynchronize());
  HSACK(hsa_init());
  g_gpu.clear();
  g_cpu.clear();
  HSACK(hsa_iterate_agents(agent_cb, nullptr));
  if (g_gpu.empty() || g_cpu.empty()) { std::fprintf(stderr, "no agents\n"); return 1; }
  hsa_agent_t gpu = g_gpu[0], cpu = g_cpu[0];
  uint32_t st_d2h = 0, st_h2d = 0, pr_d2h = 0, pr_h2d = 0;
  hsa_amd_memory_copy_engine_status(cpu, gpu, &st_d2h);
  hsa_amd_memory_copy_engine_status(gpu, cpu, &st_h2d);
  hsa_amd_memory_get_preferred_copy_engine(cpu, gpu, &pr_d2h);
  hsa_amd_memory_get_preferred_copy_engine(gpu, cpu, &pr_h2d);
  std::printf("{\"gpus\": %zu, \"cpus\": %zu, \"d2h_available\": \"0x%x\", \"h2d_available\": \"0x%x\", "
              "\"d2h_preferred\": \"0x%x\", \"h2d_preferred\": \"0x%x\", \"bytes\": %zu}\n",
              g_gpu.size(), g_cpu.size(), st_d2h, st_h2d, pr_d2h, pr_h2d, n);
  std::fflush(stdout);

  hipStream_t s;
  HIPCK(hipStreamCreate(&s));
  auto hip_rate = [&](hipMemcpyKind k) {
    double r[3];
    for (double& x : r) {
      double t = now();
      HIPCK(hipMemcpyAsync(k == hipMemcpyDeviceToHost ? host : dev,
                           k == hipMemcpyDeviceToHost ? dev : host, n, k, s));
      HIPCK(hipStreamSynchronize(s));
      x = n / (now() - t) / 1e9;
    }
    std::printf("{\"path\": \"hipMemcpyAsync\", \"dir\": \"%s\", \"GBps\": [%.1f, %.1f, %.1f]}\n",
                k == hipMemcpyDeviceToHost ? "d2h" : "h2d", r[0], r[1], r[2]);
    std::fflush(stdout);
  };
  hip_rate(hipMemcpyDeviceToHost);
  hip_rate(hipMemcpyHostToDevice);

  for (int e = -1; e < engines; ++e) {
    uint32_t eng = e < 0 ? 0 : (1u << e);
    for (int dir = 0; dir < 2; ++dir) {
      double r[3];
      hsa_status_t st = HSA_STATUS_SUCCESS;
      for (double& x : r) {
        x = dir == 0 ? hsa_copy(host, cpu, dev, gpu, n, eng, &st)
                     : hsa_copy(dev, gpu, host, cpu, n, eng, &st);
        if (st != HSA_STATUS_SUCCESS) break;
      }
      if (st != HSA_STATUS_SUCCESS) {
        std::printf("{\"engine\": %d, \"dir\": \"%s\", \"status\": \"0x%x\"}\n", e,
                    dir ? "h2d" : "d2h", (unsigned)st);
      } else {
        std::printf("{\"engine\": %d, \"dir\": \"%s\", \"GBps\": [%.1f, %.1f, %.1f]}\n", e,
                    dir ? "h2d" : "d2h", r[0], r[1], r[2]);
      }
      std::fflush(stdout);
    }
  }
  hip_rate(hipMemcpyDeviceToHost);
  HIPCK(hipStreamDestroy(s));
  HIPCK(hipFree(dev));
  HIPCK(hipHostFree(host));
  hsa_shut_down();
  return 0;
}

#ifndef SDMA_PROBE_LIB
int main(int argc, char** argv) {
  return sdma_probe_run(argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 256,
                        argc > 2 ? std::atoi(argv[2]) : 1, argc > 3 ? std::atoi(argv[3]) : 16);
}
#endif
