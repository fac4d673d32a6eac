// r05 microbenchmark: does a host->device copy slow down while a latency-bound kernel (the k-NN's shape:
// ~78k one-wave blocks of dependent gathers) runs on another stream?  hipMemcpyAsync from pinned slots
// (what host_upload.hpp does) against hsa_amd_memory_async_copy (the SDMA engines).
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)
#define HK(x) do { hsa_status_t e_ = (x); if (e_ != HSA_STATUS_SUCCESS) { std::printf("HSA %d line %d\n", (int)e_, __LINE__); std::exit(1); } } while (0)

__global__ __launch_bounds__(64) void chase(const unsigned* __restrict__ nxt, unsigned mask, int steps, unsigned* out) {
  unsigned i = (blockIdx.x * 64u + threadIdx.x) * 2654435761u & mask;
  for (int s = 0; s < steps; ++s) i = nxt[i] & mask;
  if (i == 0xffffffffu) out[0] = i;
}

static double now() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

hsa_agent_t g_gpu{}, g_cpu{};
static hsa_status_t pick(hsa_agent_t a, void*) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU && !g_gpu.handle) g_gpu = a;
  if (t == HSA_DEVICE_TYPE_CPU && !g_cpu.handle) g_cpu = a;
  return HSA_STATUS_SUCCESS;
}

int main() {
  const size_t slot = size_t(8) << 20, total = size_t(60) << 20;
  const int nslots = 4;
  std::vector<void*> pin(nslots);
  for (auto& p : pin) { CK(hipHostMalloc(&p, slot, hipHostMallocDefault)); std::memset(p, 1, slot); }
  char* d = nullptr;
  CK(hipMalloc(&d, total));
  const unsigned N = 1u << 26;  // 256 MB chase table
  unsigned* nxt = nullptr;
  unsigned* out = nullptr;
  CK(hipMalloc(&nxt, size_t(N) * 4));
  CK(hipMalloc(&out, 64));
  {
    std::vector<unsigned> h(N);
    unsigned x = 12345;
    for (unsigned i = 0; i < N; ++i) { x = x * 1664525u + 1013904223u; h[i] = x; }
    CK(hipMemcpy(nxt, h.data(), size_t(N) * 4, hipMemcpyHostToDevice));
  }
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  std::vector<hipEvent_t> ev(nslots);
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HK(hsa_iterate_agents(pick, nullptr));
  std::vector<hsa_signal_t> sig(nslots);
  for (auto& s : sig) HK(hsa_signal_create(0, 0, nullptr, &s));

  auto busy = [&](int steps) { chase<<<78125, 64, 0, a>>>(nxt, N - 1, steps, out); };
  auto copy_hip = [&]() {
    const double t0 = now();
    for (size_t c = 0, k = 0; c < total; c += slot, ++k) {
      const int s = k % nslots;
      CK(hipEventSynchronize(ev[s]));
      CK(hipMemcpyAsync(d + c, pin[s], std::min(slot, total - c), hipMemcpyHostToDevice, b));
      CK(hipEventRecord(ev[s], b));
    }
    CK(hipStreamSynchronize(b));
    return now() - t0;
  };
  bool used[4] = {};
  auto copy_hsa = [&]() {
    const double t0 = now();
    for (size_t c = 0, k = 0; c < total; c += slot, ++k) {
      const int s = k % nslots;
      if (used[s]) hsa_signal_wait_scacquire(sig[s], HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE);
      hsa_signal_store_relaxed(sig[s], 1);
      HK(hsa_amd_memory_async_copy(d + c, g_gpu, pin[s], g_cpu, std::min(slot, total - c), 0, nullptr, sig[s]));
      used[s] = true;
    }
    for (int s = 0; s < nslots; ++s)
      if (used[s]) hsa_signal_wait_scacquire(sig[s], HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_ACTIVE);
    return now() - t0;
  };
  // the busy kernel alone
  for (int steps : {100, 400}) {
    CK(hipDeviceSynchronize());
    double t0 = now();
    busy(steps);
    CK(hipStreamSynchronize(a));
    std::printf("busy kernel %d steps alone: %.3f ms\n", steps, now() - t0);
  }
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipDeviceSynchronize());
    std::printf("rep %d: hip copy alone %.3f ms", rep, copy_hip());
    std::printf(", hsa copy alone %.3f ms", copy_hsa());
    busy(400);
    std::printf(", hip copy beside busy %.3f ms", copy_hip());
    CK(hipStreamSynchronize(a));
    busy(400);
    std::printf(", hsa copy beside busy %.3f ms\n", copy_hsa());
    CK(hipStreamSynchronize(a));
  }
  std::printf("done\n");
  return 0;
}
