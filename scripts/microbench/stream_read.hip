// Streaming-read microbenchmark for the objective-pass layout question: how fast can MI355X read
// 360 MB (5M correspondences x 72 B) as (a) 12 separate streams (the CorrSoA layout), (b) one
// contiguous stream, (c) blocked SoA (per 1024 correspondences: 12 sub-streams adjacent)?
// Each variant sums the data (fp64) so nothing is optimised away.  Usage: ./stream_read [blocks]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr size_t kN = 5000000;          // correspondences
constexpr size_t kN4 = kN / 4;          // float4 groups

// (a) 6 float streams + 6 double streams, 4 correspondences per thread-iteration
__global__ __launch_bounds__(256) void soa12(const float4* f, const double2* d, size_t n4, double* out) {
  double acc = 0;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
#pragma unroll
    for (int s = 0; s < 6; ++s) { float4 v = f[s * n4 + i]; acc += v.x + v.y + v.z + v.w; }
#pragma unroll
    for (int s = 0; s < 6; ++s) { double2 a = d[s * 2 * n4 + 2 * i], b = d[s * 2 * n4 + 2 * i + 1]; acc += a.x + a.y + b.x + b.y; }
  }
  if (acc == 12345.678) out[0] = acc;
}

// (b) one contiguous stream of float4 (same byte count), 18 loads per thread-iteration
__global__ __launch_bounds__(256) void one_stream(const float4* p, size_t nvec, double* out) {
  double acc = 0;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += stride) {
    float4 v = p[i]; acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 12345.678) out[0] = acc;
}

// (c) blocked SoA: chunk of 1024 correspondences = 18 x 1 KiB sub-streams back to back (18 KiB);
// thread t of a 256-thread block reads group t of every sub-stream of its chunk
__global__ __launch_bounds__(256) void blocked(const float4* p, size_t nchunks, double* out) {
  double acc = 0;
  for (size_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const float4* base = p + c * (18 * 64);
#pragma unroll
    for (int s = 0; s < 18; ++s) {
      // each sub-stream holds 64 float4 per 256 threads? -> 1 KiB = 64 float4: use 4 lanes per vec
      float4 v = base[s * 64 + (threadIdx.x & 63)];
      acc += v.x + v.y + v.z + v.w;
    }
  }
  if (acc == 12345.678) out[0] = acc;
}

int main(int argc, char** argv) {
  int nb = argc > 1 ? atoi(argv[1]) : 256;
  const size_t bytes = kN * 72;
  void* buf;
  CK(hipMalloc(&buf, bytes + 4096));
  CK(hipMemset(buf, 0, bytes + 4096));
  double* out;
  CK(hipMalloc(&out, 8));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto time = [&](auto launch, const char* name, double nbytes) {
    for (int w = 0; w < 3; ++w) launch();
    CK(hipDeviceSynchronize());
    const int reps = 50;
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    const double us = 1e3 * ms / reps;
    printf("%-28s blocks %5d  %7.1f us  %6.2f TB/s\n", name, nb, us, nbytes / (us * 1e-6) / 1e12);
  };
  const float4* f = (const float4*)buf;
  const double2* d = (const double2*)((char*)buf + 6 * kN * 4);
  time([&] { soa12<<<nb, 256>>>(f, d, kN4, out); }, "soa12 (CorrSoA)", bytes);
  time([&] { one_stream<<<nb, 256>>>(f, bytes / 16, out); }, "one contiguous stream", bytes);
  // blocked: 18 KiB chunks (1024 correspondences at 72 B would be 72 KiB; read pattern only)
  time([&] { blocked<<<nb, 256>>>(f, bytes / (18 * 1024), out); }, "blocked 18x1KiB chunks", (double)(bytes / (18 * 1024)) * 18 * 1024);
  return 0;
}
