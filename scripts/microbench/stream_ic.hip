// Infinity-Cache residency microbenchmark for the objective pass: read a buffer of B bytes again
// and again (back-to-back launches, as consecutive BFGS passes do), in the CorrSoA layout's
// 16-B-per-lane loads, for B from 120 MB to 360 MB.  If the streamed bytes of a pass fit the
// 256 MiB Infinity Cache, the re-reads should run above the ~6 TB/s HBM rate.
// Usage: ./stream_ic [blocks]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

// grid-stride float4 stream; rev: walk back to front
__global__ __launch_bounds__(256) void stream(const float4* p, size_t nvec, int rev, double* out) {
  double acc = 0;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x; t < nvec; t += stride) {
    const size_t i = rev ? nvec - 1 - t : t;
    float4 v = p[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 12345.678) out[0] = acc;
}

// same, 8 loads in flight per lane per iteration (wave-contiguous 8 KiB pieces)
__global__ __launch_bounds__(256) void stream8(const float4* p, size_t nvec, int rev, double* out) {
  double acc = 0;
  const size_t nw = (size_t)gridDim.x * 4;
  const size_t w = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const size_t npiece = nvec / 512;
  for (size_t t = w; t < npiece; t += nw) {
    const size_t pc = rev ? npiece - 1 - t : t;
    const float4* q = p + pc * 512 + lane;
    float4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = q[64 * k];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += v[k].x + v[k].y + v[k].z + v[k].w;
  }
  if (acc == 12345.678) out[0] = acc;
}

int main(int argc, char** argv) {
  const int nb = argc > 1 ? atoi(argv[1]) : 1024;
  const size_t maxb = 360000000;
  void* buf;
  CK(hipMalloc(&buf, maxb + 4096));
  CK(hipMemset(buf, 0, maxb + 4096));
  double* out;
  CK(hipMalloc(&out, 8));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const size_t sizes[] = {120000000, 160000000, 200000000, 220000000, 240000000, 260000000, 280000000, 300000000, 360000000};
  for (int kind = 0; kind < 2; ++kind) {
    for (size_t bytes : sizes) {
      const size_t nvec = bytes / 16 / 512 * 512;
      for (int alt = 0; alt < 2; ++alt) {
        auto launch = [&](int r) {
          const int rev = alt ? (r & 1) : 0;
          if (kind == 0) stream<<<nb, 256>>>((const float4*)buf, nvec, rev, out);
          else stream8<<<nb, 256>>>((const float4*)buf, nvec, rev, out);
        };
        for (int w = 0; w < 4; ++w) launch(w);
        CK(hipDeviceSynchronize());
        const int reps = 40;
        CK(hipEventRecord(a));
        for (int r = 0; r < reps; ++r) launch(r);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        const double us = 1e3 * ms / reps;
        printf("%-8s %s blocks %5d  %6.0f MB  %7.1f us  %6.2f TB/s\n", kind ? "stream8" : "stream",
               alt ? "alternating" : "forward    ", nb, nvec * 16 / 1e6, us, nvec * 16.0 / (us * 1e-6) / 1e12);
      }
    }
  }
  return 0;
}
