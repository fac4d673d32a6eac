// Probe: can the host CPU store straight into device memory (fine-grained VRAM through the BAR)?
// Allocates a small fine-grained device buffer, reports its pointer attributes, then (argv[1] ==
// "touch") writes and reads it from the CPU and checks a kernel sees the write.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>

__global__ void read_kernel(const volatile unsigned long long* p, unsigned long long* out) { out[0] = p[0]; }

int main(int argc, char** argv) {
  unsigned long long* d = nullptr;
  hipError_t e = hipExtMallocWithFlags(reinterpret_cast<void**>(&d), 4096, hipDeviceMallocFinegrained);
  printf("fine-grained alloc: %s ptr %p\n", hipGetErrorString(e), (void*)d);
  if (e != hipSuccess) return 1;
  hipPointerAttribute_t at;
  e = hipPointerGetAttributes(&at, d);
  printf("attributes: %s type %d device %d hostPointer %p devicePointer %p isManaged %d\n", hipGetErrorString(e),
         (int)at.type, at.device, at.hostPointer, at.devicePointer, (int)at.isManaged);
  if (argc > 1 && !strcmp(argv[1], "touch")) {
    volatile unsigned long long* h = d;
    h[0] = 0x1234567890abcdefull;
    printf("cpu read back %llx\n", (unsigned long long)h[0]);
    unsigned long long* o = nullptr;
    (void)hipMalloc(&o, 8);
    read_kernel<<<1, 1>>>(d, o);
    unsigned long long v = 0;
    (void)hipMemcpy(&v, o, 8, hipMemcpyDeviceToHost);
    printf("kernel saw %llx\n", v);
  }
  return 0;
}
