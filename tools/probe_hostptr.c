/* Probe (no kernel launches): does the system ROCm runtime map hipHostMalloc memory at the
 * host address on the device (the transport passes &flags_[r] to kernels directly)? */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
int main(void) {
  hipSetDevice(0);
  int rt = 0, drv = 0;
  hipRuntimeGetVersion(&rt);
  hipDriverGetVersion(&drv);
  printf("runtime %d driver %d\n", rt, drv);
  unsigned flags[3] = {hipHostMallocCoherent | hipHostMallocMapped, hipHostMallocDefault, hipHostMallocMapped | hipHostMallocPortable};
  for (int k = 0; k < 3; ++k) {
    void* h = NULL;
    void* d = NULL;
    hipError_t e = hipHostMalloc(&h, 4096, flags[k]);
    hipError_t e2 = hipHostGetDevicePointer(&d, h, 0);
    hipPointerAttribute_t at;
    hipError_t e3 = hipPointerGetAttributes(&at, h);
    printf("flags 0x%x: alloc %d host %p dev %p (%d) attr %d type %d devptr %p hostptr %p\n", flags[k], (int)e, h, d,
           (int)e2, (int)e3, (int)at.type, at.devicePointer, at.hostPointer);
    hipHostFree(h);
  }
  return 0;
}
