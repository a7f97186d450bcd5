// Minimal HIP program for the rocprofv3 exit probe (tools/exit_probe.py): one allocation, one kernel,
// one synchronize, exit.  Under rocprofv3 it tells whether a fault after the tool's finalization comes
// from the HIP runtime's own exit handler (this program has no other library) or from libkgpu / torch.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_fill(int* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = i;
}

int main() {
  int* d = nullptr;
  const int n = 1 << 16;
  if (hipMalloc(&d, n * sizeof(int)) != hipSuccess) return 1;
  hipLaunchKernelGGL(k_fill, dim3(n / 256), dim3(256), 0, 0, d, n);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  int h = 0;
  if (hipMemcpy(&h, d + 77, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return 3;
  (void)hipFree(d);
  std::printf("exit_probe_min: %d\n", h);
  return h == 77 ? 0 : 4;
}
