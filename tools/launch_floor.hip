// Microbenchmark: per-launch floor of dependent kernels on one stream (MI355X), to size the
// per-pod launch design of kgpu.  Prints event-timed us/launch for several kernel shapes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

struct Big { void* p[120]; int x[16]; };   // ~1 KiB of kernel arguments, like kgpu::DevState

__global__ void k_empty() {}
__global__ void k_chain(const int64_t* __restrict__ src, int64_t* __restrict__ dst, int hops) {
  int64_t v = threadIdx.x;
  for (int h = 0; h < hops; ++h) v = src[(v + h) & 1023];
  if (threadIdx.x == 0) dst[blockIdx.x] = v;
}
__global__ void k_big(Big b, int64_t* dst) {
  if (threadIdx.x == 0) dst[blockIdx.x] = (int64_t)b.p[(blockIdx.x * 7) % 120] + b.x[blockIdx.x & 15];
}
__global__ void k_bigptr(const Big* b, int64_t* dst) {
  if (threadIdx.x == 0) dst[blockIdx.x] = (int64_t)b->p[(blockIdx.x * 7) % 120] + b->x[blockIdx.x & 15];
}

template <class F>
double timeit(hipStream_t s, F f, int iters = 2000) {
  for (int i = 0; i < 50; ++i) f();
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a, s);
  for (int i = 0; i < iters; ++i) f();
  hipEventRecord(b, s);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms * 1e3 / iters;
}

int main() {
  hipStream_t s; hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  int64_t *src, *dst; hipMalloc(&src, 8 * 1024); hipMalloc(&dst, 8 * 4096);
  hipMemset(src, 0, 8 * 1024);
  Big big{}; for (int i = 0; i < 120; ++i) big.p[i] = (void*)(intptr_t)i;
  Big* dbig; hipMalloc(&dbig, sizeof(Big)); hipMemcpy(dbig, &big, sizeof(Big), hipMemcpyHostToDevice);
  for (int blocks : {1, 20, 79, 512}) {
    printf("blocks=%4d  empty %.2f  chain1 %.2f  chain4 %.2f  bigarg %.2f  bigptr %.2f us/launch\n", blocks,
           timeit(s, [&] { hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(64), 0, s); }),
           timeit(s, [&] { hipLaunchKernelGGL(k_chain, dim3(blocks), dim3(64), 0, s, src, dst, 1); }),
           timeit(s, [&] { hipLaunchKernelGGL(k_chain, dim3(blocks), dim3(64), 0, s, src, dst, 4); }),
           timeit(s, [&] { hipLaunchKernelGGL(k_big, dim3(blocks), dim3(64), 0, s, big, dst); }),
           timeit(s, [&] { hipLaunchKernelGGL(k_bigptr, dim3(blocks), dim3(64), 0, s, dbig, dst); }));
  }
  // graph replay of 100 chained launches
  hipGraph_t g; hipGraphExec_t ge;
  hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(k_chain, dim3(20), dim3(64), 0, s, src, dst, 1);
  hipStreamEndCapture(s, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  printf("graph of 100 chain1 launches (20 blocks): %.2f us/launch\n",
         timeit(s, [&] { hipGraphLaunch(ge, s); }, 200) / 100.0);
  hipStreamCaptureMode m = hipStreamCaptureModeGlobal; (void)m;
  hipGraphExecDestroy(ge); hipGraphDestroy(g);
  hipGraph_t g2; hipGraphExec_t ge2;
  hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(k_big, dim3(20), dim3(64), 0, s, big, dst);
  hipStreamEndCapture(s, &g2);
  hipGraphInstantiate(&ge2, g2, nullptr, nullptr, 0);
  printf("graph of 100 bigarg launches (20 blocks): %.2f us/launch\n",
         timeit(s, [&] { hipGraphLaunch(ge2, s); }, 200) / 100.0);
  return 0;
}
