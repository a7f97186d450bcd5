// Microbenchmark: per-round cost of the all-to-all granule exchange the persistent batch kernel
// does once per pod, with no node evaluation around it.  G workgroups (256 threads), R rounds;
// every round each workgroup publishes one 8-byte granule and wave 0 polls all G granules.
//
//   mode 0: sc1 granule store, sc1 sweep of the G granules (the k_batch protocol)
//   mode 1: agent-scope atomic add on one counter per round, sc1 poll of the counter
//   mode 2: mode 0 restricted to one XCD: 8*G workgroups launched, only those whose XCC_ID
//           equals workgroup 0's take part (ranked by an atomic ticket); plain granule stores
//           (the line stays in that XCD's L2), sc1 sweeps -- speed probe only
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/xchg_bench tools/xchg_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

constexpr uint64_t kValid = 1ull << 63;
constexpr uint64_t kTimeout = 20000000ull;  // 0.2 s of s_memrealtime

__device__ __forceinline__ uint64_t ld1(const uint64_t* p) {
  return __hip_atomic_load(const_cast<uint64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st1(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int xcc_id() {
  int v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 0xF;
}

__global__ __launch_bounds__(256) void k_xchg(int mode, int G, int R, uint64_t* gran, uint32_t* ctr, int* err,
                                              int* ticket, int* xcc0, long long* t_out) {
  const int tid = threadIdx.x, lane = tid & 63;
  __shared__ int s_rank, s_stop;
  int rank = blockIdx.x;
  if (mode == 2) {
    if (tid == 0) {
      const int x = xcc_id();
      if (blockIdx.x == 0) __hip_atomic_store(xcc0, x + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      int want;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while ((want = __hip_atomic_load(xcc0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0 &&
             __builtin_amdgcn_s_memrealtime() - t0 < kTimeout) {
      }
      s_rank = (want == x + 1) ? atomicAdd(ticket, 1) : -1;
      if (s_rank >= G) s_rank = -1;
    }
    __syncthreads();
    rank = s_rank;
    if (rank < 0) return;
  }
  const uint64_t tstart = __builtin_amdgcn_s_memrealtime();
  for (int r = 0; r < R; ++r) {
    uint64_t* row = gran + (size_t)r * G;
    if (tid == 0) {
      if (mode == 1) {
        __hip_atomic_fetch_add(ctr + r, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else if (mode == 2) {
        row[rank] = kValid | (uint64_t)r;
      } else {
        st1(row + rank, kValid | (uint64_t)r);
      }
    }
    if (tid < 64) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      int stop = 0;
      for (;;) {
        bool all = true;
        if (mode == 1) {
          const uint32_t c = __hip_atomic_load(ctr + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          all = c >= (uint32_t)G;
        } else {
          for (int g = lane; g < G; g += 64)
            if (!(ld1(row + g) & kValid)) all = false;
        }
        if (__all(all)) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > kTimeout) {
          stop = 1;
          break;
        }
      }
      if (tid == 0) {
        s_stop = stop;
        if (stop) atomicExch(err, 1);
      }
    }
    __syncthreads();
    if (s_stop) return;
  }
  if (tid == 0 && rank == 0) *t_out = (long long)(__builtin_amdgcn_s_memrealtime() - tstart);
}

int main(int argc, char** argv) {
  const int R = argc > 1 ? std::atoi(argv[1]) : 2000;
  const int sizes[] = {4, 8, 20, 64, 128, 196, 256};
  uint64_t* gran;
  uint32_t* ctr;
  int *err, *ticket, *xcc0;
  long long* tout;
  CHECK(hipMalloc(&gran, sizeof(uint64_t) * (size_t)R * 256));
  CHECK(hipMalloc(&ctr, sizeof(uint32_t) * (size_t)R));
  CHECK(hipMalloc(&err, 4));
  CHECK(hipMalloc(&ticket, 4));
  CHECK(hipMalloc(&xcc0, 4));
  CHECK(hipMalloc(&tout, 8));
  for (int mode = 0; mode < 3; ++mode) {
    for (int G : sizes) {
      if (mode == 2 && G > 32) continue;
      CHECK(hipMemset(gran, 0, sizeof(uint64_t) * (size_t)R * 256));
      CHECK(hipMemset(ctr, 0, sizeof(uint32_t) * (size_t)R));
      CHECK(hipMemset(err, 0, 4));
      CHECK(hipMemset(ticket, 0, 4));
      CHECK(hipMemset(xcc0, 0, 4));
      CHECK(hipMemset(tout, 0, 8));
      const int grid = mode == 2 ? 8 * G : G;
      hipLaunchKernelGGL(k_xchg, dim3(grid), dim3(256), 0, 0, mode, G, R, gran, ctr, err, ticket, xcc0, tout);
      CHECK(hipGetLastError());
      CHECK(hipDeviceSynchronize());
      int e = 0, tk = 0;
      long long t = 0;
      CHECK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(&tk, ticket, 4, hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(&t, tout, 8, hipMemcpyDeviceToHost));
      std::printf("mode %d G %3d: %s %.0f ns/round%s\n", mode, G, e ? "TIMEOUT" : "ok", t * 10.0 / R,
                  mode == 2 ? (tk >= G ? " (one XCD)" : " (XCD short of workgroups)") : "");
      std::fflush(stdout);
    }
  }
  return 0;
}
