// Prototype measurement for DESIGN.md 4.6 ("measure a resident-server prototype rather than
// estimate it"): the host-to-host floor of one short scheduling cycle
//   launch    the host issues hipLaunchKernel of a G-workgroup grid per cycle (kgpu_schedule_one's shape);
//             every workgroup takes a ticket, the last one stores the completion word into pinned memory,
//             the host spins on it
//   resident  one persistent G-workgroup grid: workgroup 0 polls a doorbell word in pinned host memory and
//             hands the cycle number to the others through a device word (agent scope); each workgroup
//             takes its ticket as above; the host rings the doorbell and spins on the completion word
//   resident-all  the same, every workgroup polling the pinned doorbell itself (no device hand-off)
// Each cycle also reads a 256-byte "query" in every workgroup (what a resident server must fetch itself
// instead of receiving as launch arguments): from pinned host memory, from device memory, or not at all.
// Exit: the host writes -1 into the doorbell; every workgroup also leaves after ~1 s without a cycle, so
// the grid drains even if the host dies.  Stores are vector stores (global atomics), never scalar.
//   hipcc --offload-arch=gfx950 -O3 -o tools/doorbell_probe tools/doorbell_probe.hip
//   ./tools/doorbell_probe [cycles=2000]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

constexpr uint64_t kIdleTicks = 100000000ull;  // s_memrealtime runs at 100 MHz: 1 s

__device__ __forceinline__ int64_t ld_sys(const int64_t* p) {
  return __hip_atomic_load(const_cast<int64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ int64_t ld_agent(const int64_t* p) {
  return __hip_atomic_load(const_cast<int64_t*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the per-cycle work every workgroup does in both shapes: read the query, take the ticket; the last
// workgroup publishes the completion word
__device__ __forceinline__ void cycle_tail(int64_t k, const int64_t* query, int64_t* sink, unsigned* ticket,
                                           int64_t* done) {
  __shared__ int64_t q;
  if (threadIdx.x == 0) q = 0;
  if (query && threadIdx.x < 32) {
    const int64_t v = ld_sys(query + threadIdx.x);  // 256 B, one word per lane
    if (threadIdx.x == 0) q = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    sink[blockIdx.x] = q + k;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const unsigned G = gridDim.x;
    if (atomicAdd(ticket, 1u) % G == G - 1) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __hip_atomic_store(done, k, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

__global__ void k_cycle(int64_t k, const int64_t* query, int64_t* sink, unsigned* ticket, int64_t* done) {
  cycle_tail(k, query, sink, ticket, done);
}

// mode 0: workgroup 0 polls the doorbell and hands the cycle to the others through `bcast`;
// mode 1: every workgroup polls the doorbell
__global__ void k_resident(const int64_t* door, int64_t* bcast, const int64_t* query, int64_t* sink, unsigned* ticket,
                           int64_t* done, int mode) {
  __shared__ int64_t cur;
  for (int64_t k = 1;; ++k) {
    if (threadIdx.x == 0) {
      const bool host = mode == 1 || blockIdx.x == 0;
      const int64_t* src = host ? door : bcast;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      int64_t v;
      for (;;) {
        v = host ? ld_sys(src) : ld_agent(src);
        if (v >= k || v < 0) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > kIdleTicks) {
          v = -1;
          break;
        }
      }
      if (mode == 0 && blockIdx.x == 0)
        __hip_atomic_store(bcast, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      cur = v;
    }
    __syncthreads();
    if (cur < 0) return;
    cycle_tail(k, query, sink, ticket, done);
  }
}

static double pct(std::vector<double> v, double p) {
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, (size_t)(p * (double)v.size()))];
}

static void report(const char* name, int G, const std::vector<double>& us) {
  std::printf("%-14s G=%3d  p50 %6.2f us  p90 %6.2f  p99 %6.2f  min %6.2f\n", name, G, pct(us, 0.5), pct(us, 0.9),
              pct(us, 0.99), pct(us, 0.0));
}

int main(int argc, char** argv) {
  const int cycles = argc > 1 ? std::atoi(argv[1]) : 2000;
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  int64_t *door, *done, *query;
  CHECK(hipHostMalloc(&door, 64, hipHostMallocCoherent | hipHostMallocMapped));
  CHECK(hipHostMalloc(&done, 64, hipHostMallocCoherent | hipHostMallocMapped));
  CHECK(hipHostMalloc(&query, 256, hipHostMallocCoherent | hipHostMallocMapped));
  for (int i = 0; i < 32; ++i) query[i] = i;
  int64_t *bcast, *sink;
  unsigned* ticket;
  CHECK(hipMalloc(&bcast, 64));
  CHECK(hipMalloc(&sink, 8 * 1024));
  CHECK(hipMalloc(&ticket, 64));
  volatile int64_t* vdone = done;
  volatile int64_t* vdoor = door;
  using clk = std::chrono::steady_clock;
  int64_t* dquery;
  CHECK(hipMalloc(&dquery, 256));
  CHECK(hipMemcpy(dquery, query, 256, hipMemcpyHostToDevice));
  const char* qname[3] = {"pinned", "device", "none"};
  for (int qs = 0; qs < 3; ++qs)
  for (int G : {20, 79, 196}) {
    const int64_t* qp = qs == 0 ? query : (qs == 1 ? dquery : nullptr);
    std::printf("query %s: ", qname[qs]);
    // ---- launch per cycle
    {
      CHECK(hipMemset(ticket, 0, 64));
      *vdone = 0;
      std::vector<double> us;
      for (int k = 1; k <= cycles + 100; ++k) {
        const auto t0 = clk::now();
        hipLaunchKernelGGL(k_cycle, dim3(G), dim3(64), 0, s, (int64_t)k, qp, sink, ticket, done);
        const auto tl = clk::now();
        while (*vdone < k) {
          if (std::chrono::duration<double>(clk::now() - tl).count() > 2.0) {
            std::fprintf(stderr, "launch cycle %d timed out\n", k);
            return 1;
          }
        }
        const auto t1 = clk::now();
        if (k > 100) us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
      }
      CHECK(hipStreamSynchronize(s));
      report("launch", G, us);
      std::printf("query %s: ", qname[qs]);
    }
    // ---- resident, both hand-off shapes
    for (int mode = 0; mode < 2; ++mode) {
      CHECK(hipMemset(ticket, 0, 64));
      CHECK(hipMemset(bcast, 0, 64));
      *vdone = 0;
      *vdoor = 0;
      std::atomic_thread_fence(std::memory_order_seq_cst);
      hipLaunchKernelGGL(k_resident, dim3(G), dim3(64), 0, s, door, bcast, qp, sink, ticket, done, mode);
      std::vector<double> us;
      bool ok = true;
      for (int k = 1; k <= cycles + 100 && ok; ++k) {
        const auto t0 = clk::now();
        *vdoor = k;
        std::atomic_thread_fence(std::memory_order_seq_cst);
        while (*vdone < k) {
          if (std::chrono::duration<double>(clk::now() - t0).count() > 0.5) {
            std::fprintf(stderr, "resident mode %d cycle %d timed out\n", mode, k);
            ok = false;
            break;
          }
        }
        const auto t1 = clk::now();
        if (k > 100) us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
      }
      *vdoor = -1;
      std::atomic_thread_fence(std::memory_order_seq_cst);
      CHECK(hipStreamSynchronize(s));
      if (!ok) return 1;
      report(mode == 0 ? "resident-bcast" : "resident-all", G, us);
      if (mode == 0) std::printf("query %s: ", qname[qs]);
    }
  }
  CHECK(hipHostFree(door));
  CHECK(hipHostFree(done));
  CHECK(hipHostFree(query));
  CHECK(hipFree(dquery));
  CHECK(hipFree(bcast));
  CHECK(hipFree(sink));
  CHECK(hipFree(ticket));
  return 0;
}
