// Microbenchmark: latency of the config-(b) node evaluation (node_key<kFitFM, kFitSM>) on
// register-resident rows, one to four independent evaluations per lane per iteration, with
// workgroups of 256 / 512 / 1024 threads (1 / 2 / 4 waves per SIMD).  Isolates the evaluation
// from the persistent kernel's exchange (k_batch phase trace "evalA").
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -o tools/eval_bench tools/eval_bench.hip
#include "../kubernetes-1_amd/csrc/kgpu_kernels.hip"

#include <cstdio>
#include <vector>

namespace kgpu {

template <int NEV, int B, bool FRESHQ, bool PIN = false>
__global__ __launch_bounds__(B) void k_evalbench(const DevState* __restrict__ stp, const kgpu_pod_query* qs,
                                                 int iters, int64_t* out) {
  const DevState& st = *stp;
  const int tid = threadIdx.x;
  NodeRes r[NEV];
#pragma unroll
  for (int j = 0; j < NEV; ++j) {
    r[j] = load_res(st, (tid + j * B) % st.N);
    set_recips(r[j]);
  }
  kgpu_pod_query q = qs[0];
  __builtin_amdgcn_s_waitcnt(0);
  uint64_t acc = 0;
  const int64_t t0 = (int64_t)__builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
    const uint64_t tk = pod_tie_key(st.seed, it);
    if (FRESHQ) {
      q = *cp(qs + it);  // a query record never read before (as in k_batch: one per pod)
      (void)PIN;
    }
    uint64_t k[NEV];
#pragma unroll
    for (int j = 0; j < NEV; ++j) k[j] = node_key<kFitFM, kFitSM>(st, q, r[j], (tid + j * B) % st.N, tk);
#pragma unroll
    for (int j = 0; j < NEV; ++j) acc += k[j];
    r[0].rc += (int64_t)(acc & 1);  // loop-carried: the next evaluation depends on this one
  }
  const int64_t t1 = (int64_t)__builtin_amdgcn_s_memrealtime();
  if (tid == 0) out[blockIdx.x] = t1 - t0;
  if (acc == 12345) out[gridDim.x + blockIdx.x] = (int64_t)acc;
}

template <int NEV, int B, bool FRESHQ = false, bool PIN = false>
static double run(const DevState* d_st, const kgpu_pod_query* d_q, int64_t* d_out, int grid, int iters) {
  hipLaunchKernelGGL((k_evalbench<NEV, B, FRESHQ, PIN>), dim3(grid), dim3(B), 0, 0, d_st, d_q, iters, d_out);
  hipLaunchKernelGGL((k_evalbench<NEV, B, FRESHQ, PIN>), dim3(grid), dim3(B), 0, 0, d_st, d_q, iters, d_out);
  std::vector<int64_t> h(grid);
  hipMemcpy(h.data(), d_out, sizeof(int64_t) * grid, hipMemcpyDeviceToHost);
  int64_t mx = 0;
  for (auto v : h) mx = v > mx ? v : mx;
  return (double)mx * 10.0 / iters;  // 100 MHz ticks -> ns per iteration
}

}  // namespace kgpu

int main() {
  using namespace kgpu;
  const int N = 4096;
  std::vector<int64_t> ac(N), am(N), ae(N), rc(N), rm(N), re(N), zc(N), zm(N);
  std::vector<int32_t> ap(N), np(N);
  for (int i = 0; i < N; ++i) {
    ac[i] = 4000 + 1000 * (i % 7); am[i] = (int64_t)(16 + i % 5) << 30; ae[i] = 100ll << 30;
    rc[i] = 100 * (i % 11); rm[i] = (int64_t)(i % 13) << 28; re[i] = 0;
    zc[i] = rc[i] + 100; zm[i] = rm[i] + (200ll << 20);
    ap[i] = 110; np[i] = i % 17;
  }
  auto up64 = [](std::vector<int64_t>& v) { int64_t* p; hipMalloc(&p, v.size() * 8); hipMemcpy(p, v.data(), v.size() * 8, hipMemcpyHostToDevice); return p; };
  auto up32 = [](std::vector<int32_t>& v) { int32_t* p; hipMalloc(&p, v.size() * 4); hipMemcpy(p, v.data(), v.size() * 4, hipMemcpyHostToDevice); return p; };
  DevState st{};
  st.N = N; st.node_base = 0; st.n_total = N;
  st.alloc_cpu = up64(ac); st.alloc_mem = up64(am); st.alloc_eph = up64(ae);
  st.req_cpu = up64(rc); st.req_mem = up64(rm); st.req_eph = up64(re);
  st.nz_cpu = up64(zc); st.nz_mem = up64(zm);
  st.alloc_pods = up32(ap); st.num_pods = up32(np);
  st.n_scores = 2;
  st.w_of[KGPU_S_BALANCED_ALLOCATION] = 1;
  st.w_of[KGPU_S_LEAST_ALLOCATED] = 1;
  st.seed = 0x1234;
  kgpu_pod_query q{};
  q.req[0] = 500; q.req[1] = 512ll << 20; q.nz[0] = 500; q.nz[1] = 512ll << 20;
  q.score_req[0] = 500; q.score_req[1] = 512ll << 20;
  DevState* d_st; kgpu_pod_query* d_q; int64_t* d_out;
  hipMalloc(&d_st, sizeof(st)); hipMemcpy(d_st, &st, sizeof(st), hipMemcpyHostToDevice);
  const int iters = 2000;
  std::vector<kgpu_pod_query> qv(2 * iters + 1, q);
  hipMalloc(&d_q, sizeof(q) * qv.size()); hipMemcpy(d_q, qv.data(), sizeof(q) * qv.size(), hipMemcpyHostToDevice);
  hipMalloc(&d_out, 2 * 4096 * sizeof(int64_t));
  for (int grid : {20, 256}) {
    printf("grid %d: ns/iter  B=256: ev1 %.0f ev2 %.0f ev4 %.0f | B=512: ev1 %.0f ev2 %.0f ev4 %.0f | B=1024: ev1 %.0f ev2 %.0f\n",
           grid, run<1, 256>(d_st, d_q, d_out, grid, iters), run<2, 256>(d_st, d_q, d_out, grid, iters),
           run<4, 256>(d_st, d_q, d_out, grid, iters), run<1, 512>(d_st, d_q, d_out, grid, iters),
           run<2, 512>(d_st, d_q, d_out, grid, iters), run<4, 512>(d_st, d_q, d_out, grid, iters),
           run<1, 1024>(d_st, d_q, d_out, grid, iters), run<2, 1024>(d_st, d_q, d_out, grid, iters));
  }
  for (int grid : {20, 256}) {
    // fresh query per iteration: re-upload so that no cache holds them
    hipMemcpy(d_q, qv.data(), sizeof(q) * qv.size(), hipMemcpyHostToDevice);
    printf("grid %d fresh query: ns/iter  B=256: ev1 %.0f ev2 %.0f | B=512: ev4 %.0f\n", grid,
           run<1, 256, true>(d_st, d_q, d_out, grid, iters), run<2, 256, true>(d_st, d_q, d_out, grid, iters),
           run<4, 512, true>(d_st, d_q, d_out, grid, iters));
    hipMemcpy(d_q, qv.data(), sizeof(q) * qv.size(), hipMemcpyHostToDevice);
    printf("grid %d fresh query, pinned: ns/iter  B=256: ev1 %.0f ev2 %.0f | B=512: ev4 %.0f\n", grid,
           run<1, 256, true, true>(d_st, d_q, d_out, grid, iters), run<2, 256, true, true>(d_st, d_q, d_out, grid, iters),
           run<4, 512, true, true>(d_st, d_q, d_out, grid, iters));
  }
  return 0;
}
