#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
enum { kTFeas = 0, kTMaxT, kTMaxNA, kTNonIgn, kTAdjMin, kTAdjMax, kTIpaMin, kTIpaMax, kTDptsMax, kTZoned, kTFixed };
__device__ __forceinline__ int64_t tident(int op) { return op == 1 ? -(1ll << 56) : (op == 2 ? (1ll << 56) : 0); }
struct TM { int32_t acc32[8]; int64_t acc64[2]; };
template <int kForm>
__global__ void k(const int32_t* in32, const int64_t* in64, const int32_t* words, const int32_t* nsoft, int R, int soft_words,
                  int64_t* out) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  TM& M = *reinterpret_cast<TM*>(lds_raw);
  const int o_smask = 256, o_zsum = 512;
  const int tid = threadIdx.x;
  if (tid < 8) M.acc32[tid] = in32[tid];
  if (tid < 2) M.acc64[tid] = in64[tid];
  if (tid < 64) reinterpret_cast<int32_t*>(lds_raw + o_smask)[tid] = words[tid];
  if (tid < 64) reinterpret_cast<int32_t*>(lds_raw + o_zsum)[tid] = words[64 + tid];
  __syncthreads();
  const int n_soft = *nsoft;
  if constexpr (kForm == 0) {
    auto stat_of = [&](int rr) -> int64_t {
      const int i32 = rr < 6 ? rr : (rr == kTDptsMax ? 6 : 7);
      const uint32_t w32 = (uint32_t)M.acc32[i32];
      const int64_t w64 = M.acc64[rr == kTIpaMax ? 1 : 0];
      const int vi = rr - kTFixed;
      const int voff = vi < 0 ? o_smask : (vi < soft_words ? o_smask + 4 * vi : o_zsum + 4 * (vi - soft_words));
      const int32_t wv = *reinterpret_cast<const int32_t*>(lds_raw + voff);
      if (rr >= kTFixed) return vi < soft_words ? (int64_t)(uint32_t)wv : (int64_t)wv;
      if (rr == kTIpaMin) return w64 == INT64_MAX ? tident(2) : w64;
      if (rr == kTIpaMax) return w64 == INT64_MIN ? tident(1) : w64;
      if (rr == kTAdjMin) return n_soft ? (int64_t)(uint32_t)~w32 : tident(2);
      if (rr == kTAdjMax) return n_soft ? (int64_t)w32 : tident(1);
      if (rr == kTFeas || rr == kTNonIgn) return (int32_t)w32;
      return (int64_t)w32;
    };
    if (tid < R) out[tid] = stat_of(tid);
  } else if constexpr (kForm == 1) {
    if (tid < R) {
      const int i32 = tid < 6 ? tid : (tid == kTDptsMax ? 6 : 7);
      const uint32_t w32 = (uint32_t)M.acc32[i32];
      const int64_t w64 = M.acc64[tid == kTIpaMax ? 1 : 0];
      const int vi = tid - kTFixed;
      const int voff = vi < 0 ? o_smask : (vi < soft_words ? o_smask + 4 * vi : o_zsum + 4 * (vi - soft_words));
      const int32_t wv = *reinterpret_cast<const int32_t*>(lds_raw + voff);
      int64_t x;
      if (tid >= kTFixed) x = vi < soft_words ? (int64_t)(uint32_t)wv : (int64_t)wv;
      else if (tid == kTIpaMin) x = w64 == INT64_MAX ? tident(2) : w64;
      else if (tid == kTIpaMax) x = w64 == INT64_MIN ? tident(1) : w64;
      else if (tid == kTAdjMin) x = n_soft ? (int64_t)(uint32_t)~w32 : tident(2);
      else if (tid == kTAdjMax) x = n_soft ? (int64_t)w32 : tident(1);
      else if (tid == kTFeas || tid == kTNonIgn) x = (int32_t)w32;
      else x = (int64_t)w32;
      out[tid] = x;
    }
  } else {
    // the shipped form (kgpu_kernels.hip, k_tbatch's statistics publish): every candidate value computed,
    // then one select per slot kind -- no branch whose default the backend can lose
    if (tid < R) {
      const int i32 = tid < 6 ? tid : (tid == kTDptsMax ? 6 : 7);
      const uint32_t w32 = (uint32_t)M.acc32[i32];
      const int64_t w64 = M.acc64[tid == kTIpaMax ? 1 : 0];
      const int vi = tid - kTFixed;
      const int voff = vi < 0 ? o_smask : (vi < soft_words ? o_smask + 4 * vi : o_zsum + 4 * (vi - soft_words));
      const int32_t wv = *reinterpret_cast<const int32_t*>(lds_raw + voff);
      int64_t x = (int64_t)w32;  // kTMaxT, kTMaxNA, kTDptsMax, kTZoned
      x = (tid == kTFeas || tid == kTNonIgn) ? (int64_t)(int32_t)w32 : x;
      x = tid == kTAdjMax ? (n_soft ? (int64_t)w32 : tident(1)) : x;
      x = tid == kTAdjMin ? (n_soft ? (int64_t)(uint32_t)~w32 : tident(2)) : x;
      x = tid == kTIpaMax ? (w64 == INT64_MIN ? tident(1) : w64) : x;
      x = tid == kTIpaMin ? (w64 == INT64_MAX ? tident(2) : w64) : x;
      x = tid >= kTFixed ? (vi < soft_words ? (int64_t)(uint32_t)wv : (int64_t)wv) : x;
      out[tid] = x;
    }
  }
}
template __global__ void k<0>(const int32_t*, const int64_t*, const int32_t*, const int32_t*, int, int, int64_t*);
template __global__ void k<1>(const int32_t*, const int64_t*, const int32_t*, const int32_t*, int, int, int64_t*);
template __global__ void k<2>(const int32_t*, const int64_t*, const int32_t*, const int32_t*, int, int, int64_t*);

// Host side: the three forms on the same inputs, against the selection computed on the host.  Exit 2 when
// the select chain (the form k_tbatch ships) is wrong, 1 when only the branchy forms are (the miscompile
// reproduced), 0 when every form is right (a compiler without the bug).
static int64_t host_expect(int rr, const int32_t* a32, const int64_t* a64, const int32_t* words, int n_soft,
                           int soft_words) {
  const int i32 = rr < 6 ? rr : (rr == kTDptsMax ? 6 : 7);
  const uint32_t w32 = (uint32_t)a32[i32];
  const int64_t w64 = a64[rr == kTIpaMax ? 1 : 0];
  const int vi = rr - kTFixed;
  if (rr >= kTFixed) {
    const int32_t wv = vi < soft_words ? words[vi] : words[64 + vi - soft_words];
    return vi < soft_words ? (int64_t)(uint32_t)wv : (int64_t)wv;
  }
  auto id = [](int op) { return op == 1 ? -(1ll << 56) : (op == 2 ? (1ll << 56) : 0ll); };
  if (rr == kTIpaMin) return w64 == INT64_MAX ? id(2) : w64;
  if (rr == kTIpaMax) return w64 == INT64_MIN ? id(1) : w64;
  if (rr == kTAdjMin) return n_soft ? (int64_t)(uint32_t)~w32 : id(2);
  if (rr == kTAdjMax) return n_soft ? (int64_t)w32 : id(1);
  if (rr == kTFeas || rr == kTNonIgn) return (int32_t)w32;
  return (int64_t)w32;
}

int main() {
  const int soft_words = 2, zones = 3, R = kTFixed + soft_words + zones;
  int32_t a32[8] = {17, 23, -5, 9, 4, 31, 77, 1};
  int64_t a64[2] = {-12345, 67890};
  int32_t words[128];
  for (int i = 0; i < 128; ++i) words[i] = 1000 + 7 * i;
  int bad[3] = {0, 0, 0};
  for (int n_soft = 0; n_soft < 2; ++n_soft) {
    int32_t *d32, *dw, *dn;
    int64_t *d64, *dout;
    (void)hipMalloc(&d32, sizeof a32);
    (void)hipMalloc(&d64, sizeof a64);
    (void)hipMalloc(&dw, sizeof words);
    (void)hipMalloc(&dn, 4);
    (void)hipMalloc(&dout, 64 * 8);
    (void)hipMemcpy(d32, a32, sizeof a32, hipMemcpyHostToDevice);
    (void)hipMemcpy(d64, a64, sizeof a64, hipMemcpyHostToDevice);
    (void)hipMemcpy(dw, words, sizeof words, hipMemcpyHostToDevice);
    (void)hipMemcpy(dn, &n_soft, 4, hipMemcpyHostToDevice);
    for (int form = 0; form < 3; ++form) {
      (void)hipMemset(dout, 0x5A, 64 * 8);  // a recognizable stale pattern
      if (form == 0) hipLaunchKernelGGL(k<0>, dim3(1), dim3(64), 1024, 0, d32, d64, dw, dn, R, soft_words, dout);
      else if (form == 1) hipLaunchKernelGGL(k<1>, dim3(1), dim3(64), 1024, 0, d32, d64, dw, dn, R, soft_words, dout);
      else hipLaunchKernelGGL(k<2>, dim3(1), dim3(64), 1024, 0, d32, d64, dw, dn, R, soft_words, dout);
      int64_t out[64];
      (void)hipMemcpy(out, dout, sizeof out, hipMemcpyDeviceToHost);
      for (int rr = 0; rr < R; ++rr) {
        const int64_t want = host_expect(rr, a32, a64, words, n_soft, soft_words);
        if (out[rr] != want) {
          static const char* names[3] = {"lambda", "written-out", "select-chain"};
          std::printf("n_soft %d %s form: slot %d got %lld want %lld\n", n_soft, names[form], rr, (long long)out[rr],
                      (long long)want);
          bad[form] = 1;
        }
      }
    }
    (void)hipFree(d32); (void)hipFree(d64); (void)hipFree(dw); (void)hipFree(dn); (void)hipFree(dout);
  }
  std::printf("stat_select: lambda %s, written-out %s, select-chain %s\n", bad[0] ? "WRONG" : "ok", bad[1] ? "WRONG" : "ok",
              bad[2] ? "WRONG" : "ok");
  return bad[2] ? 2 : ((bad[0] || bad[1]) ? 1 : 0);
}
