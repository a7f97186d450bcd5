// kgpu_reasons.h (the Filter status reasons behind kgpu_filter_reasons) under ASan + UBSan on the CPU:
// every plugin's word, taints in spec order, scalar requests across detail bit 15 with and without a
// column reader, malformed arguments, and buffer packing at every length around the exact size.
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "kgpu_reasons.h"

#define CHECK(x)                                                   \
  do {                                                             \
    if (!(x)) {                                                    \
      std::fprintf(stderr, "check failed: %s (line %d)\n", #x, __LINE__); \
      std::exit(1);                                                \
    }                                                              \
  } while (0)

static std::vector<std::string> run(int32_t plugin, uint32_t word, const kgpu_reason_args& a,
                                    const kgpu::ScalarRead& rd, int* rc) {
  std::vector<std::string> out;
  *rc = kgpu::filter_reasons(plugin, word, a, rd, &out);
  return out;
}

int main() {
  // pools: toleration words (taint id 1 tolerated), 14 scalar requests
  std::vector<uint64_t> words = {0x2ull};
  std::vector<kgpu_scalar_req> sc;
  for (int i = 0; i < 14; ++i) sc.push_back(kgpu_scalar_req{i, i == 5 ? 0 : 1, 2, 2});
  kgpu_pools pools{};
  pools.words = words.data();
  pools.n_words = (int32_t)words.size();
  pools.scalars = sc.data();
  pools.n_scalars = (int32_t)sc.size();
  kgpu_pod_query q{};
  q.tol_nosched = kgpu_range{0, 1};
  q.scalars = kgpu_range{0, 14};
  std::vector<std::string> names;
  for (int i = 0; i < 14; ++i) names.push_back("example.com/r" + std::to_string(i));
  std::vector<const char*> cn;
  for (auto& s : names) cn.push_back(s.c_str());
  kgpu_taint_ref taints[3] = {{"soft", "x", "PreferNoSchedule", 2, 0}, {"b", "2", "NoSchedule", 1, 0},
                              {"a", "1", "NoExecute", 0, 0}};
  kgpu_reason_args a{};
  a.q = &q;
  a.pools = &pools;
  a.taints = taints;
  a.n_taints = 3;
  a.scalar_names = cn.data();
  int rc = 0;

  // TaintToleration: b (id 1) is tolerated, the PreferNoSchedule taint never counts -> a
  auto r = run(KGPU_F_TAINT_TOLERATION, 3u << 8, a, nullptr, &rc);
  CHECK(rc == KGPU_OK && r.size() == 1 && r[0] == "node(s) had taint {a: 1}, that the pod didn't tolerate");
  a.n_taints = 2;  // without a: no untolerated taint in the list -> refused
  run(KGPU_F_TAINT_TOLERATION, 3u << 8, a, nullptr, &rc);
  CHECK(rc == KGPU_E_INVAL);
  a.n_taints = 3;
  taints[2].id = 999;  // outside the query's mask
  run(KGPU_F_TAINT_TOLERATION, 3u << 8, a, nullptr, &rc);
  CHECK(rc == KGPU_E_INVAL);
  taints[2].id = 0;

  // NodeResourcesFit: pods, cpu, memory, eph, r3, then bit 15 (requests 11..13)
  const uint32_t fit = (2u << 8) | ((1u | 2u | 4u | 8u | (16u << 3) | (16u << 11)) << 16);
  run(KGPU_F_NODE_RESOURCES_FIT, fit, a, nullptr, &rc);
  CHECK(rc == KGPU_E_INVAL);  // three checked requests share bit 15 and no reader
  auto rd = [](int32_t col, int64_t* alloc, int64_t* used) {
    *alloc = col == 12 ? 1 : 8;
    *used = 0;
    return true;
  };
  r = run(KGPU_F_NODE_RESOURCES_FIT, fit, a, rd, &rc);
  CHECK(rc == KGPU_OK && r.size() == 6);
  CHECK(r[0] == "Too many pods" && r[1] == "Insufficient cpu" && r[2] == "Insufficient memory");
  CHECK(r[3] == "Insufficient ephemeral-storage" && r[4] == "Insufficient example.com/r3");
  CHECK(r[5] == "Insufficient example.com/r12");
  // only request 11 checked among 11..13: bit 15 alone names it
  sc[12].check = sc[13].check = 0;
  r = run(KGPU_F_NODE_RESOURCES_FIT, (2u << 8) | ((16u << 11) << 16), a, nullptr, &rc);
  CHECK(rc == KGPU_OK && r.size() == 1 && r[0] == "Insufficient example.com/r11");
  a.scalar_names = nullptr;
  run(KGPU_F_NODE_RESOURCES_FIT, (2u << 8) | ((16u << 11) << 16), a, nullptr, &rc);
  CHECK(rc == KGPU_E_INVAL);
  a.scalar_names = cn.data();
  q.scalars = kgpu_range{10, 9};  // beyond the pool
  run(KGPU_F_NODE_RESOURCES_FIT, (2u << 8) | (16u << 16), a, nullptr, &rc);
  CHECK(rc == KGPU_E_INVAL);
  q.scalars = kgpu_range{0, 14};

  // InterPodAffinity rules, the single-reason plugins, an unknown plugin
  for (uint32_t d = 1; d <= 3; ++d) {
    r = run(KGPU_F_INTER_POD_AFFINITY, (2u << 8) | (d << 16), a, nullptr, &rc);
    CHECK(rc == KGPU_OK && r.size() == 2 && r[0] == "node(s) didn't match pod affinity/anti-affinity");
  }
  run(KGPU_F_INTER_POD_AFFINITY, (2u << 8) | (4u << 16), a, nullptr, &rc);
  CHECK(rc == KGPU_E_INVAL);
  for (int32_t f : {KGPU_F_NODE_UNSCHEDULABLE, KGPU_F_NODE_NAME, KGPU_F_NODE_PORTS, KGPU_F_NODE_AFFINITY,
                    KGPU_F_POD_TOPOLOGY_SPREAD}) {
    r = run(f, 3u << 8, a, nullptr, &rc);
    CHECK(rc == KGPU_OK && r.size() == 1);
  }
  run(KGPU_NUM_FILTERS, 3u << 8, a, nullptr, &rc);
  CHECK(rc == KGPU_E_INVAL);

  // packing: writes only when everything fits
  r = run(KGPU_F_INTER_POD_AFFINITY, (2u << 8) | (3u << 16), a, nullptr, &rc);
  const int64_t need = kgpu::pack_reasons(r, nullptr, 0);
  CHECK(need == (int64_t)(r[0].size() + r[1].size() + 2));
  for (int64_t len = need - 2; len <= need + 2; ++len) {
    std::vector<char> buf((size_t)len, 'z');
    CHECK(kgpu::pack_reasons(r, buf.data(), len) == need);
    if (len >= need) CHECK(std::string(buf.data()) == r[0] && std::string(buf.data() + r[0].size() + 1) == r[1]);
    else CHECK(buf[0] == 'z');
  }
  std::printf("reasons ok\n");
  return 0;
}
