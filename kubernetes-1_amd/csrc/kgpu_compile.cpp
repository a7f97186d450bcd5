// kgpu_compile.cpp -- the pod / snapshot compiler behind include/kgpu_compile.h.
//
// Host C++ only (no device code): the PreFilter-time string work of every replaced plugin, done once
// per pod, and the snapshot's node columns.  Both drop-ins (the Go shim and the Python mirror) call
// these entries; the semantics, with the reference file:line each step follows, live here and nowhere
// else.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <map>
#include <new>
#include <set>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "kgpu.h"
#include "kgpu_compile.h"

namespace {

using std::string;
using std::vector;

string S(const kgpu_str& s) { return (s.p && s.n > 0) ? string(s.p, (size_t)s.n) : string(); }

constexpr const char* kHostname = "kubernetes.io/hostname";
constexpr const char* kZoneBeta = "failure-domain.beta.kubernetes.io/zone";
constexpr const char* kRegionBeta = "failure-domain.beta.kubernetes.io/region";
constexpr const char* kZone = "topology.kubernetes.io/zone";
constexpr const char* kRegion = "topology.kubernetes.io/region";
constexpr int64_t kDefaultMilliCPU = 100;                 // util/non_zero.go:30-34
constexpr int64_t kDefaultMemory = 200ll * 1024 * 1024;

struct CompileError {
  string msg;
};
struct NeedsUpload {
  string msg;
};

// ------------------------------------------------------------------ validation (apimachinery/pkg/util/validation)
bool alnum(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9'); }
bool lower_alnum(char c) { return (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); }

// ^[A-Za-z0-9]([-A-Za-z0-9_.]*[A-Za-z0-9])?$ (qualifiedNameFmt, validation.go:31-35)
bool name_chars_ok(const string& v) {
  if (v.empty() || !alnum(v.front()) || !alnum(v.back())) return false;
  for (char c : v)
    if (!alnum(c) && c != '-' && c != '_' && c != '.') return false;
  return true;
}

// DNS-1123 subdomain (validation.go:188-205): labels [a-z0-9]([-a-z0-9]*[a-z0-9])? joined by '.'
bool dns1123_subdomain_ok(const string& v) {
  if (v.empty() || v.size() > 253) return false;
  size_t i = 0;
  while (true) {
    size_t j = v.find('.', i);
    if (j == string::npos) j = v.size();
    if (j == i) return false;
    if (!lower_alnum(v[i]) || !lower_alnum(v[j - 1])) return false;
    for (size_t k = i; k < j; ++k)
      if (!lower_alnum(v[k]) && v[k] != '-') return false;
    if (j == v.size()) return true;
    i = j + 1;
  }
}

// IsQualifiedName (validation.go:42-70)
bool qualified_name_ok(const string& v) {
  size_t slash = v.find('/');
  string name = v;
  if (slash != string::npos) {
    if (v.find('/', slash + 1) != string::npos) return false;
    const string prefix = v.substr(0, slash);
    if (prefix.empty() || !dns1123_subdomain_ok(prefix)) return false;
    name = v.substr(slash + 1);
  }
  return !name.empty() && name.size() <= 63 && name_chars_ok(name);
}

// IsValidLabelValue (validation.go:82-94)
bool label_value_ok(const string& v) { return v.empty() || (v.size() <= 63 && name_chars_ok(v)); }

// strconv.ParseInt(v, 10, 64) as the Gt/Lt requirements use it (selector.go:201-214)
bool parse_int64(const string& s, int64_t& out) {
  size_t i = 0;
  bool neg = false;
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
  if (i >= s.size()) return false;
  unsigned __int128 acc = 0;
  for (; i < s.size(); ++i) {
    if (s[i] < '0' || s[i] > '9') return false;
    acc = acc * 10 + (unsigned)(s[i] - '0');
    if (acc > ((unsigned __int128)1 << 63)) return false;
  }
  if (!neg && acc == ((unsigned __int128)1 << 63)) return false;
  out = neg ? (int64_t)(0 - (uint64_t)acc) : (int64_t)acc;
  return true;
}

// ------------------------------------------------------------------ resource names (apis/core/v1/helper/helpers.go:33-143)
bool contains(const string& s, const char* sub) { return s.find(sub) != string::npos; }
bool starts_with(const string& s, const char* pre) { return s.compare(0, strlen(pre), pre) == 0; }

bool is_extended(const string& name) {
  if (name.find('/') == string::npos || contains(name, "kubernetes.io/") || starts_with(name, "requests."))
    return false;
  return qualified_name_ok("requests." + name);
}

bool is_scalar(const string& name) {
  return is_extended(name) || starts_with(name, "hugepages-") || contains(name, "kubernetes.io/") ||
         starts_with(name, "attachable-volumes-");
}

// image_locality.go:115-127 normalizedImageName
string normalized_image_name(string n) {
  const size_t c = n.rfind(':'), s = n.rfind('/');
  const long lc = c == string::npos ? -1 : (long)c, ls = s == string::npos ? -1 : (long)s;
  if (lc <= ls) n += ":latest";
  return n;
}

// v1.Toleration.ToleratesTaint (staging/src/k8s.io/api/core/v1/toleration.go:37-56)
bool tolerates(const kgpu_toleration_desc& t, const string& key, const string& value, const string& effect) {
  const string te = S(t.effect);
  if (!te.empty() && te != effect) return false;
  const string tk = S(t.key);
  if (!tk.empty() && tk != key) return false;
  const string op = S(t.op);
  if (op.empty() || op == "Equal") return S(t.value) == value;
  return op == "Exists";
}

const kgpu_kv* find_kv(const kgpu_kv* kv, int32_t n, const char* key) {
  for (int32_t i = 0; i < n; ++i)
    if (S(kv[i].key) == key) return &kv[i];
  return nullptr;
}

// GetZoneKey (pkg/util/node/node.go:148-174)
string zone_key(const kgpu_node_desc& n) {
  if (n.n_labels == 0) return string();
  const kgpu_kv* z = find_kv(n.labels, n.n_labels, kZoneBeta);
  if (!z) z = find_kv(n.labels, n.n_labels, kZone);
  const kgpu_kv* r = find_kv(n.labels, n.n_labels, kRegionBeta);
  if (!r) r = find_kv(n.labels, n.n_labels, kRegion);
  const string zone = z ? S(z->value) : string(), region = r ? S(r->value) : string();
  if (region.empty() && zone.empty()) return string();
  return region + string(":\0:", 3) + zone;
}

// ------------------------------------------------------------------ dictionaries
struct StrDict {
  std::unordered_map<string, int32_t> ids;
  vector<string> items;
  int32_t add(const string& s) {
    auto it = ids.find(s);
    if (it != ids.end()) return it->second;
    const int32_t i = (int32_t)items.size();
    ids.emplace(s, i);
    items.push_back(s);
    return i;
  }
  int32_t get(const string& s) const {
    auto it = ids.find(s);
    return it == ids.end() ? -1 : it->second;
  }
  int32_t size() const { return (int32_t)items.size(); }
};

// label keys, each with its own value dictionary (values are topology domains)
struct KeySpace {
  StrDict keys;
  vector<StrDict> vals;
  int32_t add_key(const string& k) {
    const int32_t ki = keys.add(k);
    if (ki == (int32_t)vals.size()) vals.emplace_back();
    return ki;
  }
  std::pair<int32_t, int32_t> add(const string& k, const string& v) {
    const int32_t ki = add_key(k);
    return {ki, vals[(size_t)ki].add(v)};
  }
  int32_t key(const string& k) const { return keys.get(k); }
  int32_t val(int32_t ki, const string& v) const { return ki < 0 ? -1 : vals[(size_t)ki].get(v); }
};

string join3(const string& a, const string& b, const string& c) { return a + '\0' + b + '\0' + c; }
string join2(const string& a, const string& b) { return a + '\0' + b; }

// ------------------------------------------------------------------ requests (framework/v1alpha1/types.go:262-323,549-581)
// Quantities arrive as (Value(), MilliValue()); a list is searched by name as the reference's maps are.
const kgpu_quantity* find_q(const kgpu_quantity* l, int32_t n, const char* name) {
  for (int32_t i = 0; i < n; ++i)
    if (S(l[i].name) == name) return &l[i];
  return nullptr;
}

struct PodResources {
  int64_t cpu = 0, mem = 0, eph = 0;  // computePodResourceRequest (fit.go:112-129)
  vector<std::pair<string, int64_t>> scalars;  // in first-appearance order
  int64_t nz_cpu = 0, nz_mem = 0;     // calculateResource non0CPU / non0Mem (types.go:549-581)
  bool fit_all_zero = false;

  int64_t* scalar_slot(const string& r, bool insert) {
    for (auto& kv : scalars)
      if (kv.first == r) return &kv.second;
    if (!insert) return nullptr;
    scalars.emplace_back(r, 0);
    return &scalars.back().second;
  }
  // Resource.Add (types.go:262-287): summed; pods is not a scalar
  void add(const kgpu_quantity* l, int32_t n) {
    for (int32_t i = 0; i < n; ++i) {
      const string k = S(l[i].name);
      if (k == "cpu") cpu += l[i].milli;
      else if (k == "memory") mem += l[i].value;
      else if (k == "ephemeral-storage") eph += l[i].value;
      else if (k != "pods" && is_scalar(k)) *scalar_slot(k, true) += l[i].value;
    }
  }
  // Resource.SetMaxResource (types.go:300-323)
  void max_of(const kgpu_quantity* l, int32_t n) {
    for (int32_t i = 0; i < n; ++i) {
      const string k = S(l[i].name);
      if (k == "cpu") cpu = std::max(cpu, l[i].milli);
      else if (k == "memory") mem = std::max(mem, l[i].value);
      else if (k == "ephemeral-storage") eph = std::max(eph, l[i].value);
      else if (is_scalar(k)) {
        int64_t* cur = scalar_slot(k, false);
        const int64_t v = l[i].value;
        if (v > (cur ? *cur : 0)) *scalar_slot(k, true) = v;
      }
    }
  }
};

// util.GetNonzeroRequestForResource (util/non_zero.go:54-80) over one container's requests
int64_t nonzero(const string& resource, const kgpu_quantity* req, int32_t n) {
  const kgpu_quantity* q = find_q(req, n, resource.c_str());
  if (resource == "cpu") return q ? q->milli : kDefaultMilliCPU;
  if (resource == "memory") return q ? q->value : kDefaultMemory;
  if (resource == "ephemeral-storage" || is_scalar(resource)) return q ? q->value : 0;
  return 0;
}

PodResources pod_resources(const kgpu_pod_desc& p) {
  PodResources r;
  for (int32_t i = 0; i < p.n_containers; ++i) r.add(p.containers[i].requests, p.containers[i].n_requests);
  for (int32_t i = 0; i < p.n_init_containers; ++i)
    r.max_of(p.init_containers[i].requests, p.init_containers[i].n_requests);
  if (p.n_overhead) r.add(p.overhead, p.n_overhead);
  r.fit_all_zero = r.cpu == 0 && r.mem == 0 && r.eph == 0 && r.scalars.empty();
  // NodeInfo.AddPod's NonZeroRequested delta: the non-zero defaults, overhead CPU as MilliValue
  // (types.go:571-580) -- not the scorer's Value() below
  for (int32_t i = 0; i < p.n_containers; ++i) {
    r.nz_cpu += nonzero("cpu", p.containers[i].requests, p.containers[i].n_requests);
    r.nz_mem += nonzero("memory", p.containers[i].requests, p.containers[i].n_requests);
  }
  for (int32_t i = 0; i < p.n_init_containers; ++i) {
    r.nz_cpu = std::max(r.nz_cpu, nonzero("cpu", p.init_containers[i].requests, p.init_containers[i].n_requests));
    r.nz_mem = std::max(r.nz_mem, nonzero("memory", p.init_containers[i].requests, p.init_containers[i].n_requests));
  }
  if (const kgpu_quantity* q = find_q(p.overhead, p.n_overhead, "cpu")) r.nz_cpu += q->milli;
  if (const kgpu_quantity* q = find_q(p.overhead, p.n_overhead, "memory")) r.nz_mem += q->value;
  return r;
}

// calculatePodResourceRequest (resource_allocation.go:118-142): the scorers' request, overhead added as
// Quantity.Value() for every resource, cpu included
int64_t score_request(const kgpu_pod_desc& p, const string& resource) {
  int64_t v = 0;
  for (int32_t i = 0; i < p.n_containers; ++i) v += nonzero(resource, p.containers[i].requests, p.containers[i].n_requests);
  for (int32_t i = 0; i < p.n_init_containers; ++i)
    v = std::max(v, nonzero(resource, p.init_containers[i].requests, p.init_containers[i].n_requests));
  if (const kgpu_quantity* q = find_q(p.overhead, p.n_overhead, resource.c_str())) v += q->value;
  return v;
}

// getResourceLimits (resource_limits.go:145-156): milliCPU and memory
void pod_limits(const kgpu_pod_desc& p, int64_t out[2]) {
  int64_t cpu = 0, mem = 0;
  for (int32_t i = 0; i < p.n_containers; ++i) {
    const kgpu_container_desc& c = p.containers[i];
    if (const kgpu_quantity* q = find_q(c.limits, c.n_limits, "cpu")) cpu += q->milli;
    if (const kgpu_quantity* q = find_q(c.limits, c.n_limits, "memory")) mem += q->value;
  }
  for (int32_t i = 0; i < p.n_init_containers; ++i) {
    const kgpu_container_desc& c = p.init_containers[i];
    if (const kgpu_quantity* q = find_q(c.limits, c.n_limits, "cpu")) cpu = std::max(cpu, q->milli);
    if (const kgpu_quantity* q = find_q(c.limits, c.n_limits, "memory")) mem = std::max(mem, q->value);
  }
  out[0] = cpu;
  out[1] = mem;
}

// ------------------------------------------------------------------ host-side selector evaluation
// labels.Selector.Matches of a LabelSelector (apis/meta/v1/helpers.go:34-70) against a label map; an
// unknown operator is skipped (such a selector never compiles: the callers only use matches where it did)
bool selector_matches(const kgpu_label_selector_desc& ps, const kgpu_kv* labels, int32_t n) {
  if (!ps.present) return false;
  for (int32_t i = 0; i < ps.n_match_labels; ++i) {
    const kgpu_kv* l = find_kv(labels, n, S(ps.match_labels[i].key).c_str());
    if (!l || S(l->value) != S(ps.match_labels[i].value)) return false;
  }
  for (int32_t i = 0; i < ps.n_exprs; ++i) {
    const kgpu_expr_desc& e = ps.exprs[i];
    const kgpu_kv* l = find_kv(labels, n, S(e.key).c_str());
    const string op = S(e.op);
    bool in = false;
    if (l)
      for (int32_t j = 0; j < e.n_values; ++j) in = in || S(e.values[j]) == S(l->value);
    if (op == "In" && !in) return false;
    if (op == "NotIn" && in) return false;
    if (op == "Exists" && !l) return false;
    if (op == "DoesNotExist" && l) return false;
  }
  return true;
}

// ------------------------------------------------------------------ pools
template <class T>
string bytes_of(const vector<T>& v) {
  return string(reinterpret_cast<const char*>(v.data()), v.size() * sizeof(T));
}

template <class T>
T zeroed() {
  T t;
  std::memset(&t, 0, sizeof(T));
  return t;
}

}  // namespace

struct kgpu_pool_set {
  vector<kgpu_req> reqs;
  vector<int32_t> ints;
  vector<uint64_t> words;
  vector<kgpu_node_term> node_terms;
  vector<kgpu_pref_term> pref_terms;
  vector<kgpu_spread> spreads;
  vector<kgpu_pod_term> pod_terms;
  vector<kgpu_scalar_req> scalars;
  vector<string> scalar_names;  // parallel to scalars
  vector<kgpu_port> ports;
  // content -> range, per pool (interning)
  std::unordered_map<string, kgpu_range> cache[9];

  template <class T>
  kgpu_range rng(int which, vector<T>& pool, const vector<T>& items, const string& extra = string()) {
    if (items.empty()) return kgpu_range{0, 0};
    const string key = bytes_of(items) + extra;
    auto it = cache[which].find(key);
    if (it != cache[which].end()) return it->second;
    const kgpu_range r{(int32_t)pool.size(), (int32_t)items.size()};
    pool.insert(pool.end(), items.begin(), items.end());
    cache[which].emplace(key, r);
    return r;
  }
  kgpu_range ints_range(const vector<int32_t>& xs) { return rng(1, ints, xs); }
  kgpu_range words_range(const vector<uint64_t>& ws) { return rng(2, words, ws); }
  kgpu_range reqs_range(const vector<kgpu_req>& rs) { return rng(0, reqs, rs); }
  kgpu_range scalars_range(const vector<kgpu_scalar_req>& rs, const vector<string>& names) {
    if (rs.empty()) return kgpu_range{0, 0};
    string extra;
    for (const string& n : names) extra += n + '\0';
    const size_t before = scalars.size();
    kgpu_range r = rng(7, scalars, rs, extra);
    if (scalars.size() != before) scalar_names.insert(scalar_names.end(), names.begin(), names.end());
    return r;
  }

  struct Mark {
    size_t reqs, ints;
  };
  Mark mark() const { return Mark{reqs.size(), ints.size()}; }
  // a term list that failed half-way: drop the records it appended (getAffinityTerms returns no terms)
  void rollback(const Mark& m) {
    auto drop = [](std::unordered_map<string, kgpu_range>& c, size_t n) {
      for (auto it = c.begin(); it != c.end();)
        it = ((size_t)it->second.begin + (size_t)it->second.count > n) ? c.erase(it) : std::next(it);
    };
    reqs.resize(m.reqs);
    ints.resize(m.ints);
    drop(cache[0], m.reqs);
    drop(cache[1], m.ints);
  }
};

namespace {

// ------------------------------------------------------------------ snapshot buffers
struct SnapBuf {
  vector<int64_t> alloc_cpu, alloc_mem, alloc_eph, req_cpu, req_mem, req_eph, nz_cpu, nz_mem;
  vector<int32_t> alloc_pods, num_pods;
  vector<int64_t> alloc_scalar, req_scalar;  // [S][N]
  vector<uint8_t> unschedulable;
  vector<int32_t> label_val;                 // [K][N]
  vector<uint64_t> taint_nosched, taint_prefer;  // [TW][N]
  vector<int32_t> zone_id;
  vector<int32_t> image_off, image_id, avoid_off, avoid_id;
  vector<int64_t> image_score;
  // existing pods
  vector<int32_t> pod_node, pod_ns;
  vector<uint32_t> pod_flags;
  vector<int32_t> pod_label_val;  // [PK][P]
  vector<kgpu_term> terms;
  vector<int64_t> pod_uid;
  vector<int32_t> port_count;
  vector<kgpu_port> ports;        // [slots][N]
  int32_t port_slots = 1;
  // label metadata
  vector<int32_t> key_n_values, value_off, key_empty_value;
  vector<int64_t> value_int;
  vector<uint8_t> value_int_ok;
  vector<uint8_t> key_unique;
  kgpu_pool_set pools;
  // the shard slice (views point here when sliced)
  SnapBuf* sliced = nullptr;
  ~SnapBuf() { delete sliced; }
};

template <class T>
const T* ptr_or_null(const vector<T>& v) {
  return v.empty() ? nullptr : v.data();
}

}  // namespace

struct kgpu_compiler {
  // profile
  vector<string> score_resources;  // Least + Most resource names
  std::set<string> ignored;
  vector<kgpu_default_spread> default_spreads;
  vector<string> default_spread_keys, default_spread_whens;
  // dictionaries
  KeySpace nkeys, pkeys;
  StrDict ns, taints, scalars, images, controllers, uids, ips, protos, zones;
  vector<std::pair<string, std::pair<string, string>>> taint_items;  // (key, (value, effect)) by id
  std::unordered_map<string, int32_t> node_index;
  vector<string> order;
  int32_t dims[3] = {0, 0, 1};  // S, K, TW of the last snapshot
  string err;
  SnapBuf* snap = nullptr;
  kgpu_key_meta km_view{};
  vector<int32_t> km_knv, km_off, km_empty;
  vector<int64_t> km_int;
  vector<uint8_t> km_ok;
  vector<int32_t> nl_image_off, nl_image_id, nl_avoid_off, nl_avoid_id;
  vector<int64_t> nl_image_score;
  ~kgpu_compiler() { delete snap; }

  int32_t taint_add(const string& k, const string& v, const string& e) {
    const int32_t before = taints.size();
    const int32_t id = taints.add(join3(k, v, e));
    if (taints.size() != before) taint_items.push_back({k, {v, e}});
    return id;
  }
  int32_t taint_words() const { return std::max<int32_t>(1, (taints.size() + 63) / 64); }

  StrDict* dict(int32_t d, int32_t key, bool grow) {
    switch (d) {
      case KGPU_DICT_NODE_KEY: return &nkeys.keys;
      case KGPU_DICT_POD_KEY: return &pkeys.keys;
      case KGPU_DICT_NODE_VALUE:
      case KGPU_DICT_POD_VALUE: {
        KeySpace& ks = d == KGPU_DICT_NODE_VALUE ? nkeys : pkeys;
        if (key < 0 || key >= ks.keys.size()) return nullptr;
        (void)grow;
        return &ks.vals[(size_t)key];
      }
      case KGPU_DICT_NAMESPACE: return &ns;
      case KGPU_DICT_TAINT: return &taints;
      case KGPU_DICT_SCALAR: return &scalars;
      case KGPU_DICT_IMAGE: return &images;
      case KGPU_DICT_CONTROLLER: return &controllers;
      case KGPU_DICT_UID: return &uids;
      case KGPU_DICT_IP: return &ips;
      case KGPU_DICT_PROTOCOL: return &protos;
      case KGPU_DICT_ZONE: return &zones;
      default: return nullptr;
    }
  }

  // ---------------------------------------------------------------- registration
  void register_node(const kgpu_node_desc& n) {
    for (int32_t i = 0; i < n.n_labels; ++i) nkeys.add(S(n.labels[i].key), S(n.labels[i].value));
    for (int32_t i = 0; i < n.n_taints; ++i) taint_add(S(n.taints[i].key), S(n.taints[i].value), S(n.taints[i].effect));
    for (int32_t i = 0; i < n.n_allocatable; ++i) {
      const string r = S(n.allocatable[i].name);
      if (is_scalar(r)) scalars.add(r);
    }
    for (int32_t i = 0; i < n.n_images; ++i)
      for (int32_t j = 0; j < n.images[i].n_names; ++j) images.add(S(n.images[i].names[j]));
    for (int32_t i = 0; i < n.n_avoid; ++i) controllers.add(join2(S(n.avoid[i].kind), S(n.avoid[i].uid)));
    const string z = zone_key(n);
    if (!z.empty()) zones.add(z);
  }

  void register_pod(const kgpu_pod_desc& p) {
    for (int32_t i = 0; i < p.n_labels; ++i) pkeys.add(S(p.labels[i].key), S(p.labels[i].value));
    ns.add(S(p.ns));
    for (int32_t k = 0; k < 2; ++k) {
      const kgpu_container_desc* cs = k ? p.init_containers : p.containers;
      const int32_t nc = k ? p.n_init_containers : p.n_containers;
      for (int32_t i = 0; i < nc; ++i)
        for (int32_t j = 0; j < cs[i].n_requests; ++j) {
          const string r = S(cs[i].requests[j].name);
          if (is_scalar(r)) scalars.add(r);
        }
    }
    for (int32_t i = 0; i < p.n_overhead; ++i) {
      const string r = S(p.overhead[i].name);
      if (is_scalar(r)) scalars.add(r);
    }
    for (int32_t i = 0; i < p.n_containers; ++i)
      for (int32_t j = 0; j < p.containers[i].n_ports; ++j) {
        const kgpu_port_desc& pt = p.containers[i].ports[j];
        if (pt.host_port > 0) {
          const string ip = S(pt.host_ip), pr = S(pt.protocol);
          ips.add(ip.empty() ? "0.0.0.0" : ip);
          protos.add(pr.empty() ? "TCP" : pr);
        }
      }
  }

  // ---------------------------------------------------------------- selectors
  // labels.NewRequirement validation (labels/selector.go:140-190)
  static void validate_req(const string& key, int32_t op, const vector<string>& vals) {
    if (!qualified_name_ok(key)) throw CompileError{"invalid label key \"" + key + "\""};
    if ((op == KGPU_OP_IN || op == KGPU_OP_NOTIN) && vals.empty()) throw CompileError{"values set can't be empty"};
    if ((op == KGPU_OP_EXISTS || op == KGPU_OP_DNE) && !vals.empty()) throw CompileError{"values set must be empty"};
    if (op == KGPU_OP_GT || op == KGPU_OP_LT) {
      int64_t x;
      if (vals.size() != 1 || !parse_int64(vals[0], x)) throw CompileError{"Gt/Lt needs one integer value"};
    }
    for (const string& v : vals)
      if (!label_value_ok(v)) throw CompileError{"invalid label value \"" + v + "\""};
  }

  // One requirement.  register: pod label selectors add their key and In / NotIn values to the pod key
  // space, so that a pod compiled later with that label gets the ids the selector already holds; node
  // selectors run against the snapshot's fixed node set and drop unknown values instead.
  static kgpu_req req_rec(KeySpace& ks, kgpu_pool_set& ps, const string& key, int32_t op, const vector<string>& vals,
                          bool reg) {
    int32_t ki;
    if (reg) {
      ki = ks.add_key(key);
      if (op == KGPU_OP_IN || op == KGPU_OP_NOTIN)
        for (const string& v : vals) ks.add(key, v);
    } else {
      ki = ks.key(key);
    }
    vector<int32_t> vids;
    if ((op == KGPU_OP_IN || op == KGPU_OP_NOTIN) && ki >= 0) {
      std::set<int32_t> s;
      for (const string& v : vals) {
        const int32_t vi = ks.val(ki, v);
        if (vi >= 0) s.insert(vi);
      }
      vids.assign(s.begin(), s.end());
    }
    kgpu_req r = zeroed<kgpu_req>();
    r.key = ki;
    r.op = op;
    r.vals = ps.ints_range(vids);
    r.imm = 0;
    if (op == KGPU_OP_GT || op == KGPU_OP_LT) {
      int64_t x = 0;
      if (!vals.empty() && parse_int64(vals[0], x)) r.imm = x;
    }
    return r;
  }

  static int32_t label_op(const string& op) {
    if (op == "In") return KGPU_OP_IN;
    if (op == "NotIn") return KGPU_OP_NOTIN;
    if (op == "Exists") return KGPU_OP_EXISTS;
    if (op == "DoesNotExist") return KGPU_OP_DNE;
    return -1;
  }
  static int32_t node_op(const string& op) {
    const int32_t o = label_op(op);
    if (o >= 0) return o;
    if (op == "Gt") return KGPU_OP_GT;
    if (op == "Lt") return KGPU_OP_LT;
    return -1;
  }
  static vector<string> values_of(const kgpu_expr_desc& e) {
    vector<string> v;
    v.reserve((size_t)e.n_values);
    for (int32_t i = 0; i < e.n_values; ++i) v.push_back(S(e.values[i]));
    return v;
  }

  // metav1.LabelSelectorAsSelector (apis/meta/v1/helpers.go:34-70): nil -> Nothing, matchLabels in key
  // order, then matchExpressions; an invalid requirement fails the whole selector
  kgpu_selector label_selector(kgpu_pool_set& ps, const kgpu_label_selector_desc& d) {
    kgpu_selector s = zeroed<kgpu_selector>();
    if (!d.present) {
      s.kind = KGPU_SEL_NOTHING;
      return s;
    }
    vector<std::pair<string, string>> ml;
    for (int32_t i = 0; i < d.n_match_labels; ++i) ml.emplace_back(S(d.match_labels[i].key), S(d.match_labels[i].value));
    std::sort(ml.begin(), ml.end());
    vector<kgpu_req> recs;
    for (const auto& kv : ml) {
      const vector<string> vals{kv.second};
      validate_req(kv.first, KGPU_OP_IN, vals);
      recs.push_back(req_rec(pkeys, ps, kv.first, KGPU_OP_IN, vals, true));
    }
    for (int32_t i = 0; i < d.n_exprs; ++i) {
      const kgpu_expr_desc& e = d.exprs[i];
      const int32_t op = label_op(S(e.op));
      if (op < 0) throw CompileError{"invalid pod selector operator \"" + S(e.op) + "\""};
      const vector<string> vals = values_of(e);
      validate_req(S(e.key), op, vals);
      recs.push_back(req_rec(pkeys, ps, S(e.key), op, vals, true));
    }
    s.kind = KGPU_SEL_AND;
    s.reqs = ps.reqs_range(recs);
    return s;
  }

  // NodeSelectorRequirementsAsSelector (helpers.go:237-267) body
  kgpu_range node_reqs(kgpu_pool_set& ps, const kgpu_expr_desc* ex, int32_t n, bool validate) {
    vector<kgpu_req> recs;
    for (int32_t i = 0; i < n; ++i) {
      const int32_t op = node_op(S(ex[i].op));
      if (op < 0) throw CompileError{"invalid node selector operator \"" + S(ex[i].op) + "\""};
      const vector<string> vals = values_of(ex[i]);
      if (validate) validate_req(S(ex[i].key), op, vals);
      recs.push_back(req_rec(nkeys, ps, S(ex[i].key), op, vals, false));
    }
    return ps.reqs_range(recs);
  }

  // One required NodeSelectorTerm (helpers.go:317-346; node_affinity.go:40-60): matchExpressions ANDed with
  // the metadata.name matchFields; a term that can match nothing has never_match
  kgpu_node_term node_term(kgpu_pool_set& ps, const kgpu_node_term_desc& t) {
    kgpu_node_term never = zeroed<kgpu_node_term>();
    never.field_op = -1;
    never.field_node = -1;
    never.never_match = 1;
    if (t.n_exprs == 0 && t.n_fields == 0) return never;
    kgpu_range reqs{0, 0};
    if (t.n_exprs) {
      try {
        reqs = node_reqs(ps, t.exprs, t.n_exprs, true);
      } catch (const CompileError&) {
        return never;
      }
    }
    int32_t fop = -1, fnode = -1;
    if (t.n_fields) {
      std::set<string> ins, notins;
      for (int32_t i = 0; i < t.n_fields; ++i) {
        const kgpu_expr_desc& e = t.fields[i];
        const string op = S(e.op);
        if ((op != "In" && op != "NotIn") || e.n_values != 1) return never;
        const string v = S(e.values[0]);
        if (S(e.key) != "metadata.name") {
          // fields.Set{"metadata.name": name}.Get(other key) == ""
          if ((op == "In") != (v.empty())) return never;
          continue;
        }
        (op == "In" ? ins : notins).insert(v);
      }
      bool overlap = false;
      for (const string& x : ins) overlap = overlap || notins.count(x);
      if (ins.size() > 1 || overlap) return never;
      if (!ins.empty()) {
        fop = KGPU_OP_IN;
        auto it = node_index.find(*ins.begin());
        fnode = it == node_index.end() ? -1 : it->second;
      } else if (!notins.empty()) {
        vector<int32_t> idx;
        for (const string& x : notins) {
          auto it = node_index.find(x);
          if (it != node_index.end()) idx.push_back(it->second);
        }
        if (idx.size() > 1) throw CompileError{"more than one metadata.name NotIn requirement in a term"};
        if (!idx.empty()) {
          fop = KGPU_OP_NOTIN;
          fnode = idx[0];
        }
      }
      if (t.n_exprs == 0 && fop == -1) {
        fop = KGPU_OP_NOTIN;  // fields only, all satisfied: matches every node
        fnode = -1;
      }
    }
    kgpu_node_term r = zeroed<kgpu_node_term>();
    r.reqs = reqs;
    r.field_op = fop;
    r.field_node = fnode;
    r.never_match = 0;
    return r;
  }

  // ---------------------------------------------------------------- pod terms (types.go:79-160)
  kgpu_pod_term pod_term(kgpu_pool_set& ps, const kgpu_pod_desc& pod, const kgpu_pod_term_desc& t, int32_t weight) {
    kgpu_pod_term r = zeroed<kgpu_pod_term>();
    r.weight = weight;
    r.sel = label_selector(ps, t.selector);
    std::set<string> names;
    for (int32_t i = 0; i < t.n_namespaces; ++i) names.insert(S(t.namespaces[i]));
    if (names.empty()) names.insert(S(pod.ns));
    vector<int32_t> ids;
    for (const string& n : names) ids.push_back(ns.add(n));
    r.ns = ps.ints_range(ids);
    r.topo_key = nkeys.key(S(t.topology_key));
    return r;
  }

  // getAffinityTerms / getWeightedAffinityTerms: one invalid selector drops the whole list
  vector<kgpu_pod_term> terms(kgpu_pool_set& ps, const kgpu_pod_desc& pod, const kgpu_pod_term_desc* ts, int32_t n,
                              bool weighted) {
    vector<kgpu_pod_term> out;
    if (n == 0) return out;
    const kgpu_pool_set::Mark m = ps.mark();
    try {
      for (int32_t i = 0; i < n; ++i) out.push_back(pod_term(ps, pod, ts[i], weighted ? ts[i].weight : 0));
    } catch (const CompileError&) {
      ps.rollback(m);
      out.clear();
    }
    return out;
  }

  // the four lists, in KGPU_TERM_* order
  void pod_terms(kgpu_pool_set& ps, const kgpu_pod_desc& pod, vector<kgpu_pod_term> out[4]) {
    const bool pa = pod.flags & KGPU_PD_POD_AFFINITY, paa = pod.flags & KGPU_PD_POD_ANTI;
    if (!(pod.flags & KGPU_PD_AFFINITY)) return;
    if (pa) out[KGPU_TERM_REQ_AFF] = terms(ps, pod, pod.affinity_required, pod.n_affinity_required, false);
    if (paa) out[KGPU_TERM_REQ_ANTI] = terms(ps, pod, pod.anti_required, pod.n_anti_required, false);
    if (pa) out[KGPU_TERM_PREF_AFF] = terms(ps, pod, pod.affinity_preferred, pod.n_affinity_preferred, true);
    if (paa) out[KGPU_TERM_PREF_ANTI] = terms(ps, pod, pod.anti_preferred, pod.n_anti_preferred, true);
  }

  // podMatchesAllAffinityTerms (interpodaffinity/filtering.go:334-346) on the pod itself
  bool self_match_all(const kgpu_pod_desc& pod) {
    const string own = S(pod.ns);
    for (int32_t i = 0; i < pod.n_affinity_required; ++i) {
      const kgpu_pod_term_desc& t = pod.affinity_required[i];
      bool in_ns = t.n_namespaces == 0;
      for (int32_t j = 0; j < t.n_namespaces; ++j) in_ns = in_ns || S(t.namespaces[j]) == own;
      if (!in_ns || !selector_matches(t.selector, pod.labels, pod.n_labels)) return false;
    }
    return true;
  }

  // PodTopologySpread constraints of one action (podtopologyspread/common.go:44-99): the pod's own, or
  // the profile's default constraints over the pod's DefaultSelector
  kgpu_range spreads(kgpu_pool_set& ps, const kgpu_pod_desc& pod, const char* action) {
    struct Con {
      int32_t max_skew;
      string key;
      const kgpu_label_selector_desc* sel;
    };
    vector<Con> cons;
    if (pod.n_spreads) {
      for (int32_t i = 0; i < pod.n_spreads; ++i)
        if (S(pod.spreads[i].when_unsatisfiable) == action)
          cons.push_back(Con{pod.spreads[i].max_skew, S(pod.spreads[i].topology_key), &pod.spreads[i].selector});
    } else if ((pod.flags & KGPU_PD_DEFAULT_SELECTOR) && pod.default_selector.present) {
      for (size_t i = 0; i < default_spreads.size(); ++i)
        if (default_spread_whens[i] == action)
          cons.push_back(Con{default_spreads[i].max_skew, default_spread_keys[i], &pod.default_selector});
    }
    vector<kgpu_spread> recs;
    for (const Con& c : cons) {
      kgpu_spread r = zeroed<kgpu_spread>();
      r.sel = label_selector(ps, *c.sel);
      r.max_skew = c.max_skew;
      r.key = nkeys.key(c.key);
      r.is_hostname = c.key == kHostname ? 1 : 0;
      r.self_match = selector_matches(*c.sel, pod.labels, pod.n_labels) ? 1 : 0;
      recs.push_back(r);
    }
    return ps.rng(5, ps.spreads, recs);
  }

  // ---------------------------------------------------------------- the pod query
  void compile_pod(kgpu_pool_set& ps, const kgpu_pod_desc& pod, kgpu_pod_query& q) {
    q = zeroed<kgpu_pod_query>();
    uint32_t flags = 0;
    const PodResources res = pod_resources(pod);
    q.ns = ns.add(S(pod.ns));
    q.req[0] = res.cpu;
    q.req[1] = res.mem;
    q.req[2] = res.eph;
    q.nz[0] = res.nz_cpu;
    q.nz[1] = res.nz_mem;
    q.score_req[0] = score_request(pod, "cpu");
    q.score_req[1] = score_request(pod, "memory");
    q.score_req[2] = score_request(pod, "ephemeral-storage");
    if (res.fit_all_zero) flags |= KGPU_Q_FIT_ALL_ZERO;
    // scalar requests (Fit checks them unless ignored, fit.go:247-264), then the scorers' scalar
    // resources the pod does not request
    {
      vector<kgpu_scalar_req> sc;
      vector<string> names;
      std::set<string> seen;
      for (const auto& kv : res.scalars) {
        kgpu_scalar_req r = zeroed<kgpu_scalar_req>();
        r.col = scalars.get(kv.first);
        r.check = (is_extended(kv.first) && ignored.count(kv.first)) ? 0 : 1;
        r.value = kv.second;
        r.score_value = score_request(pod, kv.first);
        sc.push_back(r);
        names.push_back(kv.first);
        seen.insert(kv.first);
      }
      for (const string& r : score_resources) {
        if (r == "cpu" || r == "memory" || r == "ephemeral-storage" || seen.count(r) || !is_scalar(r)) continue;
        kgpu_scalar_req x = zeroed<kgpu_scalar_req>();
        x.col = scalars.get(r);
        x.check = 0;
        x.value = 0;
        x.score_value = score_request(pod, r);
        sc.push_back(x);
        names.push_back(r);
        seen.insert(r);
      }
      q.scalars = ps.scalars_range(sc, names);
    }
    const string nn = S(pod.node_name);
    if (nn.empty()) {
      q.node_name = -1;
    } else {
      auto it = node_index.find(nn);
      q.node_name = it == node_index.end() ? -2 : it->second;
    }
    q.n_containers = pod.n_containers;
    // host ports (types.go:728-731)
    {
      vector<kgpu_port> want;
      for (int32_t i = 0; i < pod.n_containers; ++i)
        for (int32_t j = 0; j < pod.containers[i].n_ports; ++j) {
          const kgpu_port_desc& pt = pod.containers[i].ports[j];
          if (pt.host_port <= 0) continue;
          const string ip = S(pt.host_ip), pr = S(pt.protocol);
          kgpu_port p = zeroed<kgpu_port>();
          p.ip = ips.add(ip.empty() ? "0.0.0.0" : ip);
          p.proto = protos.add(pr.empty() ? "TCP" : pr);
          p.port = pt.host_port;
          want.push_back(p);
        }
      q.ports = ps.rng(8, ps.ports, want);
    }
    // tolerations as masks over the taint dictionary (taint_toleration.go:54-152; PreScore keeps the
    // tolerations with an empty or PreferNoSchedule effect, :103-114)
    {
      const int32_t TW = taint_words();
      vector<uint64_t> m_ns((size_t)TW, 0), m_pr((size_t)TW, 0);
      for (size_t tid = 0; tid < taint_items.size(); ++tid) {
        const string& k = taint_items[tid].first;
        const string& v = taint_items[tid].second.first;
        const string& e = taint_items[tid].second.second;
        const size_t w = tid / 64, b = tid % 64;
        if (e == "NoSchedule" || e == "NoExecute") {
          for (int32_t i = 0; i < pod.n_tolerations; ++i)
            if (tolerates(pod.tolerations[i], k, v, e)) {
              m_ns[w] |= 1ull << b;
              break;
            }
        }
        if (e == "PreferNoSchedule") {
          for (int32_t i = 0; i < pod.n_tolerations; ++i) {
            const string te = S(pod.tolerations[i].effect);
            if ((te.empty() || te == "PreferNoSchedule") && tolerates(pod.tolerations[i], k, v, e)) {
              m_pr[w] |= 1ull << b;
              break;
            }
          }
        }
      }
      q.tol_nosched = ps.words_range(m_ns);
      q.tol_prefer = ps.words_range(m_pr);
      for (int32_t i = 0; i < pod.n_tolerations; ++i)
        if (tolerates(pod.tolerations[i], "node.kubernetes.io/unschedulable", "", "NoSchedule"))
          flags |= KGPU_Q_TOLERATES_UNSCHEDULABLE;
    }
    // nodeSelector map: labels.SelectorFromSet, no validation (helper/node_affinity.go:30-36)
    {
      vector<std::pair<string, string>> sel;
      for (int32_t i = 0; i < pod.n_node_selector; ++i)
        sel.emplace_back(S(pod.node_selector[i].key), S(pod.node_selector[i].value));
      std::sort(sel.begin(), sel.end());
      vector<kgpu_req> recs;
      for (const auto& kv : sel) recs.push_back(req_rec(nkeys, ps, kv.first, KGPU_OP_IN, {kv.second}, false));
      q.node_selector = ps.reqs_range(recs);
    }
    // required node affinity (node_affinity.go:40-60, helpers.go:317-346)
    const bool na = (pod.flags & KGPU_PD_AFFINITY) && (pod.flags & KGPU_PD_NODE_AFFINITY);
    if (na && (pod.flags & KGPU_PD_NODE_REQUIRED)) {
      flags |= KGPU_Q_REQ_NODE_AFFINITY;
      vector<kgpu_node_term> recs;
      for (int32_t i = 0; i < pod.n_required_terms; ++i) recs.push_back(node_term(ps, pod.required_terms[i]));
      q.req_terms = ps.rng(3, ps.node_terms, recs);
    }
    // preferred node affinity (node_affinity.go:80-99): weight 0 skipped; an invalid term is a Score error
    {
      vector<kgpu_pref_term> prefs;
      if (na)
        for (int32_t i = 0; i < pod.n_preferred_terms; ++i) {
          const kgpu_pref_node_term_desc& t = pod.preferred_terms[i];
          if (t.weight == 0) continue;
          kgpu_pref_term r = zeroed<kgpu_pref_term>();
          r.weight = t.weight;
          if (t.preference.n_exprs == 0) {
            r.sel.kind = KGPU_SEL_NOTHING;
            prefs.push_back(r);
            continue;
          }
          try {
            r.sel.reqs = node_reqs(ps, t.preference.exprs, t.preference.n_exprs, true);
          } catch (const CompileError&) {
            flags |= KGPU_Q_SCORE_ERROR;
            continue;
          }
          r.sel.kind = KGPU_SEL_AND;
          prefs.push_back(r);
        }
      q.pref_terms = ps.rng(4, ps.pref_terms, prefs);
    }
    // ImageLocality (image_locality.go:84-98): normalized image ids per container
    {
      vector<int32_t> ims;
      bool known = false;
      for (int32_t i = 0; i < pod.n_containers; ++i) {
        const int32_t id = images.get(normalized_image_name(S(pod.containers[i].image)));
        known = known || id >= 0;
        ims.push_back(id);
      }
      q.images = ps.ints_range(ims);
      if (!known) flags |= KGPU_Q_NO_KNOWN_IMAGE;  // sumScores 0 -> score 0 (image_locality.go:53-79)
    }
    // NodePreferAvoidPods: a ReplicationController / ReplicaSet controllerRef (node_prefer_avoid_pods.go:50-66)
    q.avoid_id = -1;
    if (pod.flags & KGPU_PD_CONTROLLER) {
      const string kind = S(pod.controller_kind);
      if (kind == "ReplicationController" || kind == "ReplicaSet")
        q.avoid_id = controllers.get(join2(kind, S(pod.controller_uid)));
    }
    // PodTopologySpread
    if (pod.n_spreads) flags |= KGPU_Q_HAS_TSC;
    q.pts_hard = spreads(ps, pod, "DoNotSchedule");
    q.pts_soft = spreads(ps, pod, "ScheduleAnyway");
    // DefaultPodTopologySpread selector (default_pod_topology_spread.go:191-205); Empty(): counts are 0
    if ((pod.flags & KGPU_PD_DEFAULT_SELECTOR) && pod.default_selector.present) {
      q.dpts = label_selector(ps, pod.default_selector);
    } else {
      q.dpts = zeroed<kgpu_selector>();
      q.dpts.kind = KGPU_SEL_EMPTY;
    }
    // InterPodAffinity
    if (pod.flags & KGPU_PD_AFFINITY) {
      if (pod.flags & KGPU_PD_POD_AFFINITY) flags |= KGPU_Q_HAS_POD_AFFINITY;
      if (pod.flags & KGPU_PD_POD_ANTI) flags |= KGPU_Q_HAS_POD_ANTI;
    }
    {
      vector<kgpu_pod_term> byk[4];
      pod_terms(ps, pod, byk);
      q.ipa_req_aff = ps.rng(6, ps.pod_terms, byk[KGPU_TERM_REQ_AFF]);
      q.ipa_req_anti = ps.rng(6, ps.pod_terms, byk[KGPU_TERM_REQ_ANTI]);
      q.ipa_pref_aff = ps.rng(6, ps.pod_terms, byk[KGPU_TERM_PREF_AFF]);
      q.ipa_pref_anti = ps.rng(6, ps.pod_terms, byk[KGPU_TERM_PREF_ANTI]);
      if (!byk[KGPU_TERM_REQ_AFF].empty() && self_match_all(pod)) flags |= KGPU_Q_SELF_MATCH_ALL_AFF;
    }
    // the pod's own labels as (key, value) id pairs, in key order
    {
      vector<std::pair<string, string>> l;
      for (int32_t i = 0; i < pod.n_labels; ++i) l.emplace_back(S(pod.labels[i].key), S(pod.labels[i].value));
      std::sort(l.begin(), l.end());
      vector<int32_t> pairs;
      for (const auto& kv : l) {
        const auto kvid = pkeys.add(kv.first, kv.second);
        pairs.push_back(kvid.first);
        pairs.push_back(kvid.second);
      }
      q.labels = ps.ints_range(pairs);
    }
    if (pod.flags & KGPU_PD_TERMINATING) flags |= KGPU_Q_TERMINATING;
    q.flags = flags;
    pod_limits(pod, q.limits);
    q.priority = (pod.flags & KGPU_PD_PRIORITY) ? pod.priority : 0;  // podutil.GetPodPriority
    const string uid = S(pod.uid);
    q.uid = 1 + uids.add(uid.empty() ? S(pod.ns) + "/" + S(pod.name) : uid);
  }

  // ---------------------------------------------------------------- snapshot
  void set_order(vector<string> names, bool first_wins) {
    node_index.clear();
    node_index.reserve(names.size() * 2);
    for (size_t i = 0; i < names.size(); ++i) {
      if (first_wins) node_index.emplace(names[i], (int32_t)i);
      else node_index[names[i]] = (int32_t)i;
    }
    order = std::move(names);
  }

  void empty_columns(SnapBuf& A, size_t N) {
    for (auto* v : {&A.alloc_cpu, &A.alloc_mem, &A.alloc_eph, &A.req_cpu, &A.req_mem, &A.req_eph, &A.nz_cpu, &A.nz_mem})
      v->assign(N, 0);
    A.alloc_pods.assign(N, 0);
    A.num_pods.assign(N, 0);
    A.alloc_scalar.assign((size_t)scalars.size() * N, 0);
    A.req_scalar.assign((size_t)scalars.size() * N, 0);
    A.unschedulable.assign(N, 0);
    A.label_val.assign((size_t)nkeys.keys.size() * N, -1);
    A.taint_nosched.assign((size_t)taint_words() * N, 0);
    A.taint_prefer.assign((size_t)taint_words() * N, 0);
    A.zone_id.assign(N, -1);
  }

  // scaledImageScore (image_locality.go:100-113) CSR and the NodePreferAvoidPods CSR over `list`; spread
  // counted over `all`.  add: grow the image / controller dictionaries (a delta), else look ids up.
  void lists(const kgpu_node_desc* list, int32_t n_list, const kgpu_node_desc* all, int32_t n_all, bool add,
             vector<int32_t>& image_off, vector<int32_t>& image_id, vector<int64_t>& image_score,
             vector<int32_t>& avoid_off, vector<int32_t>& avoid_id) {
    std::unordered_map<string, std::set<string>> name_to_nodes;
    for (int32_t i = 0; i < n_all; ++i)
      for (int32_t j = 0; j < all[i].n_images; ++j)
        for (int32_t k = 0; k < all[i].images[j].n_names; ++k)
          name_to_nodes[S(all[i].images[j].names[k])].insert(S(all[i].name));
    const double N = (double)n_list;
    image_off.assign(1, 0);
    avoid_off.assign(1, 0);
    image_id.clear();
    image_score.clear();
    avoid_id.clear();
    for (int32_t i = 0; i < n_list; ++i) {
      const kgpu_node_desc& n = list[i];
      std::map<int32_t, int64_t> ims;
      for (int32_t j = 0; j < n.n_images; ++j)
        for (int32_t k = 0; k < n.images[j].n_names; ++k) {
          const string nm = S(n.images[j].names[k]);
          const double spread = (double)name_to_nodes[nm].size() / N;
          const int32_t id = add ? images.add(nm) : images.get(nm);
          ims[id] = (int64_t)((double)n.images[j].size_bytes * spread);
        }
      for (const auto& kv : ims) {
        image_id.push_back(kv.first);
        image_score.push_back(kv.second);
      }
      image_off.push_back((int32_t)image_id.size());
      std::set<int32_t> av;
      for (int32_t j = 0; j < n.n_avoid; ++j) {
        const string key = join2(S(n.avoid[j].kind), S(n.avoid[j].uid));
        av.insert(add ? controllers.add(key) : controllers.get(key));
      }
      avoid_id.insert(avoid_id.end(), av.begin(), av.end());
      avoid_off.push_back((int32_t)avoid_id.size());
    }
  }

  void node_columns(SnapBuf& A, const kgpu_node_desc* nodes, int32_t N) {
    empty_columns(A, (size_t)N);
    const size_t n = (size_t)N;
    for (int32_t i = 0; i < N; ++i) {
      const kgpu_node_desc& d = nodes[i];
      int64_t cpu = 0, mem = 0, eph = 0, pods = 0;
      for (int32_t j = 0; j < d.n_allocatable; ++j) {
        const string r = S(d.allocatable[j].name);
        if (r == "cpu") cpu += d.allocatable[j].milli;
        else if (r == "memory") mem += d.allocatable[j].value;
        else if (r == "pods") pods += d.allocatable[j].value;
        else if (r == "ephemeral-storage") eph += d.allocatable[j].value;
        else if (is_scalar(r)) {
          const int32_t col = scalars.get(r);
          if (col >= 0) A.alloc_scalar[(size_t)col * n + (size_t)i] += d.allocatable[j].value;
        }
      }
      A.alloc_cpu[(size_t)i] = cpu;
      A.alloc_mem[(size_t)i] = mem;
      A.alloc_eph[(size_t)i] = eph;
      A.alloc_pods[(size_t)i] = (int32_t)pods;
      A.unschedulable[(size_t)i] = d.unschedulable ? 1 : 0;
      for (int32_t j = 0; j < d.n_labels; ++j) {
        const int32_t ki = nkeys.key(S(d.labels[j].key));
        if (ki >= 0) A.label_val[(size_t)ki * n + (size_t)i] = nkeys.val(ki, S(d.labels[j].value));
      }
      for (int32_t j = 0; j < d.n_taints; ++j) {
        const string e = S(d.taints[j].effect);
        const int32_t tid = taints.get(join3(S(d.taints[j].key), S(d.taints[j].value), e));
        if (tid < 0) continue;
        const size_t w = (size_t)tid / 64, b = (size_t)tid % 64;
        if (e == "NoSchedule" || e == "NoExecute") A.taint_nosched[w * n + (size_t)i] |= 1ull << b;
        else if (e == "PreferNoSchedule") A.taint_prefer[w * n + (size_t)i] |= 1ull << b;
      }
      const string z = zone_key(d);
      A.zone_id[(size_t)i] = z.empty() ? -1 : zones.get(z);
    }
    lists(nodes, N, nodes, N, false, A.image_off, A.image_id, A.image_score, A.avoid_off, A.avoid_id);
  }

  // Everything after the node columns: existing pods (NodeInfo.AddPod, types.go:456-480), label value
  // metadata, key uniqueness over the whole list, the shard slice.
  void finish(SnapBuf& A, const kgpu_pod_desc* existing, int32_t n_existing, const int64_t* uids_in, int32_t base,
              int32_t cnt, kgpu_snapshot& out) {
    const size_t N = A.alloc_cpu.size();
    const int32_t S_ = scalars.size(), K = nkeys.keys.size(), TW = taint_words();
    const int32_t PK = pkeys.keys.size();
    vector<vector<std::tuple<int32_t, int32_t, int32_t>>> used((size_t)N);
    vector<int32_t> plab;
    for (int32_t e = 0; e < n_existing; ++e) {
      const kgpu_pod_desc& p = existing[e];
      auto it = node_index.find(S(p.node_name));
      if (it == node_index.end()) continue;  // NewSnapshot keeps such pods on node-less NodeInfos
      const size_t ni = (size_t)it->second;
      const PodResources res = pod_resources(p);
      A.req_cpu[ni] += res.cpu;
      A.req_mem[ni] += res.mem;
      A.req_eph[ni] += res.eph;
      for (const auto& kv : res.scalars) {
        const int32_t col = scalars.get(kv.first);
        if (col >= 0) A.req_scalar[(size_t)col * N + ni] += kv.second;
      }
      A.nz_cpu[ni] += res.nz_cpu;
      A.nz_mem[ni] += res.nz_mem;
      A.num_pods[ni] += 1;
      for (int32_t i = 0; i < p.n_containers; ++i)
        for (int32_t j = 0; j < p.containers[i].n_ports; ++j) {
          const kgpu_port_desc& pt = p.containers[i].ports[j];
          if (pt.host_port <= 0) continue;
          const string ip = S(pt.host_ip), pr = S(pt.protocol);
          used[ni].emplace_back(ips.get(ip.empty() ? "0.0.0.0" : ip), protos.get(pr.empty() ? "TCP" : pr), pt.host_port);
        }
      const int32_t slot = (int32_t)A.pod_node.size();
      A.pod_node.push_back((int32_t)ni);
      if (uids_in) A.pod_uid.push_back(uids_in[e]);
      A.pod_ns.push_back(ns.get(S(p.ns)));
      uint32_t fl = KGPU_PF_ACTIVE;
      if (p.flags & KGPU_PD_TERMINATING) fl |= KGPU_PF_TERMINATING;
      if ((p.flags & KGPU_PD_AFFINITY) && (p.flags & (KGPU_PD_POD_AFFINITY | KGPU_PD_POD_ANTI))) fl |= KGPU_PF_WITH_AFFINITY;
      A.pod_flags.push_back(fl);
      vector<int32_t> row((size_t)PK, -1);
      for (int32_t i = 0; i < p.n_labels; ++i) {
        const int32_t ki = pkeys.key(S(p.labels[i].key));
        if (ki >= 0 && ki < PK) row[(size_t)ki] = pkeys.val(ki, S(p.labels[i].value));
      }
      plab.insert(plab.end(), row.begin(), row.end());
      vector<kgpu_pod_term> byk[4];
      pod_terms(A.pools, p, byk);
      for (int32_t k = 0; k < 4; ++k)
        for (const kgpu_pod_term& t : byk[k]) {
          kgpu_term x = zeroed<kgpu_term>();
          x.pod = slot;
          x.kind = k;
          x.t = t;
          A.terms.push_back(x);
        }
    }
    const size_t P = A.pod_node.size();
    // pod_label_val [PK][P] (transposed from the rows)
    A.pod_label_val.assign((size_t)PK * P, -1);
    for (size_t i = 0; i < P; ++i)
      for (size_t k = 0; k < (size_t)PK; ++k) A.pod_label_val[k * P + i] = plab[i * (size_t)PK + k];
    size_t slots = 1;
    for (const auto& u : used) slots = std::max(slots, u.size());
    A.port_slots = (int32_t)slots;
    A.port_count.assign(N, 0);
    A.ports.assign(slots * N, zeroed<kgpu_port>());
    for (size_t i = 0; i < N; ++i) {
      std::set<std::tuple<int32_t, int32_t, int32_t>> u(used[i].begin(), used[i].end());
      size_t s = 0;
      for (const auto& t : u) {
        kgpu_port& pt = A.ports[s * N + i];
        pt.ip = std::get<0>(t);
        pt.proto = std::get<1>(t);
        pt.port = std::get<2>(t);
        ++s;
      }
      A.port_count[i] = (int32_t)u.size();
    }
    // label value metadata
    key_meta_into(K, A.key_n_values, A.value_off, A.value_int, A.value_int_ok, A.key_empty_value);
    // key_unique over the whole list (before any shard slice)
    A.key_unique.assign((size_t)K, 0);
    for (int32_t k = 0; k < K; ++k) {
      std::unordered_map<int32_t, int> seen;
      bool uniq = true;
      for (size_t i = 0; i < N && uniq; ++i) {
        const int32_t v = A.label_val[(size_t)k * N + i];
        if (v >= 0 && seen[v]++) uniq = false;
      }
      A.key_unique[(size_t)k] = uniq ? 1 : 0;
    }
    // the shard slice
    SnapBuf* V = &A;
    if (cnt >= 0 && !(base == 0 && (size_t)cnt == N)) {
      delete A.sliced;
      A.sliced = new SnapBuf();
      V = A.sliced;
      const size_t b = (size_t)base, c = (size_t)cnt;
      auto cut = [&](auto& dst, const auto& src) { dst.assign(src.begin() + (long)b, src.begin() + (long)(b + c)); };
      cut(V->alloc_cpu, A.alloc_cpu);
      cut(V->alloc_mem, A.alloc_mem);
      cut(V->alloc_eph, A.alloc_eph);
      cut(V->alloc_pods, A.alloc_pods);
      cut(V->req_cpu, A.req_cpu);
      cut(V->req_mem, A.req_mem);
      cut(V->req_eph, A.req_eph);
      cut(V->nz_cpu, A.nz_cpu);
      cut(V->nz_mem, A.nz_mem);
      cut(V->num_pods, A.num_pods);
      cut(V->unschedulable, A.unschedulable);
      cut(V->zone_id, A.zone_id);
      cut(V->port_count, A.port_count);
      auto cut2 = [&](auto& dst, const auto& src, size_t rows) {
        dst.clear();
        for (size_t r = 0; r < rows; ++r)
          dst.insert(dst.end(), src.begin() + (long)(r * N + b), src.begin() + (long)(r * N + b + c));
      };
      cut2(V->alloc_scalar, A.alloc_scalar, (size_t)S_);
      cut2(V->req_scalar, A.req_scalar, (size_t)S_);
      cut2(V->label_val, A.label_val, (size_t)K);
      cut2(V->taint_nosched, A.taint_nosched, (size_t)TW);
      cut2(V->taint_prefer, A.taint_prefer, (size_t)TW);
      cut2(V->ports, A.ports, slots);
      auto cut_csr = [&](vector<int32_t>& off, vector<int32_t>& ids, vector<int64_t>* vals, const vector<int32_t>& o,
                         const vector<int32_t>& i, const vector<int64_t>* v) {
        const int32_t lo = o[b], hi = o[b + c];
        off.clear();
        for (size_t k = b; k <= b + c; ++k) off.push_back(o[k] - lo);
        ids.assign(i.begin() + lo, i.begin() + hi);
        if (vals) vals->assign(v->begin() + lo, v->begin() + hi);
      };
      cut_csr(V->image_off, V->image_id, &V->image_score, A.image_off, A.image_id, &A.image_score);
      cut_csr(V->avoid_off, V->avoid_id, nullptr, A.avoid_off, A.avoid_id, nullptr);
    }
    // the struct
    out = zeroed<kgpu_snapshot>();
    out.n_nodes = (int32_t)(V == &A ? N : (size_t)cnt);
    out.node_base = V == &A ? 0 : base;
    out.n_total_nodes = (int32_t)N;
    out.alloc_cpu = V->alloc_cpu.data();
    out.alloc_mem = V->alloc_mem.data();
    out.alloc_eph = V->alloc_eph.data();
    out.alloc_pods = V->alloc_pods.data();
    out.req_cpu = V->req_cpu.data();
    out.req_mem = V->req_mem.data();
    out.req_eph = V->req_eph.data();
    out.nz_cpu = V->nz_cpu.data();
    out.nz_mem = V->nz_mem.data();
    out.num_pods = V->num_pods.data();
    out.n_scalar = S_;
    out.alloc_scalar = ptr_or_null(V->alloc_scalar);
    out.req_scalar = ptr_or_null(V->req_scalar);
    out.unschedulable = V->unschedulable.data();
    out.n_label_keys = K;
    out.label_val = ptr_or_null(V->label_val);
    out.key_n_values = ptr_or_null(A.key_n_values);
    out.value_off = A.value_off.data();
    out.value_int = ptr_or_null(A.value_int);
    out.value_int_ok = ptr_or_null(A.value_int_ok);
    out.key_empty_value = ptr_or_null(A.key_empty_value);
    out.taint_words = TW;
    out.taint_nosched = V->taint_nosched.data();
    out.taint_prefer = V->taint_prefer.data();
    out.port_slots = (int32_t)slots;
    out.port_count = V->port_count.data();
    out.ports = V->ports.data();
    out.image_off = V->image_off.data();
    out.image_id = ptr_or_null(V->image_id);
    out.image_score = ptr_or_null(V->image_score);
    out.avoid_off = V->avoid_off.data();
    out.avoid_id = ptr_or_null(V->avoid_id);
    out.zone_id = V->zone_id.data();
    out.n_zones = zones.size();
    out.n_pods = (int32_t)P;
    out.pod_node = ptr_or_null(A.pod_node);
    out.pod_ns = ptr_or_null(A.pod_ns);
    out.pod_flags = ptr_or_null(A.pod_flags);
    out.n_pod_label_keys = PK;
    out.n_terms = (int32_t)A.terms.size();
    out.pod_label_val = ptr_or_null(A.pod_label_val);
    out.terms = ptr_or_null(A.terms);
    kgpu_pools_view_of(A.pools, out.pools);
    out.pod_uid = uids_in ? (A.pod_uid.empty() ? nullptr : A.pod_uid.data()) : nullptr;
    out.key_unique = ptr_or_null(A.key_unique);
    dims[0] = S_;
    dims[1] = K;
    dims[2] = TW;
  }

  static void kgpu_pools_view_of(const kgpu_pool_set& ps, kgpu_pools& o) {
    o.reqs = ptr_or_null(ps.reqs);
    o.n_reqs = (int32_t)ps.reqs.size();
    o.ints = ptr_or_null(ps.ints);
    o.n_ints = (int32_t)ps.ints.size();
    o.words = ptr_or_null(ps.words);
    o.n_words = (int32_t)ps.words.size();
    o.node_terms = ptr_or_null(ps.node_terms);
    o.n_node_terms = (int32_t)ps.node_terms.size();
    o.pref_terms = ptr_or_null(ps.pref_terms);
    o.n_pref_terms = (int32_t)ps.pref_terms.size();
    o.spreads = ptr_or_null(ps.spreads);
    o.n_spreads = (int32_t)ps.spreads.size();
    o.pod_terms = ptr_or_null(ps.pod_terms);
    o.n_pod_terms = (int32_t)ps.pod_terms.size();
    o.scalars = ptr_or_null(ps.scalars);
    o.n_scalars = (int32_t)ps.scalars.size();
    o.ports = ptr_or_null(ps.ports);
    o.n_ports = (int32_t)ps.ports.size();
  }

  void key_meta_into(int32_t K, vector<int32_t>& knv, vector<int32_t>& off, vector<int64_t>& ints, vector<uint8_t>& oks,
                     vector<int32_t>& empty) {
    knv.clear();
    off.assign(1, 0);
    ints.clear();
    oks.clear();
    empty.clear();
    for (int32_t k = 0; k < K; ++k) {
      const StrDict& d = nkeys.vals[(size_t)k];
      for (const string& v : d.items) {
        int64_t x = 0;
        const bool ok = parse_int64(v, x);
        ints.push_back(ok ? x : 0);
        oks.push_back(ok ? 1 : 0);
      }
      off.push_back((int32_t)ints.size());
      empty.push_back(d.get(""));
      knv.push_back(d.size());
    }
  }

  // ---------------------------------------------------------------- node rows (deltas)
  void node_row(kgpu_pool_set& ps, const kgpu_node_desc& n, kgpu_node_row& r) {
    r = zeroed<kgpu_node_row>();
    int64_t cpu = 0, mem = 0, eph = 0, pods = 0;
    vector<int64_t> sc((size_t)dims[0], 0);
    for (int32_t j = 0; j < n.n_allocatable; ++j) {
      const string res = S(n.allocatable[j].name);
      if (res == "cpu") cpu += n.allocatable[j].milli;
      else if (res == "memory") mem += n.allocatable[j].value;
      else if (res == "pods") pods += n.allocatable[j].value;
      else if (res == "ephemeral-storage") eph += n.allocatable[j].value;
      else if (is_scalar(res)) {
        const int32_t col = scalars.add(res);
        if (col >= dims[0]) throw NeedsUpload{"new scalar resource \"" + res + "\""};
        sc[(size_t)col] += n.allocatable[j].value;
      }
    }
    r.alloc_cpu = cpu;
    r.alloc_mem = mem;
    r.alloc_eph = eph;
    r.alloc_pods = (int32_t)pods;
    r.unschedulable = n.unschedulable ? 1 : 0;
    const string z = zone_key(n);
    r.zone_id = z.empty() ? -1 : zones.add(z);
    vector<std::pair<string, string>> l;
    for (int32_t j = 0; j < n.n_labels; ++j) l.emplace_back(S(n.labels[j].key), S(n.labels[j].value));
    std::sort(l.begin(), l.end());
    vector<int32_t> pairs;
    for (const auto& kv : l) {
      const int32_t ki = nkeys.key(kv.first);
      if (ki < 0 || ki >= dims[1]) throw NeedsUpload{"new node label key \"" + kv.first + "\""};
      pairs.push_back(ki);
      pairs.push_back(nkeys.add(kv.first, kv.second).second);
    }
    r.labels = ps.ints_range(pairs);
    const int32_t TW = dims[2];
    vector<uint64_t> words((size_t)2 * TW, 0);
    bool any = false;
    for (int32_t j = 0; j < n.n_taints; ++j) {
      const string e = S(n.taints[j].effect);
      const int32_t tid = taint_add(S(n.taints[j].key), S(n.taints[j].value), e);
      const int32_t w = tid / 64, b = tid % 64;
      if (w >= TW) throw NeedsUpload{"taint dictionary outgrew " + std::to_string(TW) + " words"};
      if (e == "NoSchedule" || e == "NoExecute") words[(size_t)w] |= 1ull << b;
      else if (e == "PreferNoSchedule") words[(size_t)(TW + w)] |= 1ull << b;
    }
    for (uint64_t w : words) any = any || w;
    r.taints = any ? ps.words_range(words) : kgpu_range{0, 0};
    bool any_sc = false;
    vector<uint64_t> scw;
    for (int64_t v : sc) {
      any_sc = any_sc || v;
      scw.push_back((uint64_t)v);
    }
    r.alloc_scalar = any_sc ? ps.words_range(scw) : kgpu_range{0, 0};
    for (int32_t j = 0; j < n.n_images; ++j)
      for (int32_t k = 0; k < n.images[j].n_names; ++k) images.add(S(n.images[j].names[k]));
    for (int32_t j = 0; j < n.n_avoid; ++j) controllers.add(join2(S(n.avoid[j].kind), S(n.avoid[j].uid)));
  }
};

// ==================================================================== C ABI
namespace {
int fail(kgpu_compiler* c, int code, const string& msg) {
  if (c) c->err = msg;
  return code;
}
}  // namespace

#define KC_TRY try {
#define KC_CATCH(c)                                                  \
  }                                                                  \
  catch (const CompileError& e) {                                    \
    return fail(c, KGPU_E_INVAL, e.msg);                             \
  }                                                                  \
  catch (const NeedsUpload& e) {                                     \
    return fail(c, KGPU_E_CAPACITY, e.msg);                          \
  }                                                                  \
  catch (const std::bad_alloc&) {                                    \
    return fail(c, KGPU_E_NOMEM, "out of host memory");              \
  }                                                                  \
  catch (...) {                                                      \
    return fail(c, KGPU_E_INVAL, "unexpected exception in compiler"); \
  }

extern "C" {

int kgpu_compiler_create(const kgpu_compile_profile* prof, kgpu_compiler** out) {
  if (!out) return KGPU_E_INVAL;
  *out = nullptr;
  try {
    kgpu_compiler* c = new kgpu_compiler();
    c->ips.add("0.0.0.0");
    c->protos.add("TCP");
    c->protos.add("UDP");
    c->protos.add("SCTP");
    if (prof) {
      for (int32_t i = 0; i < prof->n_column_resources; ++i) {
        const string r = S(prof->column_resources[i]);
        if (r != "cpu" && r != "memory" && r != "ephemeral-storage") c->scalars.add(r);
        if (i < prof->n_score_resources) c->score_resources.push_back(r);
      }
      for (int32_t i = 0; i < prof->n_ignored_resources; ++i) c->ignored.insert(S(prof->ignored_resources[i]));
      for (int32_t i = 0; i < prof->n_default_spreads; ++i) {
        c->default_spreads.push_back(prof->default_spreads[i]);
        c->default_spread_keys.push_back(S(prof->default_spreads[i].topology_key));
        c->default_spread_whens.push_back(S(prof->default_spreads[i].when_unsatisfiable));
      }
    }
    *out = c;
    return KGPU_OK;
  } catch (...) {
    return KGPU_E_NOMEM;
  }
}

int kgpu_compile_struct_sizes(int32_t* out, int32_t n) {
  const int32_t sz[] = {(int32_t)sizeof(kgpu_str), (int32_t)sizeof(kgpu_kv), (int32_t)sizeof(kgpu_quantity),
                        (int32_t)sizeof(kgpu_expr_desc), (int32_t)sizeof(kgpu_label_selector_desc),
                        (int32_t)sizeof(kgpu_node_term_desc), (int32_t)sizeof(kgpu_pref_node_term_desc),
                        (int32_t)sizeof(kgpu_pod_term_desc), (int32_t)sizeof(kgpu_toleration_desc),
                        (int32_t)sizeof(kgpu_spread_desc), (int32_t)sizeof(kgpu_port_desc),
                        (int32_t)sizeof(kgpu_container_desc), (int32_t)sizeof(kgpu_pod_desc),
                        (int32_t)sizeof(kgpu_taint_desc), (int32_t)sizeof(kgpu_image_desc),
                        (int32_t)sizeof(kgpu_avoid_desc), (int32_t)sizeof(kgpu_node_desc),
                        (int32_t)sizeof(kgpu_default_spread), (int32_t)sizeof(kgpu_compile_profile),
                        (int32_t)sizeof(kgpu_key_meta), (int32_t)sizeof(kgpu_node_lists)};
  const int32_t m = (int32_t)(sizeof(sz) / sizeof(sz[0]));
  for (int32_t i = 0; i < m && i < n; ++i) out[i] = sz[i];
  return m;
}

int kgpu_compiler_destroy(kgpu_compiler* cc) {
  delete cc;
  return KGPU_OK;
}

const char* kgpu_compiler_last_error(const kgpu_compiler* cc) { return cc ? cc->err.c_str() : "no compiler"; }

int32_t kgpu_dict_add(kgpu_compiler* cc, int32_t d, int32_t key, const kgpu_str* parts, int32_t n_parts) {
  if (!cc || n_parts < 1 || !parts) return KGPU_E_INVAL;
  KC_TRY
  if (d == KGPU_DICT_TAINT) {
    if (n_parts != 3) return KGPU_E_INVAL;
    return cc->taint_add(S(parts[0]), S(parts[1]), S(parts[2]));
  }
  if (d == KGPU_DICT_NODE_VALUE || d == KGPU_DICT_POD_VALUE) {
    KeySpace& ks = d == KGPU_DICT_NODE_VALUE ? cc->nkeys : cc->pkeys;
    if (key < 0 || key >= ks.keys.size()) return KGPU_E_INVAL;
    return ks.vals[(size_t)key].add(S(parts[0]));
  }
  if (d == KGPU_DICT_NODE_KEY) return cc->nkeys.add_key(S(parts[0]));
  if (d == KGPU_DICT_POD_KEY) return cc->pkeys.add_key(S(parts[0]));
  StrDict* sd = cc->dict(d, key, true);
  if (!sd) return KGPU_E_INVAL;
  if (d == KGPU_DICT_CONTROLLER) {
    if (n_parts != 2) return KGPU_E_INVAL;
    return sd->add(join2(S(parts[0]), S(parts[1])));
  }
  return sd->add(S(parts[0]));
  KC_CATCH(cc)
}

int32_t kgpu_dict_get(const kgpu_compiler* cc, int32_t d, int32_t key, const kgpu_str* parts, int32_t n_parts) {
  if (!cc || n_parts < 1 || !parts) return -1;
  try {
    const StrDict* sd = const_cast<kgpu_compiler*>(cc)->dict(d, key, false);
    if (!sd) return -1;
    if (d == KGPU_DICT_TAINT) return n_parts == 3 ? sd->get(join3(S(parts[0]), S(parts[1]), S(parts[2]))) : -1;
    if (d == KGPU_DICT_CONTROLLER) return n_parts == 2 ? sd->get(join2(S(parts[0]), S(parts[1]))) : -1;
    return sd->get(S(parts[0]));
  } catch (...) {
    return -1;
  }
}

int32_t kgpu_dict_size(const kgpu_compiler* cc, int32_t d, int32_t key) {
  if (!cc) return KGPU_E_INVAL;
  const StrDict* sd = const_cast<kgpu_compiler*>(cc)->dict(d, key, false);
  return sd ? sd->size() : 0;
}

int64_t kgpu_dict_item(const kgpu_compiler* cc, int32_t d, int32_t key, int32_t id, char* buf, int64_t len) {
  if (!cc) return KGPU_E_INVAL;
  const StrDict* sd = const_cast<kgpu_compiler*>(cc)->dict(d, key, false);
  if (!sd || id < 0 || id >= sd->size()) return KGPU_E_INVAL;
  const string& s = sd->items[(size_t)id];
  if (buf && len >= (int64_t)s.size()) std::memcpy(buf, s.data(), s.size());
  return (int64_t)s.size();
}

int kgpu_dict_add_many(kgpu_compiler* cc, int32_t d, int32_t key, const char* chars, const int64_t* offsets, int32_t n,
                       int32_t* ids_out) {
  if (!cc || n < 0 || (n > 0 && (!chars || !offsets))) return KGPU_E_INVAL;
  if (d == KGPU_DICT_TAINT || d == KGPU_DICT_CONTROLLER) return KGPU_E_INVAL;
  KC_TRY
  for (int32_t i = 0; i < n; ++i) {
    const kgpu_str s{chars + offsets[i], offsets[i + 1] - offsets[i]};
    const int32_t id = kgpu_dict_add(cc, d, key, &s, 1);
    if (id < 0) return id;
    if (ids_out) ids_out[i] = id;
  }
  return KGPU_OK;
  KC_CATCH(cc)
}

int kgpu_compiler_register_node(kgpu_compiler* cc, const kgpu_node_desc* n) {
  if (!cc || !n) return KGPU_E_INVAL;
  KC_TRY
  cc->register_node(*n);
  return KGPU_OK;
  KC_CATCH(cc)
}

int kgpu_compiler_register_pod(kgpu_compiler* cc, const kgpu_pod_desc* p) {
  if (!cc || !p) return KGPU_E_INVAL;
  KC_TRY
  cc->register_pod(*p);
  return KGPU_OK;
  KC_CATCH(cc)
}

int kgpu_compiler_set_order(kgpu_compiler* cc, const char* chars, const int64_t* offsets, int32_t n, int32_t first_wins) {
  if (!cc || n < 0 || (n > 0 && (!chars || !offsets))) return KGPU_E_INVAL;
  KC_TRY
  vector<string> names;
  names.reserve((size_t)n);
  for (int32_t i = 0; i < n; ++i) names.emplace_back(chars + offsets[i], (size_t)(offsets[i + 1] - offsets[i]));
  cc->set_order(std::move(names), first_wins != 0);
  return KGPU_OK;
  KC_CATCH(cc)
}

int kgpu_compiler_dims(const kgpu_compiler* cc, int32_t out[3]) {
  if (!cc || !out) return KGPU_E_INVAL;
  for (int k = 0; k < 3; ++k) out[k] = cc->dims[k];
  return KGPU_OK;
}

int kgpu_pools_create(kgpu_pool_set** out) {
  if (!out) return KGPU_E_INVAL;
  try {
    *out = new kgpu_pool_set();
    return KGPU_OK;
  } catch (...) {
    *out = nullptr;
    return KGPU_E_NOMEM;
  }
}

int kgpu_pools_destroy(kgpu_pool_set* ps) {
  delete ps;
  return KGPU_OK;
}

int kgpu_pools_view(const kgpu_pool_set* ps, kgpu_pools* out) {
  if (!ps || !out) return KGPU_E_INVAL;
  kgpu_compiler::kgpu_pools_view_of(*ps, *out);
  return KGPU_OK;
}

int kgpu_pools_scalar_name(const kgpu_pool_set* ps, int32_t i, kgpu_str* out) {
  if (!ps || !out || i < 0 || (size_t)i >= ps->scalar_names.size()) return KGPU_E_INVAL;
  out->p = ps->scalar_names[(size_t)i].data();
  out->n = (int64_t)ps->scalar_names[(size_t)i].size();
  return KGPU_OK;
}

int kgpu_compile_pod(kgpu_compiler* cc, kgpu_pool_set* ps, const kgpu_pod_desc* pod, kgpu_pod_query* out) {
  if (!cc || !ps || !pod || !out) return KGPU_E_INVAL;
  KC_TRY
  cc->compile_pod(*ps, *pod, *out);
  return KGPU_OK;
  KC_CATCH(cc)
}

int kgpu_compile_pods(kgpu_compiler* cc, kgpu_pool_set* ps, const kgpu_pod_desc* pods, int32_t n, kgpu_pod_query* out,
                      int32_t* status) {
  if (!cc || !ps || n < 0 || (n > 0 && (!pods || !out || !status))) return KGPU_E_INVAL;
  int failures = 0;
  for (int32_t i = 0; i < n; ++i) {
    status[i] = kgpu_compile_pod(cc, ps, &pods[i], &out[i]);
    if (status[i] != KGPU_OK) {
      std::memset(&out[i], 0, sizeof(kgpu_pod_query));
      if (status[i] == KGPU_E_NOMEM) return KGPU_E_NOMEM;
      ++failures;
    }
  }
  return failures;
}

int kgpu_compile_snapshot(kgpu_compiler* cc, const kgpu_node_desc* nodes, int32_t n_nodes, const kgpu_pod_desc* existing,
                          int32_t n_existing, const int64_t* uids, int32_t shard_base, int32_t shard_count,
                          kgpu_snapshot* out) {
  if (!cc || !out || n_nodes < 0 || n_existing < 0 || (n_nodes > 0 && !nodes) || (n_existing > 0 && !existing))
    return KGPU_E_INVAL;
  if (shard_count >= 0 && (shard_base < 0 || shard_base + shard_count > n_nodes)) return KGPU_E_INVAL;
  KC_TRY
  vector<string> names;
  names.reserve((size_t)n_nodes);
  for (int32_t i = 0; i < n_nodes; ++i) names.push_back(S(nodes[i].name));
  cc->set_order(std::move(names), false);
  SnapBuf* b = new SnapBuf();
  delete cc->snap;
  cc->snap = b;
  cc->node_columns(*b, nodes, n_nodes);
  cc->finish(*b, existing, n_existing, uids, shard_base, shard_count, *out);
  return KGPU_OK;
  KC_CATCH(cc)
}

int kgpu_compile_snapshot_columns(kgpu_compiler* cc, const kgpu_snapshot* c, const kgpu_pod_desc* existing,
                                  int32_t n_existing, const int64_t* uids, int32_t shard_base, int32_t shard_count,
                                  kgpu_snapshot* out) {
  if (!cc || !c || !out || n_existing < 0 || (n_existing > 0 && !existing)) return KGPU_E_INVAL;
  const int32_t N = c->n_nodes;
  if (N < 0 || (size_t)N != cc->order.size()) return fail(cc, KGPU_E_INVAL, "columns and node order differ in length");
  if (c->n_scalar != cc->scalars.size() || c->n_label_keys != cc->nkeys.keys.size() ||
      c->taint_words != cc->taint_words())
    return fail(cc, KGPU_E_INVAL, "column counts differ from the dictionaries");
  if (shard_count >= 0 && (shard_base < 0 || shard_base + shard_count > N)) return KGPU_E_INVAL;
  KC_TRY
  SnapBuf* b = new SnapBuf();
  delete cc->snap;
  cc->snap = b;
  const size_t n = (size_t)N;
  auto take = [n](auto& dst, const auto* src, size_t rows) {
    if (src) dst.assign(src, src + rows * n);
  };
  cc->empty_columns(*b, n);
  take(b->alloc_cpu, c->alloc_cpu, 1);
  take(b->alloc_mem, c->alloc_mem, 1);
  take(b->alloc_eph, c->alloc_eph, 1);
  take(b->alloc_pods, c->alloc_pods, 1);
  take(b->unschedulable, c->unschedulable, 1);
  take(b->zone_id, c->zone_id, 1);
  take(b->alloc_scalar, c->alloc_scalar, (size_t)c->n_scalar);
  take(b->label_val, c->label_val, (size_t)c->n_label_keys);
  take(b->taint_nosched, c->taint_nosched, (size_t)c->taint_words);
  take(b->taint_prefer, c->taint_prefer, (size_t)c->taint_words);
  if (c->image_off) {
    b->image_off.assign(c->image_off, c->image_off + n + 1);
    b->image_id.assign(c->image_id, c->image_id + b->image_off[n]);
    b->image_score.assign(c->image_score, c->image_score + b->image_off[n]);
  } else {
    b->image_off.assign(n + 1, 0);
  }
  if (c->avoid_off) {
    b->avoid_off.assign(c->avoid_off, c->avoid_off + n + 1);
    b->avoid_id.assign(c->avoid_id, c->avoid_id + b->avoid_off[n]);
  } else {
    b->avoid_off.assign(n + 1, 0);
  }
  cc->finish(*b, existing, n_existing, uids, shard_base, shard_count, *out);
  return KGPU_OK;
  KC_CATCH(cc)
}

int kgpu_compile_node_row(kgpu_compiler* cc, kgpu_pool_set* ps, const kgpu_node_desc* node, kgpu_node_row* out) {
  if (!cc || !ps || !node || !out) return KGPU_E_INVAL;
  KC_TRY
  cc->node_row(*ps, *node, *out);
  return KGPU_OK;
  KC_CATCH(cc)
}

int kgpu_compiler_key_meta(kgpu_compiler* cc, kgpu_key_meta* out) {
  if (!cc || !out) return KGPU_E_INVAL;
  KC_TRY
  const int32_t K = cc->dims[1];
  cc->key_meta_into(K, cc->km_knv, cc->km_off, cc->km_int, cc->km_ok, cc->km_empty);
  out->n_keys = K;
  out->n_values = (int32_t)cc->km_int.size();
  out->key_n_values = ptr_or_null(cc->km_knv);
  out->value_off = cc->km_off.data();
  out->value_int = ptr_or_null(cc->km_int);
  out->value_int_ok = ptr_or_null(cc->km_ok);
  out->key_empty_value = ptr_or_null(cc->km_empty);
  return KGPU_OK;
  KC_CATCH(cc)
}

int kgpu_compile_node_lists(kgpu_compiler* cc, const kgpu_node_desc* list, int32_t n_list, const kgpu_node_desc* all,
                            int32_t n_all, kgpu_node_lists* out) {
  if (!cc || !out || n_list < 0 || n_all < 0 || (n_list > 0 && !list) || (n_all > 0 && !all)) return KGPU_E_INVAL;
  KC_TRY
  cc->lists(list, n_list, all, n_all, true, cc->nl_image_off, cc->nl_image_id, cc->nl_image_score, cc->nl_avoid_off,
            cc->nl_avoid_id);
  out->n_nodes = n_list;
  out->n_images = (int32_t)cc->nl_image_id.size();
  out->n_avoid = (int32_t)cc->nl_avoid_id.size();
  out->pad = 0;
  out->image_off = cc->nl_image_off.data();
  out->image_id = ptr_or_null(cc->nl_image_id);
  out->image_score = ptr_or_null(cc->nl_image_score);
  out->avoid_off = cc->nl_avoid_off.data();
  out->avoid_id = ptr_or_null(cc->nl_avoid_id);
  return KGPU_OK;
  KC_CATCH(cc)
}

}  // extern "C"
